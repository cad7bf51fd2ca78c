#!/bin/bash
# paths-in-flight sweep (chunk size) on the C3 bench
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for mp in 1048576 4194304 16777216 67108864; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --max-paths $mp > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  echo "$mp $(tail -1 gpurun_out/sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms_per_step_rank0'])")"
done
