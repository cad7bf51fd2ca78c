#!/bin/bash
# default lib with and without the slice counters (RTG_FETCH8 env) at 1 and 8 simulated ranks
R=$GRAFT_REPO_ROOT; cd $R
for n in 1 8; do for f in 1 0 1 0; do
  RTG_FETCH8=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --shard-of $n > gpurun_out/f8.log 2>&1 || { tail -5 gpurun_out/f8.log; exit 1; }
  echo "N=$n fetch8=$f $(tail -1 gpurun_out/f8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms_per_step_rank0'])")"
done; done
