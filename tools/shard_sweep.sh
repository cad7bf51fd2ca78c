#!/bin/bash
# per-GPU rate when the C3 frame is split over N ranks (rank 0's tiles rendered alone)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for n in 1 2 4 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --shard-of $n > gpurun_out/sh.log 2>&1 || { tail -5 gpurun_out/sh.log; exit 1; }
  echo "N=$n $(tail -1 gpurun_out/sh.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'x', '$n', '=', round(d['value']*$n), d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done
