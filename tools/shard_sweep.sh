#!/bin/bash
# per-GPU rate when the C3 frame is split over N ranks (rank 0's tiles rendered alone), with the film
# exchange a rank of N adds (shard_exchange: pack + scatter measured, the RCCL transfer modelled)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for n in 1 2 4 8; do
  # 10 x N steps: about the same wall time at every N (at N >= 4 the frames run in the pipeline,
  # whose first and last frames have no neighbour to overlap)
  timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --steps $((10 * n)) --shard-of $n > gpurun_out/sh.log 2>&1 || { tail -5 gpurun_out/sh.log; exit 1; }
  echo "N=$n $(tail -1 gpurun_out/sh.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); x=d.get('shard_exchange') or {}
print(d['value'], 'x', '$n', '=', round(d['value']*$n), 'ms/step', d['ms_per_step'], d['kernel_ms_per_step_rank0'], 'exchange_ms', x.get('total_ms'), 'job_ms', x.get('projected_job_ms_per_step'))")"
done
