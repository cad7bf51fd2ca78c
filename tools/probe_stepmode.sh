#!/bin/bash
# bench.py --step-mode full / lean / pipe on shard-of 8 and C3, two interleaved rounds
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for round in 1 2; do for cfg in "--shard-of 8 --steps 30 --warmup 3" "--config C3 --steps 10 --warmup 2"; do for m in ${MODES:-full lean pipe}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 $cfg --step-mode $m > gpurun_out/sm.log 2> gpurun_out/sm.err || { tail -5 gpurun_out/sm.err; exit 1; }
  echo "$cfg $m $(tail -1 gpurun_out/sm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], d['config'].get('chunk_spp'))")"
done; done; done
