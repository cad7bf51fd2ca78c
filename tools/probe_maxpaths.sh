#!/bin/bash
# C3 with the render cut into pipelined chunks (--max-paths): default (one 64M-path chunk) vs 16M / 8M
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for round in 1 2; do for mp in 0 16777216 8388608; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --config C3 --steps 10 --warmup 4 --max-paths $mp > gpurun_out/mp.log 2> gpurun_out/mp.err || { tail -5 gpurun_out/mp.err; exit 1; }
  echo "C3 max_paths=$mp $(tail -1 gpurun_out/mp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], d['config'].get('chunk_spp'))")"
done; done
