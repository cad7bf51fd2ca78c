#!/bin/bash
# Round 6 (late): C5 at 1024 spp with the 50 % / 60 % chunk memory budgets, with and without a warm-up
# step (a first step includes the chunk buffers' allocation).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for w in 0 1; do for lib in a_mem50 b_mem60; do
  RTG_LIB=$R/raytracingrenderer_amd/lib/ab/$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --config C5 --spp 1024 --steps 1 --warmup $w > gpurun_out/c5a.log 2> gpurun_out/c5a.err || { tail -5 gpurun_out/c5a.err; exit 1; }
  echo "warmup=$w $lib $(tail -1 gpurun_out/c5a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], d['config'].get('chunk_spp'))")"
done; done
