#!/bin/bash
# per-launch wave start/end percentiles (RTG_WAVETIME build in lib/ab/wt.so) at shard-of 1 and 8
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for n in 1 8; do
  RTG_LIB=$R/raytracingrenderer_amd/lib/ab/wt.so RTG_WAVETIME=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --shard-of $n > gpurun_out/wt$n.log 2>&1 || { tail -5 gpurun_out/wt$n.log; exit 1; }
  echo "== shard-of $n"; grep wavetime gpurun_out/wt$n.log | tail -7
done
