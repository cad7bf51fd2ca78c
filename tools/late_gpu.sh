#!/bin/bash
# shard sweep (per-GPU rate at N = 1, 2, 4, 8) and C5 at full size through the native CLI group path
# (the 4096^2 result_1024.hdr stays in /tmp on the box; the PNG and the log come back)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out /tmp/c5
bash tools/shard_sweep.sh > gpurun_out/shard_sweep.txt 2>&1 &&
cd /tmp/c5 && timeout -k 10 120 $R/raytracingrenderer_amd/lib/rtg_render -scene $R/assets/coffee -envmap GI.hdr \
  -width 4096 -height 4096 -skipMissing 1 -SPP 1024 -gpus 1 -batch 1024 -timeLimit 0 -outputFilename c5.png > $R/gpurun_out/c5_full_cli.log 2>&1 &&
md5sum result_1024.hdr >> $R/gpurun_out/c5_full_cli.log && cp c5.png $R/gpurun_out/c5_full.png
