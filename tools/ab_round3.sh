#!/bin/bash
# round-2 late A/B: shade grid (env knob on the default lib) and tail refill (lib variants), C3 / shard-of 8 / C2
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/ab.sh > gpurun_out/tr_c3.txt 2>&1 &&
BENCH_ARGS="--shard-of 8" bash tools/ab.sh > gpurun_out/tr_s8.txt 2>&1 &&
bash tools/ab_env.sh RTG_SHADE_GRID=0 RTG_SHADE_GRID=1 RTG_SHADE_GRID=4 > gpurun_out/sg_c3.txt 2>&1 &&
BENCH_ARGS="--shard-of 8" bash tools/ab_env.sh RTG_SHADE_GRID=0 RTG_SHADE_GRID=1 > gpurun_out/sg_s8.txt 2>&1
