#!/bin/bash
# Round 6, seventh GPU pass: queue entries sorted by ray direction octant (RTG_SORT_OCT) A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06g; mkdir -p $O
AB_SETS="--steps 10;--steps 40 --shard-of 8;--config C4 --spp 64 --steps 1;--config C5 --spp 32 --steps 1" bash tools/ab_leaf.sh 2>&1 | tee $O/ab_sortoct.txt
