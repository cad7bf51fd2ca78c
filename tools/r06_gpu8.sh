#!/bin/bash
# Round 6, eighth GPU pass: more traversal waves per SIMD (7 with a 20-entry LDS stack, 8 with 16) A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06h; mkdir -p $O
AB_SETS="--steps 10;--steps 40 --shard-of 8;--config C4 --spp 64 --steps 1;--config C2 --steps 20" bash tools/ab_leaf.sh 2>&1 | tee $O/ab_waves.txt
