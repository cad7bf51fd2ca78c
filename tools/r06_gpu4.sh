#!/bin/bash
# Round 6, fourth GPU pass: per-launch trace time and rays (C3, shard-of 8) for the tail analysis,
# and the small-scene image without leaf boxes (C2) against the product.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06d; mkdir -p $O
timeout -k 10 200 python -u tools/launch_profile.py > $O/lp1.json 2> $O/lp1.err || { tail -20 $O/lp1.err; exit 1; }
timeout -k 10 200 python -u tools/launch_profile.py --shard-of 8 > $O/lp8.json 2> $O/lp8.err || { tail -20 $O/lp8.err; exit 1; }
cat $O/lp1.json $O/lp8.json
AB_SETS="--config C2 --steps 20;--steps 10" bash tools/ab_leaf.sh 2>&1 | tee $O/ab_small.txt
