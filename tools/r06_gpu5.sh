#!/bin/bash
# Round 6, fifth GPU pass: the GPU suite on the product (small-scene image without leaf boxes), then
# the camera-launch grid and the small-scene pop-park A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
AB_SETS="--steps 40 --shard-of 8;--config C2 --steps 20;--steps 10" bash tools/ab_leaf.sh 2>&1 | tee $O/ab_cam.txt
