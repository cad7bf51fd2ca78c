#!/bin/bash
# Round 6 session 2: GPU suite + smoke + bench + shard-of-8 on the tree, then the C4 / C5 A/B of the
# 7-wave traversal against round 6's first build (lib/ab: a_r06base, b_w7).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
NO_GROUP=1 TAG=r06s2 bash tools/gpu_check.sh || exit 1
CFGS="C4 C5" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/ab_w7_c45.txt 2>&1; rc=$?; cat gpurun_out/ab_w7_c45.txt; exit $rc
