#!/bin/bash
# Round 6 (session 2): k_trace register layout / waves-per-SIMD A/B (lib/ab variants from tools/mkab.sh)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CFGS="${CFGS:-C3 S8}" timeout -k 10 1100 bash tools/ab_cfg.sh > gpurun_out/ab_w7.txt 2>&1; rc=$?; cat gpurun_out/ab_w7.txt; exit $rc
