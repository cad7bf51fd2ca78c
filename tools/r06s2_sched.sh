#!/bin/bash
# Round 6 (late): LLVM scheduling strategies for the traversal's unit at 7 waves (lib/ab: a_prod, b_ilp,
# c_memc, d_iilp).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CFGS="${CFGS:-C3 S8 C2}" timeout -k 10 1000 bash tools/ab_cfg.sh > gpurun_out/ab_sched.txt 2>&1; rc=$?; cat gpurun_out/ab_sched.txt; exit $rc
