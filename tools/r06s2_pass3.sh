#!/bin/bash
# Round 6 session 2, pass 3: GPU suite + smoke with the grouped contribution fold, then its A/B
# (lib/ab: a_u12 = the product, b_u1 = one plane per group as before, c_u6).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r06b_gputest_fold.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/r06b_gputest_fold.log; exit 1; }
tail -1 gpurun_out/r06b_gputest_fold.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06b_smoke_fold.log 2>&1 \
  || { echo "smoke failed"; cat gpurun_out/r06b_smoke_fold.log; exit 1; }
cat gpurun_out/r06b_smoke_fold.log
CFGS="${CFGS:-C2 C3 C5}" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/ab_fold.txt 2>&1; rc=$?; cat gpurun_out/ab_fold.txt; exit $rc
