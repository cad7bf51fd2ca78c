#!/bin/bash
# Round 6 session 2, pass 2: the GPU suite and smoke on the PEND2 build, then a refill / fetch re-check
# at 7 waves (lib/ab: b_pend2 = the product, r8 / r16 refill thresholds, f128 fetch batch).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r06b_gputest_pend2.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/r06b_gputest_pend2.log; exit 1; }
tail -1 gpurun_out/r06b_gputest_pend2.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06b_smoke_pend2.log 2>&1 \
  || { echo "smoke failed"; cat gpurun_out/r06b_smoke_pend2.log; exit 1; }
cat gpurun_out/r06b_smoke_pend2.log
CFGS="${CFGS:-C3 S8}" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/ab_refill.txt 2>&1; rc=$?; cat gpurun_out/ab_refill.txt; exit $rc
