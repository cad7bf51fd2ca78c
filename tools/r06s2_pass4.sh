#!/bin/bash
# Round 6 session 2, pass 4: the GPU suite (with the small-scene deep-stack case) and smoke on the final tree.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/prof_out/r06_gputest_final.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/prof_out/r06_gputest_final.log; exit 1; }
grep -c PASSED gpurun_out/prof_out/r06_gputest_final.log; grep deep_bvh gpurun_out/prof_out/r06_gputest_final.log; tail -1 gpurun_out/prof_out/r06_gputest_final.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/prof_out/r06_smoke.log 2>&1 \
  || { echo "smoke failed"; cat gpurun_out/prof_out/r06_smoke.log; exit 1; }
cat gpurun_out/prof_out/r06_smoke.log
