#!/bin/bash
# Round 6 (late): a third parked-leaf slot (lib/ab: a_prod, b_pend3), then the GPU parity suite on b_pend3.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CFGS="${CFGS:-C3 S8 C4 C5}" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/ab_pend3.txt 2>&1 || { cat gpurun_out/ab_pend3.txt; exit 1; }
cat gpurun_out/ab_pend3.txt
RTG_LIB=$R/raytracingrenderer_amd/lib/ab/b_pend3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "not build_ids" > gpurun_out/r06b_gputest_pend3.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/r06b_gputest_pend3.log; exit 1; }
tail -1 gpurun_out/r06b_gputest_pend3.log
