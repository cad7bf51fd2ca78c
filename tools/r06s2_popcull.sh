#!/bin/bash
# Round 6 (late): pop-time distance culling A/B (lib/ab: a_prod, b_pc1 = RTG_POPCULL with one pop per
# step, c_pc2 = two), then the GPU parity suite on b_pc1 (its build id is the variant's, so the
# build-id test is deselected).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CFGS="${CFGS:-C3 S8 C4}" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/ab_popcull.txt 2>&1 || { cat gpurun_out/ab_popcull.txt; exit 1; }
cat gpurun_out/ab_popcull.txt
RTG_LIB=$R/raytracingrenderer_amd/lib/ab/b_pc1.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "not build_ids" > gpurun_out/r06b_gputest_popcull.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/r06b_gputest_popcull.log; exit 1; }
tail -1 gpurun_out/r06b_gputest_popcull.log
