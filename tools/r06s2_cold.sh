#!/bin/bash
# Round 6 (late): the traversal's cold operands through one pointer (RTG_TRACE_COLD) at 7 and 8 waves
# per SIMD (lib/ab: a_prod, b_cold7, c_cold8), then the GPU parity suite on c_cold8.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CFGS="${CFGS:-C3 S8 C4}" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/ab_cold.txt 2>&1 || { cat gpurun_out/ab_cold.txt; exit 1; }
cat gpurun_out/ab_cold.txt
RTG_LIB=$R/raytracingrenderer_amd/lib/ab/c_cold8.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "not build_ids and not kernel_resources" > gpurun_out/r06b_gputest_cold8.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/r06b_gputest_cold8.log; exit 1; }
tail -1 gpurun_out/r06b_gputest_cold8.log
