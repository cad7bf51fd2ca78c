#!/bin/bash
# parity of the last variant in lib/ab (GPU parity + north-star suites), then the config A/B (CFGS)
cd $GRAFT_REPO_ROOT
LAST=$(ls raytracingrenderer_amd/lib/ab/*.so | tail -1)
RTG_LIB=$PWD/$LAST timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_north_star.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || { echo PARITY FAIL; tail -30 gpurun_out/ab_parity.log; exit 1; }
echo "parity $LAST: $(tail -1 gpurun_out/ab_parity.log)"
CFGS=${CFGS:-"C3 S8 C4"} timeout -k 10 900 bash tools/ab_cfg.sh
