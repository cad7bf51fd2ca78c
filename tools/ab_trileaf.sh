#!/bin/bash
# tri-leaf tree variants: wide-walk parity of the last variant, then the config A/B (tools/ab_cfg.sh)
cd $GRAFT_REPO_ROOT
LAST=$(ls raytracingrenderer_amd/lib/ab/*.so | tail -1)
RTG_LIB=$PWD/$LAST timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "wide_walk or adversarial or cull_equivalence or grazing or c3_full or synthetic or c1 or c2_shape or depths" > gpurun_out/ab_trileaf_parity.log 2>&1 || { echo PARITY FAIL; tail -30 gpurun_out/ab_trileaf_parity.log; exit 1; }
echo "parity $LAST: $(tail -1 gpurun_out/ab_trileaf_parity.log)"
CFGS=${CFGS:-"C3 C4 C2 S8"} timeout -k 10 1000 bash tools/ab_cfg.sh
