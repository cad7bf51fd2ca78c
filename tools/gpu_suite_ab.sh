#!/bin/bash
# The -m gpu suite on the product build, then the config A/B of the variants in lib/ab
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${TAG:-r05}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputest.log
CFGS=${CFGS:-"C3 C4 S8"} timeout -k 10 1000 bash tools/ab_cfg.sh
