#!/bin/bash
# GPU parity suite against one A/B variant (RTG_LIB), then the interleaved A/B bench (tools/ab.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
if [ -n "$ABT_LIB" ]; then
  RTG_LIB=$R/raytracingrenderer_amd/lib/ab/$ABT_LIB.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_pytest.log 2>&1 || { tail -30 gpurun_out/abt_pytest.log; exit 1; }
  tail -1 gpurun_out/abt_pytest.log
fi
bash tools/ab.sh
