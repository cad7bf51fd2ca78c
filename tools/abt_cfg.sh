#!/bin/bash
# GPU parity suite against one A/B variant (ABT_LIB), then A/B bench on C3 and C2 (interleaved, 2 rounds)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
if [ -n "$ABT_LIB" ]; then
  RTG_LIB=$R/raytracingrenderer_amd/lib/ab/$ABT_LIB.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_pytest.log 2>&1 || { tail -30 gpurun_out/abt_pytest.log; exit 1; }
  tail -1 gpurun_out/abt_pytest.log
fi
for cfg in ${CFGS:-C3 C2}; do for round in 1 2; do for lib in raytracingrenderer_amd/lib/ab/*.so; do
  RTG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config $cfg --steps 3 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "$cfg $(basename $lib) $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms_per_step_rank0'])")"
done; done; done
