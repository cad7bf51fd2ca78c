#!/bin/bash
# Tail-mode subtree donation (RTG_STEAL build in lib/ab/b_steal.so): GPU parity suite with it, then
# C3 at shard-of 8 and 1 against the default build (lib/ab/a_base.so), two rounds
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
RTG_LIB=$R/raytracingrenderer_amd/lib/ab/b_steal.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/steal_pytest.log 2>&1 || { tail -30 gpurun_out/steal_pytest.log; exit 1; }
tail -1 gpurun_out/steal_pytest.log
for round in 1 2; do for sh in 8 1; do for lib in a_base b_steal; do
  RTG_LIB=$R/raytracingrenderer_amd/lib/ab/$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --shard-of $sh > gpurun_out/st.log 2>&1 || { tail -5 gpurun_out/st.log; exit 1; }
  echo "shard-of $sh $lib $(tail -1 gpurun_out/st.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done; done; done
