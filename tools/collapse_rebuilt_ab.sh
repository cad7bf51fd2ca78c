R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "tree_source or wide_walk" > gpurun_out/ts.log 2>&1 || { tail -30 gpurun_out/ts.log; exit 1; }
tail -1 gpurun_out/ts.log
for cfg in C3 C4 C2; do for v in "greedy 0.6 4" "dp 0.6 2" "dp 1.0 4"; do
  set -- $v
  RTG_COLLAPSE=$1 RTG_DP_CTRI=$2 RTG_DP_LEAF=$3 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --config $cfg > gpurun_out/col.log 2>&1 || { tail -5 gpurun_out/col.log; exit 1; }
  echo "$cfg $v $(tail -1 gpurun_out/col.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['kernel_ms_per_step_rank0'], 'slots', r['walk_box_tests_per_ray'], 'tris', r['walk_tri_tests_per_ray'], 'pops', r['pops_per_ray'])")"
done; done
