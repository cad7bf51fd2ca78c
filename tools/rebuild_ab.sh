#!/bin/bash
# Wide tree cut from the reference BVH2 (RTG_REBUILD=0) vs an own 3-axis SAH tree over the reference
# leaves (RTG_REBUILD=1): parity suite with the rebuilt tree, then C3 (and $CFGS) benches alternated
R=$GRAFT_REPO_ROOT; cd $R
RTG_REBUILD=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rb_pytest.log 2>&1 || { tail -30 gpurun_out/rb_pytest.log; exit 1; }
tail -1 gpurun_out/rb_pytest.log
for round in 1 2; do
for cfg in "" $CFGS; do
for v in 0 1; do
  RTG_REBUILD=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 ${cfg:+--config $cfg} > gpurun_out/rb.log 2>&1 || { tail -5 gpurun_out/rb.log; exit 1; }
  echo "cfg=${cfg:-C3} rebuild=$v $(tail -1 gpurun_out/rb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['kernel_ms_per_step_rank0'], 'setup', d.get('setup_s'), 'slots', r.get('walk_box_tests_per_ray'), 'tris', r.get('walk_tri_tests_per_ray'), 'pops', r.get('pops_per_ray'))")"
done; done; done
