#!/bin/bash
# A/B with the walk counters: value, kernel ms, node steps / box tests / triangle tests per ray
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for round in ${AB_ROUNDS:-1 2}; do
for lib in raytracingrenderer_amd/lib/ab/*.so; do
  RTG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 $BENCH_ARGS > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "$(basename $lib) $(tail -1 gpurun_out/ab.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}
print(d['value'], d['kernel_ms_per_step_rank0'], 'steps', r.get('node_steps_per_ray'), 'box', r.get('walk_box_tests_per_ray'), 'tri', r.get('walk_tri_tests_per_ray'), 'fetch', r.get('fetches_per_ray'))")"
done; done
