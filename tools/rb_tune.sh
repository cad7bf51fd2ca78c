#!/bin/bash
# rebuild_over_leaves knobs (RTG_RB_WEIGHT / RTG_RB_SWEEP / RTG_RB_BINS) on C3, C2, C4 (64 spp)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for cfg in "--config C3" "--config C2" "--config C4 --spp 64"; do
for v in "0 2048 64" "1 2048 64" "1 16384 64" "1 2048 256"; do
  set -- $v
  RTG_RB_WEIGHT=$1 RTG_RB_SWEEP=$2 RTG_RB_BINS=$3 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 $cfg > gpurun_out/rb.log 2>&1 || { tail -5 gpurun_out/rb.log; exit 1; }
  echo "$cfg w=$1 sweep=$2 bins=$3 $(tail -1 gpurun_out/rb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['kernel_ms_per_step_rank0']['trace'], 'setup', d.get('setup_s'), 'slots', r.get('walk_box_tests_per_ray'), 'tris', r.get('walk_tri_tests_per_ray'))")"
done; done
