#!/bin/bash
# A/B of the lib variants in raytracingrenderer_amd/lib/ab over several configs, 2 interleaved rounds:
# C3 (headline), C2, C4 at 64 spp, C5 at 32 spp, S8 / S4 / S2 (rank 0's C3 share at 8 / 4 / 2 ranks). Prints value and kernel ms per step.
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
CFGS=${CFGS:-"C3 C2 C4 C5"}
for round in 1 2; do
for cfg in $CFGS; do
for lib in raytracingrenderer_amd/lib/ab/*.so; do
  case $cfg in
    C3) args="--config C3 --steps 10 --warmup ${C3_WARMUP:-2}";;
    C2) args="--config C2 --steps 20 --warmup 2";;
    C4) args="--config C4 --spp 64 --steps 2 --warmup 1";;
    C5) args="--config C5 --spp 32 --steps 2 --warmup 1";;
    S8) args="--shard-of 8 --steps 30 --warmup 3";;
    S2) args="--shard-of 2 --steps 10 --warmup 4";;
    S4) args="--shard-of 4 --steps 20 --warmup 2";;
  esac
  RTG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 $args > gpurun_out/ab.log 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  echo "$cfg $(basename $lib) $(tail -1 gpurun_out/ab.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], 'fetch/ray', r['fetches']['per_ray'], 'node', r['node_steps_per_ray'], 'tri', r['walk_tri_tests_per_ray'], 'util', r['lane_util_node_leaf'])")"
done; done; done
