#!/bin/bash
# Round 6 A/B of the traversal's leaf handling (RTG_LEAF_MINWALK, RTG_LEAF_SWAP): every lib in
# raytracingrenderer_amd/lib/ab x every workload in AB_SETS, interleaved, 2 rounds; prints traced
# Mray/s, ms/step, kernel ms and the counting pass's lane utilisation / idle reasons.
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
IFS=';' read -ra SETS <<< "${AB_SETS:---steps 20;--steps 40 --shard-of 8;--config C4 --spp 64 --steps 1}"
for set in "${SETS[@]}"; do
for round in 1 2; do
for lib in raytracingrenderer_amd/lib/ab/*.so; do
  RTG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 $set > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "[$set] $(basename $lib) $(tail -1 gpurun_out/ab.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], 'util', r['lane_util_node_leaf'], r['lane_idle_node'], 'steps/ray', r['node_steps_per_ray'])")"
done; done; done
