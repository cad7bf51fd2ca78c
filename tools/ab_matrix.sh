#!/bin/bash
# A/B matrix: every lib in raytracingrenderer_amd/lib/ab x every bench.py flag set in AB_FLAGS ('|'-separated,
# an empty entry = defaults) x every workload in AB_SETS (';'-separated), interleaved, 2 rounds.
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
IFS=';' read -ra SETS <<< "${AB_SETS:---steps 20;--steps 40 --shard-of 8;--config C2 --steps 40}"
IFS='|' read -ra FLAGS <<< "${AB_FLAGS:-}"
[ ${#FLAGS[@]} -eq 0 ] && FLAGS=("")
for set in "${SETS[@]}"; do
for round in 1 2; do
for lib in raytracingrenderer_amd/lib/ab/*.so; do
for f in "${FLAGS[@]}"; do
  RTG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline $set $f > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "[$set] $(basename $lib) ${f:-default} $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done; done; done; done
