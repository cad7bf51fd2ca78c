#!/bin/bash
# A/B of lib variants at simulated world sizes (bench --shard-of N): per-GPU rate
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for n in ${SHARDS:-1 8}; do for lib in raytracingrenderer_amd/lib/ab/*.so; do
  RTG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --shard-of $n > gpurun_out/abs.log 2>&1 || { tail -5 gpurun_out/abs.log; exit 1; }
  echo "N=$n $(basename $lib) $(tail -1 gpurun_out/abs.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done; done
