#!/bin/bash
# RTG_STEAL variants (lib/ab/*.so) at shard-of 8 and 1, two rounds
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for round in 1 2; do for sh in 8 1; do for lib in raytracingrenderer_amd/lib/ab/*.so; do
  RTG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --shard-of $sh > gpurun_out/st.log 2>&1 || { tail -5 gpurun_out/st.log; exit 1; }
  echo "shard-of $sh $(basename $lib) $(tail -1 gpurun_out/st.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done; done; done
