#!/bin/bash
# A/B of environment knobs over the side configs (C2, C4, C5 at 32 spp): ab_cfg_env.sh "RTG_X=0" "RTG_X=1" ...
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for args in "--config C2 --steps 2" "--config C4 --steps 1 --warmup 1" "--config C5 --spp 32 --steps 1 --warmup 1"; do
for kv in "$@"; do
  env $kv timeout -k 10 400 python bench.py --no-cpu-baseline $args > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
  echo "$kv $(tail -1 gpurun_out/cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done; done
