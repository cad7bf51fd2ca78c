#!/bin/bash
# side measurements of the other BASELINE configs (C3 is the headline bench line)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for args in "--config C2 --steps 20 --warmup 2" "--config C4 --steps 1 --warmup 1" "--config C5 --spp 32 --steps 1 --warmup 1"; do
  timeout -k 10 400 python bench.py --no-cpu-baseline $args > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
  tail -1 gpurun_out/cfg.log >> gpurun_out/configs.jsonl
  tail -1 gpurun_out/cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['value'], d['unit'], d['ms_per_step'], 'ms/step', d['rays_per_path'], 'rays/path', d['kernel_ms_per_step_rank0'])"
done
