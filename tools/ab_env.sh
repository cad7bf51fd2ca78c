#!/bin/bash
# A/B of environment knobs on one build: ab_env.sh "RTG_X=0" "RTG_X=1" ... (interleaved, 2 rounds)
# BENCH_ARGS adds bench.py arguments (e.g. "--config C2").
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for round in 1 2; do
for kv in "$@"; do
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 $BENCH_ARGS > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "$kv $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['kernel_ms_per_step_rank0'], 'fetch/ray', r['fetches_per_ray'], 'frac', r['frac'], 'nsteps/ray', r['node_steps_per_ray'], 'pops', r['pops_per_ray'], 'cullable', r['cullable_pops_per_ray'])")"
done; done
