#!/bin/bash
# run-to-run spread of the default bench line (three runs, one box) and the shard sweep
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --dropin-frames 0 $([ $i -gt 1 ] && echo --no-cpu-baseline) > gpurun_out/rb$i.json 2> gpurun_out/rb$i.err || { tail -5 gpurun_out/rb$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rb$i.json').read().strip().splitlines()[-1]); print('run $i', d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], d['roofline']['frac'])"
done | tee gpurun_out/prof_out/r05_bench_repeats.txt
timeout -k 10 600 bash tools/shard_sweep.sh | tee gpurun_out/prof_out/r05_shard_sweep.txt
