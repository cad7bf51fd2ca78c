#!/bin/bash
# Round 6 (late): the default bench line three times on one box (run-to-run spread of the headline).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof_out
for i in 1 2 3; do
  timeout -k 10 400 python bench.py > gpurun_out/rep.log 2>&1 || { tail -20 gpurun_out/rep.log; exit 1; }
  tail -1 gpurun_out/rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(json.dumps({'run': $i, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'ms_per_frame': d['ms_per_frame'], 'kernel_ms_per_step_rank0': d['kernel_ms_per_step_rank0'], 'roofline_frac': d['roofline']['frac'], 'dropin_queued_ms_per_frame': d['dropin']['queued']['ms_per_frame'], 'cpu_mrays': d['cpu_baseline']['value'], 'gpu_over_cpu_ms_per_frame': d['gpu_over_cpu']['ms_per_frame']}))" | tee -a gpurun_out/prof_out/r06_bench_repeats.jsonl
done
