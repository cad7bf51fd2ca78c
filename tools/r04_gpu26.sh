# the default bench line on the final build (profiles/r04_bench.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -5 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log > gpurun_out/r04_bench_final.json
python3 -c "import json; d=json.load(open('gpurun_out/r04_bench_final.json')); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], d['dropin']['queued'], d['cpu_baseline']['value'])"
