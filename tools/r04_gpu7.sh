# chunk splitting through the pipeline (timing events no longer force one chunk at a time)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for round in 1 2; do
for mp in 0 33554432 16777216; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --steps 10 --warmup 2 --max-paths $mp > gpurun_out/ab.log 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  echo "N1 mp=$mp $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done
for mp in 0 4194304 3000000 2097152; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --steps 40 --warmup 3 --shard-of 8 --max-paths $mp > gpurun_out/ab.log 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  echo "S8 mp=$mp $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done; done
