set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "chunks or many_samples or adaptive or c3_full" > gpurun_out/r02_chunk_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r02_chunk_tests.log; exit 1; }
tail -1 gpurun_out/r02_chunk_tests.log
for args in "--config C4 --steps 1 --warmup 1" "--config C4 --steps 1 --warmup 1 --max-paths 1073741824" "--config C5 --spp 32 --steps 1 --warmup 1" "--config C5 --spp 32 --steps 1 --warmup 1 --max-paths 1073741824"; do
  timeout -k 10 400 python bench.py --no-cpu-baseline $args > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
  echo "$args: $(tail -1 gpurun_out/cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done
