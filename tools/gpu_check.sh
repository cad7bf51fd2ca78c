#!/bin/bash
# One GPU call: the -m gpu suite, smoke() (build ids + bit-exact film), the default bench line, the
# shard-of-8 line (with the rehearsed film exchange) and the 8-rank group rehearsal on one GPU.
# Every step has its own time limit and the chain stops at the first failure.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TAG=${TAG:-r05}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -3 gpurun_out/${TAG}_gputest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  || { echo "smoke failed"; cat gpurun_out/${TAG}_smoke.log; exit 1; }
cat gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['mrays_reference_equivalent_per_s'], d['kernel_ms_per_step_rank0'], d['roofline']['frac'])"
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --shard-of 8 > gpurun_out/${TAG}_shard8.json 2> gpurun_out/${TAG}_shard8.err \
  || { echo "shard8 failed"; tail -20 gpurun_out/${TAG}_shard8.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_shard8.json').read().strip().splitlines()[-1]); print('shard8', d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], d['shard_exchange'])"
if [ -z "$NO_GROUP" ]; then
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --devices 0,0,0,0,0,0,0,0 --verify-film > gpurun_out/${TAG}_group8.json 2> gpurun_out/${TAG}_group8.err \
  || { echo "group8 failed"; tail -20 gpurun_out/${TAG}_group8.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_group8.json').read().strip().splitlines()[-1]); print('group8', d['value'], d.get('film_reduce_bit_exact'), d['group']['reduce_ms_per_step'], d['group']['rank_render_ms'])"
fi
