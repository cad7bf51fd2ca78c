#!/bin/bash
# A/B of the two-chunk-pipeline modes (RTG_PIPES / RTG_STAGGER) at 1 and 8 simulated ranks,
# plus the GPU parity suite with the pipelined mode on.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pab
RTG_PIPES=2 RTG_STAGGER=${PAB_STAGGER:-2} timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pab/pytest.log 2>&1 || { tail -30 gpurun_out/pab/pytest.log; exit 1; }
tail -2 gpurun_out/pab/pytest.log
for shard in ${PAB_SHARDS:-8 1}; do
for v in "1 0" "2 0" "2 1" "2 2" "1 0"; do
set -- $v
RTG_PIPES=$1 RTG_STAGGER=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --shard-of $shard > gpurun_out/pab/b.log 2>&1 || { tail -20 gpurun_out/pab/b.log; exit 1; }
echo "shard $shard pipes $1 stagger $2: $(tail -1 gpurun_out/pab/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'ms', d['ms_per_step'])")"
done; done
