#!/bin/bash
# quick GPU iteration: parity subset + bench (no CPU baseline)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/quick_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/quick_pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/quick_pytest.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/quick_bench.log 2>&1 || { tail -20 gpurun_out/quick_bench.log; exit 1; }
tail -1 gpurun_out/quick_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'roof', d['roofline'])"
