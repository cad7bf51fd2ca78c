#!/bin/bash
# kernel trace of one timed bench step (no counting passes): per-launch durations -> gpurun_out/ktq/
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
rm -rf $R/gpurun_out/ktq
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ktq -o ktq --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 1 $* > $R/gpurun_out/ktq.log 2>&1 || { tail -20 $R/gpurun_out/ktq.log; exit 1; }
grep '^{' $R/gpurun_out/ktq.log | cut -c1-200
