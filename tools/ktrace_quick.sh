#!/bin/bash
# per-dispatch kernel times of one bench run (rocprofv3 kernel trace) -> gpurun_out/kq/
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kq -o kq --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 1 $BENCH_ARGS > $R/gpurun_out/kq.log 2>&1
