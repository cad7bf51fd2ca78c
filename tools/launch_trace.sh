#!/bin/bash
# rocprofv3 kernel trace of bench.py at the given simulated rank counts (per-launch timeline)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/lt; cd /tmp && export TMPDIR=/tmp
for n in ${LT_SHARDS:-1 8}; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/lt/n$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1 --shard-of $n > $GRAFT_REPO_ROOT/gpurun_out/lt/b$n.log 2>&1 || exit 1
done
