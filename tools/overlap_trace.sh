#!/bin/bash
# Kernel timelines (rocprofv3 --kernel-trace, no counters) of the shard-of-8 C3 bench with one and
# with two chunk pipelines: do kernels of the two streams overlap, and where does a step's time go
# (kernel busy vs gaps)? Summarised by tools/timeline.py.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/ovl; cd /tmp; export TMPDIR=/tmp
for v in "1 0" "2 2"; do
  set -- $v
  RTG_PIPES=$1 RTG_STAGGER=$2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ovl/p$1 -o kt -- \
    python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --shard-of ${OVL_SHARD:-8} > $R/gpurun_out/ovl/p$1.log 2>&1 || { tail -20 $R/gpurun_out/ovl/p$1.log; exit 1; }
  tail -1 $R/gpurun_out/ovl/p$1.log
  python3 $R/tools/timeline.py $(find $R/gpurun_out/ovl/p$1 -name '*kernel_trace.csv') > $R/gpurun_out/ovl/p$1.txt
  cat $R/gpurun_out/ovl/p$1.txt
done
