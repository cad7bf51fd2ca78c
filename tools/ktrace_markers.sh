#!/bin/bash
# rocprofv3 kernel trace + roctx marker trace (the rtg:generate / rtg:trace b / rtg:shade b /
# rtg:accumulate ranges of render_impl) of one bench run -> gpurun_out/km_<tag>/ ; then the per-step
# timeline (kernel busy time, gaps between kernels) with tools/timeline.py
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-c3}
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $R/gpurun_out/km_$TAG -o km --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 --dropin-frames 0 $BENCH_ARGS > $R/gpurun_out/km_$TAG.log 2>&1 \
  || { echo "profile failed"; tail -20 $R/gpurun_out/km_$TAG.log; exit 1; }
K=$(find $R/gpurun_out/km_$TAG -name '*kernel_trace.csv' | head -1)
M=$(find $R/gpurun_out/km_$TAG -name '*marker_api_trace.csv' | head -1)
echo "kernel trace: $K"; echo "marker trace: $M"
python3 $R/tools/timeline.py $K
[ -n "$M" ] && head -5 $M && cut -d, -f1-8 $M | grep -c rtg
