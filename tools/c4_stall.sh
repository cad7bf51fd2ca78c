#!/bin/bash
# C4 large-chunk host time: HIP API + kernel trace of one C4 step with 1G paths in flight (each
# step time-limited; no PMC counters in this run)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c4stall; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --config C4 --steps 1 --warmup 1 --max-paths 1073741824 > $O/plain.log 2>&1 || { echo plain failed; tail -5 $O/plain.log; exit 1; }
tail -1 $O/plain.log | cut -c1-400
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --stats -d $O/tr -o tr --output-format csv -- python3 $R/bench.py --no-cpu-baseline --config C4 --steps 1 --warmup 1 --max-paths 1073741824 > $O/tr.log 2>&1 || { echo trace failed; tail -5 $O/tr.log; exit 1; }
ls $O/tr
