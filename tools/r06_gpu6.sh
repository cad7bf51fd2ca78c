#!/bin/bash
# Round 6, sixth GPU pass: an RCCL communicator's effect on librtg's kernels (tools/rccl_probe.py
# under rocprofv3 kernel-trace stats), three orders.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in none pg_first pg_after; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$m -o kt --output-format csv -- python3 $R/tools/rccl_probe.py --mode $m > $O/$m.log 2>&1 || { tail -20 $O/$m.log; exit 1; }
  tail -1 $O/$m.log
  grep -h "k_accumulate_pm\|k_shade<false, true>\|k_trace<false, false>" $O/$m/kt_kernel_stats.csv | cut -d, -f1-4
done
cd $R
AB_SETS="--steps 10;--config C2 --steps 20;--config C5 --spp 32 --steps 1;--config C4 --spp 64 --steps 1" bash tools/ab_leaf.sh 2>&1 | tee $O/ab_shade_early.txt
