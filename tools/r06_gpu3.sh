#!/bin/bash
# Round 6, third GPU pass: PMC traffic of every config's bench line (tools/pmc_config.sh), and the
# kernel trace of a group of one with and without an RCCL communicator (which kernels slow down).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06c; mkdir -p $O
bash tools/pmc_config.sh C3 "--steps 1 --warmup 0" 64 || exit 1
bash tools/pmc_config.sh C2 "--steps 1 --warmup 0" 64 || exit 1
bash tools/pmc_config.sh C4 "--steps 1 --warmup 0" 256 || exit 1
bash tools/pmc_config.sh C5 "--steps 1 --warmup 0" 32 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g1r -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --dropin-frames 0 --steps 3 --step-mode full --devices 0 > $O/g1r.log 2>&1 || { tail -20 $O/g1r.log; exit 1; }
RTG_GROUP_NO_RCCL1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g1n -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --dropin-frames 0 --steps 3 --step-mode full --devices 0 > $O/g1n.log 2>&1 || { tail -20 $O/g1n.log; exit 1; }
cd $R
for d in g1r g1n; do echo "== $d"; head -8 $O/$d/kt_kernel_stats.csv | cut -c1-160; python3 tools/kernel_gaps.py $O/$d $d; done
