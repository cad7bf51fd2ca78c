#!/bin/bash
# Round 6 (late): traversal counters on the final (7-wave) build, C3 at 8 spp: TA busy / stalls, L2 and
# L1 hit rates, L1 -> L2 read latency. One rocprofv3 --pmc run per pass; the chain stops at the first
# failure. Summary: tools/pmc_kernels.py.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/deep; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --dropin-frames 0 --steps 1 --warmup 0 --spp 8"
i=0
for line in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TCC_HIT_sum TCC_MISS_sum" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
            "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $line -d $O/p$i -o p$i --output-format csv -- python3 $B > $O/p$i.log 2>&1 || { echo "pass $i failed ($?): $line"; tail -5 $O/p$i.log; exit 1; }
done
cd $R && python3 tools/pmc_kernels.py $O/p1 $O/p2 $O/p3 $O/p4 $O/p5 | tee $O/summary.txt
