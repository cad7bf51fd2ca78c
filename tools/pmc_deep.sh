#!/bin/bash
# Traversal-kernel counter passes (each its own rocprofv3 --pmc run, no tracing domains).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/deep; cd /tmp; export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --spp 8"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 100 rocprofv3 --pmc $line -d $R/gpurun_out/deep/p$i -o p$i --output-format csv -- python3 $B > $R/gpurun_out/deep/p$i.log 2>&1 || { echo "pass $i failed: $line"; grep -m1 "Could not\|error" $R/gpurun_out/deep/p$i.log; }
done <<'PASSES'
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum
TCC_HIT_sum TCC_MISS_sum
TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum
TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum
PASSES
echo done
