#!/bin/bash
# k_trace counter passes on the C3 bench workload at 8 spp (each its own rocprofv3 --pmc run, no
# tracing domains); summarised by tools/pmc_kernels.py into gpurun_out/pmct/summary.json
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/pmct; cd /tmp; export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --spp 8"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 100 rocprofv3 --pmc $line -d $R/gpurun_out/pmct/p$i -o p$i --output-format csv -- python3 $B > $R/gpurun_out/pmct/p$i.log 2>&1 || { echo "pass $i failed: $line"; grep -m1 "Could not\|rror" $R/gpurun_out/pmct/p$i.log; exit 1; }
done <<'PASSES'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
TCC_HIT_sum TCC_MISS_sum
GRBM_GUI_ACTIVE GRBM_COUNT
PASSES
cd $R && python3 tools/pmc_kernels.py gpurun_out/pmct/p* > gpurun_out/pmct/summary.txt; cat gpurun_out/pmct/summary.txt
