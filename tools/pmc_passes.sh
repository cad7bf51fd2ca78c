#!/bin/bash
# Counter passes for the wavefront kernels (each its own rocprofv3 --pmc run, no tracing domains),
# summarised per kernel by tools/pmc_kernels.py. usage: tools/pmc_passes.sh OUTDIR [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-passes}; shift; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --spp 8 $*"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 100 rocprofv3 --pmc $line -d $OUT/p$i -o p$i --output-format csv -- python3 $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $line"; grep -m1 "Could not\|error" $OUT/p$i.log; exit 1; }
done <<'PASSES'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum
TCC_HIT_sum TCC_MISS_sum
TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum
PASSES
python3 $R/tools/pmc_kernels.py $OUT/p* > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
