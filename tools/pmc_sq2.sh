#!/bin/bash
# SQ instruction-mix passes for the traversal kernels (each its own rocprofv3 --pmc run)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/sq; cd /tmp; export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --spp 8"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 100 rocprofv3 --pmc $line -d $R/gpurun_out/sq/p$i -o p$i --output-format csv -- python3 $B > $R/gpurun_out/sq/p$i.log 2>&1 || { echo "pass $i failed: $line"; grep -m1 "Could not\|rror" $R/gpurun_out/sq/p$i.log; exit 1; }
done <<'PASSES'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_WAIT_ANY
SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F32
PASSES
echo done
