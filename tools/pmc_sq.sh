#!/bin/bash
# SQ / TCC counter passes on a short bench run (each pass its own rocprofv3 call)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1 || true
B="python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --spp 8"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES -d $R/gpurun_out/sq1 -o sq1 --output-format csv -- $B > $R/gpurun_out/sq1.log 2>&1 || { echo sq1 failed; tail -5 $R/gpurun_out/sq1.log; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/tcc -o tcc --output-format csv -- $B > $R/gpurun_out/tcc.log 2>&1 || { echo tcc failed; tail -5 $R/gpurun_out/tcc.log; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/sq2 -o sq2 --output-format csv -- $B > $R/gpurun_out/sq2.log 2>&1 || { echo sq2 failed; tail -5 $R/gpurun_out/sq2.log; }
echo done
