# k_shade / k_trace counter passes on a short C3 bench (each pass its own rocprofv3 --pmc run)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/pmcs; cd /tmp; export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --spp 16 --dropin-frames 0"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $line -d $R/gpurun_out/pmcs/p$i -o p$i --output-format csv -- python3 $B > $R/gpurun_out/pmcs/p$i.log 2>&1 || { echo "pass $i failed: $line"; tail -3 $R/gpurun_out/pmcs/p$i.log; exit 1; }
done <<'PASSES'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum
TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
FETCH_SIZE
WRITE_SIZE
PASSES
python3 $R/tools/pmc_kernels.py $R/gpurun_out/pmcs/p* > $R/gpurun_out/r04_pmc_shade.txt 2>&1
echo done
