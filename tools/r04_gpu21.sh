# LLVM scheduling strategies for the whole device library (same instructions, different order)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFGS="C3 S8 C2 C5" timeout -k 10 1100 bash tools/ab_cfg.sh > gpurun_out/r04_sched_ab.txt 2>&1 || { echo ab failed; tail -5 gpurun_out/r04_sched_ab.txt; exit 1; }
cat gpurun_out/r04_sched_ab.txt
