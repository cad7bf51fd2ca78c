# k_shade at 8 waves/SIMD (64 VGPRs, 7 spilled) vs 7 (72 VGPRs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFGS="C3 C5 C2" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/r04_shadew8_ab.txt 2>&1 || { echo ab failed; tail -5 gpurun_out/r04_shadew8_ab.txt; exit 1; }
cat gpurun_out/r04_shadew8_ab.txt
