# k_shade with queue reservation before the BSDF sample: GPU parity suite, then A/B against the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_gputest_early.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04_gputest_early.log; exit 1; }
tail -2 gpurun_out/r04_gputest_early.log
CFGS="C3 C5 C2" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/r04_early_ab.txt 2>&1 || { echo ab failed; tail -5 gpurun_out/r04_early_ab.txt; exit 1; }
cat gpurun_out/r04_early_ab.txt
