# k_shade with the small-scene walk in its own unit (max-ilp): GPU parity suite, then A/B against the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_gputest_smallilp.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04_gputest_smallilp.log; exit 1; }
tail -2 gpurun_out/r04_gputest_smallilp.log
CFGS="C2 C3" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/r04_smallilp_ab.txt 2>&1 || { echo ab failed; tail -5 gpurun_out/r04_smallilp_ab.txt; exit 1; }
cat gpurun_out/r04_smallilp_ab.txt
