# new GPU parity cases: adversarial mesh families rendered against the oracle
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k adversarial -v --timeout 120 --timeout-method thread > gpurun_out/r04_gputest_adversarial.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r04_gputest_adversarial.log; exit 1; }
tail -12 gpurun_out/r04_gputest_adversarial.log
