# full GPU suite on the current build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04_gputest.log 2>&1
echo "pytest rc $?" >> gpurun_out/r04_gputest.log
