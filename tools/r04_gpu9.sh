set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r04_gputest_small.log 2>&1
echo "pytest rc $?" >> gpurun_out/r04_gputest_small.log
CFGS="C2 C3" tools/ab_cfg.sh > gpurun_out/r04_ab_small.txt 2>&1
