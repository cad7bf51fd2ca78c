set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_north_star.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gputest_shade.log 2>&1
echo "pytest rc $?" >> gpurun_out/r04_gputest_shade.log
tools/ab_cfg.sh > gpurun_out/r04_ab_shade.txt 2>&1
