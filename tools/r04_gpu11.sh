set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r04_gputest_cam.log 2>&1
echo "pytest rc $?" >> gpurun_out/r04_gputest_cam.log
tools/ab_cfg.sh > gpurun_out/r04_ab_cam.txt 2>&1
