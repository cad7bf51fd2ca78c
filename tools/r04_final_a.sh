# round-end evidence, part A: GPU parity suite on the final build, then the profile refresh
# (kernel stats, PMC traffic, default bench line, smoke, side configs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_gputest_final.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04_gputest_final.log; exit 1; }
tail -2 gpurun_out/r04_gputest_final.log
RND=r04 bash tools/refresh_profiles.sh || { echo refresh failed; exit 1; }
echo done
