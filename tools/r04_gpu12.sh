set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 100 python -u tools/r04_churn.py 300 > gpurun_out/r04_churn_default.log 2>&1 || { echo churn failed; exit 1; }
timeout -k 10 200 python -u tools/dropin_probe.py --policy queued --reps 2 --no-coalesce > gpurun_out/r04_probe_prio.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/dropin_probe.py --policy queued --reps 2 >> gpurun_out/r04_probe_prio.txt 2>&1 || exit 1
bash tools/refresh_profiles.sh > gpurun_out/r04_refresh.log 2>&1
