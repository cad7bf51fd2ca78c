set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dropin -o dq -- python3 tools/dropin_probe.py --policy queued --reps 1 > gpurun_out/r04_probe_prof.txt 2>&1 && \
python3 tools/overlap.py $(find gpurun_out/prof_dropin -name "dq_kernel_trace.csv" | head -1) --last-ms 150 > gpurun_out/r04_overlap.txt 2>&1
