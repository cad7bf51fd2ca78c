# drop-in probe per lib variant in lib/ab (queued policy, each call issued / coalesced), then a profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lib in raytracingrenderer_amd/lib/ab/*.so; do
  echo "== $lib"
  RTG_LIB=$PWD/$lib timeout -k 10 200 python -u tools/dropin_probe.py --policy queued --reps 2 --no-coalesce || exit 1
done > gpurun_out/r04_probe_variants.txt 2>&1
timeout -k 10 200 python -u tools/dropin_probe.py --policy queued --reps 2 >> gpurun_out/r04_probe_variants.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dropin2 -o dq -- python3 tools/dropin_probe.py --policy queued --reps 1 --no-coalesce > gpurun_out/r04_probe_prof.txt 2>&1 && \
python3 tools/overlap.py $(find gpurun_out/prof_dropin2 -name "dq_kernel_trace.csv" | head -1) --last-ms 150 > gpurun_out/r04_overlap2.txt 2>&1
