# drop-in probe (queued, coalesced) per lib variant in lib/ab, 2 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for round in 1 2; do
for lib in raytracingrenderer_amd/lib/ab/*.so; do
  echo "== $lib"
  RTG_LIB=$PWD/$lib timeout -k 10 200 python -u tools/dropin_probe.py --policy queued --reps 2 || exit 1
done; done > gpurun_out/r04_probe_coalesce.txt 2>&1
