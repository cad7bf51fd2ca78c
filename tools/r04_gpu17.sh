# drop-in frames coalesced up to 64M paths (one chunk for 64 one-spp calls) vs 16M (pipelined)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEPS=5 timeout -k 10 900 bash tools/ab_dropin.sh > gpurun_out/r04_dropin_c64_ab.txt 2>&1 || { echo ab failed; tail -5 gpurun_out/r04_dropin_c64_ab.txt; exit 1; }
cat gpurun_out/r04_dropin_c64_ab.txt
