# round-end evidence, part B: k_shade / k_trace counter passes and the shard sweep on the final build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/r04_pmc_shade.sh || { echo pmc failed; exit 1; }
timeout -k 10 900 bash tools/shard_sweep.sh > gpurun_out/r04_shard_sweep.txt 2>&1 || { echo sweep failed; tail -5 gpurun_out/r04_shard_sweep.txt; exit 1; }
cat gpurun_out/r04_shard_sweep.txt
