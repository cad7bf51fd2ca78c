set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_a -o a --output-format csv -- python3 -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/pmc_a.log 2>&1; echo "a rc=$?"
RTG_NULL_STREAM=1 timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_b -o b --output-format csv -- python3 -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/pmc_b.log 2>&1; echo "b rc=$?"
