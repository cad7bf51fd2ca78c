set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
RTG_NULL_STREAM=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_c -o c --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $R/gpurun_out/pmc_c.log 2>&1; echo "c rc=$?"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_d -o d --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --spp 4 > $R/gpurun_out/pmc_d.log 2>&1; echo "d rc=$?"
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --max-paths 67108864 > $R/gpurun_out/big.log 2>&1; echo "big rc=$?"; tail -1 $R/gpurun_out/big.log
