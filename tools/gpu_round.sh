#!/bin/bash
# GPU session: smoke, bench, rocprof kernel-trace stats, PMC passes (each step time-limited)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 > $R/gpurun_out/prof_kt.log 2>&1 || { echo kt failed; tail -20 $R/gpurun_out/prof_kt.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o fetch --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $R/gpurun_out/prof_fetch.log 2>&1 || { echo fetch failed; tail -20 $R/gpurun_out/prof_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o write --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $R/gpurun_out/prof_write.log 2>&1 || { echo write failed; tail -20 $R/gpurun_out/prof_write.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $R/gpurun_out/prof_dram -o dram --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 > $R/gpurun_out/prof_dram.log 2>&1 || { echo dram failed; tail -20 $R/gpurun_out/prof_dram.log; exit 1; }
echo all done
