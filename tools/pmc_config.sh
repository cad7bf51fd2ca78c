#!/bin/bash
# PMC traffic of one config's bench line (round 6: every config line carries `traffic`): kernel-trace
# stats + FETCH_SIZE, WRITE_SIZE and the DRAM share of L2 read requests, each its own rocprofv3 run,
# summarised by tools/pmc_summary.py into gpurun_out/prof_out/${RND}_pmc_traffic_<cfg>.json.
# usage: tools/pmc_config.sh C2 "--steps 1 --warmup 0" 64
set -o pipefail
CFG=$1; ARGS=$2; SPP=$3
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_$CFG; mkdir -p $O $R/gpurun_out/prof_out
RND=${RND:-r06}
B="$R/bench.py --no-cpu-baseline --dropin-frames 0 --config $CFG --spp $SPP $ARGS"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $B > $O/kt.log 2>&1 || { echo kt failed; tail -20 $O/kt.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $B > $O/fetch.log 2>&1 || { echo fetch failed; tail -20 $O/fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $B > $O/write.log 2>&1 || { echo write failed; tail -20 $O/write.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $O/dram -o dram --output-format csv -- python3 $B > $O/dram.log 2>&1 || { echo dram failed; tail -20 $O/dram.log; exit 1; }
cd $R
lc=$(echo $CFG | tr A-Z a-z)
python3 tools/pmc_summary.py $O/fetch/fetch_counter_collection.csv $O/write/write_counter_collection.csv $O/kt/kt_kernel_stats.csv \
  $R/gpurun_out/prof_out/${RND}_pmc_traffic_$lc.json $O/dram/dram_counter_collection.csv $CFG $SPP > /dev/null || exit 1
cp $R/gpurun_out/prof_out/${RND}_pmc_traffic_$lc.json profiles/
cp $O/kt/kt_kernel_stats.csv $R/gpurun_out/prof_out/${RND}_kernel_stats_$lc.csv
python3 -c "import json; d=json.load(open('profiles/${RND}_pmc_traffic_$lc.json')); print('$CFG', d.get('extend_kernel'), d.get('extend_hbm_bytes_per_launch'))"
