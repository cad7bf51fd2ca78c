#!/bin/bash
# Round-end evidence in one call: rocprofv3 kernel-trace stats + PMC passes (separate runs: FETCH_SIZE,
# WRITE_SIZE, DRAM requests, SQ_INSTS_VALU), their summaries (pmc_summary.py -> ${RND}_pmc_traffic.json,
# valu_issue.py -> ${RND}_valu_issue.json, also copied to profiles/ on the box so the bench line that
# follows reads them), then the default bench line, smoke and the side configs. Copy
# gpurun_out/prof_out/* to profiles/ afterwards.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof_out
RND=${RND:-r05}
O=$R/gpurun_out
B="$R/bench.py --no-cpu-baseline --dropin-frames 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_kt -o kt --output-format csv -- python3 $B --steps 2 > $O/prof_kt.log 2>&1 || { echo kt failed; tail -20 $O/prof_kt.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch -o fetch --output-format csv -- python3 $B --steps 1 --warmup 0 > $O/prof_fetch.log 2>&1 || { echo fetch failed; tail -20 $O/prof_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write -o write --output-format csv -- python3 $B --steps 1 --warmup 0 > $O/prof_write.log 2>&1 || { echo write failed; tail -20 $O/prof_write.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $O/prof_dram -o dram --output-format csv -- python3 $B --steps 1 --warmup 0 > $O/prof_dram.log 2>&1 || { echo dram failed; tail -20 $O/prof_dram.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $O/prof_valu -o valu --output-format csv -- python3 $B --steps 1 --warmup 0 > $O/prof_valu.log 2>&1 || { echo valu failed; tail -20 $O/prof_valu.log; exit 1; }
cd $R
python3 tools/pmc_summary.py $O/prof_fetch/fetch_counter_collection.csv $O/prof_write/write_counter_collection.csv $O/prof_kt/kt_kernel_stats.csv $O/prof_out/${RND}_pmc_traffic.json $O/prof_dram/dram_counter_collection.csv > /dev/null
python3 tools/valu_issue.py $O/prof_valu/valu_counter_collection.csv $O/prof_out/${RND}_valu_issue.json > /dev/null
cp $O/prof_out/${RND}_pmc_traffic.json $O/prof_out/${RND}_valu_issue.json profiles/
cp $O/prof_kt/kt_kernel_stats.csv $O/prof_out/${RND}_kernel_stats.csv
cp $O/prof_out/${RND}_kernel_stats.csv profiles/
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | tee $O/prof_out/${RND}_bench.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/prof_out/${RND}_smoke.log 2>&1 || { echo smoke failed; tail -20 $O/prof_out/${RND}_smoke.log; exit 1; }
rm -f $O/configs.jsonl
bash tools/configs_bench.sh && cp $O/configs.jsonl $O/prof_out/${RND}_configs_bench.jsonl
