#!/bin/bash
# Round-6 final evidence, part 1: the GPU suite, PMC traffic of every config line on the final build
# (tools/pmc_config.sh), the VALU issue pass (C3), the default bench line, smoke, the side configs.
# Copy gpurun_out/prof_out/* to profiles/ afterwards.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out; mkdir -p $O/prof_out
RND=r06
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/prof_out/${RND}_gputest_final.log 2>&1 || { tail -30 $O/prof_out/${RND}_gputest_final.log; exit 1; }
tail -1 $O/prof_out/${RND}_gputest_final.log
bash tools/pmc_config.sh C3 "--steps 1 --warmup 0" 64 || exit 1
bash tools/pmc_config.sh C2 "--steps 1 --warmup 0" 64 || exit 1
bash tools/pmc_config.sh C4 "--steps 1 --warmup 0" 256 || exit 1
bash tools/pmc_config.sh C5 "--steps 1 --warmup 0" 32 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $O/prof_valu -o valu --output-format csv -- python3 $R/bench.py --no-cpu-baseline --dropin-frames 0 --steps 1 --warmup 0 > $O/prof_valu.log 2>&1 || { echo valu failed; tail -20 $O/prof_valu.log; exit 1; }
cd $R
python3 tools/valu_issue.py $O/prof_valu/valu_counter_collection.csv $O/prof_out/${RND}_valu_issue.json > /dev/null || exit 1
cp $O/prof_out/${RND}_valu_issue.json profiles/
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | tee $O/prof_out/${RND}_bench.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/prof_out/${RND}_smoke.log 2>&1 || { echo smoke failed; tail -20 $O/prof_out/${RND}_smoke.log; exit 1; }
rm -f $O/configs.jsonl
bash tools/configs_bench.sh && cp $O/configs.jsonl $O/prof_out/${RND}_configs_bench.jsonl
