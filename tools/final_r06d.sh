#!/bin/bash
# Round-6 final evidence on the 7-wave build, part 2: PMC traffic and kernel stats of every config line
# (tools/pmc_config.sh) and the VALU issue pass (C3). Copy gpurun_out/prof_out/* to profiles/ afterwards.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out; mkdir -p $O/prof_out
RND=r06
bash tools/pmc_config.sh C3 "--steps 1 --warmup 0" 64 || exit 1
bash tools/pmc_config.sh C2 "--steps 1 --warmup 0" 64 || exit 1
bash tools/pmc_config.sh C4 "--steps 1 --warmup 0" 256 || exit 1
bash tools/pmc_config.sh C5 "--steps 1 --warmup 0" 32 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $O/prof_valu -o valu --output-format csv -- python3 $R/bench.py --no-cpu-baseline --dropin-frames 0 --steps 1 --warmup 0 > $O/prof_valu.log 2>&1 || { echo valu failed; tail -20 $O/prof_valu.log; exit 1; }
cd $R
python3 tools/valu_issue.py $O/prof_valu/valu_counter_collection.csv $O/prof_out/${RND}_valu_issue.json > /dev/null || exit 1
