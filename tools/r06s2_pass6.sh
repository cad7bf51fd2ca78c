#!/bin/bash
# Round 6 (late), pass 6 on the final tree (half-HBM memory budget restored): GPU suite, smoke, the side configs and
# C5 at full size through the CLI. Copy gpurun_out/prof_out/* to profiles/ afterwards.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out; mkdir -p $O/prof_out
RND=r06
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/prof_out/${RND}_gputest_final.log 2>&1 || { tail -30 $O/prof_out/${RND}_gputest_final.log; exit 1; }
tail -1 $O/prof_out/${RND}_gputest_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/prof_out/${RND}_smoke.log 2>&1 || { echo smoke failed; tail -20 $O/prof_out/${RND}_smoke.log; exit 1; }
cat $O/prof_out/${RND}_smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/prof_out/${RND}_bench.json
python3 -c "import json; d=json.load(open('$O/prof_out/${RND}_bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
rm -f $O/configs.jsonl
bash tools/configs_bench.sh && cp $O/configs.jsonl $O/prof_out/${RND}_configs_bench.jsonl || exit 1
mkdir -p /tmp/c5 && cd /tmp/c5 && timeout -k 10 300 $R/raytracingrenderer_amd/lib/rtg_render -scene $R/assets/coffee -skipMissing 1 -envmap GI.hdr -width 4096 -height 4096 -SPP 1024 -gpus 1 -batch 1024 -timeLimit 0 > $O/prof_out/${RND}_c5_full_cli.log 2>&1 || { tail -5 $O/prof_out/${RND}_c5_full_cli.log; exit 1; }
md5sum result_1024.hdr >> $O/prof_out/${RND}_c5_full_cli.log; tail -4 $O/prof_out/${RND}_c5_full_cli.log
