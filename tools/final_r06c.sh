#!/bin/bash
# Round-6 final evidence on the 7-wave build, part 1: the GPU suite, smoke, the default bench line and
# the side configs. Copy gpurun_out/prof_out/* to profiles/ afterwards.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out; mkdir -p $O/prof_out
RND=r06
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/prof_out/${RND}_gputest_final.log 2>&1 || { tail -30 $O/prof_out/${RND}_gputest_final.log; exit 1; }
tail -1 $O/prof_out/${RND}_gputest_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/prof_out/${RND}_smoke.log 2>&1 || { echo smoke failed; tail -20 $O/prof_out/${RND}_smoke.log; exit 1; }
cat $O/prof_out/${RND}_smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | tee $O/prof_out/${RND}_bench.json
rm -f $O/configs.jsonl
bash tools/configs_bench.sh && cp $O/configs.jsonl $O/prof_out/${RND}_configs_bench.jsonl
