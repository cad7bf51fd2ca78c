#!/bin/bash
# Round 6 (late): the default bench line on the final tree.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof_out
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log > gpurun_out/prof_out/r06_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/prof_out/r06_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['lane_util_node_leaf'], r['lane_idle_node'])"
