#!/bin/bash
# Round-5 final evidence: the new queued/user-stream test, the profile refresh (kernel stats, PMC,
# VALU, bench line, smoke, side configs), and the kernel + marker timeline of the pipelined shard-of-8 step.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "user_stream or queued" > gpurun_out/tq.log 2>&1 || { tail -20 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
RND=r05 bash tools/refresh_profiles.sh || exit 1
TAG=s8pipe BENCH_ARGS="--shard-of 8" bash tools/ktrace_markers.sh > gpurun_out/prof_out/r05_s8_pipeline_timeline.txt 2>&1 || { tail gpurun_out/prof_out/r05_s8_pipeline_timeline.txt; exit 1; }
head -20 gpurun_out/prof_out/r05_s8_pipeline_timeline.txt
