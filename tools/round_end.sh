#!/bin/bash
# Round-end evidence on the current build: the locality-matched replay (C3, C2, shard-of 8), then
# tools/refresh_profiles.sh (kernel stats, PMC traffic, bench line, smoke, side configs).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof_out
RND=${RND:-r03}
timeout -k 10 500 python tools/roof_replay.py > gpurun_out/prof_out/${RND}_roof_replay.jsonl 2> gpurun_out/rr.err || { echo replay failed; tail -5 gpurun_out/rr.err; exit 1; }
cp gpurun_out/prof_out/${RND}_roof_replay.jsonl profiles/${RND}_roof_replay.jsonl
timeout -k 10 400 python tools/roof_replay.py --config C2 > gpurun_out/prof_out/${RND}_roof_replay_c2.jsonl 2> gpurun_out/rr.err || { echo replay c2 failed; tail -5 gpurun_out/rr.err; exit 1; }
timeout -k 10 400 python tools/roof_replay.py --shard-of 8 > gpurun_out/prof_out/${RND}_roof_replay_shard8.jsonl 2> gpurun_out/rr.err || { echo replay s8 failed; tail -5 gpurun_out/rr.err; exit 1; }
RND=$RND timeout -k 10 900 bash tools/refresh_profiles.sh
