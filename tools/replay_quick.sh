#!/bin/bash
# C3 and C2 replay ceilings only (tools/roof_replay.py), for a quick check of the replay itself
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/replay2
timeout -k 10 500 python tools/roof_replay.py > gpurun_out/replay2/c3.jsonl 2> gpurun_out/replay2/c3.err || { tail -5 gpurun_out/replay2/c3.err; exit 1; }
tail -1 gpurun_out/replay2/c3.jsonl
timeout -k 10 500 python tools/roof_replay.py --config C2 > gpurun_out/replay2/c2.jsonl 2> gpurun_out/replay2/c2.err || { tail -5 gpurun_out/replay2/c2.err; exit 1; }
tail -1 gpurun_out/replay2/c2.jsonl
