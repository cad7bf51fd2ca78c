#!/bin/bash
# Replay ceilings of every bench line at the line's own chunk shape (tools/roof_replay.py; the
# capture and the timed launches are chunk 0 of a render of exactly one chunk of that shape):
#   C3 (64 spp, one 64M-path chunk), C3 at shard-of 8, C2 (64 spp), C5 (16 spp: the C5 line's
#   chunks), C4 (128 spp: the C4 line's 256 spp run as 2 x 128)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/replay
RND=${RND:-r05}
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python tools/roof_replay.py "$@" > gpurun_out/replay/${RND}_roof_replay_${name}.jsonl 2> gpurun_out/replay/${name}.err \
    || { echo "replay $name failed"; tail -5 gpurun_out/replay/${name}.err; return 1; }
  tail -1 gpurun_out/replay/${RND}_roof_replay_${name}.jsonl
}
run c3 500 && run shard8 400 --shard-of 8 && run c2 400 --config C2 && run c5_16spp 600 --config C5 --spp 16 \
  && run c4_128spp 900 --config C4 --spp 128
