#!/bin/bash
# Round-end scaling evidence on the current build (the replays are tools/replay_all.sh, the profiles
# tools/refresh_profiles.sh): the shard sweep, the 8-rank group rehearsal on one GPU, and the full C5
# frame through the CLI (an RCCL group of one device).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof_out
RND=${RND:-r05}
O=$R/gpurun_out
timeout -k 10 500 bash tools/shard_sweep.sh > $O/prof_out/${RND}_shard_sweep.txt 2>&1 || { echo sweep failed; cat $O/prof_out/${RND}_shard_sweep.txt; exit 1; }
cat $O/prof_out/${RND}_shard_sweep.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --devices 0,0,0,0,0,0,0,0 --verify-film > $O/g8.log 2> $O/g8.err \
  || { echo "group8 failed"; tail -20 $O/g8.err; exit 1; }
tail -1 $O/g8.log > $O/prof_out/${RND}_group8_rehearsal.json
mkdir -p $O/c5 && cd $O/c5 && timeout -k 10 300 $R/raytracingrenderer_amd/lib/rtg_render -scene $R/assets/coffee -skipMissing 1 -envmap GI.hdr \
  -width 4096 -height 4096 -SPP 1024 -gpus 1 -batch 1024 > $O/prof_out/${RND}_c5_full_cli.log 2>&1 || { echo c5 failed; tail $O/prof_out/${RND}_c5_full_cli.log; exit 1; }
md5sum $O/c5/result_1024.hdr >> $O/prof_out/${RND}_c5_full_cli.log; tail -4 $O/prof_out/${RND}_c5_full_cli.log
