#!/bin/bash
# Round-6 final evidence on the 7-wave build, part 3: shard sweeps (pipelined and waited-for steps), the 8-rank group
# rehearsal with lean steps and --verify-film, the group of one, and C5 at full size through the CLI.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out; mkdir -p $O/prof_out
RND=r06
bash tools/shard_sweep.sh > $O/prof_out/${RND}_shard_sweep.txt 2>&1 || { cat $O/prof_out/${RND}_shard_sweep.txt; exit 1; }
cat $O/prof_out/${RND}_shard_sweep.txt
for n in 1 2 4 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --steps 10 --shard-of $n --step-mode full > $O/shw.log 2>&1 || { tail -5 $O/shw.log; exit 1; }
  echo "N=$n waited $(tail -1 $O/shw.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); x=d.get('shard_exchange') or {}
print(d['value'], 'ms/step', d['ms_per_step'], d['kernel_ms_per_step_rank0'], 'exchange_ms', x.get('total_ms'), 'job_ms', x.get('projected_job_ms_per_step'))")"
done | tee $O/prof_out/${RND}_shard_sweep_waited.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --steps 10 --devices 0,0,0,0,0,0,0,0 --verify-film > $O/g8.log 2>&1 || { tail -5 $O/g8.log; exit 1; }
tail -1 $O/g8.log > $O/prof_out/${RND}_group8_rehearsal.json
timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --steps 30 --devices 0 > $O/g1.log 2>&1 || { tail -5 $O/g1.log; exit 1; }
tail -1 $O/g1.log > $O/prof_out/${RND}_group1.json
mkdir -p /tmp/c5 && cd /tmp/c5 && timeout -k 10 300 $R/raytracingrenderer_amd/lib/rtg_render -scene $R/assets/coffee -skipMissing 1 -envmap GI.hdr -width 4096 -height 4096 -SPP 1024 -gpus 1 -batch 1024 -timeLimit 0 > $O/prof_out/${RND}_c5_full_cli.log 2>&1 || { tail -5 $O/prof_out/${RND}_c5_full_cli.log; exit 1; }
md5sum result_1024.hdr >> $O/prof_out/${RND}_c5_full_cli.log; tail -4 $O/prof_out/${RND}_c5_full_cli.log
cd $R
for n in 1 8; do
  timeout -k 10 300 python tools/launch_profile.py --shard-of $n > $O/lp.log 2>&1 || { tail -5 $O/lp.log; exit 1; }
  tail -1 $O/lp.log >> $O/prof_out/${RND}_launch_profile.jsonl
done
bash tools/dist_rehearse.sh > $O/prof_out/${RND}_torchrun_rehearsal.json 2>&1 || { cat $O/prof_out/${RND}_torchrun_rehearsal.json; exit 1; }
cat $O/prof_out/${RND}_torchrun_rehearsal.json | cut -c1-300
