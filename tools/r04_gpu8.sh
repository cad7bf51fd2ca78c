# C5 replay ceiling, C5 8-rank rehearsal balance, drop-in + shard-of-8 after the pipeline policy change
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/roof_replay.py --config C5 --spp 4 --reps 2 > gpurun_out/r04_roof_replay_c5_4spp.jsonl 2> gpurun_out/r04_roof_replay_c5.err || { echo replay failed; tail -5 gpurun_out/r04_roof_replay_c5.err; }
timeout -k 10 400 python -u bench.py --config C5 --devices 0,0,0,0,0,0,0,0 --verify-film --steps 1 --warmup 1 > gpurun_out/r04_c5_group8.json 2> gpurun_out/r04_c5_group8.err || { echo group8 failed; tail -5 gpurun_out/r04_c5_group8.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_bench2.json 2> gpurun_out/r04_bench2.err || exit 1
timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --shard-of 8 > gpurun_out/r04_shard8.json 2> gpurun_out/r04_shard8.err || exit 1
echo done
