# replay ceilings of the current build (camera rays per pixel changed launch 0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/roof_replay.py > gpurun_out/r04_roof_replay.jsonl 2> gpurun_out/r04_rr_c3.err || { echo c3 failed; tail -3 gpurun_out/r04_rr_c3.err; exit 1; }
timeout -k 10 400 python -u tools/roof_replay.py --shard-of 8 > gpurun_out/r04_roof_replay_shard8.jsonl 2> gpurun_out/r04_rr_s8.err || { echo s8 failed; exit 1; }
timeout -k 10 400 python -u tools/roof_replay.py --config C2 > gpurun_out/r04_roof_replay_c2.jsonl 2> gpurun_out/r04_rr_c2.err || { echo c2 failed; exit 1; }
timeout -k 10 400 python -u tools/roof_replay.py --config C5 --spp 4 > gpurun_out/r04_roof_replay_c5_4spp.jsonl 2> gpurun_out/r04_rr_c5.err || { echo c5 failed; exit 1; }
timeout -k 10 600 python -u tools/roof_replay.py --config C4 --spp 32 > gpurun_out/r04_roof_replay_c4_32spp.jsonl 2> gpurun_out/r04_rr_c4.err || { echo c4 failed; exit 1; }
echo done
