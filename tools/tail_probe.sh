cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 200 python tools/wavetime.py --shard-of 1 > gpurun_out/wt1.txt 2>&1 && \
timeout -k 10 200 python tools/wavetime.py --shard-of 8 > gpurun_out/wt8.txt 2>&1 && \
timeout -k 10 400 python tools/roof_replay.py --shard-of 8 > gpurun_out/rr8.jsonl 2>&1
