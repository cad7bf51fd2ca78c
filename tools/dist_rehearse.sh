#!/bin/bash
# N=2 rehearsal of bench.py's multi-rank path on a one-GPU box: two ranks share cuda:0, gloo for
# the film reduce; rank 0 checks the reduced film against a solo render of every tile.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
RTG_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 0 --spp 8 --no-cpu-baseline \
  --verify-film > gpurun_out/dist2.log 2>&1 || { tail -30 gpurun_out/dist2.log; exit 1; }
grep '^{' gpurun_out/dist2.log | tail -1
