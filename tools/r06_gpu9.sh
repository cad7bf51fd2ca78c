#!/bin/bash
# Round 6: GPU suite after the group-of-one copy, torchrun rehearsal (2 ranks, gloo, one GPU), group of one.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
bash tools/dist_rehearse.sh | tee $O/dist2.json || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --steps 30 --devices 0 > $O/g1.log 2>&1 || { tail -5 $O/g1.log; exit 1; }
tail -1 $O/g1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('g1', d['value'], d['ms_per_step'], d['group']['reduce_ms_per_step'], d['group']['uses_rccl'])"
