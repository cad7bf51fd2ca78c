#!/bin/bash
# Round 6, second GPU pass: the group of one with / without an RCCL communicator against the
# single handle, then the leaf-handling A/B (tools/ab_leaf.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06b; mkdir -p $O
B="python -u bench.py --no-cpu-baseline --dropin-frames 0 --steps 30"
for round in 1 2; do
  timeout -k 10 200 $B > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
  echo "c3 $(tail -1 $O/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
  timeout -k 10 200 $B --devices 0 > $O/g1.log 2>&1 || { tail -20 $O/g1.log; exit 1; }
  echo "g1 rccl $(tail -1 $O/g1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], d['group']['uses_rccl'])")"
  RTG_GROUP_NO_RCCL1=1 timeout -k 10 200 $B --devices 0 > $O/g1n.log 2>&1 || { tail -20 $O/g1n.log; exit 1; }
  echo "g1 none $(tail -1 $O/g1n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], d['group']['uses_rccl'])")"
done
AB_SETS="--steps 20;--steps 40 --shard-of 8;--config C4 --spp 64 --steps 1" bash tools/ab_leaf.sh 2>&1 | tee $O/ab_leaf.txt
