#!/bin/bash
# A/B of a bench.py flag on one build (interleaved, 2 rounds): AB_FLAG (e.g. --fused-shadow) against
# the default, on each BENCH_ARGS set given as ';'-separated AB_SETS (default: C3, C3 --shard-of 8, C2).
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
IFS=';' read -ra SETS <<< "${AB_SETS:---steps 20;--steps 40 --shard-of 8;--config C2 --steps 40}"
for set in "${SETS[@]}"; do
for round in 1 2; do
for f in "" "$AB_FLAG"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $set $f > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "[$set] ${f:-default} $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])")"
done; done; done
