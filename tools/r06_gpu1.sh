#!/bin/bash
# Round 6, first GPU pass: the GPU suite, the queued group path (bench --devices), the count hand-off
# (kernel trace: no copyBuffer, trace -> shade gaps at N = 1 and shard-of 2), short bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06a; mkdir -p $O
B="python -u bench.py --no-cpu-baseline --dropin-frames 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 $B --steps 30 > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
tail -1 $O/c3.log > $O/c3.json
timeout -k 10 200 $B --steps 30 --devices 0 > $O/g1.log 2>&1 || { tail -20 $O/g1.log; exit 1; }
tail -1 $O/g1.log > $O/g1.json
timeout -k 10 300 $B --steps 10 --devices 0,0,0,0,0,0,0,0 --verify-film > $O/g8.log 2>&1 || { tail -20 $O/g8.log; exit 1; }
tail -1 $O/g8.log > $O/g8.json
timeout -k 10 200 $B --steps 80 --shard-of 8 > $O/s8.log 2>&1 || { tail -20 $O/s8.log; exit 1; }
tail -1 $O/s8.log > $O/s8.json
timeout -k 10 200 $B --steps 30 --shard-of 8 --step-mode full > $O/s8w.log 2>&1 || { tail -20 $O/s8w.log; exit 1; }
tail -1 $O/s8w.log > $O/s8w.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt1 -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --dropin-frames 0 --steps 3 --step-mode full > $O/kt1.log 2>&1 || { tail -20 $O/kt1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt2 -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --dropin-frames 0 --steps 5 --shard-of 2 --step-mode full > $O/kt2.log 2>&1 || { tail -20 $O/kt2.log; exit 1; }
cd $R
python3 tools/kernel_gaps.py $O/kt1 "C3 N=1" | tee $O/gaps.jsonl
python3 tools/kernel_gaps.py $O/kt2 "C3 shard-of 2" | tee -a $O/gaps.jsonl
for f in c3 g1 g8 s8 s8w; do python3 -c "
import json,sys; d=json.load(open('$O/$f.json')); g=d.get('group',{})
print('$f', d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'], d.get('film_reduce_bit_exact'), g.get('reduce_ms_per_step'), d.get('timed_step','')[:40])"; done
