#!/bin/bash
# A/B of the lib variants in raytracingrenderer_amd/lib/ab on the batched bench step AND the drop-in
# frame loop (bench.py's dropin leg: 1-spp calls, queued / sync / sync + film read), interleaved,
# $ROUNDS rounds (default 2). BENCH_ARGS adds bench.py flags (e.g. "--config C2").
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for round in $(seq 1 ${ROUNDS:-2}); do
for lib in raytracingrenderer_amd/lib/ab/*.so; do
  RTG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 $BENCH_ARGS \
    > gpurun_out/ab.log 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  echo "$(basename $lib) $(tail -1 gpurun_out/ab.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); di=d.get('dropin') or {}
print(d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'],
      'dropin', {k: (v['ms_per_frame'], v['film_equals_batched']) for k, v in di.items() if isinstance(v, dict)},
      di.get('queued_over_batched'))")"
done; done
