#!/bin/bash
# lib variants on the default C3 line with its drop-in leg (queued / queued_each / sync frames), 2 rounds
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for round in 1 2; do for lib in raytracingrenderer_amd/lib/ab/*.so; do
  RTG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/abd.log 2> gpurun_out/abd.err || { tail -5 gpurun_out/abd.err; exit 1; }
  echo "$(basename $lib) $(tail -1 gpurun_out/abd.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); di=d['dropin']; print(d['value'], d['ms_per_step'], 'queued', di['queued']['ms_per_frame'], 'queued_each', di['queued_each']['ms_per_frame'], 'sync', di['sync']['ms_per_frame'])")"
done; done
