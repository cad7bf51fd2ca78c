# final build: config C5 at full size through the CLI (one RCCL group of one device), and the
# headline bench repeated three times (spread of `value`)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/c5full
export TMPDIR=/tmp
( cd gpurun_out/c5full && timeout -k 10 300 $R/raytracingrenderer_amd/lib/rtg_render -scene $R/assets/coffee -width 4096 -height 4096 -skipMissing 1 -envmap GI.hdr -SPP 1024 -gpus 1 -batch 1024 -timeLimit 100 -outputFilename result_1024.hdr > ../r04_c5_full_cli.log 2>&1 && md5sum result_1024.hdr >> ../r04_c5_full_cli.log && rm -f result_1024.hdr ) || { echo c5 failed; tail -5 gpurun_out/r04_c5_full_cli.log; exit 1; }
cat gpurun_out/r04_c5_full_cli.log
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 > gpurun_out/rep.log 2>&1 || { echo bench failed; tail -5 gpurun_out/rep.log; exit 1; }
  tail -1 gpurun_out/rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rep', $k, d['value'], d['ms_per_step'], d['kernel_ms_per_step_rank0'])" | tee -a gpurun_out/r04_bench_repeats.txt
done
