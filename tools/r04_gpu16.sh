# per-kernel time of C2 and C5 (kernel-trace stats)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --dropin-frames 0 --config C2 --steps 5 --warmup 1 > $O/kt_c2.log 2>&1 || { echo c2 failed; tail -5 $O/kt_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --dropin-frames 0 --config C5 --spp 32 --steps 1 --warmup 1 > $O/kt_c5.log 2>&1 || { echo c5 failed; tail -5 $O/kt_c5.log; exit 1; }
for c in c2 c5; do echo "== $c"; cut -d, -f1-5 $O/kt_$c/kt_kernel_stats.csv | head -12; done
