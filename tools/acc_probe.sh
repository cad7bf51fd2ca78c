cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_acc.log 2>&1; rc=$?; tail -3 gpurun_out/gputest_acc.log; [ $rc -eq 0 ] && \
BENCH_ARGS="--config C5 --spp 32 --warmup 1" bash tools/ab.sh > gpurun_out/ab5.txt && bash tools/ab.sh > gpurun_out/ab1.txt
