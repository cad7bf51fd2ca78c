cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
RTG_LIB=$GRAFT_REPO_ROOT/raytracingrenderer_amd/lib/ab/b_fuse2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_north_star.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_fuse.log 2>&1; rc=$?; tail -3 gpurun_out/gputest_fuse.log; [ $rc -eq 0 ] && \
BENCH_ARGS="--shard-of 8" bash tools/ab.sh > gpurun_out/ab8.txt && bash tools/ab.sh > gpurun_out/ab1.txt && BENCH_ARGS="--config C2" bash tools/ab.sh > gpurun_out/ab2.txt
