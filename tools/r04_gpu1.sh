set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "queued_frames or queue_segment or tiles_and_chunks or many_samples" > gpurun_out/r04_gputest_pipe.log 2>&1 && \
ROUNDS=1 tools/ab_dropin.sh > gpurun_out/r04_ab_dropin.txt 2>&1
