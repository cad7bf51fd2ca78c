set -o pipefail
cd $GRAFT_REPO_ROOT
RTG_LIB=$GRAFT_REPO_ROOT/raytracingrenderer_amd/lib/ab/b_f8.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "c1 or tiles or c3_full or synthetic or many_samples or adaptive or light_tracer or radiosity" > gpurun_out/f8_pytest.log 2>&1 || { tail -20 gpurun_out/f8_pytest.log; exit 1; }
tail -1 gpurun_out/f8_pytest.log
SHARDS="8 1 8" bash tools/ab_shard.sh
