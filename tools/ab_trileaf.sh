cd $GRAFT_REPO_ROOT
RTG_LIB=$PWD/raytracingrenderer_amd/lib/ab/trileaf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "wide_walk or adversarial or cull_equivalence or grazing or c3_full or synthetic or c1" > gpurun_out/ab_trileaf_parity.log 2>&1 || { echo PARITY FAIL; tail -30 gpurun_out/ab_trileaf_parity.log; exit 1; }
tail -2 gpurun_out/ab_trileaf_parity.log
CFGS="C3 C4 C2 S8" timeout -k 10 1000 bash tools/ab_cfg.sh
