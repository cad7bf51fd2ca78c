# bench line with the VALU sub-objects (short run) and the bench contract test
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-frames 0 --steps 5 > gpurun_out/b25.log 2>&1 || { tail -5 gpurun_out/b25.log; exit 1; }
tail -1 gpurun_out/b25.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['valu'], d['roofline_shade']['valu'])"
timeout -k 10 300 python -u -m pytest tests/test_bench.py -m gpu -q --timeout 250 --timeout-method thread 2>&1 | tail -2
