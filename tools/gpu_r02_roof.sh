set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r02_roof
O=$R/gpurun_out/r02_roof
timeout -k 10 120 ./tools/micro/roof > $O/sweep.jsonl 2>&1 || { echo sweep failed; cat $O/sweep.jsonl; exit 1; }
cat $O/sweep.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- $R/tools/micro/roof 1024 0 64 > $O/fetch.log 2>&1 || { echo fetch failed; tail $O/fetch.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/hit -o hit --output-format csv -- $R/tools/micro/roof 1024 0 64 > $O/hit.log 2>&1 || { echo hit failed; tail $O/hit.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/rdreq -o rdreq --output-format csv -- $R/tools/micro/roof 1024 0 64 > $O/rdreq.log 2>&1 || { echo rdreq failed; tail $O/rdreq.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/fetch69 -o fetch69 --output-format csv -- $R/tools/micro/roof 69 0 64 > $O/fetch69.log 2>&1 || { echo fetch69 failed; tail $O/fetch69.log; exit 1; }
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "reference_classes" > $O/reftests.log 2>&1 || { echo reftests failed; tail -30 $O/reftests.log; exit 1; }
tail -2 $O/reftests.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
