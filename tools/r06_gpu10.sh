#!/bin/bash
# Round 6: the RCCL self-send tests (ncclSend/ncclRecv on a one-GPU box), then the full GPU suite.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r06j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -x -v --timeout 120 --timeout-method thread -k "group" > $O/group_tests.log 2>&1 || { tail -30 $O/group_tests.log; exit 1; }
grep -c PASSED $O/group_tests.log; tail -1 $O/group_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
