#!/bin/bash
# n = 3 with a third route slot (MsgProp on the fast lane): the suite, the MultiNode lines, then
# same-box A/B against the two-slot engine (k2) and the 1024-group route variant (rg10)
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r4
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r4/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4/gpu_tests.log
SKIP_TESTS=1 bash tools/gpu_r4_mn.sh || exit 1
bash tools/ab.sh "cfg2 cfg5 follow" k2 full rg10 || exit 1
bash tools/ab.sh "cfg2 cfg5" k2 full rg10 || exit 1
