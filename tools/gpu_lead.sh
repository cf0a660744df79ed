#!/bin/bash
# k_lead check: the n >= 5 parity tests on the default build, then cfg3 / cfg4 A/B of the given variants
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/lead
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/lead/gpu_tests.log 2>&1 || { tail -60 gpurun_out/lead/gpu_tests.log; exit 1; }
tail -2 gpurun_out/lead/gpu_tests.log
bash tools/ab.sh "cfg3 cfg4" "$@"
