#!/bin/bash
# Round 4: the whole -m gpu suite, then the multinode lines and the engine lines on the current build.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r4
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r4/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4/gpu_tests.log
SKIP_TESTS=1 bash tools/gpu_r4_mn.sh
