#!/bin/bash
# Round 4: the whole -m gpu suite on the current build, then same-box A/B of engine builds.
#   WLS="cfg2 cfg3" VERS="base full" bash tools/gpu_r4_ab.sh
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r4
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread $TESTARGS \
    > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r4/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/r4/gpu_tests.log
fi
bash tools/ab.sh "${WLS:-cfg2}" ${VERS:-base full}
