#!/bin/bash
# GPU suite on the default build, then an A/B of variants on the given workloads:
#   gpurun -- bash tools/gpu_ab_tests.sh "<workloads>" full v1 v2 ...
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/abt
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/abt/gpu_tests.log 2>&1 || { tail -60 gpurun_out/abt/gpu_tests.log; exit 1; }
tail -2 gpurun_out/abt/gpu_tests.log
WLS=$1; shift
bash tools/ab.sh "$WLS" "$@"
