#!/bin/bash
# GPU parity tests then a short bench:  gpurun -- bash tools/gpu_quick.sh
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/q
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/q/gpu_tests.log 2>&1 || { tail -40 gpurun_out/q/gpu_tests.log; exit 1; }
tail -2 gpurun_out/q/gpu_tests.log
bash tools/variants.sh full "$@"
