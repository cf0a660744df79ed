#!/bin/bash
# MultiNode host-side tests on the GPU:  gpurun -- bash tools/gpu_mn.sh
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/mn
timeout -k 10 300 python3 -u -m pytest tests/test_multinode_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mn/tests.log 2>&1 || { tail -60 gpurun_out/mn/tests.log; exit 1; }
tail -15 gpurun_out/mn/tests.log
