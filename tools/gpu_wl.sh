#!/bin/bash
# GPU parity tests, then the cfg4 / cfg3 bench lines:  gpurun -- bash tools/gpu_wl.sh
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/wl
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/wl/gpu_tests.log 2>&1 || { tail -40 gpurun_out/wl/gpu_tests.log; exit 1; }
tail -2 gpurun_out/wl/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --workload cfg4 --steps 5 --warmup 1 > gpurun_out/wl/cfg4.json 2> gpurun_out/wl/cfg4.err || { tail -20 gpurun_out/wl/cfg4.err; exit 1; }
cat gpurun_out/wl/cfg4.json
timeout -k 10 300 python3 -u bench.py --workload cfg3 --steps 6 --warmup 2 > gpurun_out/wl/cfg3.json 2> gpurun_out/wl/cfg3.err || { tail -20 gpurun_out/wl/cfg3.err; exit 1; }
cat gpurun_out/wl/cfg3.json
