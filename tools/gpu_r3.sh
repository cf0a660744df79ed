#!/bin/bash
# Round-3 GPU check: the whole -m gpu suite (new log-index tests first), smoke, default bench.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r3
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  ${TESTS:-tests} > gpurun_out/r3/gpu_tests.log 2>&1 \
  || { tail -40 gpurun_out/r3/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1
tail -1 gpurun_out/r3/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r3/bench.json 2> gpurun_out/r3/bench.err
tail -1 gpurun_out/r3/bench.json
