#!/bin/bash
# suite on the LDS-slot build, then cfg3 / cfg4 A/B against the previous engine, then the tick line
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r4 gpurun_out/r04f
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r4/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4/gpu_tests.log
bash tools/ab.sh "cfg4 cfg3" prelds full || exit 1
bash tools/ab.sh "cfg4 cfg3" prelds full || exit 1
timeout -k 10 300 python3 bench.py --workload tick > gpurun_out/r04f/tick.json 2> gpurun_out/r04f/tick.err || exit 1
tail -c 500 gpurun_out/r04f/tick.json
