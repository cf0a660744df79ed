#!/bin/bash
# The GPU suite, smoke and the default bench line on one box:
#   gpurun --timeout 1200 -- bash tools/gpu_suite.sh <tag>
# Every GPU step has its own time limit; the first failure ends the script.
TAG=${1:-suite}
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/$TAG/gpu_tests.log 2>&1 || { tail -60 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$TAG/gpu_tests.log
[ -n "$NO_SMOKE" ] && exit 0
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 \
  || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err \
  || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
tail -c 400 gpurun_out/$TAG/bench.json; echo
