#!/bin/bash
# Round-4 GPU check: selected tests first ($FIRST), then the whole -m gpu suite, smoke, default bench.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r4
if [ -n "$FIRST" ]; then
  timeout -k 10 900 python3 -u -m pytest $FIRST -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/r4/gpu_first.log 2>&1 || { tail -60 gpurun_out/r4/gpu_first.log; exit 1; }
  tail -3 gpurun_out/r4/gpu_first.log
fi
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread $DESEL \
    > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r4/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/r4/gpu_tests.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1
  tail -1 gpurun_out/r4/smoke.log
fi
timeout -k 10 300 python3 bench.py $BENCH_ARGS > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.err
tail -1 gpurun_out/r4/bench.json
