#!/bin/bash
# Round-4 final evidence: the suite, smoke, the default line, then per-workload profiles (A: cfg2 follow tick
# cfg3; B: cfg4 cfg5 + e2e / wire / multinode lines)
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r04f gpurun_out/r4
if [ "${PART:-A}" = A ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r4/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/r4/gpu_tests.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04f/smoke.log 2>&1 \
    || { tail -20 gpurun_out/r04f/smoke.log; exit 1; }
  tail -1 gpurun_out/r04f/smoke.log
  timeout -k 10 300 python3 bench.py > gpurun_out/r04f/bench.json 2> gpurun_out/r04f/bench.err || { tail -20 gpurun_out/r04f/bench.err; exit 1; }
  tail -c 300 gpurun_out/r04f/bench.json; echo
  WLS="cfg2 follow tick cfg3" bash tools/profile_r04.sh || exit 1
else
  WLS="cfg4 cfg5" bash tools/profile_r04.sh || exit 1
  for W in e2e wire; do
    timeout -k 10 300 python3 bench.py --workload $W > gpurun_out/r04f/$W.json 2> gpurun_out/r04f/$W.err || { tail -20 gpurun_out/r04f/$W.err; exit 1; }
    tail -c 200 gpurun_out/r04f/$W.json; echo
  done
  SKIP_TESTS=1 bash tools/gpu_r4_mn.sh || exit 1
fi
