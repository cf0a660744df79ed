#!/bin/bash
# Round-4 closing evidence after the tick split: the whole GPU suite, smoke, the default line,
# the tick profile (trace + FETCH/WRITE passes + line), the MultiNode lines
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r04f gpurun_out/r4
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r4/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04f/smoke.log 2>&1 \
  || { tail -20 gpurun_out/r04f/smoke.log; exit 1; }
tail -1 gpurun_out/r04f/smoke.log
[ -n "$AB" ] && { bash tools/ab.sh "$AB" prev full prev full || exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/r04f/bench.json 2> gpurun_out/r04f/bench.err || { tail -20 gpurun_out/r04f/bench.err; exit 1; }
tail -c 300 gpurun_out/r04f/bench.json; echo
WLS="${PWLS:-tick}" bash tools/profile_r04.sh || exit 1
[ -n "$MN" ] && { SKIP_TESTS=1 bash tools/gpu_r4_mn.sh || exit 1; }
exit 0
