#!/bin/bash
# Round-4 evidence on the final build, part A: smoke, the default bench line, then per-workload
# profiles (trace + FETCH/WRITE passes + bench line with cpu_baseline).  Part B: PART=B.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r04f
if [ "${PART:-A}" = A ]; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04f/smoke.log 2>&1 \
    || { tail -20 gpurun_out/r04f/smoke.log; exit 1; }
  tail -1 gpurun_out/r04f/smoke.log
  timeout -k 10 300 python3 bench.py > gpurun_out/r04f/bench.json 2> gpurun_out/r04f/bench.err || { tail -20 gpurun_out/r04f/bench.err; exit 1; }
  tail -c 400 gpurun_out/r04f/bench.json
  WLS="cfg2 follow tick" bash tools/profile_r04.sh || exit 1
else
  WLS="cfg4 cfg5" bash tools/profile_r04.sh || exit 1
  for W in e2e wire; do
    timeout -k 10 300 python3 bench.py --workload $W > gpurun_out/r04f/$W.json 2> gpurun_out/r04f/$W.err || { tail -20 gpurun_out/r04f/$W.err; exit 1; }
    tail -c 300 gpurun_out/r04f/$W.json; echo
  done
fi
