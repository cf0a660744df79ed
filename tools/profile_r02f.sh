#!/bin/bash
# Final round-2 evidence on the judged build:  gpurun -- bash tools/profile_r02f.sh
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out/r02f
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r02f/gpu_tests.log 2>&1
tail -2 gpurun_out/r02f/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02f/smoke.log 2>&1 && tail -1 gpurun_out/r02f/smoke.log
bash tools/profile_round.sh r02f || exit 1
for wl in cfg3 cfg4 cfg5; do
  timeout -k 10 300 python3 bench.py --workload $wl > gpurun_out/r02f/bench_$wl.json 2> gpurun_out/r02f/bench_$wl.err || { echo "bench $wl failed"; exit 1; }
  echo "bench $wl done"
done
bash tools/trace_wl.sh r02f_tr cfg4 cfg5 || exit 1
