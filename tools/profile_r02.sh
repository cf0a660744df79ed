#!/bin/bash
# Round-2 evidence on the GPU box:  gpurun -- bash tools/profile_r02.sh
#   GPU tests + smoke, the cfg2 profile round (trace + FETCH/WRITE passes + bench line with the
#   measured traffic), traffic passes for cfg3 / cfg4, bench lines of every workload, traces.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out/r02
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r02/gpu_tests.log 2>&1
tail -2 gpurun_out/r02/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 && tail -1 gpurun_out/r02/smoke.log
bash tools/profile_round.sh r02 || exit 1
for wl in cfg4 cfg3; do bash tools/prof_pmc_wl.sh r02_$wl $wl 6 || exit 1; done
for wl in cfg3 cfg4 cfg5 tick wire e2e multinode; do
  timeout -k 10 300 python3 bench.py --workload $wl > gpurun_out/r02/bench_$wl.json 2> gpurun_out/r02/bench_$wl.err || { echo "bench $wl failed"; exit 1; }
  echo "bench $wl done"
done
bash tools/trace_wl.sh r02_tr cfg5 tick wire || exit 1
