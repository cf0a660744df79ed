#!/bin/bash
# The rest of the round-2 evidence (after tools/profile_r02.sh's cfg2 round and cfg4 passes):
#   gpurun -- bash tools/profile_r02b.sh
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out/r02
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r02/gpu_tests_b.log 2>&1
tail -2 gpurun_out/r02/gpu_tests_b.log
bash tools/prof_pmc_wl.sh r02_cfg3 cfg3 6 || exit 1
for wl in cfg3 cfg4 cfg5 tick wire e2e multinode; do
  timeout -k 10 300 python3 bench.py --workload $wl > gpurun_out/r02/bench_$wl.json 2> gpurun_out/r02/bench_$wl.err || { echo "bench $wl failed"; exit 1; }
  echo "bench $wl done"
done
timeout -k 10 300 python3 bench.py --workload multinode --groups 1048576 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02/bench_multinode_1m.json 2> gpurun_out/r02/bench_multinode_1m.err || echo "multinode 1m failed"
bash tools/trace_wl.sh r02_tr cfg5 tick wire || exit 1
