#!/bin/bash
# Kernel trace + HBM traffic passes of one bench workload:
#   gpurun -- bash tools/prof_pmc_wl.sh <tag> <workload> [steps]
# (one counter group per rocprofv3 pass, MI355X_MICROARCH.md; folded by tools/prof_summary.py)
set -euo pipefail
TAG=$1; WL=$2; STEPS=${3:-10}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --workload $WL --steps "$STEPS" --warmup 3 --no-cpu-baseline > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
echo "$TAG trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --workload $WL --steps 4 --warmup 2 --no-cpu-baseline --no-profile > "$OUT/pmc_fetch.log" 2>&1
echo "$TAG fetch done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py --workload $WL --steps 4 --warmup 2 --no-cpu-baseline --no-profile > "$OUT/pmc_write.log" 2>&1
echo "$TAG write done"
python3 tools/prof_summary.py "$OUT" --tag "$TAG" --out "$OUT/summary" > "$OUT/summary.log"
echo "$TAG summary done"
