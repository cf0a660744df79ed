#!/bin/bash
# Kernel-trace stats for every bench workload:  gpurun -- bash tools/prof_all.sh <tag>
set -euo pipefail
TAG=${1:-pa}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
for WL in ${WLS:-cfg2 cfg5 cfg3 cfg4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$WL" -o run -- \
      python3 bench.py --workload $WL --steps 10 --warmup 3 --no-cpu-baseline --no-profile > "$OUT/$WL.json" 2> "$OUT/$WL.err"
  echo "$WL done"
done
