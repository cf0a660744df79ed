#!/bin/bash
# Kernel-trace stats of bench workloads:  gpurun -- bash tools/trace_wl.sh <tag> [workload...]
# (HB_LIB=<path> traces a variant build of the engine)
set -euo pipefail
TAG=${1:-tr}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
for WL in ${@:-cfg2}; do
  echo "== $WL ${HB_LIB:-}"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$WL" -o run -- \
      python3 bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline --no-profile > "$OUT/$WL.json" 2> "$OUT/$WL.err"
  python3 - "$OUT/$WL" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-40s %5s %9.2f us" % (r["Name"].split("(")[0].replace("void ", "")[:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
