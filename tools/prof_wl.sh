#!/bin/bash
# Kernel traces of the cfg3 / cfg4 bench lines:  gpurun -- bash tools/prof_wl.sh <tag> [lib variant] [workloads]
set -euo pipefail
TAG=${1:-pw}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
if [ -n "${2:-}" ] && [ "$2" != full ]; then export HB_LIB=$ROOT/etcd_amd/libhipbatch_$2.so; fi
for w in ${3:-cfg4 cfg3}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$w" -o run -- \
      python3 bench.py --workload $w --steps 4 --warmup 1 --no-cpu-baseline > "$OUT/$w.json" 2> "$OUT/$w.err"
  echo "== $w"; python3 - "$OUT/$w" <<'PY'
import csv, glob, sys
st = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(st[0])):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs'])/1e3:9.1f} pct {float(r['Percentage']):5.1f}")
PY
done
