#!/bin/bash
# Round profile on the GPU box:  gpurun -- bash tools/profile_round.sh rNN
#   1. rocprofv3 --kernel-trace --stats over bench.py   (per-kernel average durations)
#   2. PMC pass FETCH_SIZE  (own run, MI355X_MICROARCH.md: one counter group per pass)
#   3. PMC pass WRITE_SIZE
#   4. plain bench.py (the JSON line, with the traffic the passes measured)
# WL=<workload> (default cfg2) profiles another bench line (cfg3 / cfg4 / cfg5 / tick); BA= adds bench args.
# Outputs under gpurun_out/<tag>/; tools/prof_summary.py folds them into profiles/.
set -euo pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
STEPS=${STEPS:-20}
# WL=<workload>[:<replicas>] (e.g. follow:5)
SPEC=${WL:-cfg2}; W0=${SPEC%%:*}
WA="--workload $W0"; [ "$SPEC" != "$W0" ] && WA="$WA --replicas ${SPEC#*:}"
WA="$WA ${BA:-}"  # BA=<more bench args> (e.g. --role-order)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $WA --steps "$STEPS" --warmup 5 --no-cpu-baseline > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
echo "trace done"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py $WA --steps 5 --warmup 2 --no-cpu-baseline --no-profile > "$OUT/pmc_fetch.log" 2>&1
echo "fetch done"
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py $WA --steps 5 --warmup 2 --no-cpu-baseline --no-profile > "$OUT/pmc_write.log" 2>&1
echo "write done"
python3 tools/prof_summary.py "$OUT" --tag "$TAG" --out "$OUT/summary" > "$OUT/summary.log"
echo "summary done"
# the summary goes where it is committed (profiles/), so the line's traffic_source names that file
cp "$OUT/summary/${TAG}_traffic.json" "$ROOT/profiles/"
timeout -k 10 300 python3 bench.py $WA ${CPUB:---no-cpu-baseline} --traffic-json "profiles/${TAG}_traffic.json" > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench done"
tail -1 "$OUT/bench.json"
