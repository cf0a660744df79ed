#!/bin/bash
# Kernel trace + one SQ counter pass:  gpurun -- bash tools/prof_quick.sh <tag>
set -euo pipefail
TAG=${1:-pq}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-profile > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
echo trace done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d "$OUT/sq1" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile > "$OUT/sq1.log" 2>&1
echo sq done
