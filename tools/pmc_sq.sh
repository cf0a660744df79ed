#!/bin/bash
# SQ-counter pass over a short bench run (one PMC group per rocprofv3 run).
#   gpurun -- bash tools/pmc_sq.sh <tag>      (BENCH_ARGS="--workload cfg4 ..." to pick the workload)
set -euo pipefail
TAG=${1:-sq}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
BA=${BENCH_ARGS:---steps 5 --warmup 2}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d "$OUT/sq1" -o run -- python3 bench.py $BA --no-cpu-baseline --no-profile > "$OUT/sq1.log" 2>&1
python3 tools/pmc_sum.py "$OUT/sq1" ${FILTER:-}
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT \
  --output-format csv -d "$OUT/sq2" -o run -- python3 bench.py $BA --no-cpu-baseline --no-profile > "$OUT/sq2.log" 2>&1
python3 tools/pmc_sum.py "$OUT/sq2" ${FILTER:-}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $BA --no-cpu-baseline --no-profile > "$OUT/fetch.log" 2>&1
python3 tools/pmc_sum.py "$OUT/fetch" ${FILTER:-}
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $BA --no-cpu-baseline --no-profile > "$OUT/write.log" 2>&1
python3 tools/pmc_sum.py "$OUT/write" ${FILTER:-}
