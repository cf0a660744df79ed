#!/bin/bash
# wire bench line + kernel trace:  gpurun -- bash tools/gpu_wire.sh
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/wi
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_wire_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/wi/tests.log 2>&1 || { tail -30 gpurun_out/wi/tests.log; exit 1; }
tail -1 gpurun_out/wi/tests.log
timeout -k 10 300 python3 -u bench.py --workload wire --steps 10 --warmup 2 > gpurun_out/wi/wire.json 2> gpurun_out/wi/wire.err || { tail -20 gpurun_out/wi/wire.err; exit 1; }
cat gpurun_out/wi/wire.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wi/trace -o run -- \
    python3 bench.py --workload wire --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/wi/wire_trace.json 2> gpurun_out/wi/trace.err
python3 - <<'PY'
import csv, glob
st = glob.glob("gpurun_out/wi/trace/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(st[0])):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs'])/1e3:9.1f} pct {float(r['Percentage']):5.1f}")
PY
