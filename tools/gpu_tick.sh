#!/bin/bash
# tick bench line + kernel trace:  gpurun -- bash tools/gpu_tick.sh
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/tk
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --workload tick --steps 20 --warmup 3 > gpurun_out/tk/tick.json 2> gpurun_out/tk/tick.err || { tail -20 gpurun_out/tk/tick.err; exit 1; }
cat gpurun_out/tk/tick.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tk/trace -o run -- \
    python3 bench.py --workload tick --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/tk/tick_trace.json 2> gpurun_out/tk/trace.err
python3 - <<'PY'
import csv, glob
st = glob.glob("gpurun_out/tk/trace/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(st[0])):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs'])/1e3:9.1f} pct {float(r['Percentage']):5.1f}")
PY
