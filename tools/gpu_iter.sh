#!/bin/bash
# Perf iteration: engine parity tests, then bench lines of variant builds, then
# the aux workloads ($WLS) on the main build.
#   gpurun -- bash tools/gpu_iter.sh <tag> <variant>...   (variants as tools/variants.sh)
set -e
TAG=$1; shift
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests/test_parity_gpu.py tests/test_follower_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -40 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
bash tools/variants.sh "$@"
for WL in ${WLS:-}; do
  timeout -k 10 300 python3 bench.py --workload $WL --no-cpu-baseline > gpurun_out/$TAG/$WL.json 2> gpurun_out/$TAG/$WL.err
  python3 -c "import json;d=json.loads(open('gpurun_out/$TAG/$WL.json').read().strip().splitlines()[-1]);print('$WL', '%.4g'%d['value'], 'ms/step %.4f'%d['ms_per_step'], d.get('phases',{}).get('isolated'), d.get('parity_sanity'))"
done
