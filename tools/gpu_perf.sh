# Perf iteration: parity tests of the engine, then cfg2 / cfg5 bench lines (no CPU baseline).
set -e
TAG=${1:-perf}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -40 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
for WL in ${WLS:-cfg2 cfg5}; do
  timeout -k 10 300 python3 bench.py --workload $WL --no-cpu-baseline > gpurun_out/$TAG/$WL.json 2> gpurun_out/$TAG/$WL.err
  python3 -c "import json;d=json.loads(open('gpurun_out/$TAG/$WL.json').read().strip().splitlines()[-1]);print('$WL', '%.4g'%d['value'], 'ms/step %.4f'%d['ms_per_step'], d['phases'].get('isolated'), 'frac', d['roofline']['frac'], 'step_frac', d['roofline'].get('step_frac'), d['parity_sanity'])"
done
