#!/bin/bash
# MultiNode 1k-group A/B: small-step device path on / off (HB_SMALL_STEP), after the small-step tests
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out/abmn13
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_small_step_gpu.py > gpurun_out/abmn13/tests.log 2>&1 || { tail -30 gpurun_out/abmn13/tests.log; exit 1; }
tail -1 gpurun_out/abmn13/tests.log
for rep in 1 2 3; do
for v in 0 1; do
  HB_SMALL_STEP=$v timeout -k 10 120 python3 bench.py --workload multinode --groups 1000 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/abmn13/mn_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abmn13/mn_${v}_$rep.json').read().strip().splitlines()[-1]);h=d['host_phases_s_per_step'];print('small $v rep=$rep', round(d['value']/1e6,3),'M', round(d['ms_per_step']*1e3,1),'us', {k:round(v*1e6) for k,v in h.items() if v>2e-6})"
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abmn13/trace -- ./tools/mnprof/mnprof 1000 300 3 4 > gpurun_out/abmn13/trace_run.txt 2>&1
