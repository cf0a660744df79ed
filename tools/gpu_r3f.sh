#!/bin/bash
# cfg2: FastLane vs LeadLane for n = 3; serialized vs overlapped stages
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r3f
bash tools/ab.sh "cfg2 cfg5" full lead3 lead3w4 full lead3 || exit 1
for O in "" "--overlap" "" "--overlap"; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline $O > gpurun_out/r3f/ov.json 2> gpurun_out/r3f/ov.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r3f/ov.json').read().strip().splitlines()[-1]); print('cfg2 $O', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1), d['pipeline'], d['roofline']['frac'])"
done
HB_LIB=$PWD/etcd_amd/libhipbatch_lead3.so timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3f/lead3_tests.log 2>&1; tail -2 gpurun_out/r3f/lead3_tests.log
