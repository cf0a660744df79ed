#!/bin/bash
# MultiNode API end-to-end bench lines:  gpurun -- bash tools/gpu_mnbench.sh
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/mnb
timeout -k 10 300 python3 -u -m pytest tests/test_multinode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mnb/tests.log 2>&1 || { tail -40 gpurun_out/mnb/tests.log; exit 1; }
tail -2 gpurun_out/mnb/tests.log
timeout -k 10 200 python3 -u bench.py --workload multinode --groups 1000 --steps 200 --warmup 20 > gpurun_out/mnb/g1k.json 2> gpurun_out/mnb/g1k.err || { tail -20 gpurun_out/mnb/g1k.err; exit 1; }
cat gpurun_out/mnb/g1k.json
timeout -k 10 300 python3 -u bench.py --workload multinode --groups 1048576 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/mnb/g1m.json 2> gpurun_out/mnb/g1m.err || { tail -20 gpurun_out/mnb/g1m.err; exit 1; }
cat gpurun_out/mnb/g1m.json; cat gpurun_out/mnb/g1m.err
