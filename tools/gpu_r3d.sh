#!/bin/bash
# GPU suite (eager heads default), cfg2 / e2e lines, gprof of the host MultiNode path at 1k and 1M groups
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r3d
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/r3d/gpu_tests.log 2>&1 || { tail -60 gpurun_out/r3d/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3d/gpu_tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r3d/cfg2.json 2> gpurun_out/r3d/cfg2.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r3d/cfg2.json').read().strip().splitlines()[-1]); print('cfg2', '%.4g'%d['value'], d['ms_per_step'], d['phases']['isolated'])"
timeout -k 10 300 python3 bench.py --workload e2e --no-cpu-baseline > gpurun_out/r3d/e2e.json 2> gpurun_out/r3d/e2e.err || { tail -5 gpurun_out/r3d/e2e.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3d/e2e.json').read().strip().splitlines()[-1]); print('e2e', '%.3g'%d['value'], d['ms_per_step'], d['bytes_per_step'], d['pcie_gbs'], d.get('host_expand_ms_per_step'), d['parity_sanity'])"
cd gpurun_out/r3d
timeout -k 10 200 ../../tools/mnprof/mnprof 1000 400 3 1 && gprof ../../tools/mnprof/mnprof gmon.out > gprof_1k.txt && head -40 gprof_1k.txt | tail -34
rm -f gmon.out
timeout -k 10 300 ../../tools/mnprof/mnprof 1048576 3 3 1 && gprof ../../tools/mnprof/mnprof gmon.out > gprof_1m.txt && head -40 gprof_1m.txt | tail -34
