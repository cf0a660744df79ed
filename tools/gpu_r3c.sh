#!/bin/bash
# GPU suite, lazy-vs-eager ring heads A/B, MultiNode 1k / 1M bulk lines, profiler probe
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r3c
bash tools/gpu_ab_tests.sh "cfg2 cfg3 cfg5" full eager || exit 1
for G in 1000 1048576; do
  ST=20; [ $G -gt 100000 ] && ST=4
  timeout -k 10 400 python3 bench.py --workload multinode --groups $G --steps $ST --warmup 2 --mn-mode bulk \
    --no-cpu-baseline > gpurun_out/r3c/mn_${G}.json 2> gpurun_out/r3c/mn_${G}.err || { tail -5 gpurun_out/r3c/mn_${G}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r3c/mn_${G}.json').read().strip().splitlines()[-1]); print('mn $G', '%.3g'%d['value'], d['ms_per_step'], d['split_s_per_step'], d['host_phases_s_per_step'])"
done
which perf gprof valgrind ltrace 2>/dev/null; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; true
timeout -k 10 300 python3 bench.py --workload e2e --no-cpu-baseline > gpurun_out/r3c/e2e.json 2> gpurun_out/r3c/e2e.err || { tail -5 gpurun_out/r3c/e2e.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3c/e2e.json').read().strip().splitlines()[-1]); print('e2e', '%.3g'%d['value'], d['ms_per_step'], d['bytes_per_step'], d['split_ms_per_step'], d.get('host_expand_ms_per_step'))"
