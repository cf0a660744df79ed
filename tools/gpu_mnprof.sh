#!/bin/bash
# MultiNode host phases at 1M groups (bulk), JSON lines to gpurun_out/mnp/
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/mnp
for T in ${THREADS:-16 8}; do
  timeout -k 10 300 python3 bench.py --workload multinode --groups ${G:-1048576} --steps 4 --warmup 2 --mn-mode bulk \
    --mn-threads $T --no-cpu-baseline > gpurun_out/mnp/mn_$T.json 2> gpurun_out/mnp/mn_$T.err || { tail -5 gpurun_out/mnp/mn_$T.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/mnp/mn_$T.json').read().strip().splitlines()[-1]); print('threads $T', '%.3g'%d['value'], d['ms_per_step'], d['split_s_per_step'], d['host_phases_s_per_step'])"
done
nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
