#!/bin/bash
# GPU suite, cfg4 vote-broadcast A/B, MultiNode 1k / 1M with pool spin 0 / 50 / 200 us
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r3e
bash tools/gpu_ab_tests.sh "cfg4" full novb full novb || exit 1
for SP in 0 50 200; do
for G in 1000 1048576; do
  ST=20; [ $G -gt 100000 ] && ST=4
  HBN_SPIN_US=$SP timeout -k 10 400 python3 bench.py --workload multinode --groups $G --steps $ST --warmup 2 --mn-mode bulk \
    --no-cpu-baseline > gpurun_out/r3e/mn_${G}_$SP.json 2> gpurun_out/r3e/mn_${G}_$SP.err || { tail -5 gpurun_out/r3e/mn_${G}_$SP.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r3e/mn_${G}_$SP.json').read().strip().splitlines()[-1]); print('mn $G spin $SP', '%.3g'%d['value'], round(d['ms_per_step'],3), {k: round(v*1e3,3) for k,v in d['split_s_per_step'].items()}, {k: round(v*1e3,3) for k,v in d['host_phases_s_per_step'].items() if v})"
done
done
