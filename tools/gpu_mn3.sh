#!/bin/bash
# Round-3 MultiNode host path: GPU tests of the MultiNode files, then bulk vs per-call on one box.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/mn3
timeout -k 10 400 python3 -u -m pytest tests/test_multinode_gpu.py tests/test_follower_gpu.py -m gpu -x -v --timeout 180 \
  --timeout-method thread > gpurun_out/mn3/tests.log 2>&1 || { tail -40 gpurun_out/mn3/tests.log; exit 1; }
tail -2 gpurun_out/mn3/tests.log
for G in 1000 1048576; do
  ST=20; [ $G -gt 100000 ] && ST=4
  for M in bulk percall; do
    timeout -k 10 400 python3 bench.py --workload multinode --groups $G --steps $ST --warmup 2 --mn-mode $M \
      --no-cpu-baseline > gpurun_out/mn3/mn_${G}_${M}.json 2> gpurun_out/mn3/mn_${G}_${M}.err || { tail -5 gpurun_out/mn3/mn_${G}_${M}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/mn3/mn_${G}_${M}.json').read().strip().splitlines()[-1]); print('$G $M', '%.3g'%d['value'], d['ms_per_step'], d['split_s_per_step'], d['parity_sanity'])"
  done
done
