#!/bin/bash
# Round 4 host MultiNode: its GPU tests, then the multinode bench lines (1k and 1M groups),
# then optional engine A/Bs:  WLS="cfg3 cfg4" VERS="full lu1" bash tools/gpu_r4_mn.sh
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r4
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_multinode_gpu.py tests/test_follower_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r4/mn_tests.log 2>&1 || { tail -60 gpurun_out/r4/mn_tests.log; exit 1; }
  tail -2 gpurun_out/r4/mn_tests.log
fi
for G in ${MN_GROUPS:-1000 1048576}; do
  S=20; W=2; [ $G -gt 100000 ] && { S=4; W=2; }
  timeout -k 10 300 python3 bench.py --workload multinode --groups $G --steps $S --warmup $W $MN_ARGS \
    > gpurun_out/r4/mn_$G.json 2> gpurun_out/r4/mn_$G.err || { tail -20 gpurun_out/r4/mn_$G.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4/mn_$G.json').read().strip().splitlines()[-1]); print($G, '%.4g' % d['value'], 'ms/round %.3f' % d['ms_per_step'], d['split_s_per_step'], d['host_phases_s_per_step'], d.get('cpu_baseline', {}).get('value'))"
  grep round gpurun_out/r4/mn_$G.err | tail -6 | tr '\n' ' '; echo
done
[ -n "$WLS" ] && bash tools/ab.sh "$WLS" ${VERS:-full}
exit 0
