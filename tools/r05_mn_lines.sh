#!/bin/bash
# round 5 MultiNode lines (1k groups = BASELINE configs[0] shape, and 1M groups) with their cpu_baseline
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out/r05_mn
for rep in 1 2; do
  for G in ${MN_GROUPS:-1000 1048576}; do
    S=200; W=20; [ $G -gt 4096 ] && S=4 && W=2
    timeout -k 10 500 python3 bench.py --workload multinode --groups $G --steps $S --warmup $W > gpurun_out/r05_mn/multinode_${G}_$rep.json 2> gpurun_out/r05_mn/multinode_${G}_$rep.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/r05_mn/multinode_${G}_$rep.json').read().strip().splitlines()[-1]);print('$G rep $rep', round(d['value']/1e6,3),'M', round(d['ms_per_step'],3),'ms', 'cpu', round(d['cpu_baseline']['value']/1e6,3), {k:round(v*1e3,2) for k,v in d['split_s_per_step'].items()})"
  done
done
