#!/bin/bash
# round 5 MultiNode lines (1k groups = BASELINE configs[0] shape, and 1M groups), each run twice
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out/r05_mn
for rep in 1 2; do
  [ $rep = 1 ] || timeout -k 10 200 python3 bench.py --workload multinode --groups 1000 --steps 200 --warmup 20 > gpurun_out/r05_mn/multinode_1000_$rep.json 2> gpurun_out/r05_mn/multinode_1000_$rep.err || exit 1
  timeout -k 10 500 python3 bench.py --workload multinode --groups 1048576 --steps 4 --warmup 2 > gpurun_out/r05_mn/multinode_1048576_$rep.json 2> gpurun_out/r05_mn/multinode_1048576_$rep.err || exit 1
  for G in 1000 1048576; do
    python3 -c "import json;d=json.loads(open('gpurun_out/r05_mn/multinode_${G}_$rep.json').read().strip().splitlines()[-1]);print('$G rep $rep', round(d['value']/1e6,3),'M', round(d['ms_per_step'],3),'ms', 'cpu', round(d['cpu_baseline']['value']/1e6,3), {k:round(v*1e3,2) for k,v in d['split_s_per_step'].items()})"
  done
done
