#!/bin/bash
# MultiNode A/B of the host library: the tree's build vs a variant directory (HBNB_DIR=etcd_amd/vhead)
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out/abmn15
for rep in 1 2 3; do
for v in new head; do
  D=""; [ $v = head ] && D="HBNB_DIR=$PWD/etcd_amd/vhead"
  env $D timeout -k 10 400 python3 bench.py --workload multinode --groups 1048576 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/abmn15/mn1m_${v}_$rep.json 2> gpurun_out/abmn15/mn1m_${v}_$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abmn15/mn1m_${v}_$rep.json').read().strip().splitlines()[-1]);h=d['host_phases_s_per_step'];print('1M $v $rep', round(d['value']/1e6,3),'M', round(d['ms_per_step'],1),'ms', {k:round(v*1e3,1) for k,v in h.items() if v>5e-4}, {k:round(v*1e3,1) for k,v in d['split_s_per_step'].items()})"
done; done
for rep in 1 2 3; do for v in new head; do
  D=""; [ $v = head ] && D="HBNB_DIR=$PWD/etcd_amd/vhead"
  env $D timeout -k 10 120 python3 bench.py --workload multinode --groups 1000 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/abmn15/mn1k_$v.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abmn15/mn1k_$v.json').read().strip().splitlines()[-1]);print('1k $v', round(d['value']/1e6,3),'M', round(d['ms_per_step']*1e3,1),'us')"
done; done
