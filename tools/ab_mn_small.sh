#!/bin/bash
# MultiNode A/B: bulk ingestion over the small-phase partners (HBN_SMALL_BULK); 1M groups with the
# application thread pinned or not, and the other workers on the caller's NUMA node (HBN_PIN_NODE)
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out/abmn12
for rep in 1 2 3; do
for v in "0" "512"; do
  A=""; [ $v != 0 ] && A="HBN_SMALL_BULK=$v"
  env $A timeout -k 10 120 python3 bench.py --workload multinode --groups 1000 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/abmn12/mn_${v}_$rep.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abmn12/mn_${v}_$rep.json').read().strip().splitlines()[-1]);h=d['host_phases_s_per_step'];print('bulk $v rep=$rep', round(d['value']/1e6,3),'M', round(d['ms_per_step']*1e3,1),'us', {k:round(v*1e6) for k,v in h.items() if v>2e-6})"
done; done
for v in "0 pin" "0 nopin" "1 pin" "1 nopin"; do
  set -- $v
  P=""; [ $2 = nopin ] && P="--mn-no-pin"
  HBN_PIN_NODE=$1 timeout -k 10 400 python3 bench.py --workload multinode --groups 1048576 --steps 4 --warmup 2 --no-cpu-baseline $P > gpurun_out/abmn12/mn1m_$1_$2.json 2> gpurun_out/abmn12/mn1m_$1_$2.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abmn12/mn1m_$1_$2.json').read().strip().splitlines()[-1]);h=d['host_phases_s_per_step'];print('1M $v', round(d['value']/1e6,3),'M', round(d['ms_per_step'],1),'ms', {k:round(v*1e3,1) for k,v in h.items() if v>2e-4}, {k:round(v*1e3,1) for k,v in d['split_s_per_step'].items()})"
done
