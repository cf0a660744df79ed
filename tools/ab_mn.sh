#!/bin/bash
# Same-box A/B of host MultiNode builds:  bash tools/ab_mn.sh "<groups>" main var_g4 ...
# (variant = etcd_amd/<name>/ holding libhbnode.so + libhbnode_bench.so; "main" = etcd_amd/)
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/abmn
GS=$1; shift
for rep in 1 2; do
  for G in $GS; do
    for v in "$@"; do
      d=$PWD/etcd_amd/$v; [ "$v" = main ] && d=$PWD/etcd_amd
      S=20; [ $G -gt 100000 ] && S=4
      HBNB_DIR=$d timeout -k 10 300 python3 bench.py --workload multinode --groups $G --steps $S --warmup 2 --no-cpu-baseline \
        > gpurun_out/abmn/$G.$v.$rep.json 2>/dev/null || { echo "$G $v failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/abmn/$G.$v.$rep.json').read().strip().splitlines()[-1]); h=d['host_phases_s_per_step']; print('$G $v rep $rep', '%.4g' % d['value'], 'ms %.3f' % d['ms_per_step'], 'replay %.0f build %.0f adv %.0f resp %.0f prop %.0f us' % (h['event_replay']*1e6, h['ready_build']*1e6, h['advance']*1e6, h['bulk_responses']*1e6, h['bulk_proposals']*1e6))"
    done
  done
done
