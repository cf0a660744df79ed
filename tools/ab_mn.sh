#!/bin/bash
# Same-box A/B of host MultiNode builds or settings:
#   bash tools/ab_mn.sh "<groups>" main var_g4 env:HBN_SMALL_WAYS=1 env:HBN_SPIN_US=0,HBN_PIN_L3=0 ...
# (a build variant = etcd_amd/<name>/ holding libhbnode.so + libhbnode_bench.so; "main" = etcd_amd/;
#  "env:A=x,B=y" = the main build with those environment variables)
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/abmn
GS=$1; shift
for rep in 1 2 3; do
  for G in $GS; do
    for v in "$@"; do
      d=$PWD/etcd_amd; ENVS=""
      case "$v" in
        main) ;;
        env:*) ENVS=$(echo "${v#env:}" | tr ',' ' ') ;;
        *) d=$PWD/etcd_amd/$v ;;
      esac
      S=200; W=20; [ $G -gt 4096 ] && S=20 && W=2; [ $G -gt 100000 ] && S=4
      tag=$(echo "$v" | tr ':=,/' '____')
      env HBNB_DIR=$d $ENVS timeout -k 10 400 python3 bench.py --workload multinode --groups $G --steps $S --warmup $W \
        --no-cpu-baseline > gpurun_out/abmn/$G.$tag.$rep.json 2>/dev/null || { echo "$G $v failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/abmn/$G.$tag.$rep.json').read().strip().splitlines()[-1]); h=d['host_phases_s_per_step']; print('$G $v rep $rep', '%.4g' % d['value'], 'ms %.3f' % d['ms_per_step'], 'replay %.0f build %.0f adv %.0f resp %.0f prop %.0f us' % (h['event_replay']*1e6, h['ready_build']*1e6, h['advance']*1e6, h['bulk_responses']*1e6, h['bulk_proposals']*1e6))"
    done
  done
done
