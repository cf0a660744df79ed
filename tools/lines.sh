#!/bin/bash
# The host-facing bench lines of a round (wire, e2e, MultiNode 1k and 1M groups,
# each with its cpu_baseline), REPS times each MultiNode size:
#   gpurun -- bash tools/lines.sh <tag>          (LINES="wire e2e mn" to pick)
# The kernel lines with profiles come from tools/profile.sh.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-lines}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for L in ${LINES:-wire e2e mn}; do
  case $L in
    wire|e2e)
      timeout -k 10 300 python3 bench.py --workload $L --cpu-seconds 10 > $OUT/$L.json 2> $OUT/$L.err \
        || { tail -20 $OUT/$L.err; exit 1; }
      tail -c 300 $OUT/$L.json; echo ;;
    mn)
      for rep in $(seq 1 ${REPS:-2}); do
        for G in ${MN_GROUPS:-1000 1048576}; do
          S=200; W=20; [ $G -gt 4096 ] && S=4 && W=2
          timeout -k 10 500 python3 bench.py --workload multinode --groups $G --steps $S --warmup $W ${MN_ARGS:-} \
            > $OUT/multinode_${G}_$rep.json 2> $OUT/multinode_${G}_$rep.err || { tail -20 $OUT/multinode_${G}_$rep.err; exit 1; }
          python3 -c "import json;d=json.loads(open('$OUT/multinode_${G}_$rep.json').read().strip().splitlines()[-1]);print('$G rep $rep', round(d['value']/1e6,3),'M', round(d['ms_per_step'],3),'ms', 'cpu', round((d.get('cpu_baseline') or {}).get('value',0)/1e6,3))"
        done
      done ;;
  esac
done
