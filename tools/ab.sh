#!/bin/bash
# A/B of engine builds on bench workloads:  gpurun -- bash tools/ab.sh "<workloads>" v1 v2 ...
# (etcd_amd/libhipbatch_<v>.so built beforehand; "full" = etcd_amd/libhipbatch.so)
# A workload "name:n" runs with --replicas n (e.g. follow:5).
# A variant "env:NAME=VAL" runs the full build with that environment variable;
# "arg:--flag" runs the full build with that bench.py flag.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/ab
WLS=$1; shift
for SPEC in $WLS; do
  WL=${SPEC%%:*}; RA=""; [ "$SPEC" != "$WL" ] && RA="--replicas ${SPEC#*:}"
  for v in "$@"; do
    lib=$PWD/etcd_amd/libhipbatch_$v.so; [ "$v" = full ] && lib=$PWD/etcd_amd/libhipbatch.so
    EV=""; XA=""
    case $v in env:*) lib=$PWD/etcd_amd/libhipbatch.so; EV=${v#env:};; arg:*) lib=$PWD/etcd_amd/libhipbatch.so; XA=${v#arg:};; esac
    env HB_LIB=$lib $EV timeout -k 10 300 python3 bench.py --workload $WL $RA --steps 20 --warmup 5 --no-cpu-baseline $XA \
      > "gpurun_out/ab/$WL${RA:+_r}.${v//[:=\/ ]/_}.json"
    F="gpurun_out/ab/$WL${RA:+_r}.${v//[:=\/ ]/_}.json" WL=$SPEC V=$v python3 - <<'PY'
import json, os
v, wl = os.environ["V"], os.environ["WL"]
d = json.loads(open(os.environ["F"]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(wl, v, "%.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"], "frac", r.get("frac"), "launch_us", r.get("launch_us_timed"),
      json.dumps(d.get("phases", {}).get("isolated")), d["parity_sanity"])
PY
  done
done
