#!/bin/bash
# cfg4 / cfg3 bench lines of diagnostic engine builds:  gpurun -- bash tools/variants_wl.sh v1 v2 ...
# (etcd_amd/libhipbatch_<v>.so, built beforehand; "full" = etcd_amd/libhipbatch.so)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/varwl
for v in "$@"; do
  lib=$PWD/etcd_amd/libhipbatch_$v.so; [ "$v" = full ] && lib=$PWD/etcd_amd/libhipbatch.so
  for wl in cfg4 cfg3; do
    HB_LIB=$lib timeout -k 10 200 python3 bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/varwl/${v}_$wl.json
    V=$v W=$wl python3 - <<'PY'
import json, os
v, wl = os.environ["V"], os.environ["W"]
d = json.loads(open(f"gpurun_out/varwl/{v}_{wl}.json").read().strip().splitlines()[-1])
print(v, wl, round(d["value"] / 1e9, 3), "ms/step", round(d["ms_per_step"], 3), json.dumps(d.get("phases")), d.get("parity_sanity"))
PY
  done
done
