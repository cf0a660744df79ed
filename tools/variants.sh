#!/bin/bash
# Time diagnostic builds of the engine side by side:  gpurun -- bash tools/variants.sh v1 v2 ...
# (etcd_amd/libhipbatch_<v>.so, built beforehand; "full" = etcd_amd/libhipbatch.so)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/var
for v in "$@"; do
  lib=$PWD/etcd_amd/libhipbatch_$v.so; [ "$v" = full ] && lib=$PWD/etcd_amd/libhipbatch.so
  HB_LIB=$lib timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/var/$v.json
  V=$v python3 - <<'PY'
import json, os
v = os.environ["V"]
d = json.loads(open(f"gpurun_out/var/{v}.json").read().strip().splitlines()[-1])
print(v, round(d["value"] / 1e9, 3), "ms/step", round(d["ms_per_step"] * 1e3, 1), "frac", d["roofline"]["frac"],
      json.dumps(d["phases"]), d["parity_sanity"])
PY
done
