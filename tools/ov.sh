#!/bin/bash
# overlap vs no overlap, with and without apply-phase events:  gpurun -- bash tools/ov.sh
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/ov
for args in "" "--no-profile" "--overlap" "--overlap --no-profile"; do
  timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline $args > gpurun_out/ov/o.json
  A="$args" python3 - <<'PY'
import json, os
d = json.loads(open("gpurun_out/ov/o.json").read().strip().splitlines()[-1])
print(repr(os.environ["A"]), round(d["value"] / 1e9, 3), round(d["ms_per_step"] * 1e3, 1),
      (d["roofline"] or {}).get("frac"), d["parity_sanity"])
PY
done
