#!/bin/bash
# Round-4 profiles: trace + FETCH/WRITE passes + bench line (with its cpu_baseline) per workload.
#   WLS="cfg3 follow" bash tools/profile_r04.sh
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for W in ${WLS:-cfg2 cfg3 cfg4 cfg5 follow tick}; do
  CPUB="--cpu-seconds 10" WL=$W bash tools/profile_round.sh r04_$W > gpurun_out/r04_$W.log 2>&1 || { tail -20 gpurun_out/r04_$W.log; exit 1; }
  tail -1 gpurun_out/r04_$W.log | cut -c1-300
  grep -A3 "Whole step" gpurun_out/r04_$W/summary/r04_${W}_summary.md | head -3
done
