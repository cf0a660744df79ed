#!/bin/bash
# Profiles of bench lines (trace + FETCH/WRITE passes + the line with its cpu_baseline):
#   WLS="cfg2 cfg3" gpurun -- bash tools/profile.sh r05
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=${1:-r05}
for W in ${WLS:-cfg2 cfg3 cfg4 cfg5 follow tick}; do
  CPUB="--cpu-seconds 10" WL=$W bash tools/profile_round.sh ${R}_$W > gpurun_out/${R}_$W.log 2>&1 || { tail -20 gpurun_out/${R}_$W.log; exit 1; }
  tail -1 gpurun_out/${R}_$W.log | cut -c1-300
  grep -A3 "Whole step" gpurun_out/${R}_$W/summary/${R}_${W}_summary.md | head -3
done
