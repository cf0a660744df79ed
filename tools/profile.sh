#!/bin/bash
# Profiles of bench lines (trace + FETCH/WRITE passes + the line with its cpu_baseline):
#   WLS="cfg2 cfg3" gpurun -- bash tools/profile.sh r05
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=${1:-r05}
for W in ${WLS:-cfg2 cfg3 cfg4 cfg5 follow follow:5 mixed tick}; do
  T=${W/:/n}  # follow:5 -> follown5
  CPUB="--cpu-seconds 10" WL=$W bash tools/profile_round.sh ${R}_$T > gpurun_out/${R}_$T.log 2>&1 || { tail -20 gpurun_out/${R}_$T.log; exit 1; }
  tail -1 gpurun_out/${R}_$T.log | cut -c1-300
  grep -A3 "Whole step" gpurun_out/${R}_$T/summary/${R}_${T}_summary.md | head -3
done
