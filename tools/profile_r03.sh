#!/bin/bash
# Round-3 profiles: SQ counters of the cfg2 step, then trace + FETCH/WRITE passes + bench line per workload
cd ${GRAFT_REPO_ROOT:-$(pwd)}
BENCH_ARGS="--steps 5 --warmup 2" FILTER=k_ bash tools/pmc_sq.sh r03_sq_cfg2 > gpurun_out/r03_sq_cfg2.txt 2>&1 || exit 1
head -30 gpurun_out/r03_sq_cfg2.txt | cut -c1-300
for W in cfg2 cfg3 cfg4 cfg5; do
  WL=$W bash tools/profile_round.sh r03_$W > gpurun_out/r03_$W.log 2>&1 || { tail -20 gpurun_out/r03_$W.log; exit 1; }
  tail -1 gpurun_out/r03_$W.log | cut -c1-200
  grep -A3 "Whole step" gpurun_out/r03_$W/summary/r03_${W}_summary.md | head -3
done
