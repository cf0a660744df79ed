#!/bin/bash
# Round-3 evidence on one build: -m gpu suite, smoke, the default bench line, profiles of
# cfg2 / cfg3 / cfg4 / cfg5 (trace + FETCH / WRITE passes + bench line), e2e and MultiNode lines.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/fin
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread \
  > gpurun_out/fin/gpu_tests.log 2>&1 || { tail -40 gpurun_out/fin/gpu_tests.log; exit 1; }
tail -1 gpurun_out/fin/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 || { tail -20 gpurun_out/fin/smoke.log; exit 1; }
tail -1 gpurun_out/fin/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/fin/bench.json 2> gpurun_out/fin/bench.err || { tail -20 gpurun_out/fin/bench.err; exit 1; }
tail -1 gpurun_out/fin/bench.json | cut -c1-300
for W in cfg2 cfg3 cfg4 cfg5; do
  WL=$W bash tools/profile_round.sh r03_$W > gpurun_out/r03_$W.log 2>&1 || { tail -20 gpurun_out/r03_$W.log; exit 1; }
  grep "Whole step" gpurun_out/r03_$W/summary/r03_${W}_summary.md
done
timeout -k 10 300 python3 bench.py --workload e2e --no-cpu-baseline > gpurun_out/fin/e2e.json 2> gpurun_out/fin/e2e.err || exit 1
for G in 1000 1048576; do
  ST=20; [ $G -gt 100000 ] && ST=4
  timeout -k 10 400 python3 bench.py --workload multinode --groups $G --steps $ST --warmup 2 \
    --no-cpu-baseline > gpurun_out/fin/mn_$G.json 2> gpurun_out/fin/mn_$G.err || exit 1
done
for W in tick wire; do
  timeout -k 10 300 python3 bench.py --workload $W > gpurun_out/fin/$W.json 2> gpurun_out/fin/$W.err || exit 1
done
echo done
