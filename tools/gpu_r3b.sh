#!/bin/bash
# Round-3 check of HEAD: whole -m gpu suite, smoke, default bench, MultiNode 1k / 1M bulk vs per-call.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r3b
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/r3b/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3b/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3b/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b/smoke.log 2>&1 || { tail -20 gpurun_out/r3b/smoke.log; exit 1; }
tail -1 gpurun_out/r3b/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.err || { tail -20 gpurun_out/r3b/bench.err; exit 1; }
tail -1 gpurun_out/r3b/bench.json
for G in 1000 1048576; do
  ST=20; [ $G -gt 100000 ] && ST=4
  for M in bulk percall; do
    timeout -k 10 400 python3 bench.py --workload multinode --groups $G --steps $ST --warmup 2 --mn-mode $M \
      --no-cpu-baseline > gpurun_out/r3b/mn_${G}_${M}.json 2> gpurun_out/r3b/mn_${G}_${M}.err || { tail -5 gpurun_out/r3b/mn_${G}_${M}.err; exit 1; }
    tail -1 gpurun_out/r3b/mn_${G}_${M}.json
  done
done
