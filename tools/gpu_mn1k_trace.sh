#!/bin/bash
# 1k-group MultiNode cycle on the device timeline: kernel + memory-copy trace (no counters)
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/mn1k; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/mn1k/trace -o run -- \
  python3 bench.py --workload multinode --groups 1000 --steps 200 --warmup 2 --no-cpu-baseline > gpurun_out/mn1k/bench.json 2> gpurun_out/mn1k/bench.err || exit 1
tail -c 300 gpurun_out/mn1k/bench.json
ls gpurun_out/mn1k/trace | head
