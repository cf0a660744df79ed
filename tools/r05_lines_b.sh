#!/bin/bash
# round 5 evidence, part B: follower / mixed / tick profiles, then the wire, e2e and MultiNode lines
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r05_lines
WLS="follow follow:5 mixed tick" bash tools/profile.sh r05 || exit 1
for W in wire e2e; do
  timeout -k 10 300 python3 bench.py --workload $W --cpu-seconds 10 > gpurun_out/r05_lines/$W.json 2> gpurun_out/r05_lines/$W.err \
    || { tail -20 gpurun_out/r05_lines/$W.err; exit 1; }
  tail -c 300 gpurun_out/r05_lines/$W.json; echo
done
for G in 1000 1048576; do
  S=20; [ $G -gt 100000 ] && S=4
  timeout -k 10 600 python3 bench.py --workload multinode --groups $G --steps $S --warmup 2 > gpurun_out/r05_lines/multinode_$G.json \
    2> gpurun_out/r05_lines/multinode_$G.err || { tail -20 gpurun_out/r05_lines/multinode_$G.err; exit 1; }
  tail -c 300 gpurun_out/r05_lines/multinode_$G.json; echo
done
