#!/bin/bash
# round 5: the default line, then A/Bs of the leader lane (LDS vs registers) and the new lines
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r05c
timeout -k 10 300 python3 bench.py > gpurun_out/r05c/bench.json 2> gpurun_out/r05c/bench.err \
  || { tail -20 gpurun_out/r05c/bench.err; exit 1; }
tail -c 600 gpurun_out/r05c/bench.json; echo
bash tools/ab.sh "cfg3 cfg4 follow:5 mixed follow" full reg || exit 1
