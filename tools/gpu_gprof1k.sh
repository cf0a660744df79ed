#!/bin/bash
# gprof of the host MultiNode path at 1k groups (single thread, bulk API)
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/gp1k; cd gpurun_out/gp1k
timeout -k 10 200 ../../tools/mnprof/mnprof 1000 4000 3 1 && gprof -b ../../tools/mnprof/mnprof gmon.out > gprof_1k.txt && head -45 gprof_1k.txt | cut -c1-200
rm -f gmon.out
