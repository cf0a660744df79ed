#!/bin/bash
# leader lane A/B (full: LDS lane rolled sends; ldsc: compile-time-slot sends; reg: registers)
# and the direct-claim microbench
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r05f
timeout -k 10 120 ./tools/microbench/claim_mb > gpurun_out/r05f/claim_mb.txt 2>&1 || { cat gpurun_out/r05f/claim_mb.txt; exit 1; }
cat gpurun_out/r05f/claim_mb.txt
bash tools/ab.sh "cfg3 follow:5 mixed" full ldsc reg || exit 1
