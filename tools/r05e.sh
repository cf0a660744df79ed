#!/bin/bash
# leader lane A/B: full (LDS lane, rolled sends), ldsc (LDS lane, compile-time-slot sends), reg (register lane)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/ab.sh "cfg3 follow:5 mixed" full ldsc reg || exit 1
bash tools/prof_wl.sh r05e_ldsc ldsc cfg3 || exit 1
