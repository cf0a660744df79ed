#!/bin/bash
# round 5: GPU suite + smoke + default line, then A/Bs of the leader lane (LDS vs registers)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_suite.sh r05b || exit 1
bash tools/ab.sh "cfg3 cfg4 follow:5 mixed follow" full reg || exit 1
