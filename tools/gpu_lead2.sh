#!/bin/bash
# GPU suite on the default build, cfg3 / cfg4 A/B of occupancy variants, then a cfg3 kernel trace
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_lead.sh "$@" || exit 1
bash tools/prof_wl.sh plead3 full cfg3
