#!/bin/bash
# kernel traces of cfg3 with the LDS leader lane (full) and the register lane (reg)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/prof_wl.sh r05d_full full cfg3 || exit 1
bash tools/prof_wl.sh r05d_reg reg cfg3 || exit 1
