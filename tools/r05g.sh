#!/bin/bash
# the role deal in X-mode k_apply_fast (deal) vs without (ldsc); both LDS lane + compile-time sends
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/ab.sh "mixed follow follow:5" deal ldsc || exit 1
bash tools/prof_wl.sh r05g_deal deal "mixed cfg3" || exit 1
