# Selected GPU tests: gpu_tests_sel.sh <tag> <pytest args...>
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG
timeout -k 10 1100 python3 -u -m pytest "$@" -m gpu -x -v --timeout 900 --timeout-method thread --durations=15 > gpurun_out/$TAG/tests.log 2>&1 || { tail -60 gpurun_out/$TAG/tests.log; exit 1; }
tail -25 gpurun_out/$TAG/tests.log
