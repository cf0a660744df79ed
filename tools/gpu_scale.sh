# New scale / multi-rank GPU parity tests only.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/scale
timeout -k 10 1100 python3 -u -m pytest tests/test_scale_gpu.py -m gpu -x -v --timeout 900 --timeout-method thread --durations=0 > gpurun_out/scale/tests.log 2>&1 || { tail -60 gpurun_out/scale/tests.log; exit 1; }
tail -15 gpurun_out/scale/tests.log
