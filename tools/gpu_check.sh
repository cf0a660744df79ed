set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/v1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v1/gpu_tests.log 2>&1 || { tail -30 gpurun_out/v1/gpu_tests.log; exit 1; }
tail -3 gpurun_out/v1/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v1/smoke.log 2>&1
tail -1 gpurun_out/v1/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/v1/bench.json 2> gpurun_out/v1/bench.err
tail -1 gpurun_out/v1/bench.json
