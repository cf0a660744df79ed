# Round-2 GPU check: GPU tests, smoke, cfg2 / cfg5 / e2e bench lines.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r2
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r2/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r2/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1
tail -1 gpurun_out/r2/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err
tail -1 gpurun_out/r2/bench.json
timeout -k 10 300 python3 bench.py --workload cfg5 --no-cpu-baseline > gpurun_out/r2/cfg5.json 2> gpurun_out/r2/cfg5.err
tail -1 gpurun_out/r2/cfg5.json
timeout -k 10 300 python3 bench.py --workload e2e > gpurun_out/r2/e2e.json 2> gpurun_out/r2/e2e.err
tail -1 gpurun_out/r2/e2e.json
