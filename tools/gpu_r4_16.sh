cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r04f
bash tools/ab_mn.sh "1000 1048576" main var_g4 || exit 1
timeout -k 10 300 python3 bench.py --workload tick > gpurun_out/r04f/tick.json 2> gpurun_out/r04f/tick.err || exit 1
tail -c 700 gpurun_out/r04f/tick.json; echo
timeout -k 10 300 python3 bench.py --workload e2e > gpurun_out/r04f/e2e.json 2> gpurun_out/r04f/e2e.err || exit 1
tail -c 400 gpurun_out/r04f/e2e.json
