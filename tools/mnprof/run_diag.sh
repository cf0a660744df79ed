cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out/mnprof && cd gpurun_out/mnprof && \
timeout -k 10 200 ../../tools/mnprof/mnprof 1000 4000 3 1 > run.txt 2>&1 && gprof -b ../../tools/mnprof/mnprof gmon.out > gprof.txt && rm -f gmon.out && \
cd ../.. && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --stats --output-format csv -d gpurun_out/mnprof/trace -- ./tools/mnprof/mnprof 1000 300 3 1 > gpurun_out/mnprof/trace_run.txt 2>&1
