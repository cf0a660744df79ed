#!/bin/bash
# rocprofv3 kernel + HIP API + copy trace of the 1k-group MultiNode loop (tools/mnprof)
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out/${1:-mntrace}
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --stats --output-format csv \
  -d gpurun_out/${1:-mntrace}/trace -- ./tools/mnprof/mnprof 1000 300 7 4 > gpurun_out/${1:-mntrace}/trace_run.txt 2>&1
