#!/bin/bash
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/r3g
bash tools/gpu_ab_tests.sh "cfg2 cfg5 cfg3" full wide sacc full wide sacc || exit 1
HB_LIB=$PWD/etcd_amd/libhipbatch_sacc.so timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3g/sacc_tests.log 2>&1; tail -2 gpurun_out/r3g/sacc_tests.log
