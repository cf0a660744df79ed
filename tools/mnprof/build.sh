#!/bin/bash
# Build the gprof driver (host MultiNode code compiled -pg into the executable).
set -e
cd "$(dirname "$0")/../.."
g++ -O2 -g -pg -std=c++17 -o tools/mnprof/mnprof etcd_amd/csrc/hbnode.cpp etcd_amd/csrc/hbnode_bench.cpp \
    tools/mnprof/main.cpp -Letcd_amd -lhipbatch -Wl,-rpath,'$ORIGIN/../../etcd_amd' -lpthread
