set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/var
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/var/gpu_tests.log 2>&1 || { tail -30 gpurun_out/var/gpu_tests.log; exit 1; }
tail -2 gpurun_out/var/gpu_tests.log
for v in full nomsg nostep p9w4 p8w3; do
  HB_LIB=$PWD/etcd_amd/libhipbatch_$v.so timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/var/$v.json
  python3 -c "import json;d=json.loads(open('gpurun_out/var/$v.json').read().strip().splitlines()[-1]);print('$v',round(d['value']/1e9,3),d['phases'],d['parity_sanity'])"
done
