"""Phase timestamps of k_apply_fast (diagnostic build etcd_amd/libhipbatch_STAMPS.so,
-DHB_X_STAMPS): per-workgroup cycle deltas between phases and the realtime
(100 MHz) start/end spread over the launch.  Runs the cfg2 step like bench.py.

  HB_LIB=$PWD/etcd_amd/libhipbatch_STAMPS.so python3 tools/stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from etcd_amd import synth
    from etcd_amd.hipbatch import Engine, lib
    G, n = 1 << 20, 3
    groups, _ = synth.steady_groups(G, n, seed=0x5EED0002, with_runs=False)
    batch = synth.cfg2_batch(groups, 0, seed=0x5EED0002)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    eng = Engine(G, max_replicas=n, max_inflight=256, max_batch=len(batch["group"]), stream=stream)
    eng.load_groups(groups)
    d = {k: torch.from_numpy(batch[k].view(np.int32 if batch[k].dtype == np.uint32 else np.int64)).to(dev)
         for k in ("group", "info", "term", "index", "props")}
    for k in range(6):
        eng.step(d["group"], d["info"], d["term"], d["index"] + k, None, d["props"], host=False)
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    NB = G // 256
    out = np.zeros(NB * 8, dtype=np.uint64)
    L = lib()
    L.hb_x_stamps.argtypes = [C.c_void_p, C.c_uint32]
    assert L.hb_x_stamps(out.ctypes.data, NB * 8) == 0
    st = out.reshape(NB, 8).astype(np.int64)
    names = ["loads landed", "proposal", "messages", "store+stats"]
    cols = [(0, 1), (1, 2), (2, 3), (3, 5)]
    print("phase cycles per workgroup (median / p10 / p90):")
    for nm, (a, b) in zip(names, cols):
        dd = st[:, b] - st[:, a]
        print(f"  {nm:16s} {np.median(dd):9.0f} {np.percentile(dd, 10):9.0f} {np.percentile(dd, 90):9.0f}")
    tot = st[:, 5] - st[:, 0]
    print(f"  {'total':16s} {np.median(tot):9.0f} {np.percentile(tot, 10):9.0f} {np.percentile(tot, 90):9.0f}")
    rt0, rt1 = st[:, 6], st[:, 7]
    t0 = rt0.min()
    life = (rt1 - rt0) * 10  # ns
    print(f"realtime: launch span {(rt1.max() - t0) * 10 / 1e3:.1f} us, WG lifetime median {np.median(life) / 1e3:.2f} us "
          f"p90 {np.percentile(life, 90) / 1e3:.2f} us; clock ~{np.median(tot) / np.median(life):.2f} GHz")
    # concurrency over time
    edges = np.arange(0, (rt1.max() - t0) + 50, 50)
    conc = [int(((rt0 - t0 <= e) & (rt1 - t0 > e)).sum()) for e in edges]
    print("live WGs every 0.5 us:", conc)
    starts = np.sort(rt0 - t0) * 10 / 1e3
    print("WG start quantiles (us):", [round(float(np.percentile(starts, q)), 1) for q in (0, 10, 25, 50, 75, 90, 100)])


if __name__ == "__main__":
    main()
