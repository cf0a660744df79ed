"""Host owner routing (include/hbroute.h, libhbnode.so) against its Python
mirror etcd_amd/shard.py (ShardMap): the same owner hash and local slots, each
rank's messages in arrival order (raft/multinode.go:233-237), for dense and
sparse group-id spaces, 1..8 ranks, unknown ids, and the threaded chunking at
sizes that split the stream over many threads."""
import os
import re

import numpy as np
import pytest

from etcd_amd import synth
from etcd_amd.shard import NativeRouter, ShardMap, owner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_router_exports_every_declared_function():
    from etcd_amd import multinode
    L = multinode.lib()
    txt = open(os.path.join(ROOT, "include", "hbroute.h")).read()
    names = sorted(set(re.findall(r"^\s*(?:int|uint32_t|uint64_t)\s+(hbn_[a-z_]+)\s*\(", txt, re.M)))
    assert len(names) == 7
    for n in names:
        assert hasattr(L, n), f"libhbnode.so does not export {n}"


def test_owner_matches_splitmix():
    from etcd_amd import multinode
    L = multinode.lib()
    ids = np.random.default_rng(1).integers(0, 1 << 63, 1000, dtype=np.uint64)
    for w in (1, 2, 3, 8):
        want = owner(ids, w)
        assert [L.hbn_owner(int(x), w) for x in ids[:200]] == want[:200].tolist()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("dense", [True, False])
def test_route_equals_shardmap(world, dense):
    rng = np.random.default_rng(world * 10 + dense)
    G = 50_000
    ids = np.arange(G, dtype=np.uint64) if dense else \
        np.unique(rng.integers(0, 1 << 64, G + 100, dtype=np.uint64))[:G]
    rng.shuffle(ids)
    r = NativeRouter(ids, world, threads=7)
    # a stream of 600k messages (several 64K chunks per thread), 1 % of them for unknown groups
    gids = ids[rng.integers(0, G, 600_000)]
    unk = rng.random(len(gids)) < 0.01
    gids[unk] = np.uint64(1 << 62) + rng.integers(0, 1 << 20, int(unk.sum()), dtype=np.uint64)
    out, n_unk = r.route(gids)
    assert n_unk == int(unk.sum())
    total = 0
    for k in range(world):
        sm = ShardMap(ids, world, k)
        assert np.array_equal(r.local_ids(k), sm.local_ids)
        known = ~unk
        idx, slots = sm.route_local(gids[known])
        want_pos = np.nonzero(known)[0][idx]
        pos, slot = out[k]
        assert np.array_equal(pos, want_pos), f"rank {k}: positions"
        assert np.array_equal(slot, slots), f"rank {k}: slots"
        total += len(pos)
    assert total + n_unk == len(gids)


def test_route_one_rank_only_and_edge_cases():
    ids = np.arange(1000, dtype=np.uint64)
    r = NativeRouter(ids, 4, threads=2)
    out, _ = r.route(ids[::-1], ranks=[2])
    sm = ShardMap(ids, 4, 2)
    idx, slots = sm.route_local(ids[::-1])
    assert list(out) == [2] and np.array_equal(out[2][0], idx) and np.array_equal(out[2][1], slots)
    out, n_unk = r.route(np.zeros(0, np.uint64))
    assert n_unk == 0 and all(len(p) == 0 for p, _ in out.values())
    with pytest.raises(ValueError):  # a duplicate id
        NativeRouter(np.array([5, 7, 5], np.uint64), 2)
    with pytest.raises(ValueError):  # world 0
        NativeRouter(ids, 0)
    big = np.array([np.uint64(2**64 - 1), np.uint64(3)], np.uint64)  # the all-ones id (the hash's empty key)
    r2 = NativeRouter(big, 2)
    out, n_unk = r2.route(np.array([2**64 - 1, 3, 4], np.uint64))
    assert n_unk == 1 and sum(len(p) for p, _ in out.values()) == 2


def test_route_global_ack_stream_like_the_bench():
    """bench.py's cfg2/cfg5 host leg at a reduced size: the global ack stream of
    2 x 200k groups routed to each of 8 ranks equals ShardMap.route_local with
    the dense table."""
    G_total, world = 200_000, 8
    ids = np.arange(G_total, dtype=np.uint64)
    gid, _ = synth.global_ack_stream(G_total, 3)
    out, n_unk = NativeRouter(ids, world).route(gid)
    assert n_unk == 0
    for k in range(world):
        sm = ShardMap(ids, world, k)
        idx, slots = sm.route_local(gid, sm.dense_slots(G_total))
        assert np.array_equal(out[k][0], idx) and np.array_equal(out[k][1], slots)


def test_router_out_of_memory_is_an_error_code():
    """A failed allocation inside the router is HB_ENOMEM (MemoryError here),
    not a C++ exception through the C ABI (which would abort the host).  The
    child caps its address space just above what it holds, then asks for a
    sparse router whose hash table (96 MB) cannot fit."""
    import subprocess
    import sys
    code = (
        "import resource, numpy as np\n"
        "from etcd_amd.shard import NativeRouter\n"
        "from etcd_amd import multinode; multinode.lib()\n"
        "ids = np.arange(4_000_000, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)\n"
        "vm = [int(l.split()[1]) for l in open('/proc/self/status') if l.startswith('VmSize:')][0] * 1024\n"
        "resource.setrlimit(resource.RLIMIT_AS, (vm + (32 << 20), resource.RLIM_INFINITY))\n"
        "try:\n"
        "    NativeRouter(ids, 2, threads=1)\n"
        "    print('created')\n"
        "except MemoryError:\n"
        "    print('enomem')\n")
    if "libasan" in os.environ.get("LD_PRELOAD", ""):
        pytest.skip("under ASan (tests/test_sanitizers.py) operator new aborts on out-of-memory instead of throwing")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == "enomem"
