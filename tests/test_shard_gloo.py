"""Multi-rank sharding path on CPU (gloo, world_size 2).

Each rank owns the groups with splitmix64(id) % world == rank, routes a
message batch by the same hash, steps its shard through the C oracle (the
engine needs a GPU; its parity with the oracle is tested in
test_parity_gpu.py) and the per-rank statistics are summed with one
all-reduce — the only collective of the multi-GPU design.  The result must
equal stepping all groups in one process.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from etcd_amd import abi, synth
from etcd_amd.shard import ShardMap, owner, reduce_stats

G_TOTAL = 3000
N = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batch():
    g, runs = synth.steady_groups(G_TOTAL, N, seed=21, last_hi=1 << 12)
    b = synth.cfg2_batch(g, 0, seed=22)
    return g, runs, b


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.pyoracle import OracleGroups
        g, runs, b = _global_batch()
        ids = np.arange(G_TOTAL, dtype=np.uint64)
        sm = ShardMap(ids, world, rank)
        local = sm.local_ids.astype(np.int64)
        og = OracleGroups(g[local], [runs[i] for i in local], 256)
        # route the arrival-ordered batch: this rank's messages, order kept — by the
        # host router of libhbnode (include/hbroute.h), checked against ShardMap
        from etcd_amd.shard import NativeRouter
        routed, unknown = NativeRouter(ids, world).route(b["group"].astype(np.uint64), ranks=[rank])
        idx, slots = routed[rank]
        idx = idx.astype(np.int64)
        assert unknown == 0 and np.array_equal(idx, sm.route(b["group"].astype(np.uint64))[rank])
        lb = {k: (v[idx] if (v is not None and k != "props") else v) for k, v in b.items()}
        lb["group"] = slots
        assert np.array_equal(slots, sm.local_slot(b["group"][idx].astype(np.uint64)).astype(np.uint32))
        lb["props"] = b["props"][local]
        _, st = og.step(lb)
        t = torch.from_numpy(st.astype(np.int64))
        reduce_stats(t, dist)
        counts = torch.tensor([len(sm)], dtype=torch.int64)
        dist.all_reduce(counts)
        if rank == 0:
            out.put((t.numpy().tolist(), int(counts.item())))
    finally:
        dist.destroy_process_group()


def test_sharded_stats_equal_single_process():
    from oracle.pyoracle import OracleGroups
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    stats, count = q.get(timeout=10)
    g, runs, b = _global_batch()
    _, st = OracleGroups(g, runs, 256).step(b)
    assert count == G_TOTAL
    assert stats == st.astype(np.int64).tolist()
    assert stats[abi.HB_STAT_COMMITS] == G_TOTAL


def test_owner_is_a_partition():
    ids = np.arange(100_000, dtype=np.uint64)
    for world in (1, 2, 4, 8):
        own = owner(ids, world)
        assert own.min() >= 0 and own.max() < world
        cnt = np.bincount(own, minlength=world)
        assert cnt.sum() == len(ids)
        assert cnt.min() > 0.95 * len(ids) / world  # balanced hash
        maps = [ShardMap(ids, world, r) for r in range(world)]
        allids = np.concatenate([m.local_ids for m in maps])
        assert np.array_equal(np.sort(allids), ids)
        m = maps[world - 1]
        slots = m.local_slot(m.local_ids)
        assert np.array_equal(slots, np.arange(len(m)))
        other = ids[own != world - 1][:10]
        assert (m.local_slot(other) == -1).all()


def test_routed_batch_partitions_the_global_stream():
    """bench.py's host routing (cfg2 / cfg5 at N GPUs): every rank scans one
    global arrival stream and keeps its own messages; over all ranks each
    group gets exactly one ack per follower, and a rank's messages keep their
    global arrival order."""
    import bench
    from etcd_amd.synth import global_ack_stream
    G_per, n = 5000, 3
    for world in (1, 2, 4):
        gid, frm = global_ack_stream(G_per * world, n)
        total = 0
        for rank in range(world):
            groups, batch, G_total, route = bench.routed_batch(G_per, world, rank, n)
            assert G_total == G_per * world and route["local_msgs"] == len(batch["group"])
            cnt = np.bincount(batch["group"], minlength=len(groups))
            assert (cnt == n - 1).all()
            sm = ShardMap(np.arange(G_total, dtype=np.uint64), world, rank)
            mine = np.nonzero(owner(gid, world) == rank)[0]
            assert np.array_equal(sm.local_ids[batch["group"]], gid[mine])  # arrival order kept
            assert np.array_equal((batch["info"] >> 4) & 0xF, frm[mine])
            assert np.array_equal(batch["index"], groups["last_index"][batch["group"]] + np.uint64(1))
            total += len(batch["group"])
        assert total == G_per * world * (n - 1)
