"""Multi-GPU sharding of raft groups.

Groups are independent (raft/multinode.go:125-131), so they shard by a hash of
the group id over the GPUs of a node with no data-path collective:
gpu = splitmix64(group_id) % world.  The host routes every message by the same
hash; each GPU owns a dense local slot space.  The only collective is one
all-reduce of the per-step statistics (RCCL over xGMI on GPUs, gloo in CPU
tests).
"""
import os

import numpy as np

from .synth import splitmix64


def owner(group_ids, world):
    """GPU rank that owns each global group id."""
    if world == 1:
        return np.zeros(len(group_ids), dtype=np.int64)
    return (splitmix64(np.asarray(group_ids, dtype=np.uint64)) % np.uint64(world)).astype(np.int64)


class ShardMap:
    """Global group id <-> (rank, local slot) for one rank."""

    def __init__(self, group_ids, world, rank):
        ids = np.asarray(group_ids, dtype=np.uint64)
        own = owner(ids, world)
        self.world, self.rank = world, rank
        self.local_ids = ids[own == rank]               # local slot -> global id
        self._sorted = np.argsort(self.local_ids, kind="stable")
        self._keys = self.local_ids[self._sorted]

    def __len__(self):
        return len(self.local_ids)

    def local_slot(self, gids):
        """Local slots of global ids owned by this rank (-1 if not owned)."""
        gids = np.asarray(gids, dtype=np.uint64)
        pos = np.searchsorted(self._keys, gids)
        pos = np.minimum(pos, len(self._keys) - 1) if len(self._keys) else pos
        hit = (len(self._keys) > 0) & (self._keys[pos] == gids) if len(self._keys) else np.zeros(len(gids), bool)
        out = np.full(len(gids), -1, dtype=np.int64)
        out[hit] = self._sorted[pos[hit]]
        return out

    def route(self, gids):
        """Split a message batch by owner rank: returns rank -> indices (arrival order kept)."""
        own = owner(gids, self.world)
        return {r: np.nonzero(own == r)[0] for r in range(self.world)}

    def dense_slots(self, id_space):
        """Lookup table global id -> local slot (-1 when another rank owns it) for
        the dense id space [0, id_space): one gather per routed message instead
        of a binary search."""
        t = np.full(id_space, -1, dtype=np.int32)
        t[self.local_ids.astype(np.int64)] = np.arange(len(self.local_ids), dtype=np.int32)
        return t

    def route_local(self, gids, table=None):
        """This rank's messages of an arrival-ordered batch: (indices into the
        batch, local slots), arrival order kept.  `table` = dense_slots() for a
        dense id space (else the sorted-id search of local_slot)."""
        gids = np.asarray(gids, dtype=np.uint64)
        idx = np.nonzero(owner(gids, self.world) == self.rank)[0]
        sel = gids[idx]
        slots = table[sel.astype(np.int64)] if table is not None else self.local_slot(sel)
        return idx, slots.astype(np.uint32)


def reduce_stats(stats_tensor, dist=None):
    """Sum a per-rank HB_STAT_COUNT u64 vector over ranks (one all-reduce)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(stats_tensor)
    return stats_tensor


class NativeRouter:
    """The owner routing of libhbnode.so (include/hbroute.h): one pass over an
    arrival-ordered stream on host threads, every rank's (stream positions,
    local slots) at once, order kept.  Same shard map as ShardMap (owner =
    splitmix64(id) % world, local slot = position among the rank's ids)."""

    def __init__(self, group_ids, world, threads=0):
        # (hipbatch.lib() binds the engine to torch's HIP runtime whatever the
        # import order: tests/test_runtime_bind.py)
        import ctypes as C
        from .multinode import lib
        self._L = L = lib()
        self._C = C
        ids = np.ascontiguousarray(group_ids, dtype=np.uint64)
        self.world = world
        self.threads = threads or min(16, os.cpu_count() or 1)
        self._h = C.c_void_p()
        rc = L.hbn_router_create(ids.ctypes.data_as(C.c_void_p), len(ids), world, self.threads, C.byref(self._h))
        if rc == -2:  # HB_ENOMEM
            raise MemoryError("hbn_router_create: out of host memory")
        if rc != 0:
            raise ValueError(f"hbn_router_create: {rc}")

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.hbn_router_destroy(self._h)
            self._h = None

    def local_ids(self, rank):
        C = self._C
        n = self._L.hbn_router_local_count(self._h, rank)
        out = np.zeros(n, np.uint64)
        self._L.hbn_router_local_ids(self._h, rank, out.ctypes.data_as(C.c_void_p))
        return out

    def route(self, gids, ranks=None):
        """{rank: (positions u64, local slots u32)} for `ranks` (default all),
        plus the count of messages for unknown groups."""
        C = self._C
        gids = np.ascontiguousarray(gids, dtype=np.uint64)
        W = self.world
        counts = np.zeros(W, np.uint64)
        unk = C.c_uint64()
        rc = self._L.hbn_route(self._h, gids.ctypes.data_as(C.c_void_p), len(gids), counts.ctypes.data_as(C.c_void_p),
                               C.byref(unk))
        if rc == -2:
            raise MemoryError("hbn_route: out of host memory")
        if rc != 0:
            raise ValueError(f"hbn_route: {rc}")
        ranks = range(W) if ranks is None else ranks
        out = {k: (np.empty(int(counts[k]), np.uint64), np.empty(int(counts[k]), np.uint32)) for k in ranks}
        pos = (C.c_void_p * W)(*[out[k][0].ctypes.data if k in out else None for k in range(W)])
        slot = (C.c_void_p * W)(*[out[k][1].ctypes.data if k in out else None for k in range(W)])
        rc = self._L.hbn_route_take(self._h, pos, slot)
        if rc != 0:
            raise ValueError(f"hbn_route_take: {rc}")
        return out, int(unk.value)
