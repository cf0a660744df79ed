"""MemoryStorage of the MultiNode host library (etcd_amd/libhbnode.so) against
the reference's own storage tests, raft/storage_test.go:27-245 (tables
transcribed), plus Entry.Size (what limitSize sums) against the protobuf
library's encoding of the same entries.  CPU only: the storage is host code."""
import pytest

from etcd_amd.multinode import Entry, MemoryStorage, NO_LIMIT, entry_size


def E(i, t, data=None, typ=0):
    return Entry(Term=t, Index=i, Type=typ, Data=data)


ENTS = [E(3, 3), E(4, 4), E(5, 5)]


def ents_of(s):
    """s.ents as the Go tests read it: the dummy at FirstIndex-1, then every entry."""
    first, last = s.FirstIndex(), s.LastIndex()
    out = []
    for i in range(first - 1, last + 1):
        t, err = s.Term(i)
        assert err is None
        out.append((i, t))
    return out


@pytest.mark.parametrize("i,werr,wterm", [(2, "ErrCompacted", 0), (3, None, 3), (4, None, 4), (5, None, 5)])
def test_storage_term(i, werr, wterm):  # raft/storage_test.go:27-51
    s = MemoryStorage(ENTS)
    assert s.Term(i) == (wterm, werr)


def test_storage_entries():  # raft/storage_test.go:53-87
    ents = [E(3, 3), E(4, 4), E(5, 5), E(6, 6)]
    sz = [entry_size(e) for e in ents]
    tests = [
        (2, 6, NO_LIMIT, "ErrCompacted", None),
        (3, 4, NO_LIMIT, "ErrCompacted", None),
        (4, 5, NO_LIMIT, None, [E(4, 4)]),
        (4, 6, NO_LIMIT, None, [E(4, 4), E(5, 5)]),
        (4, 7, NO_LIMIT, None, [E(4, 4), E(5, 5), E(6, 6)]),
        (4, 7, 0, None, [E(4, 4)]),
        (4, 7, sz[1] + sz[2], None, [E(4, 4), E(5, 5)]),
        (4, 7, sz[1] + sz[2] + sz[3] // 2, None, [E(4, 4), E(5, 5)]),
        (4, 7, sz[1] + sz[2] + sz[3] - 1, None, [E(4, 4), E(5, 5)]),
        (4, 7, sz[1] + sz[2] + sz[3], None, [E(4, 4), E(5, 5), E(6, 6)]),
    ]
    for k, (lo, hi, mx, werr, went) in enumerate(tests):
        s = MemoryStorage(ents)
        got, err = s.Entries(lo, hi, mx)
        assert err == werr, k
        assert got == went, k


def test_storage_last_index():  # :89-109
    s = MemoryStorage(ENTS)
    assert s.LastIndex() == 5
    s.Append([E(6, 5)])
    assert s.LastIndex() == 6


def test_storage_first_index():  # :111-131
    s = MemoryStorage(ENTS)
    assert s.FirstIndex() == 4
    s.Compact(4)
    assert s.FirstIndex() == 5


@pytest.mark.parametrize("i,werr,windex,wterm,wlen", [(2, "ErrCompacted", 3, 3, 3), (3, "ErrCompacted", 3, 3, 3),
                                                      (4, None, 4, 4, 2), (5, None, 5, 5, 1)])
def test_storage_compact(i, werr, windex, wterm, wlen):  # :133-165
    s = MemoryStorage(ENTS)
    assert s.Compact(i) == werr
    got = ents_of(s)
    assert got[0] == (windex, wterm)
    assert len(got) == wlen


@pytest.mark.parametrize("i", [4, 5])
def test_storage_create_snapshot(i):  # :167-192
    s = MemoryStorage(ENTS)
    snap, err = s.CreateSnapshot(i, [1, 2, 3], b"data")
    assert err is None
    assert (snap.Index, snap.Term, snap.Nodes, snap.Data) == (i, i, [1, 2, 3], b"data")
    assert s.Snapshot() == snap
    # older than the existing snapshot (raft/storage.go:165-167)
    assert s.CreateSnapshot(i, [1], b"x")[1] == "ErrSnapOutOfDate"


@pytest.mark.parametrize("entries,went", [
    ([E(3, 3), E(4, 4), E(5, 5)], [(3, 3), (4, 4), (5, 5)]),
    ([E(3, 3), E(4, 6), E(5, 6)], [(3, 3), (4, 6), (5, 6)]),
    ([E(3, 3), E(4, 4), E(5, 5), E(6, 5)], [(3, 3), (4, 4), (5, 5), (6, 5)]),
    ([E(2, 3), E(3, 3), E(4, 5)], [(3, 3), (4, 5)]),  # truncate incoming, truncate existing, append
    ([E(4, 5)], [(3, 3), (4, 5)]),  # truncate the existing entries and append
    ([E(6, 5)], [(3, 3), (4, 4), (5, 5), (6, 5)]),  # direct append
])
def test_storage_append(entries, went):  # :194-245
    s = MemoryStorage(ENTS)
    assert s.Append(entries) is None
    assert ents_of(s) == went


def test_storage_append_keeps_payloads_and_panics_on_gap():
    s = MemoryStorage()
    s.Append([E(1, 1, b"a"), E(2, 1, b""), E(3, 2)])
    got, err = s.Entries(1, 4)
    assert err is None and [e.Data for e in got] == [b"a", b"", None]
    from etcd_amd.multinode import RaftPanic
    with pytest.raises(RaftPanic, match="missing log entry"):
        s.Append([E(9, 2)])
    assert MemoryStorage().Entries(1, 1)[1] == "ErrUnavailable"  # only the dummy entry


def test_apply_snapshot_and_initial_state():
    from etcd_amd.multinode import HardState, Snapshot
    s = MemoryStorage()
    s.SetHardState(HardState(1, 0, 3))
    s.ApplySnapshot(Snapshot(Index=2, Term=1, Nodes=[1, 2]))
    s.Append([E(3, 1, b"foo")])
    hs, nodes = s.InitialState()
    assert hs == HardState(1, 0, 3) and nodes == [1, 2]
    assert (s.FirstIndex(), s.LastIndex()) == (3, 3)
    assert s.Term(2) == (1, None)


def test_entry_size_matches_protobuf_encoding():
    """Entry.Size() == len(protobuf encoding of the Entry) (gogo Size, raft/raftpb/raft.pb.go)."""
    import numpy as np
    from . import wire_util as W
    rng = np.random.default_rng(1)
    for _ in range(200):
        e = E(int(rng.integers(0, 1 << 40)), int(rng.integers(0, 1 << 20)),
              bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)) if rng.random() < .7 else None,
              int(rng.integers(0, 2)))
        assert entry_size(e) == len(W.pb_entry(e.Type, e.Term, e.Index, e.Data))
