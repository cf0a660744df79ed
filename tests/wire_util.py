"""Test infrastructure for wire ingestion: raftpb.Message encoders and a
malformed-record corpus.

gogo_marshal restates the reference's generated encoder byte for byte
(Message.MarshalTo raft/raftpb/raft.pb.go:1271-1330, Snapshot :1236-1262,
SnapshotMetadata :1201-1234, ConfState :1374-1392, Entry, encodeVarintRaft
:1446-1454).  pb_message builds the same schema (raft/raftpb/raft.proto) with
the protobuf library, an encoder independent of both decoders.
"""
import numpy as np

from etcd_amd import abi


def varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def key(field, wt):
    return varint((field << 3) | wt)


def _entry(e):
    t, term, index, data = e
    b = key(1, 0) + varint(t) + key(2, 0) + varint(term) + key(3, 0) + varint(index)
    if data is not None:
        b += key(4, 2) + varint(len(data)) + data
    return b


def _snapshot(snap):
    data, nodes, index, term = snap if snap else (None, (), 0, 0)
    conf = b"".join(key(1, 0) + varint(n) for n in nodes)
    meta = key(1, 2) + varint(len(conf)) + conf + key(2, 0) + varint(index) + key(3, 0) + varint(term)
    b = b""
    if data is not None:
        b += key(1, 2) + varint(len(data)) + data
    return b + key(2, 2) + varint(len(meta)) + meta


def gogo_marshal(type, to=0, frm=0, term=0, log_term=0, index=0, entries=(), commit=0, snapshot=None,
                 reject=False, hint=0):
    """Message.MarshalTo: every required field, in field order, entries and
    the (non-nullable) snapshot included."""
    b = (key(1, 0) + varint(type) + key(2, 0) + varint(to) + key(3, 0) + varint(frm) + key(4, 0) + varint(term) +
         key(5, 0) + varint(log_term) + key(6, 0) + varint(index))
    for e in entries:
        eb = _entry(e)
        b += key(7, 2) + varint(len(eb)) + eb
    sb = _snapshot(snapshot)
    b += key(8, 0) + varint(commit) + key(9, 2) + varint(len(sb)) + sb
    b += key(10, 0) + bytes([1 if reject else 0]) + key(11, 0) + varint(hint)
    return b


_PB = None


def pb_classes():
    """raftpb.Message & co. from raft/raftpb/raft.proto through the protobuf library."""
    global _PB
    if _PB is not None:
        return _PB
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="raftpb_test.proto", package="raftpb", syntax="proto2")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
    REQ, OPT, REP = F.LABEL_REQUIRED, F.LABEL_OPTIONAL, F.LABEL_REPEATED
    U64, BYTES, MSG, I32, BOOL = F.TYPE_UINT64, F.TYPE_BYTES, F.TYPE_MESSAGE, F.TYPE_INT32, F.TYPE_BOOL
    msg("Entry", [("Type", 1, I32, REQ, None), ("Term", 2, U64, REQ, None), ("Index", 3, U64, REQ, None),
                  ("Data", 4, BYTES, OPT, None)])
    msg("ConfState", [("nodes", 1, U64, REP, None)])
    msg("SnapshotMetadata", [("conf_state", 1, MSG, REQ, ".raftpb.ConfState"), ("index", 2, U64, REQ, None),
                             ("term", 3, U64, REQ, None)])
    msg("Snapshot", [("data", 1, BYTES, OPT, None), ("metadata", 2, MSG, REQ, ".raftpb.SnapshotMetadata")])
    msg("Message", [("type", 1, I32, REQ, None), ("to", 2, U64, REQ, None), ("from", 3, U64, REQ, None),
                    ("term", 4, U64, REQ, None), ("logTerm", 5, U64, REQ, None), ("index", 6, U64, REQ, None),
                    ("entries", 7, MSG, REP, ".raftpb.Entry"), ("commit", 8, U64, REQ, None),
                    ("snapshot", 9, MSG, REQ, ".raftpb.Snapshot"), ("reject", 10, BOOL, REQ, None),
                    ("rejectHint", 11, U64, REQ, None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    _PB = {n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"raftpb.{n}"))
           for n in ("Message", "Entry", "Snapshot")}
    return _PB


def pb_message(type, to=0, frm=0, term=0, log_term=0, index=0, commit=0, reject=False, hint=0, entries=()):
    M = pb_classes()["Message"]
    m = M()
    m.type, m.to, m.term, m.logTerm, m.index, m.commit, m.reject, m.rejectHint = \
        type, to, term, log_term, index, commit, reject, hint
    setattr(m, "from", frm)
    for t, et, ei, data in entries:
        e = m.entries.add()
        e.Type, e.Term, e.Index = t, et, ei
        if data is not None:
            e.Data = data
    m.snapshot.metadata.index = 0
    m.snapshot.metadata.term = 0
    m.snapshot.metadata.conf_state.SetInParent()
    return m.SerializeToString()


# ---------------------------------------------------------------------------- corpora
RESP_TYPES = (abi.HB_MSG_APP_RESP, abi.HB_MSG_VOTE_RESP, abi.HB_MSG_HEARTBEAT_RESP)


def response_records(G, n_per_group, peers, rng, reject_p=0.1):
    """Well-formed gogo-encoded responses addressed to random groups."""
    recs, groups = [], []
    N = G * n_per_group
    g = rng.integers(0, G, N)
    for k in range(N):
        gi = int(g[k])
        t = int(rng.choice(RESP_TYPES))
        frm = int(peers[gi, int(rng.integers(0, 3))])
        rej = bool(rng.random() < reject_p)
        recs.append(gogo_marshal(t, to=int(peers[gi, 0]), frm=frm, term=int(rng.integers(0, 1 << 20)),
                                 log_term=int(rng.integers(0, 50)), index=int(rng.integers(0, 1 << 40)),
                                 commit=int(rng.integers(0, 1 << 30)), reject=rej,
                                 hint=int(rng.integers(0, 1 << 33)) if rej else 0))
        groups.append(gi)
    return recs, np.array(groups, np.uint32)


def _unknown_field(rng, depth=0):
    f = int(rng.integers(12, 4000))
    wt = int(rng.choice([0, 1, 2, 3, 5]))
    if wt == 0:
        return key(f, 0) + varint(int(rng.integers(0, 1 << 63)))
    if wt == 1:
        return key(f, 1) + bytes(rng.integers(0, 256, 8, dtype=np.uint8))
    if wt == 5:
        return key(f, 5) + bytes(rng.integers(0, 256, 4, dtype=np.uint8))
    if wt == 2:
        b = bytes(rng.integers(0, 256, int(rng.integers(0, 12)), dtype=np.uint8))
        return key(f, 2) + varint(len(b)) + b
    inner = b"".join(_unknown_field(rng, depth + 1) for _ in range(int(rng.integers(0, 3)))) if depth < 3 else b""
    return key(f, 3) + inner + key(f, 4)


def mutate(rec, rng):
    """One adversarial variant of a record (each kind exercises a decoder rule)."""
    r = bytearray(rec)
    kind = int(rng.integers(0, 14))
    if kind == 0 and len(r) > 1:                       # truncation -> ErrUnexpectedEOF
        return bytes(r[: int(rng.integers(0, len(r)))]), "trunc"
    if kind == 1:                                      # a byte flip anywhere
        i = int(rng.integers(0, len(r)))
        r[i] ^= 1 << int(rng.integers(0, 8))
        return bytes(r), "flip"
    if kind == 2:                                      # a repeated varint field ORs in
        f = int(rng.choice([1, 3, 4, 6, 10, 11]))
        return bytes(r) + key(f, 0) + varint(int(rng.integers(0, 1 << 40))), "repeat"
    if kind == 3:                                      # unknown fields (all wire types, nested groups)
        pos = int(rng.integers(0, 2))
        u = b"".join(_unknown_field(rng) for _ in range(int(rng.integers(1, 4))))
        return (u + bytes(r)) if pos == 0 else (bytes(r) + u), "unknown"
    if kind == 4:                                      # non-minimal varint value
        return key(4, 0) + b"\x85\x80\x80\x00" + bytes(r), "nonminimal"
    if kind == 5:                                      # non-minimal key (the skip restart quirk)
        return bytes(r) + b"\xe0\x80\x00" + varint(5), "nonminimal-key"
    if kind == 6:                                      # an over-long varint (> 10 bytes)
        return bytes(r) + key(6, 0) + b"\xff" * 12 + b"\x01", "longvarint"
    if kind == 7:                                      # wrong wire type for a known field
        f = int(rng.integers(1, 12))
        return bytes(r) + key(f, 1 if f not in (7, 9) else 0) + b"\x00" * 8, "wrongwt"
    if kind == 8:                                      # illegal wire type in an unknown field
        return bytes(r) + key(int(rng.integers(12, 100)), int(rng.choice([6, 7]))), "illegal"
    if kind == 9:                                      # negative length (Go panics)
        return bytes(r) + key(int(rng.choice([7, 9, 20])), 2) + varint((1 << 64) - 20), "neglen"
    if kind == 10:                                     # field number aliasing through int32(key >> 3)
        return bytes(r) + varint(((1 << 32) + 4) << 3) + varint(int(rng.integers(0, 1 << 20))), "alias"
    if kind == 11:                                     # a malformed Entry (its error is ignored)
        bad = key(4, 2) + varint(50) + b"\x01"
        return bytes(r) + key(7, 2) + varint(len(bad)) + bad, "badentry"
    if kind == 12:                                     # a malformed Snapshot (its error propagates)
        bad = key(2, 2) + varint(3) + key(1, 0) + b"\x80"
        return bytes(r) + key(9, 2) + varint(len(bad)) + bad, "badsnap"
    # a group whose inner field moves the index backwards (Go never returns)
    loop = key(30, 3) + key(31, 2) + varint((1 << 64) - 12) + key(30, 4)
    return bytes(r) + loop, "loop"


def pack(recs):
    """Records -> (bytes u8, off u64, len u32)."""
    lens = np.array([len(r) for r in recs], np.uint32)
    off = np.zeros(len(recs), np.uint64)
    if len(recs) > 1:
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    data = np.frombuffer(b"".join(recs), dtype=np.uint8).copy() if recs else np.zeros(1, np.uint8)
    return data, off, lens


def pb_entry(type, term, index, data):
    """raftpb.Entry through the protobuf library (independent of the gogo Size restatement)."""
    e = pb_classes()["Entry"]()
    e.Type, e.Term, e.Index = type, term, index
    if data is not None:
        e.Data = data
    return e.SerializeToString()
