"""Wire ingestion on the CPU: the oracle's restatement of the reference's
raftpb decoder (oracle/wire_oracle.c) against encodings from the protobuf
library and the reference's own encoder (restated in wire_util.gogo_marshal),
plus the generated decoder's quirks, each on a hand-made record.

Parity anchor: raft/raftpb/raft.pb.go (gogo-generated Unmarshal / MarshalTo)
and gogo proto.Skip; the reference ships no wire test vectors for Message, so
the independent protobuf encoder is the golden source for well-formed records.
"""
import numpy as np
import pytest

from etcd_amd import abi
from oracle.pyoracle import decode_batch, unmarshal_message

from . import wire_util as W

OK, ERR, PANIC, DEEP = 0, 1, 2, 3


def _fields(m):
    return (m.type, m.to, m.from_, m.term, m.log_term, m.index, m.commit, bool(m.reject), m.reject_hint)


@pytest.mark.parametrize("seed", range(4))
def test_protobuf_library_encodings_decode(seed):
    rng = np.random.default_rng(seed)
    for _ in range(300):
        f = dict(type=int(rng.integers(0, 12)), to=int(rng.integers(0, 1 << 63)), frm=int(rng.integers(0, 1 << 63)),
                 term=int(rng.integers(0, 1 << 63)), log_term=int(rng.integers(0, 1 << 20)),
                 index=int(rng.integers(0, 1 << 63)), commit=int(rng.integers(0, 1 << 40)),
                 reject=bool(rng.integers(0, 2)), hint=int(rng.integers(0, 1 << 63)))
        ents = [(int(rng.integers(0, 2)), int(rng.integers(0, 9)), int(rng.integers(0, 99)),
                 bytes(rng.integers(0, 256, int(rng.integers(0, 5)), dtype=np.uint8)) if rng.random() < .5 else None)
                for _ in range(int(rng.integers(0, 3)))]
        rc, m = unmarshal_message(W.pb_message(**f, entries=ents))
        assert rc == OK
        assert _fields(m) == (f["type"], f["to"], f["frm"], f["term"], f["log_term"], f["index"], f["commit"],
                              f["reject"], f["hint"])
        assert m.nentries == len(ents)


def test_gogo_encoder_matches_protobuf_library():
    """The restated MarshalTo produces what the protobuf library parses."""
    M = W.pb_classes()["Message"]
    rng = np.random.default_rng(9)
    for _ in range(200):
        vals = [int(rng.integers(0, 1 << 40)) for _ in range(7)]
        b = W.gogo_marshal(4, *vals[:5], commit=vals[5], reject=bool(vals[6] & 1), hint=vals[6],
                           entries=[(0, 3, 4, b"xy")], snapshot=(b"s", (1, 2), 7, 8))
        m = M()
        m.ParseFromString(b)
        assert (m.to, getattr(m, "from"), m.term, m.logTerm, m.index, m.commit, m.rejectHint) == \
            (vals[0], vals[1], vals[2], vals[3], vals[4], vals[5], vals[6])
        assert m.snapshot.metadata.index == 7 and list(m.snapshot.metadata.conf_state.nodes) == [1, 2]
        rc, o = unmarshal_message(b)
        assert rc == OK and o.index == vals[4] and o.nentries == 1


def test_vectorized_encoder_matches_gogo():
    """synth.encode_responses (the bench's encoder) == the restated MarshalTo."""
    from etcd_amd import synth
    rng = np.random.default_rng(2)
    N = 400
    t = rng.choice(W.RESP_TYPES, N).astype(np.uint64)
    to, frm = rng.integers(0, 1 << 20, N), rng.integers(0, 1 << 62, N)
    term, idx = rng.integers(0, 1 << 40, N), rng.integers(0, 1 << 63, N)
    rej, hint = rng.integers(0, 2, N), rng.integers(0, 1 << 45, N)
    data, off, ln = synth.encode_responses(t, to, frm, term, idx, rej, hint)
    for i in range(N):
        want = W.gogo_marshal(int(t[i]), to=int(to[i]), frm=int(frm[i]), term=int(term[i]), index=int(idx[i]),
                              reject=bool(rej[i]), hint=int(hint[i]))
        assert bytes(data[int(off[i]):int(off[i]) + int(ln[i])]) == want, i


def test_appresp_wire_size():
    """A steady-state MsgAppResp as the reference encodes it."""
    b = W.gogo_marshal(abi.HB_MSG_APP_RESP, to=1, frm=2, term=7, index=1 << 20)
    assert len(b) == 30 and b[:2] == b"\x08\x04"


def test_quirks():
    base = W.gogo_marshal(abi.HB_MSG_APP_RESP, to=1, frm=2, term=5, index=100, reject=True, hint=3)
    # a repeated varint field ORs into the value
    rc, m = unmarshal_message(base + W.key(6, 0) + W.varint(0x1000))
    assert rc == OK and m.index == 100 | 0x1000
    # Reject is assigned: the last occurrence wins
    rc, m = unmarshal_message(base + W.key(10, 0) + W.varint(0))
    assert rc == OK and m.reject == 0
    # MessageType is int32: bits past 31 vanish, bit 31 makes it negative
    rc, m = unmarshal_message(W.key(1, 0) + b"\x80\x80\x80\x80\x7f")
    assert rc == OK and m.type == -268435456  # 0x7F << 28 kept to 32 bits = 0xF0000000
    # field numbers alias through int32(key >> 3)
    rc, m = unmarshal_message(W.varint(((1 << 32) + 6) << 3) + W.varint(77))
    assert rc == OK and m.index == 77
    # bits shifted past 63 are dropped (over-long varints still parse)
    rc, m = unmarshal_message(W.key(4, 0) + b"\xff" * 12 + b"\x01")
    assert rc == OK and m.term == (1 << 63) - 1 + (1 << 63)
    # truncated / wrong wire type / illegal wire type
    assert unmarshal_message(base[:-1])[0] == ERR
    assert unmarshal_message(base + W.key(4, 2) + b"\x00")[0] == ERR
    assert unmarshal_message(base + W.key(40, 7))[0] == ERR
    # unknown fields of every wire type are skipped
    u = (W.key(40, 0) + W.varint(5) + W.key(41, 1) + b"\x00" * 8 + W.key(42, 2) + b"\x02ab" +
         W.key(43, 5) + b"\x00" * 4 + W.key(44, 3) + W.key(45, 0) + b"\x01" + W.key(44, 4))
    rc, m = unmarshal_message(u + base)
    assert rc == OK and m.index == 100 and m.term == 5
    # an unknown fixed64 running past the end is an EOF error
    assert unmarshal_message(base + W.key(41, 1) + b"\x00" * 3)[0] == ERR
    # a malformed Entry is ignored; a malformed Snapshot is an error
    bad = W.key(4, 2) + W.varint(50) + b"\x01"
    assert unmarshal_message(base + W.key(7, 2) + W.varint(len(bad)) + bad)[0] == OK
    bad = W.key(2, 2) + W.varint(3) + W.key(1, 0) + b"\x80"
    assert unmarshal_message(base + W.key(9, 2) + W.varint(len(bad)) + bad)[0] == ERR
    # negative lengths: Go panics on the slice bounds
    assert unmarshal_message(base + W.key(9, 2) + b"\xff" * 9 + b"\x01")[0] == PANIC
    assert unmarshal_message(base + W.key(50, 2) + W.varint((1 << 64) - 20))[0] == PANIC
    # ... unless index + skippy still moves forward: then Go reads on (here to an EOF)
    assert unmarshal_message(base + W.key(50, 2) + b"\xff" * 9 + b"\x01")[0] == ERR
    # a group whose inner field jumps backwards never returns in Go
    loop = W.key(30, 3) + W.key(31, 2) + W.varint((1 << 64) - 12) + W.key(30, 4)  # next = 0
    assert unmarshal_message(base + loop)[0] == PANIC
    back = W.key(30, 3) + W.key(31, 2) + W.varint((1 << 64) - 20) + W.key(30, 4)  # index < 0
    assert unmarshal_message(base + back)[0] == PANIC
    # an unknown field whose length cancels its own key (skippy = 0): Message.Unmarshal never returns
    k50 = W.key(50, 2)
    assert unmarshal_message(base + k50 + W.varint((1 << 64) - (len(k50) + 10)))[0] == PANIC
    # groups nested past 16 levels go to the host
    deep = b"".join(W.key(60, 3) for _ in range(20)) + b"".join(W.key(60, 4) for _ in range(20))
    assert unmarshal_message(base + deep)[0] == DEEP
    shallow = b"".join(W.key(60, 3) for _ in range(5)) + b"".join(W.key(60, 4) for _ in range(5))
    assert unmarshal_message(base + shallow)[0] == OK
    # a non-minimal key: the skip restarts at index - minimal_len(key)
    rc, _ = unmarshal_message(base + b"\xe0\x80\x00" + W.varint(5))
    assert rc in (OK, ERR, PANIC)
    # the empty record is a valid, all-zero message (MsgHup)
    rc, m = unmarshal_message(b"")
    assert rc == OK and m.type == 0


def test_decode_batch_contract():
    """Statuses and the batch record (local / host types, bad groups, slots)."""
    G = 4
    peers = np.zeros((G, abi.HB_MAX_REPLICAS), np.uint64)
    peers[:, :3] = [[11, 12, 13]] * G
    group_n = np.full(G, 3, np.uint32)
    recs = [W.gogo_marshal(abi.HB_MSG_APP_RESP, frm=12, term=3, index=9),
            W.gogo_marshal(abi.HB_MSG_VOTE_RESP, frm=13, term=4, reject=True),
            W.gogo_marshal(abi.HB_MSG_HEARTBEAT_RESP, frm=99, term=4),
            W.gogo_marshal(abi.HB_MSG_HUP, frm=12),
            W.gogo_marshal(abi.HB_MSG_APP, frm=12, entries=[(0, 1, 2, b"x")]),
            W.gogo_marshal(abi.HB_MSG_APP_RESP, frm=12, term=3, index=9, reject=True, hint=4),
            W.gogo_marshal(abi.HB_MSG_APP_RESP, frm=12)[:-1]]
    grp = np.array([0, 1, 2, 3, 0, 7, 1], np.uint32)
    data, off, ln = W.pack(recs)
    o = decode_batch(data, off, ln, grp, G, group_n, peers)
    assert list(o["status"]) == [abi.HB_WIRE_OK, abi.HB_WIRE_OK, abi.HB_WIRE_OK, abi.HB_WIRE_LOCAL,
                                 abi.HB_WIRE_HOST, abi.HB_WIRE_BADGROUP, abi.HB_WIRE_ERROR]
    assert list(o["group"][:3]) == [0, 1, 2] and (o["group"][3:] == 0xFFFFFFFF).all()
    assert o["info"][0] == abi.hb_info(abi.HB_MSG_APP_RESP, 1)
    assert o["info"][1] == abi.hb_info(abi.HB_MSG_VOTE_RESP, 2, reject=True)
    assert o["info"][2] == abi.hb_info(abi.HB_MSG_HEARTBEAT_RESP, abi.HB_SLOT_NONE)
    assert o["term"][0] == 3 and o["index"][0] == 9


def test_mutated_corpus_runs():
    """Every mutation kind decodes to some status without crashing the oracle."""
    rng = np.random.default_rng(3)
    base = [W.gogo_marshal(abi.HB_MSG_APP_RESP, frm=2, term=int(t), index=int(i))
            for t, i in zip(rng.integers(0, 99, 100), rng.integers(0, 1 << 30, 100))]
    seen = {}
    for r in base * 10:
        m, kind = W.mutate(r, rng)
        rc, _ = unmarshal_message(m)
        seen.setdefault(kind, set()).add(rc)
    assert len(seen) == 14
    assert seen["trunc"] <= {OK, ERR} and seen["neglen"] == {PANIC} and seen["loop"] == {PANIC}
    assert seen["badentry"] == {OK} and seen["badsnap"] == {ERR} and seen["illegal"] == {ERR}
