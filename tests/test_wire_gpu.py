"""GPU parity of wire ingestion: hb_decode (k_decode) against the oracle's
restatement of the reference decoder, record by record (status and batch
record bit-exact), and decode -> step end to end against the oracle."""
import numpy as np
import pytest

from etcd_amd import abi, synth
from oracle.pyoracle import decode_batch

from . import wire_util as W
from .parity_util import Pair, assert_events_equal, assert_groups_equal

pytestmark = pytest.mark.gpu


def _dev(torch, a):
    a = np.ascontiguousarray(a)
    view = {np.dtype(np.uint8): np.uint8, np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}[a.dtype]
    return torch.from_numpy(a.view(view)).cuda()


def _decode_dev(eng, torch, data, off, ln, grp):
    n = len(off)
    out = {"group": torch.empty(n, dtype=torch.int32, device="cuda"),
           "info": torch.empty(n, dtype=torch.int32, device="cuda"),
           "term": torch.empty(n, dtype=torch.int64, device="cuda"),
           "index": torch.empty(n, dtype=torch.int64, device="cuda"),
           "hint": torch.empty(n, dtype=torch.int64, device="cuda")}
    status = torch.empty(n, dtype=torch.uint8, device="cuda")
    eng.decode(_dev(torch, data), _dev(torch, off), _dev(torch, ln), _dev(torch, grp), out, status)
    torch.cuda.synchronize()
    return out, status


def _peers(G, n):
    p = np.zeros((G, abi.HB_MAX_REPLICAS), np.uint64)
    p[:, :n] = np.arange(1, n + 1, dtype=np.uint64)  # the oracle's ids: slot + 1
    return p


@pytest.mark.parametrize("seed", [1, 2])
def test_decode_corpus_bit_exact(seed):
    import torch
    from etcd_amd.hipbatch import Engine
    G = 3000
    rng = np.random.default_rng(seed)
    g, _ = synth.steady_groups(G, 3, seed=seed, with_runs=False)
    eng = Engine(G, max_replicas=3, max_inflight=8, max_batch=1 << 16)
    eng.load_groups(g)
    peers = _peers(G, 3)
    peers[::7, 1] = 99  # some groups do not know node 2
    eng.load_peers(peers)
    good, grp = W.response_records(G, 3, peers, rng)
    recs = list(good)
    for r in good[:6000]:
        recs.append(W.mutate(r, rng)[0])
    grp = np.concatenate([grp, rng.integers(0, G + 50, len(recs) - len(grp)).astype(np.uint32)])
    data, off, ln = W.pack(recs)
    out, status = _decode_dev(eng, torch, data, off, ln, grp)
    ora = decode_batch(data, off, ln, grp, G, np.full(G, 3, np.uint32), peers)
    st = status.cpu().numpy()
    bad = np.nonzero(st != ora["status"])[0]
    assert len(bad) == 0, f"status differs at {bad[:5]}: dev {st[bad[:5]]} ora {ora['status'][bad[:5]]}"
    for k, dt in (("group", np.uint32), ("info", np.uint32), ("term", np.uint64), ("index", np.uint64),
                  ("hint", np.uint64)):
        d = out[k].cpu().numpy().view(dt)
        bad = np.nonzero(d != ora[k])[0]
        assert len(bad) == 0, f"{k} differs at {bad[:5]}"
    counts = np.bincount(st, minlength=6)
    assert counts[abi.HB_WIRE_OK] > 0 and counts[abi.HB_WIRE_ERROR] > 0 and counts[abi.HB_WIRE_PANIC] > 0


def test_decode_then_step_cfg2():
    """cfg2 acks as the reference encodes them -> hb_decode -> hb_step equals
    the oracle stepping its own decode of the same bytes."""
    import torch
    G, n = 4000, 3
    g, runs = synth.steady_groups(G, n, seed=5)
    pair = Pair(g, runs, n, 256, max_batch=G * n + 16)
    peers = _peers(G, n)
    pair.eng.load_peers(peers)
    for step in range(3):
        b = synth.cfg2_batch(g, step, seed=50 + step)
        recs = [W.gogo_marshal(abi.HB_MSG_APP_RESP, to=1, frm=int((inf >> 4) & 0xF) + 1, term=int(t), index=int(i))
                for inf, t, i in zip(b["info"], b["term"], b["index"])]
        data, off, ln = W.pack(recs)
        out, status = _decode_dev(pair.eng, torch, data, off, ln, b["group"])
        assert (status.cpu().numpy() == abi.HB_WIRE_OK).all()
        props = torch.from_numpy(b["props"].view(np.int32)).cuda()
        pair.eng.step(out["group"], out["info"], out["term"], out["index"], out["hint"], props, host=False)
        dev_ev, dev_st = pair.eng.events(), pair.eng.stats()
        ora = decode_batch(data, off, ln, b["group"], G, np.full(G, n, np.uint32), peers)
        ob = dict(group=ora["group"], info=ora["info"], term=ora["term"], index=ora["index"], hint=ora["hint"],
                  props=b["props"])
        ora_ev, ora_st = pair.og.step(ob)
        assert_events_equal(dev_ev, ora_ev, f"wire step {step}")
        assert np.array_equal(dev_st, ora_st)
        assert_groups_equal(pair.eng.get_groups(), pair.og.groups(), f"wire step {step}")
        assert dev_st[abi.HB_STAT_COMMITS] == G


def test_decode_slots_beyond_n_and_load_order():
    """From -> slot looks only at slots < n of the group (raft/multinode.go:235
    drops the rest as non-members), whichever of hb_load_peers /
    hb_load_groups came first; groups of different n share one handle."""
    import torch
    from etcd_amd.hipbatch import Engine
    G = 2048
    rng = np.random.default_rng(9)
    g3, _ = synth.steady_groups(G // 2, 3, seed=3, with_runs=False)
    g5, _ = synth.steady_groups(G // 2, 5, seed=4, with_runs=False)
    eng = Engine(G, max_replicas=5, max_inflight=8, max_batch=1 << 16)
    peers = np.zeros((G, abi.HB_MAX_REPLICAS), np.uint64)
    peers[:, :5] = np.arange(1, 6, dtype=np.uint64)  # ids beyond n = 3 are set: they must not match
    eng.load_peers(peers)       # before the groups (n comes from hb_load_groups)
    eng.load_groups(g3, first=0)
    eng.load_groups(g5, first=G // 2)
    eng.load_peers(peers[G // 2:], first=G // 2)  # and after
    N = 6 * G
    grp = rng.integers(0, G, N).astype(np.uint32)
    frm = rng.integers(1, 7, N)
    recs = [W.gogo_marshal(abi.HB_MSG_APP_RESP, to=1, frm=int(f), term=7, index=int(i))
            for f, i in zip(frm, rng.integers(0, 1 << 40, N))]
    data, off, ln = W.pack(recs)
    out, status = _decode_dev(eng, torch, data, off, ln, grp)
    nn = np.where(np.arange(G) < G // 2, 3, 5).astype(np.uint32)
    ora = decode_batch(data, off, ln, grp, G, nn, peers)
    assert np.array_equal(status.cpu().numpy(), ora["status"])
    info = out["info"].cpu().numpy().view(np.uint32)
    assert np.array_equal(info, ora["info"])
    slot = (info >> 4) & 0xF
    assert ((slot == abi.HB_SLOT_NONE) == ((frm > nn[grp]) | (frm > 5))).all()
