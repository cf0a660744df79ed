"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py):
seeded cases with the expected event stream, statistics and group records per
step.  CPU: the oracle still reproduces them.  GPU: the engine reproduces them
through the C ABI, with no oracle involved."""
import glob
import os

import numpy as np
import pytest

from etcd_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))
BATCH_KEYS = ("group", "info", "term", "index", "hint", "props", "edesc", "eoff", "peoff", "commit", "eterm")


def load(path):
    d = np.load(path, allow_pickle=False)
    return {k: d[k] for k in d.files}


def batch(d, k):
    return {f: d[f"b{k}_{f}"] for f in BATCH_KEYS if f"b{k}_{f}" in d}


def ins_of(d):
    if "ins_gs" not in d:
        return None
    out, o = {}, 0
    for (g, s), n in zip(d["ins_gs"].tolist(), d["ins_len"].tolist()):
        out[(g, s)] = d["ins_vals"][o:o + n]
        o += n
    return out


def unflat(d, key, width):
    if f"{key}_gs" not in d:
        return None
    out, o = {}, 0
    for g, n in zip(d[f"{key}_gs"].tolist(), d[f"{key}_n"].tolist()):
        v = d[f"{key}_vals"][o:o + n * width]
        out[g] = v.tolist() if width == 1 else [tuple(x) for x in v.reshape(-1, 2).tolist()]
        o += n * width
    return out


def test_fixtures_present():
    names = {os.path.basename(p) for p in FIXTURES}
    assert {"cfg2_n3.npz", "cfg2_n5.npz", "storm_n7.npz", "fuzz_n5.npz", "sized_n3.npz",
            "follower_n3.npz", "commitzero_n5.npz"} <= names


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_golden(path):
    from tests.golden.make_golden import cases, oracle_for
    name = os.path.basename(path)[:-4]
    case = next(c for c in cases() if c[0] == name)
    want = load(path)
    _, nmax, W, groups, runs, ins, batches, extra = case
    og = oracle_for(groups, runs, W, ins, extra)
    assert np.array_equal(og.groups(), want["init"])
    for k, b in enumerate(batches):
        ev, st = og.step(b)
        ev = ev[np.argsort(ev["group"], kind="stable")]
        assert np.array_equal(ev, want[f"ev{k}"]), f"{name} step {k}: events"
        assert np.array_equal(st, want[f"st{k}"]), f"{name} step {k}: stats"
        assert np.array_equal(og.groups(), want[f"gr{k}"]), f"{name} step {k}: groups"


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_engine_reproduces_golden(path):
    from etcd_amd.hipbatch import Engine
    d = load(path)
    init = d["init"]
    eng = Engine(len(init), max_replicas=int(d["nmax"]), max_inflight=int(d["W"]),
                 max_msg_size=int(d["max_msg_size"]), max_batch=1 << 14)
    eng.load_groups(init)
    if unflat(d, "sz", 1):
        eng.load_entry_sizes(unflat(d, "sz", 1))
    if unflat(d, "tr", 2):
        eng.load_term_runs(unflat(d, "tr", 2))
    # the log index covers every group's log and anything a fixture step appends
    sized = int(d["max_msg_size"]) not in (0, abi.HB_NO_LIMIT)
    eng.reserve_log(np.arange(len(init), dtype=np.uint32), 4096 if sized else None, 256)
    for (g, s), vals in (ins_of(d) or {}).items():
        eng.set_inflights(g, s, int(init[g]["pr"][s]["ins_start"]), vals)
    name = os.path.basename(path)[:-4]
    for k in range(int(d["steps"])):
        eng.step_batch(batch(d, k), host=True)
        ev = eng.events()
        ev = ev[np.argsort(ev["group"], kind="stable")]  # (order is promised per group only)
        assert np.array_equal(ev, d[f"ev{k}"]), f"{name} step {k}: events"
        st = eng.stats()
        assert np.array_equal(st, d[f"st{k}"]), f"{name} step {k}: stats {st} vs {d[f'st{k}']}"
        got, want = eng.get_groups(), d[f"gr{k}"]
        assert np.array_equal(got["fault"], want["fault"]), f"{name} step {k}: faults"
        live = want["fault"] == 0  # after a panic only the fault code is specified
        assert np.array_equal(got[live], want[live]), f"{name} step {k}: group records"
