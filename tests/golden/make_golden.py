"""Generate the committed golden fixtures (tests/golden/*.npz).

Test infrastructure only.  Each fixture is a small seeded case stepped by the
C oracle (oracle/raft_oracle.c, the restatement pinned by the reference's own
known-answer tests, tests/test_oracle_kat.py): the initial group records, the
batches, and per step the expected event stream, statistics and group records.
The reference (Go) cannot run in this image or on the GPU box (SURVEY.md
§8(c)), so these are oracle outputs frozen as data: tests/test_golden.py checks
that the oracle still reproduces them (CPU) and that the engine reproduces
them without the oracle (GPU).

  python tests/golden/make_golden.py        # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from etcd_amd import abi, synth  # noqa: E402
from oracle.pyoracle import OracleGroups  # noqa: E402

BATCH_KEYS = ("group", "info", "term", "index", "hint", "props", "edesc", "eoff", "peoff", "commit", "eterm")


def _follower_batches(g, runs, ins, W, term_runs, seeds):
    """Follower-side messages mixed with leader-side ones, each step drawn from
    the state the previous steps left (a scratch oracle)."""
    og = OracleGroups(g, runs, W, abi.HB_NO_LIMIT, ins)
    og.load_term_runs(term_runs)
    out = []
    for s in seeds:
        a = synth.random_batch(g, 300, seed=s, props=False)
        b = synth.follower_messages(og.groups(), og.term, 300, seed=s + 1, deep=0.3)
        m = synth.merge_batches(a, b, seed=s + 2)
        og.step(m)
        out.append(m)
    return out


def cases():
    """(name, nmax, W, groups, runs, ins, [batch per step], extra) — extra:
    max_msg_size, entry sizes {group: [...]}, older term runs {group: [...]}"""
    g, runs = synth.steady_groups(96, 3, seed=0x601D01, last_hi=1 << 12)
    yield "cfg2_n3", 3, 256, g, runs, None, [synth.cfg2_batch(g, k, seed=0x601D02) for k in range(3)], {}
    g, runs = synth.steady_groups(64, 5, seed=0x601D03, last_hi=1 << 12)
    yield "cfg2_n5", 5, 256, g, runs, None, [synth.cfg2_batch(g, k, seed=0x601D04) for k in range(2)], {}
    g, runs = synth.election_groups(64, 7, seed=0x601D05)
    yield "storm_n7", 7, 8, g, runs, None, [synth.cfg4_storm_batch(g, seed=0x601D06)], {}
    g, runs, ins = synth.random_groups(128, 5, seed=0x601D07, W=8)
    yield "fuzz_n5", 5, 8, g, runs, ins, [synth.random_batch(g, 600, seed=0x601D08 + k) for k in range(2)], {}
    # a finite MaxSizePerMsg: limitSize over the entries' gogo sizes, the whole log's sizes loaded
    g, runs, ins = synth.random_groups(128, 3, seed=0x601D09, W=8)
    sizes = synth.window_sizes(g, runs, seed=0x601D0A, frac_full=1.0)
    bs = [synth.attach_entry_descs(synth.random_batch(g, 500, seed=0x601D0B + k), len(g), seed=0x601D0C + k)
          for k in range(2)]
    yield "sized_n3", 3, 8, g, runs, ins, bs, {"max_msg_size": 150, "sizes": sizes}
    # the follower side: MsgApp (conflicts, rejections, probes into older runs), MsgHeartbeat, MsgSnap, MsgVote
    g, runs, ins = synth.random_groups(160, 3, seed=0x601D0D, W=8)
    tr = synth.older_runs(g, runs)
    yield "follower_n3", 3, 8, g, runs, ins, _follower_batches(g, runs, ins, 8, tr, [0x601D0E, 0x601D1E]), \
        {"term_runs": tr}
    # r.Commit = 0 before a group's first Step (hb_group.commit_zero) beside r.Commit == committed
    g, runs, ins = synth.random_groups(160, 5, seed=0x601D0F, W=8, commit_zero_p=0.5)
    tr = synth.older_runs(g, runs)
    yield "commitzero_n5", 5, 8, g, runs, ins, _follower_batches(g, runs, ins, 8, tr, [0x601D2E, 0x601D3E]), \
        {"term_runs": tr}


def oracle_for(groups, runs, W, ins, extra):
    og = OracleGroups(groups, runs, W, extra.get("max_msg_size", abi.HB_NO_LIMIT), ins)
    if extra.get("sizes"):
        og.load_sizes(extra["sizes"])
    if extra.get("term_runs"):
        og.load_term_runs(extra["term_runs"])
    return og


def flat(d, width):
    """{group: [items]} -> (groups u32, counts u32, flat values) for the fixture"""
    gs = sorted(d)
    vals = [x for g in gs for x in (d[g] if width == 1 else [v for r in d[g] for v in r])]
    return (np.array(gs, dtype=np.uint32), np.array([len(d[g]) for g in gs], dtype=np.uint32),
            np.array(vals, dtype=np.uint64))


def make(name, nmax, W, groups, runs, ins, batches, extra):
    og = oracle_for(groups, runs, W, ins, extra)
    out = {"nmax": np.array(nmax), "W": np.array(W), "init": og.groups(), "steps": np.array(len(batches)),
           "max_msg_size": np.array(extra.get("max_msg_size", abi.HB_NO_LIMIT), dtype=np.uint64)}
    if extra.get("sizes"):
        out["sz_gs"], out["sz_n"], out["sz_vals"] = flat(extra["sizes"], 1)
    if extra.get("term_runs"):
        out["tr_gs"], out["tr_n"], out["tr_vals"] = flat(extra["term_runs"], 2)
    if ins:
        keys = sorted(ins)
        out["ins_gs"] = np.array(keys, dtype=np.uint32).reshape(-1, 2)
        out["ins_len"] = np.array([len(ins[k]) for k in keys], dtype=np.uint32)
        out["ins_vals"] = np.concatenate([np.asarray(ins[k], dtype=np.uint64) for k in keys])
    for k, b in enumerate(batches):
        for f in BATCH_KEYS:
            if b.get(f) is not None:
                out[f"b{k}_{f}"] = np.ascontiguousarray(b[f])
        ev, st = og.step(b)
        order = np.argsort(ev["group"], kind="stable")
        out[f"ev{k}"] = ev[order]
        out[f"st{k}"] = st
        out[f"gr{k}"] = og.groups()
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    return out


if __name__ == "__main__":
    for c in cases():
        o = make(*c)
        print(c[0], {k: v.shape for k, v in o.items() if k.startswith("ev")})
