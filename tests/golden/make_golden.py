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

BATCH_KEYS = ("group", "info", "term", "index", "hint", "props")


def cases():
    """(name, nmax, W, groups, runs, ins, [batch per step])"""
    g, runs = synth.steady_groups(96, 3, seed=0x601D01, last_hi=1 << 12)
    yield "cfg2_n3", 3, 256, g, runs, None, [synth.cfg2_batch(g, k, seed=0x601D02) for k in range(3)]
    g, runs = synth.steady_groups(64, 5, seed=0x601D03, last_hi=1 << 12)
    yield "cfg2_n5", 5, 256, g, runs, None, [synth.cfg2_batch(g, k, seed=0x601D04) for k in range(2)]
    g, runs = synth.election_groups(64, 7, seed=0x601D05)
    yield "storm_n7", 7, 8, g, runs, None, [synth.cfg4_storm_batch(g, seed=0x601D06)]
    g, runs, ins = synth.random_groups(128, 5, seed=0x601D07, W=8)
    yield "fuzz_n5", 5, 8, g, runs, ins, [synth.random_batch(g, 600, seed=0x601D08 + k) for k in range(2)]


def make(name, nmax, W, groups, runs, ins, batches):
    og = OracleGroups(groups, runs, W, abi.HB_NO_LIMIT, ins)
    out = {"nmax": np.array(nmax), "W": np.array(W), "init": og.groups(), "steps": np.array(len(batches))}
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
