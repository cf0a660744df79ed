"""cfg3 / cfg4 bench streams through the oracle (CPU): the streams the bench
replays must hit the paths they are meant to hit."""
import numpy as np

from etcd_amd import abi, synth
from oracle.pyoracle import OracleGroups


def test_cfg4_storm_repeats():
    """Every step of the repeatable storm steps every group down, campaigns and
    tallies n-1 votes; decided = won + lost, and the terms stay inside [T, T+4k+3]."""
    G, n = 2000, 7
    g, runs = synth.election_groups(G, n, seed=3)
    og = OracleGroups(g, runs, 16)
    b = synth.cfg4_storm_batch(g, seed=4)
    t0 = g["term"].astype(np.int64)
    for k in range(3):
        bk = dict(b, term=synth.storm_terms(b["term"], k))
        _, st = og.step(bk)
        assert st[abi.HB_STAT_VOTERESP] == G * (n - 1)
        assert st[abi.HB_STAT_FAULTS] == 0
        assert st[abi.HB_STAT_WON] > 0 and st[abi.HB_STAT_LOST] > 0
        now = og.groups()
        t = now["term"].astype(np.int64)
        assert (t >= t0 + 4 * k + 2).all() and (t <= t0 + 4 * k + 3).all()
        # a winner still steps down on a later higher-term vote response
        assert 0 < int((now["state"] == abi.HB_STATE_LEADER).sum()) <= int(st[abi.HB_STAT_WON])


def test_cfg3_open_loop_mix():
    """The open-loop cfg3 stream keeps leaders replicating with a Probe /
    Replicate / paused mix, rejects, heartbeats and commits, without faults."""
    G, n, W = 3000, 5, 8
    g, runs = synth.lagging_groups(G, n, seed=0x5EED0003, W=W)
    og = OracleGroups(g, runs, W)
    rng = np.random.default_rng(5)
    seen_probe = seen_repl = 0
    for k in range(5):
        now = og.groups()
        b = synth.cfg3_open_batch(now, rng)
        _, st = og.step(b)
        assert st[abi.HB_STAT_FAULTS] == 0
        assert st[abi.HB_STAT_APPRESP] > 0 and st[abi.HB_STAT_COMMITS] > 0
        after = og.groups()
        prs = after["pr"][:, 1:n]
        seen_probe += int((prs["state"] == abi.HB_PR_PROBE).sum())
        seen_repl += int((prs["state"] == abi.HB_PR_REPLICATE).sum())
        assert (after["state"] == abi.HB_STATE_LEADER).all()
    assert seen_probe > 0 and seen_repl > 0
