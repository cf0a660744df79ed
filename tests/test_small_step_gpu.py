"""Small steps (a MultiNode node's Ready cycle over a few thousand groups):
the one-workgroup partitions (`k_pack_one` for a single 4,096-group bucket: a
stable compaction; `k_radix_small` otherwise: histogram, column scan and
scatter of at most 8 tiles of 2048 messages in one launch) and the
one-workgroup event-word compaction (`k_words_small`) against the tiled
kernels they stand in for (`HB_SMALL_STEP=0` at hb_create) and the oracle:
each group's events in the same order, the same compact words, the same state.
"""
import numpy as np
import pytest

from etcd_amd import abi, synth

from .parity_util import Pair, sort_events

pytestmark = pytest.mark.gpu

DRAWS = np.random.default_rng(7).integers(0, 1 << 63, 4096, dtype=np.uint64)


def _pairs(monkeypatch, make):
    """The same groups on two engines: small steps on (default) and off."""
    a = make()
    monkeypatch.setenv("HB_SMALL_STEP", "0")
    try:
        b = make()
    finally:
        monkeypatch.delenv("HB_SMALL_STEP")
    return a, b


def _same(a, b, batch, ctx):
    ev_a, st_a, _ = a.step(batch, ctx=ctx + " small")
    ev_b, st_b, _ = b.step(batch, ctx=ctx + " tiled")
    # (each group's events in its order: the order the engine promises across groups)
    assert np.array_equal(sort_events(ev_a), sort_events(ev_b)), f"{ctx}: events differ"
    assert np.array_equal(st_a, st_b)
    wa, ca = a.eng.event_words()
    wb, cb = b.eng.event_words()
    assert np.array_equal(ca, cb), f"{ctx}: words per chunk differ"
    assert np.array_equal(sort_events(a.eng.expand_words(wa, ca)), sort_events(b.eng.expand_words(wb, cb)))


# 1 tile, exactly 1 / 8 tiles, one message past 1 and past 8 (9 tiles: the tiled path on both)
# (1,800 groups: one bucket, k_pack_one; 20,000: five buckets, k_radix_small)
@pytest.mark.parametrize("nmsg", [1, 2047, 2048, 2049, 16384, 16385])
@pytest.mark.parametrize("nmax", [3, 5, 7])
@pytest.mark.parametrize("G", [1800, 20000])
def test_small_partition_matches_tiled(monkeypatch, G, nmsg, nmax):
    g, runs, ins = synth.random_groups(G, nmax, seed=nmsg + nmax, W=8)
    a, b = _pairs(monkeypatch, lambda: Pair(g, runs, nmax, 8, ins=ins, max_batch=1 << 15))
    for k in range(2):
        batch = synth.random_batch(g, nmsg, seed=31 * nmsg + k)
        if k == 1 and nmsg > 40:  # messages of groups beyond capacity: dropped by the partition
            batch["group"] = batch["group"].copy()
            batch["group"][::37] = G + 3000
        _same(a, b, batch, f"n={nmax} nmsg={nmsg} step {k}")


@pytest.mark.parametrize("nmax", [3, 5])
@pytest.mark.parametrize("G", [1500, 9000])
def test_small_partition_follower_side(monkeypatch, G, nmax):
    """X mode (m.Commit with every record: the extensions beside the records)."""
    g, runs, ins = synth.random_groups(G, nmax, seed=90 + nmax, W=8)
    a, b = _pairs(monkeypatch, lambda: Pair(g, runs, nmax, 8, ins=ins, max_batch=1 << 15, term_runs=True))
    for p in (a, b):
        p.set_timers(synth.random_timers(len(g), seed=5), DRAWS)
    now = a.og.groups()
    for k in range(3):
        f = synth.follower_messages(now, a.og.term, 2500, seed=40 + k)
        batch = synth.merge_batches(synth.random_batch(g, 2500, seed=50 + k), f, seed=60 + k)
        _same(a, b, batch, f"follower n={nmax} step {k}")
        now = a.og.groups()


def test_small_step_multinode_cycle(monkeypatch):
    """The BASELINE configs[0] shape: 1,000 groups x 3, a proposal and two acks
    per group (3,000 messages: two tiles), several cycles."""
    G = 1000
    g, runs = synth.steady_groups(G, 3, seed=12, last_hi=1 << 20)
    a, b = _pairs(monkeypatch, lambda: Pair(g, runs, 3, 256, max_batch=G * 3 + 16))
    for step in range(3):
        _same(a, b, synth.cfg2_batch(g, step, seed=70 + step), f"cycle {step}")
        assert a.eng.stats()[abi.HB_STAT_COMMITS] == G
