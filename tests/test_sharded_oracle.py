"""CPU: the sharded oracle (the full-size GPU parity tests' checker) equals the
single oracle over the same batches — events (global group ids and arrival
positions), statistics, group records and inflight windows."""
import numpy as np
import pytest

from etcd_amd import abi, synth
from oracle.pyoracle import OracleGroups, ShardedOracleGroups

from .parity_util import assert_events_equal, assert_groups_equal


@pytest.mark.parametrize("shards", [3, 7])
def test_sharded_storm_equals_single(shards):
    g, runs = synth.election_groups(3001, 7, seed=71, with_runs="flat")
    a, b = OracleGroups(g, runs, 8), ShardedOracleGroups(g, runs, 8, shards=shards)
    bt = synth.cfg4_storm_batch(g, seed=72)
    for k in range(2):
        bb = dict(bt, term=synth.storm_terms(bt["term"], k))
        ea, sa = a.step(bb)
        eb, sb = b.step(bb)
        assert_events_equal(eb, ea, f"storm {k}")
        assert np.array_equal(sa, sb)
        assert_groups_equal(b.groups(), a.groups(), f"storm {k}")


def test_sharded_cfg3_stream_equals_single():
    g, runs = synth.lagging_groups(2500, 5, seed=3, W=8, with_runs="flat")
    a, b = OracleGroups(g, runs, 8), ShardedOracleGroups(g, runs, 8, shards=4)
    rng = np.random.default_rng(1)
    now = a.groups()
    for k in range(3):
        bt = synth.cfg3_open_batch(now, rng)
        ea, sa = a.step(bt)
        eb, sb = b.step(bt)
        assert_events_equal(eb, ea, f"cfg3 {k}")
        assert np.array_equal(sa, sb)
        now = a.groups()
        assert_groups_equal(b.groups(), now, f"cfg3 {k}")
        assert np.array_equal(b.log_info(), a.log_info())
        for gi in range(0, 2500, 61):
            for s in range(5):
                assert np.array_equal(a.inflights(gi, s), b.inflights(gi, s))


def test_sharded_maps_proposal_arrivals_back():
    """MsgProp drops / forwards carry the arrival position: global after the merge."""
    g, runs, _ = synth.random_groups(800, 5, seed=9, W=8)
    a, b = OracleGroups(g, runs, 8), ShardedOracleGroups(g, runs, 8, shards=5)
    bt = synth.random_batch(g, 4000, seed=10)
    ea, sa = a.step(bt)
    eb, sb = b.step(bt)
    assert_events_equal(eb, ea, "fuzz")
    assert np.array_equal(sa, sb)
    assert np.any(np.isin(ea["type"], [abi.HB_EV_PROP_FWD, abi.HB_EV_PROP_DROP]))


def test_sharded_oracle_follower_batches_equal_one_oracle():
    """The sharded oracle re-bases each message's entries per shard and maps
    the follower side's arrival-indexed events (HB_EV_FOLLOW) back: on the
    follow workload and on random follower-side traffic it equals one oracle
    over the whole batch."""
    from etcd_amd import synth
    from oracle.pyoracle import OracleGroups, ShardedOracleGroups
    G = 3000
    g, runs = synth.follow_groups(G, 3, seed=5, last_hi=1 << 12)
    one = OracleGroups(g, runs, 256)
    many = ShardedOracleGroups(g, runs, 256, shards=7)
    for step in range(2):
        b = synth.follow_batch(g, step, seed=6, ents=2)
        e1, s1 = one.step(b)
        e2, s2 = many.step(b)
        o1, o2 = np.argsort(e1["group"], kind="stable"), np.argsort(e2["group"], kind="stable")
        assert np.array_equal(e1[o1], e2[o2]) and np.array_equal(s1, s2)
        assert s1[abi.HB_STAT_COMMITS] == G and s1[abi.HB_STAT_ENTRIES] == 2 * G
    f = synth.follower_messages(one.groups(), one.term, 4000, seed=8)
    e1, s1 = one.step(f)
    e2, s2 = many.step(f)
    o1, o2 = np.argsort(e1["group"], kind="stable"), np.argsort(e2["group"], kind="stable")
    assert np.array_equal(e1[o1], e2[o2]) and np.array_equal(s1, s2)
    assert np.array_equal(one.groups(), many.groups())
