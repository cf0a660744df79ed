"""GPU parity on the exact headline paths, at their real sizes.

bench.py's cfg2 line (BASELINE.json configs[1]) runs 1,048,576 groups x 3 at
W = 256: 256 buckets of 4,096 groups, i.e. the ONE-pass bucket sort, 1,024-group
k_route<2> workgroups and k_apply_fast<3> over 4,096 partitions.  Its cfg3 line
(configs[2]) runs 1,048,576 x 5 at W = 256 through k_route<8> and
k_apply_lead<5>.  The other large tests use 1.1M groups (two passes) or W = 8;
these pin the benchmarked geometry itself against the C oracle (16 shards on 16
cores): every event, statistic and group record of every step, plus live
inflight windows of sampled groups, whose ring words lie beyond 4 GB offsets
(ring[s][W][G] is 2 x 256 x 2^20 x 8 B = 4.3 GB below slot 2).
Reference: raft/raft.go:494-546 (stepLeader MsgProp / MsgAppResp),
raft/progress.go:172-237 (inflights).
"""
import numpy as np
import pytest

from etcd_amd import abi, synth

from .parity_util import Pair

pytestmark = pytest.mark.gpu

G_HEAD = 1 << 20


def _sample_windows(pair, now, rng, n, k=256):
    """Compare the live inflight windows of k random groups (every follower slot)."""
    seen = 0
    for gi in rng.integers(0, len(now), k):
        for s in range(1, n):
            p = now[gi]["pr"][s]
            if p["state"] == abi.HB_PR_REPLICATE and p["ins_count"]:
                start, vals = pair.eng.get_inflights(int(gi), s)
                assert start == p["ins_start"], f"g{gi}/s{s} start"
                assert np.array_equal(vals, pair.og.inflights(int(gi), s)), f"g{gi}/s{s} window"
                seen += 1
    return seen


@pytest.mark.timeout(900)
def test_cfg2_headline_geometry_full_size():
    """bench.py cfg2 at its size: the bench's own groups (seed 0x5EED0002) and
    global arrival stream (synth.global_ack_stream, one rank), two full steps
    (proposal + both acks per group: one commit each), then two steps where only
    follower 1 acks / nobody acks, so follower 2 holds a live window of 1 then 2
    entries (and follower 1 of 1) — sampled word by word."""
    n = 3
    g, runs = synth.steady_groups(G_HEAD, n, seed=0x5EED0002, with_runs="flat")
    gid, frm = synth.global_ack_stream(G_HEAD, n)
    slots = gid.astype(np.uint32)
    pair = Pair(g, runs, n, 256, max_batch=len(slots), oracle_shards=16)
    for step in range(2):
        b = synth.cfg2_local_batch(g, slots, frm, step)
        _, st, now = pair.step(b, ctx=f"headline step {step}", check_inflights=False)
        assert st[abi.HB_STAT_COMMITS] == G_HEAD and st[abi.HB_STAT_APPRESP] == 2 * G_HEAD
        assert st[abi.HB_STAT_FAULTS] == 0
        assert np.array_equal(now["committed"], g["last_index"] + np.uint64(step + 1))
    # step 3: only follower 1 acks (the newest index); step 4: proposals only
    one = frm == 1
    b = synth.cfg2_local_batch(g, slots[one], frm[one], 2)
    _, st, now = pair.step(b, ctx="headline step 2 (follower 1 only)", check_inflights=False)
    assert st[abi.HB_STAT_COMMITS] == G_HEAD
    b = dict(group=np.zeros(0, np.uint32), info=np.zeros(0, np.uint32), term=np.zeros(0, np.uint64),
             index=np.zeros(0, np.uint64), hint=None, props=np.ones(G_HEAD, np.uint32))
    _, st, now = pair.step(b, ctx="headline step 3 (proposals only)", check_inflights=False)
    assert st[abi.HB_STAT_COMMITS] == 0 and st[abi.HB_STAT_ENTRIES] == G_HEAD
    assert np.all(now["pr"][:, 2]["ins_count"] == 2) and np.all(now["pr"][:, 1]["ins_count"] == 1)
    assert _sample_windows(pair, now, np.random.default_rng(7), n) >= 400


@pytest.mark.timeout(900)
def test_cfg3_headline_geometry_full_size():
    """bench.py cfg3 at its size: 1,048,576 leaders x 5 at W = 256 (the bench's
    seed and open-loop generator: lagging / stale / rejecting acks, heartbeat
    responses, unreachable, 1-4 entries per group), three steps against the
    oracle, live windows of sampled groups compared word by word."""
    n = 5
    g, runs = synth.lagging_groups(G_HEAD, n, seed=0x5EED0003, W=256, with_runs="flat")
    pair = Pair(g, runs, n, 256, max_batch=2 * G_HEAD * n + G_HEAD, oracle_shards=16)
    rng = np.random.default_rng(0x5EED0003)
    now = pair.og.groups()
    for k in range(3):
        _, st, now = pair.step(synth.cfg3_open_batch(now, rng), ctx=f"cfg3 headline {k}", check_inflights=False)
        assert st[abi.HB_STAT_FAULTS] == 0 and st[abi.HB_STAT_APPRESP] > 3 * G_HEAD
    assert _sample_windows(pair, now, np.random.default_rng(8), n) >= 200


@pytest.mark.timeout(900)
def test_follow_workload_full_size():
    """bench.py --workload follow at its size: 1,048,576 groups x 3 that this
    node follows, each receiving its leader's MsgApp (one entry) and a
    MsgHeartbeat per step, through k_apply_fast's follower lane; two steps
    against the oracle (16 shards): every event, statistic and group record."""
    g, runs = synth.follow_groups(G_HEAD, 3, seed=0x5EED0006, with_runs="flat")
    pair = Pair(g, runs, 3, 256, max_batch=2 * G_HEAD, oracle_shards=16)
    for step in range(2):
        _, st, now = pair.step(synth.follow_batch(g, step), ctx=f"follow step {step}", check_inflights=False)
        assert st[abi.HB_STAT_COMMITS] == G_HEAD and st[abi.HB_STAT_ENTRIES] == G_HEAD
        assert st[abi.HB_STAT_MSGS] == 2 * G_HEAD and st[abi.HB_STAT_FAULTS] == 0
        assert np.array_equal(now["last_index"], g["last_index"] + np.uint64(step + 1))


@pytest.mark.timeout(900)
def test_mixed_workload_full_size():
    """bench.py --workload mixed at its size: 1,048,576 groups x 3, this node
    leading 1/3 (a proposal + both followers' MsgAppResp) and following 2/3 (its
    leader's MsgApp with one entry + MsgHeartbeat), all in ONE X-mode batch
    (raft/multinode.go:233-237: one Ready cycle steps both roles); two steps
    against the oracle (16 shards): every event, statistic and group record."""
    g, runs = synth.mixed_groups(G_HEAD, 3, seed=0x5EED0007, with_runs="flat")
    n_led = int((g["state"] == abi.HB_STATE_LEADER).sum())
    pair = Pair(g, runs, 3, 256, max_batch=2 * G_HEAD, oracle_shards=16)
    for step in range(2):
        b, _ = synth.mixed_batch(g, step, seed=0x5EED0007)
        _, st, now = pair.step(b, ctx=f"mixed step {step}", check_inflights=False)
        assert st[abi.HB_STAT_COMMITS] == G_HEAD and st[abi.HB_STAT_ENTRIES] == G_HEAD
        assert st[abi.HB_STAT_APPRESP] == 2 * n_led and st[abi.HB_STAT_FAULTS] == 0
        assert np.array_equal(now["last_index"], g["last_index"] + np.uint64(step + 1))


@pytest.mark.timeout(900)
def test_follow_workload_n5_full_size():
    """bench.py --workload follow --replicas 5 at its size: 1,048,576 followed
    groups x 5, MsgApp + MsgHeartbeat each per step, against the oracle."""
    g, runs = synth.follow_groups(G_HEAD, 5, seed=0x5EED0006, with_runs="flat")
    pair = Pair(g, runs, 5, 256, max_batch=2 * G_HEAD, oracle_shards=16)
    for step in range(2):
        _, st, now = pair.step(synth.follow_batch(g, step), ctx=f"follow n5 step {step}", check_inflights=False)
        assert st[abi.HB_STAT_COMMITS] == G_HEAD and st[abi.HB_STAT_MSGS] == 2 * G_HEAD
        assert st[abi.HB_STAT_FAULTS] == 0
