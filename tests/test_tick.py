"""Tick (MultiNode.Tick -> tickHeartbeat / tickElection, raft/raft.go:362-382,
isElectionTimeout :765-771) in the oracle, against the reference's own tests.

The reference draws r.rand.Int() from rand.New(rand.NewSource(id)); Go's
math/rand is not available here, so the stream is an input (as it is for the
engine, hb_set_rand) and the tests pin the algorithm with the reference's
draw-independent assertions plus exact timeouts for chosen draws."""
import numpy as np
import pytest

from etcd_amd import abi, synth
from oracle.pyoracle import OracleGroups, Raft

LEADER, FOLLOWER, CANDIDATE = abi.HB_STATE_LEADER, abi.HB_STATE_FOLLOWER, abi.HB_STATE_CANDIDATE
MSG_VOTE, MSG_HEARTBEAT = abi.HB_MSG_VOTE, abi.HB_MSG_HEARTBEAT
RNG_DRAWS = np.random.default_rng(7).integers(0, 1 << 63, 100_000, dtype=np.uint64)


def _msgs(r):
    return sorted((m.From, m.To, m.Term, m.Type) for m in r.readMessages())


def test_leader_bcast_beat():
    """TestLeaderBcastBeat raft/raft_paper_test.go:109-132."""
    hi = 1
    r = Raft(1, [1, 2, 3], election=10, heartbeat=hi, draws=RNG_DRAWS)
    r.becomeCandidate()
    r.becomeLeader()
    for _ in range(10):
        r.appendEntry(1)
    for _ in range(hi):
        r.tick()
    assert _msgs(r) == [(1, 2, 1, MSG_HEARTBEAT), (1, 3, 1, MSG_HEARTBEAT)]


@pytest.mark.parametrize("hi", [2, 3, 5])
def test_leader_beats_every_heartbeat_tick(hi):
    r = Raft(1, [1, 2, 3], election=10, heartbeat=hi, draws=RNG_DRAWS)
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    for k in range(1, 4 * hi + 1):
        r.tick()
        beats = [m for m in _msgs(r) if m[3] == MSG_HEARTBEAT]
        assert len(beats) == (2 if k % hi == 0 else 0), k
        assert r.elapsed == k % hi


@pytest.mark.parametrize("state", [FOLLOWER, CANDIDATE])
def test_nonleader_start_election(state):
    """testNonleaderStartElection raft/raft_paper_test.go:134-190: 2*et ticks
    always time out, whatever the draws."""
    et = 10
    for seed in range(5):
        draws = np.random.default_rng(seed).integers(0, 1 << 63, 64, dtype=np.uint64)
        r = Raft(1, [1, 2, 3], election=et, heartbeat=1, draws=draws)
        if state == FOLLOWER:
            r.becomeFollower(1, 2)
        else:
            r.becomeCandidate()
        for _ in range(2 * et):
            r.tick()
        assert r.Term == 2 and r.state == CANDIDATE
        assert _msgs(r) == [(1, 2, 2, MSG_VOTE), (1, 3, 2, MSG_VOTE)]


@pytest.mark.parametrize("state", [FOLLOWER, CANDIDATE])
def test_election_timeout_randomized(state):
    """testNonleaderElectionTimeoutRandomized raft/raft_paper_test.go:310-333:
    every timeout in (et, 2et) occurs; and each one is exactly the first tick
    t >= et with t - et > draw % et (one draw per tick from t = et)."""
    et = 10
    r = Raft(1, [1, 2, 3], election=et, heartbeat=1, draws=RNG_DRAWS)
    timeouts = set()
    pos = 0
    for _ in range(50 * et):
        if state == FOLLOWER:
            r.becomeFollower(r.Term + 1, 2)
        else:
            r.becomeCandidate()
        r.readMessages()
        time = 0
        while not r.readMessages():
            r.tick()
            time += 1
        want = et
        while not (want - et > int(RNG_DRAWS[pos]) % et):
            pos += 1
            want += 1
        pos += 1
        assert time == want
        timeouts.add(time)
    for d in range(et + 1, 2 * et):
        assert d in timeouts, d
    assert r.r.rand_pos == pos


def test_not_promotable_never_campaigns():
    """tickElection :363-366: a node outside prs keeps elapsed at 0."""
    r = Raft(4, [1, 2, 3], election=3, heartbeat=1, draws=RNG_DRAWS)
    for _ in range(20):
        r.tick()
        assert r.elapsed == 0
    assert r.state == FOLLOWER and not r.readMessages() and r.r.rand_pos == 0


def test_single_node_tick_wins():
    """A one-node group times out, campaigns and becomes leader in one tick."""
    r = Raft(1, [1], election=2, heartbeat=1, draws=np.array([0, 0, 0], np.uint64))
    r.tick()
    r.tick()  # d = 0: draw 0 % 2 = 0, not > 0
    assert r.state == FOLLOWER
    r.tick()  # d = 1 > 0
    assert r.state == LEADER and r.Term == 1 and r.committed == 1


def test_tick_batch_matches_per_group_ticks():
    """orc_tick_batch (MultiNode.Tick over every group) = each group's tick."""
    G = 300
    g, runs, ins = synth.random_groups(G, 5, seed=3, W=8)
    og = OracleGroups(g, runs, 8, inflights=ins)
    t = synth.random_timers(G, seed=4)
    og.load_timers(t)
    draws = RNG_DRAWS[:2000]
    total_msgs = 0
    for k in range(30):
        ev, st = og.tick(draws)
        total_msgs += int(st[abi.HB_STAT_MSGS])
        assert st[abi.HB_STAT_FAULTS] == 0
    now = og.timers()
    assert total_msgs > 0
    assert (now["rand_pos"] >= t["rand_pos"]).all()


def test_tick_draws_exhausted_faults():
    G = 4
    g, runs = synth.election_groups(G, 3, seed=1)
    og = OracleGroups(g, runs, 8)
    t = np.zeros(G, abi.TIMER_DTYPE)
    t["election_tick"], t["heartbeat_tick"], t["elapsed"] = 2, 1, 5
    t["rand_pos"] = [0, 1, 2, 3]
    og.load_timers(t)
    ev, st = og.tick(np.array([5, 5], np.uint64))
    assert st[abi.HB_STAT_FAULTS] == 2
    f = og.groups()["fault"]
    assert list(f) == [0, 0, abi.HB_FAULT_RAND_EXHAUSTED, abi.HB_FAULT_RAND_EXHAUSTED]
    assert (ev[ev["type"] == abi.HB_EV_FAULT]["x"] == abi.HB_NO_INDEX).all()
