"""Known-answer tests that pin the C parity oracle to the reference.

Each test transcribes one of the reference's own Go tests (file:line cited) onto
the oracle (oracle/raft_oracle.c).  The Go toolchain is absent from this image,
so these tables ARE the oracle's pin (DESIGN.md "Parity").  Substitutions are
named where a test drives a follower-side path the engine does not cover.
"""
import numpy as np
import pytest

from etcd_amd import abi
from oracle.pyoracle import Inflights, Msg, Progress, Raft

P, R, S = abi.HB_PR_PROBE, abi.HB_PR_REPLICATE, abi.HB_PR_SNAPSHOT
F, Cd, L = abi.HB_STATE_FOLLOWER, abi.HB_STATE_CANDIDATE, abi.HB_STATE_LEADER
None_ = 0


# ---------------------------------------------------------------- inflights
def test_inflights_add():  # raft/progress_test.go:22-94
    inf = Inflights(10)
    for i in range(5):
        inf.add(i)
    assert inf.as_tuple() == (0, 5, 10, [0, 1, 2, 3, 4, 0, 0, 0, 0, 0])
    for i in range(5, 10):
        inf.add(i)
    assert inf.as_tuple() == (0, 10, 10, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9])
    in2 = Inflights(10, start=5)
    for i in range(5):
        in2.add(i)
    assert in2.as_tuple() == (5, 5, 10, [0, 0, 0, 0, 0, 0, 1, 2, 3, 4])
    for i in range(5, 10):
        in2.add(i)
    assert in2.as_tuple() == (5, 10, 10, [5, 6, 7, 8, 9, 0, 1, 2, 3, 4])
    with pytest.raises(RuntimeError):  # add panics when full (raft/progress.go:192-194)
        in2.add(10)


def test_inflight_free_to():  # raft/progress_test.go:96-167
    inf = Inflights(10)
    for i in range(10):
        inf.add(i)
    inf.freeTo(4)
    assert inf.as_tuple() == (5, 5, 10, list(range(10)))
    inf.freeTo(8)
    assert inf.as_tuple() == (9, 1, 10, list(range(10)))
    for i in range(10, 15):
        inf.add(i)
    inf.freeTo(12)
    assert inf.as_tuple() == (3, 2, 10, [10, 11, 12, 13, 14, 5, 6, 7, 8, 9])
    inf.freeTo(14)
    assert inf.as_tuple() == (5, 0, 10, [10, 11, 12, 13, 14, 5, 6, 7, 8, 9])


def test_inflight_free_first_one():  # raft/progress_test.go:169-189
    inf = Inflights(10)
    for i in range(10):
        inf.add(i)
    inf.freeFirstOne()
    assert inf.as_tuple() == (1, 9, 10, list(range(10)))


# ---------------------------------------------------------------- Progress
@pytest.mark.parametrize("p,wnext", [  # raft/raft_test.go:51-83
    (dict(State=R, Match=1, Next=5), 2),
    (dict(State=S, Match=1, Next=5, PendingSnapshot=10), 11),
    (dict(State=S, Match=1, Next=5, PendingSnapshot=0), 2),
])
def test_progress_become_probe(p, wnext):
    pr = Progress(**p)
    pr.becomeProbe()
    assert (pr.State, pr.Match, pr.Next) == (P, 1, wnext)


def test_progress_become_replicate():  # raft/raft_test.go:85-99
    pr = Progress(State=P, Match=1, Next=5)
    pr.becomeReplicate()
    assert (pr.State, pr.Match, pr.Next) == (R, 1, 2)


def test_progress_become_snapshot():  # raft/raft_test.go:101-115
    pr = Progress(State=P, Match=1, Next=5)
    pr.becomeSnapshot(10)
    assert (pr.State, pr.Match, pr.PendingSnapshot) == (S, 1, 10)


@pytest.mark.parametrize("update,wm,wn,wok", [  # raft/raft_test.go:117-148
    (2, 3, 5, False), (3, 3, 5, False), (4, 4, 5, True), (5, 5, 6, True)])
def test_progress_update(update, wm, wn, wok):
    pr = Progress(Match=3, Next=5)
    assert pr.maybeUpdate(update) == wok
    assert (pr.Match, pr.Next) == (wm, wn)


@pytest.mark.parametrize("state,m,n,rejected,last,w,wn", [  # raft/raft_test.go:150-212
    (R, 5, 10, 5, 5, False, 10), (R, 5, 10, 4, 4, False, 10), (R, 5, 10, 9, 9, True, 6),
    (P, 0, 0, 0, 0, False, 0), (P, 0, 10, 5, 5, False, 10), (P, 0, 10, 9, 9, True, 9),
    (P, 0, 2, 1, 1, True, 1), (P, 0, 1, 0, 0, True, 1), (P, 0, 10, 9, 2, True, 3),
    (P, 0, 10, 9, 0, True, 1)])
def test_progress_maybe_decr(state, m, n, rejected, last, w, wn):
    pr = Progress(State=state, Match=m, Next=n)
    assert pr.maybeDecrTo(rejected, last) == w
    assert (pr.Match, pr.Next) == (m, wn)


@pytest.mark.parametrize("state,paused,w", [  # raft/raft_test.go:214-238
    (P, False, False), (P, True, True), (R, False, False), (R, True, False),
    (S, False, True), (S, True, True)])
def test_progress_is_paused(state, paused, w):
    assert Progress(State=state, Paused=paused).isPaused() == w


def test_progress_resume():  # raft/raft_test.go:240-261
    pr = Progress(Next=2, Paused=True)
    pr.maybeDecrTo(1, 1)
    assert not pr.Paused
    pr.p.Paused = 1
    pr.maybeUpdate(2)
    assert not pr.Paused


def test_progress_resume_by_heartbeat():  # raft/raft_test.go:264-275
    r = Raft(1, [1, 2])
    r.becomeCandidate()
    r.becomeLeader()
    r.pr(2).Paused = 1
    r.Step(Msg(abi.HB_MSG_BEAT, From=1, To=1))
    assert r.pr(2).Paused == 0


def test_progress_paused():  # raft/raft_test.go:277-288
    r = Raft(1, [1, 2])
    r.becomeCandidate()
    r.becomeLeader()
    for _ in range(3):
        r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
    assert len(r.readMessages()) == 1


# ---------------------------------------------------------------- commit
COMMIT_TABLE = [  # raft/raft_test.go:706-748 (matches, log terms, smTerm, w)
    ([1], [1], 1, 1), ([1], [1], 2, 0), ([2], [1, 2], 2, 2), ([1], [2], 2, 1),
    ([2, 1, 1], [1, 2], 1, 1), ([2, 1, 1], [1, 1], 2, 0), ([2, 1, 2], [1, 2], 2, 2),
    ([2, 1, 2], [1, 1], 2, 0),
    ([2, 1, 1, 1], [1, 2], 1, 1), ([2, 1, 1, 1], [1, 1], 2, 0), ([2, 1, 1, 2], [1, 2], 1, 1),
    ([2, 1, 1, 2], [1, 1], 2, 0), ([2, 1, 2, 2], [1, 2], 2, 2), ([2, 1, 2, 2], [1, 1], 2, 0),
]


@pytest.mark.parametrize("matches,terms,smterm,w", COMMIT_TABLE)
def test_commit(matches, terms, smterm, w):
    sm = Raft(1, [1], ents=[(i + 1, t) for i, t in enumerate(terms)], hard=(smterm, 0, 0))
    for j, m in enumerate(matches):
        sm.setProgress(j + 1, m, m + 1)
    sm.maybeCommit()
    assert sm.committed == w


def test_commit_to():  # raft/log_test.go:399-429
    for commit, wcommit, wpanic in [(3, 3, False), (1, 2, False), (4, 0, True)]:
        r = Raft(1, [1], ents=[(1, 1), (2, 2), (3, 3)])
        r.r.log.committed = 2
        r.commitTo(commit)
        if wpanic:
            assert r.fault == abi.HB_FAULT_COMMIT_RANGE
        else:
            assert r.committed == wcommit and r.fault == 0


def test_term():  # raft/log_test.go:629-658
    offset, num = 100, 100
    r = Raft(1, [1], snapshot=(offset, 1), ents=[(offset + i, i) for i in range(1, num)])
    for index, w in [(offset - 1, 0), (offset, 1), (offset + num // 2, num // 2),
                     (offset + num - 1, num - 1), (offset + num, 0)]:
        assert r.term(index) == w


def test_term_with_unstable_snapshot():  # raft/log_test.go:660-688
    storagesnapi, unstablesnapi = 100, 105
    r = Raft(1, [1], snapshot=(unstablesnapi, 1))  # restore() -> firstIndex = 106
    for index, w in [(storagesnapi, 0), (storagesnapi + 1, 0), (unstablesnapi - 1, 0),
                     (unstablesnapi, 1)]:
        assert r.term(index) == w


# ---------------------------------------------------------------- leader responses
@pytest.mark.parametrize("index,reject,wmatch,wnext,wmsgnum,windex,wcommitted", [
    (3, True, 0, 3, 0, 0, 0), (2, True, 0, 2, 1, 1, 0), (2, False, 2, 4, 2, 2, 2),
    (0, False, 0, 3, 0, 0, 0)])
def test_leader_app_resp(index, reject, wmatch, wnext, wmsgnum, windex, wcommitted):
    # raft/raft_test.go:1175-1229 — log {1: term 0, 2: term 1}; becomes leader at term 1
    sm = Raft(1, [1, 2, 3], ents=[(1, 0), (2, 1)])
    sm.becomeCandidate()
    sm.becomeLeader()
    sm.readMessages()
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=2, Index=index, Term=sm.Term, Reject=reject, RejectHint=index))
    p = sm.pr(2)
    assert (p.Match, p.Next) == (wmatch, wnext)
    msgs = sm.readMessages()
    assert len(msgs) == wmsgnum
    for m in msgs:
        assert (m.Index, m.Commit) == (windex, wcommitted)


def test_msg_app_resp_wait_reset():  # raft/raft_test.go:944-1002
    sm = Raft(1, [1, 2, 3])
    sm.becomeCandidate()
    sm.becomeLeader()
    sm.bcastAppend()
    sm.readMessages()
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=2, Index=1))
    assert sm.Commit == 1
    sm.readMessages()
    sm.Step(Msg(abi.HB_MSG_PROP, From=1, Entries=1))
    msgs = sm.readMessages()
    assert len(msgs) == 1
    assert (msgs[0].Type, msgs[0].To, msgs[0].nents, msgs[0].ent_lo) == (abi.HB_MSG_APP, 2, 1, 2)
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=3, Index=1))
    msgs = sm.readMessages()
    assert len(msgs) == 1
    assert (msgs[0].Type, msgs[0].To, msgs[0].nents, msgs[0].ent_lo) == (abi.HB_MSG_APP, 3, 1, 2)


def test_handle_heartbeat_resp():  # raft/raft_test.go:883-940
    sm = Raft(1, [1, 2], ents=[(1, 1), (2, 2), (3, 3)])
    sm.becomeCandidate()
    sm.becomeLeader()
    sm.commitTo(sm.lastIndex)
    sm.Step(Msg(abi.HB_MSG_HEARTBEAT_RESP, From=2))
    msgs = sm.readMessages()
    assert [m.Type for m in msgs] == [abi.HB_MSG_APP]
    sm.Step(Msg(abi.HB_MSG_HEARTBEAT_RESP, From=2))
    assert sm.readMessages() == []
    sm.bcastHeartbeat()
    sm.Step(Msg(abi.HB_MSG_HEARTBEAT_RESP, From=2))
    msgs = sm.readMessages()
    assert [m.Type for m in msgs] == [abi.HB_MSG_HEARTBEAT, abi.HB_MSG_APP]
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=2, Index=msgs[1].Index + msgs[1].nents))
    sm.readMessages()
    sm.bcastHeartbeat()
    sm.Step(Msg(abi.HB_MSG_HEARTBEAT_RESP, From=2))
    msgs = sm.readMessages()
    assert [m.Type for m in msgs] == [abi.HB_MSG_HEARTBEAT]


def test_recv_msg_unreachable():  # raft/raft_test.go:1442-1463
    r = Raft(1, [1, 2], ents=[(1, 1), (2, 1), (3, 1)])
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    p = r.pr(2)
    p.Match = 3
    # becomeReplicate + optimisticUpdate(5)
    p.State, p.Next = R, 4
    p.Next = 6
    r.Step(Msg(abi.HB_MSG_UNREACHABLE, From=2, To=1))
    assert (r.pr(2).State, r.pr(2).Next) == (P, r.pr(2).Match + 1)


@pytest.mark.parametrize("state,nxt,wnext", [(R, 2, 3 + 1 + 1 + 1), (P, 2, 2)])
def test_leader_increase_next(state, nxt, wnext):  # raft/raft_test.go:1330-1360
    sm = Raft(1, [1, 2], ents=[(1, 1), (2, 1), (3, 1)])
    sm.becomeCandidate()
    sm.becomeLeader()
    sm.pr(2).State = state
    sm.pr(2).Next = nxt
    sm.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
    assert sm.pr(2).Next == wnext


def test_send_append_for_progress_probe():  # raft/raft_test.go:1362-1403
    r = Raft(1, [1, 2])
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    p = r.pr(2)
    p.State, p.Next = P, p.Match + 1  # becomeProbe
    for _ in range(3):
        r.appendEntry()
        r.sendAppend(2)
        msg = r.readMessages()
        assert len(msg) == 1 and msg[0].Index == 0
        assert r.pr(2).Paused == 1
        for _ in range(10):
            r.appendEntry()
            r.sendAppend(2)
            assert len(r.readMessages()) == 0
        r.Step(Msg(abi.HB_MSG_BEAT, From=1, To=1))  # heartbeatTimeout = 1
        msg = r.readMessages()
        assert len(msg) == 1 and msg[0].Type == abi.HB_MSG_HEARTBEAT


def test_send_append_for_progress_replicate():  # raft/raft_test.go:1405-1420
    r = Raft(1, [1, 2])
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    p = r.pr(2)
    p.State, p.Next = R, p.Match + 1
    for _ in range(10):
        r.appendEntry()
        r.sendAppend(2)
        assert len(r.readMessages()) == 1


def test_send_append_for_progress_snapshot():  # raft/raft_test.go:1422-1440
    r = Raft(1, [1, 2])
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    p = r.pr(2)
    p.State, p.PendingSnapshot = S, 10
    for _ in range(10):
        r.appendEntry()
        r.sendAppend(2)
        assert len(r.readMessages()) == 0


def test_bcast_beat():  # raft/raft_test.go:1231-1284
    offset = 1000
    sm = Raft(1, [1, 2, 3], snapshot=(offset, 1))
    sm.Term = 1
    sm.becomeCandidate()
    sm.becomeLeader()
    for _ in range(10):
        sm.appendEntry()
    sm.pr(2).Match, sm.pr(2).Next = 5, 6
    sm.pr(3).Match, sm.pr(3).Next = sm.lastIndex, sm.lastIndex + 1
    sm.Step(Msg(abi.HB_MSG_BEAT))
    msgs = sm.readMessages()
    assert len(msgs) == 2
    want = {2: min(sm.committed, 5), 3: min(sm.committed, sm.lastIndex)}
    for m in msgs:
        assert m.Type == abi.HB_MSG_HEARTBEAT and m.Index == 0 and m.LogTerm == 0 and m.nents == 0
        assert m.Commit == want.pop(m.To)


@pytest.mark.parametrize("state,wmsg", [(L, 2), (Cd, 0), (F, 0)])
def test_recv_msg_beat(state, wmsg):  # raft/raft_test.go:1286-1328
    sm = Raft(1, [1, 2, 3], ents=[(1, 0), (2, 1)])
    sm.Term = 1
    sm.r.state = state
    sm.Step(Msg(abi.HB_MSG_BEAT, From=1, To=1))
    msgs = sm.readMessages()
    assert len(msgs) == wmsg
    assert all(m.Type == abi.HB_MSG_HEARTBEAT for m in msgs)


# ---------------------------------------------------------------- flow control
def _leader_with_replicating_2(max_inflight=256):
    r = Raft(1, [1, 2], max_inflight=max_inflight)
    r.becomeCandidate()
    r.becomeLeader()
    p = r.pr(2)
    p.State, p.Next = R, p.Match + 1  # pr2.becomeReplicate()
    return r


def test_msg_app_flow_control_full():  # raft/raft_flow_control_test.go:26-56
    r = _leader_with_replicating_2()
    for i in range(256):
        r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
        assert len(r.readMessages()) == 1
    assert r.pr(2).ins.count == 256
    for i in range(10):
        r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
        assert len(r.readMessages()) == 0


def test_msg_app_flow_control_move_forward():  # raft/raft_flow_control_test.go:62-101
    r = _leader_with_replicating_2()
    for i in range(256):
        r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
        r.readMessages()
    for tt in range(2, 256):
        r.Step(Msg(abi.HB_MSG_APP_RESP, From=2, To=1, Index=tt))
        r.readMessages()
        r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
        assert len(r.readMessages()) == 1
        assert r.pr(2).ins.count == r.pr(2).ins.size
        for i in range(tt):
            r.Step(Msg(abi.HB_MSG_APP_RESP, From=2, To=1, Index=i))
            assert r.pr(2).ins.count == r.pr(2).ins.size


def test_msg_app_flow_control_recv_heartbeat():  # raft/raft_flow_control_test.go:105-155
    r = _leader_with_replicating_2()
    for i in range(256):
        r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
        r.readMessages()
    for tt in range(1, 5):
        assert r.pr(2).ins.count == 256
        for i in range(tt):
            r.Step(Msg(abi.HB_MSG_HEARTBEAT_RESP, From=2, To=1))
            r.readMessages()
            assert r.pr(2).ins.count < 256
        r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
        assert len(r.readMessages()) == 1
        for i in range(10):
            r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
            assert len(r.readMessages()) == 0
        r.Step(Msg(abi.HB_MSG_HEARTBEAT_RESP, From=2, To=1))
        r.readMessages()


# ---------------------------------------------------------------- snapshots
def _snap_leader(peers):
    # newTestRaft(1, peers) + restore(testingSnap{Index 11, Term 11, Nodes [1 2]})
    sm = Raft(1, [1, 2], snapshot=(11, 11))
    sm.becomeCandidate()
    sm.becomeLeader()
    return sm


def test_sending_snapshot_set_pending_snapshot():  # raft/raft_snap_test.go:33-49
    sm = _snap_leader([1])
    sm.pr(2).Next = sm.firstIndex
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=2, To=1, Index=sm.pr(2).Next - 1, Reject=True))
    assert sm.pr(2).PendingSnapshot == 11


def test_pending_snapshot_pause_replication():  # raft/raft_snap_test.go:51-66
    sm = _snap_leader([1, 2])
    p = sm.pr(2)
    p.State, p.PendingSnapshot = S, 11
    sm.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
    assert len(sm.readMessages()) == 0


def test_snapshot_failure():  # raft/raft_snap_test.go:68-89
    sm = _snap_leader([1, 2])
    p = sm.pr(2)
    p.Next = 1
    p.State, p.PendingSnapshot = S, 11
    sm.Step(Msg(abi.HB_MSG_SNAP_STATUS, From=2, To=1, Reject=True))
    p = sm.pr(2)
    assert (p.PendingSnapshot, p.Next, p.Paused) == (0, 1, 1)


def test_snapshot_succeed():  # raft/raft_snap_test.go:91-112
    sm = _snap_leader([1, 2])
    p = sm.pr(2)
    p.Next = 1
    p.State, p.PendingSnapshot = S, 11
    sm.Step(Msg(abi.HB_MSG_SNAP_STATUS, From=2, To=1, Reject=False))
    p = sm.pr(2)
    assert (p.PendingSnapshot, p.Next, p.Paused) == (0, 12, 1)


def test_snapshot_abort():  # raft/raft_snap_test.go:114-134
    sm = _snap_leader([1, 2])
    p = sm.pr(2)
    p.Next = 1
    p.State, p.PendingSnapshot = S, 11
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=2, To=1, Index=11))
    p = sm.pr(2)
    assert (p.PendingSnapshot, p.Next) == (0, 12)


# ---------------------------------------------------------------- elections / terms
ELECTION_TABLE = [  # raft/raft_paper_test.go:192-232
    (1, {}, L), (3, {2: True, 3: True}, L), (3, {2: True}, L),
    (5, {2: True, 3: True, 4: True, 5: True}, L), (5, {2: True, 3: True, 4: True}, L),
    (5, {2: True, 3: True}, L),
    (3, {2: False, 3: False}, F), (5, {2: False, 3: False, 4: False, 5: False}, F),
    (5, {2: True, 3: False, 4: False, 5: False}, F),
    (3, {}, Cd), (5, {2: True}, Cd), (5, {2: False, 3: False}, Cd), (5, {}, Cd),
]


@pytest.mark.parametrize("size,votes,state", ELECTION_TABLE)
def test_leader_election_in_one_round_rpc(size, votes, state):
    r = Raft(1, list(range(1, size + 1)))
    r.Step(Msg(abi.HB_MSG_HUP, From=1, To=1))
    for id_, vote in votes.items():
        r.Step(Msg(abi.HB_MSG_VOTE_RESP, From=id_, To=1, Reject=not vote))
    assert r.state == state
    assert r.Term == 1


def _commit_noop_entry(r):  # raft/raft_paper_test.go:907-925
    r.bcastAppend()
    for m in r.readMessages():
        assert m.Type == abi.HB_MSG_APP and m.nents == 1
        r.Step(Msg(abi.HB_MSG_APP_RESP, From=m.To, To=m.From, Term=m.Term, Index=m.Index + m.nents))
    r.readMessages()


def test_leader_commit_entry():  # raft/raft_paper_test.go:436-469
    r = Raft(1, [1, 2, 3])
    r.becomeCandidate()
    r.becomeLeader()
    _commit_noop_entry(r)
    li = r.lastIndex
    r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
    for m in r.readMessages():
        r.Step(Msg(abi.HB_MSG_APP_RESP, From=m.To, To=m.From, Term=m.Term, Index=m.Index + m.nents))
    assert r.committed == li + 1
    msgs = sorted(r.readMessages(), key=lambda m: m.To)
    for i, m in enumerate(msgs):
        assert (m.To, m.Type, m.Commit) == (i + 2, abi.HB_MSG_APP, li + 1)


@pytest.mark.parametrize("size,acceptors,wack", [  # raft/raft_paper_test.go:474-509
    (1, {}, True), (3, {}, False), (3, {2}, True), (3, {2, 3}, True), (5, {}, False),
    (5, {2}, False), (5, {2, 3}, True), (5, {2, 3, 4}, True), (5, {2, 3, 4, 5}, True)])
def test_leader_acknowledge_commit(size, acceptors, wack):
    r = Raft(1, list(range(1, size + 1)))
    r.becomeCandidate()
    r.becomeLeader()
    _commit_noop_entry(r)
    li = r.lastIndex
    r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
    for m in r.readMessages():
        if m.To in acceptors:
            r.Step(Msg(abi.HB_MSG_APP_RESP, From=m.To, To=m.From, Term=m.Term, Index=m.Index + m.nents))
    assert (r.committed > li) == wack


@pytest.mark.parametrize("index,wcommit", [(1, 0), (2, 0), (3, 3)])
def test_leader_only_commits_log_from_current_term(index, wcommit):  # raft/raft_paper_test.go:866-895
    r = Raft(1, [1, 2], ents=[(1, 1), (2, 2)], hard=(2, 0, 0))
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
    r.Step(Msg(abi.HB_MSG_APP_RESP, From=2, To=1, Term=r.Term, Index=index))
    assert r.committed == wcommit


@pytest.mark.parametrize("state", [F, Cd, L])
def test_update_term_from_message(state):  # raft/raft_paper_test.go:54-74
    # The Go test steps a MsgApp (follower-side handling, off the engine path);
    # the term gate (raft/raft.go:473-480) is type independent except for MsgVote,
    # so a MsgHeartbeatResp exercises the same transition.
    r = Raft(1, [1, 2, 3])
    if state == F:
        r.becomeFollower(1, 2)
    elif state == Cd:
        r.becomeCandidate()
    else:
        r.becomeCandidate()
        r.becomeLeader()
    r.Step(Msg(abi.HB_MSG_HEARTBEAT_RESP, From=2, Term=2))
    assert (r.Term, r.state, r.lead) == (2, F, 2)


def test_reject_stale_term_message():  # raft/raft_paper_test.go:80-94
    r = Raft(1, [1, 2, 3], hard=(2, 0, 0))
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    before = bytes(r.to_group())
    r.Step(Msg(abi.HB_MSG_APP_RESP, From=2, Term=r.Term - 1, Index=1))
    assert bytes(r.to_group()) == before
    assert r.readMessages() == []


STATE_TRANSITION = [  # raft/raft_test.go:1068-1119 (from, to, wallow, wterm, wlead)
    (F, F, True, 1, None_), (F, Cd, True, 1, None_), (F, L, False, 0, None_),
    (Cd, F, True, 0, None_), (Cd, Cd, True, 1, None_), (Cd, L, True, 0, 1),
    (L, F, True, 1, None_), (L, Cd, False, 1, None_), (L, L, True, 0, 1),
]


@pytest.mark.parametrize("frm,to,wallow,wterm,wlead", STATE_TRANSITION)
def test_state_transition(frm, to, wallow, wterm, wlead):
    sm = Raft(1, [1])
    sm.r.state = frm
    if to == F:
        sm.becomeFollower(wterm, wlead)
    elif to == Cd:
        sm.becomeCandidate()
    else:
        sm.becomeLeader()
    if not wallow:
        assert sm.fault != 0
        return
    assert sm.fault == 0
    assert (sm.Term, sm.lead) == (wterm, wlead)


@pytest.mark.parametrize("state,wstate,wterm,windex", [(F, F, 3, 0), (Cd, F, 3, 0), (L, F, 3, 1)])
def test_all_server_stepdown(state, wstate, wterm, windex):  # raft/raft_test.go:1121-1173
    # MsgApp is replaced by MsgAppResp (same term-gate behaviour, lead = From);
    # MsgVote keeps lead = None.
    for mtype, wlead in [(abi.HB_MSG_VOTE, None_), (abi.HB_MSG_APP_RESP, 2)]:
        sm = Raft(1, [1, 2, 3])
        if state == F:
            sm.becomeFollower(1, None_)
        elif state == Cd:
            sm.becomeCandidate()
        else:
            sm.becomeCandidate()
            sm.becomeLeader()
        sm.Step(Msg(mtype, From=2, Term=3, LogTerm=3))
        assert (sm.state, sm.Term, sm.lastIndex, sm.lead) == (wstate, wterm, windex, wlead)


def test_multinode_start_campaign_single():  # raft/multinode_test.go:246-300 (raft-level part)
    # CreateGroup on an empty log with peers [1]: becomeFollower(1, None), conf entry
    # at index 1 term 1 committed; Campaign -> leader at term 2, noop at 2, commit 2.
    r = Raft(1, [1], ents=[(1, 1)])
    r.becomeFollower(1, None_)
    r.r.log.committed = 1
    r.Step(Msg(abi.HB_MSG_HUP))
    assert (r.state, r.lead, r.Term, r.Vote, r.committed, r.lastIndex) == (L, 1, 2, 1, 2, 2)
    r.Step(Msg(abi.HB_MSG_PROP, From=1, Entries=1))
    assert (r.committed, r.lastIndex) == (3, 3)


# ---------------------------------------------------------------- MaxSizePerMsg (limitSize)
def test_limit_size():  # raft/util_test.go:49-75
    import ctypes as C
    from oracle.pyoracle import lib
    ents = [(4, 4), (5, 5), (6, 6)]  # pb.Entry{Index, Term}: Type 0, Data nil
    sz = [int(lib().orc_entry_size(abi.hb_ent_desc(0, 0, False), t, i)) for i, t in ents]
    assert sz == [6, 6, 6]
    tests = [
        (2 ** 64 - 1, 3),
        (0, 1),  # even if maxsize is zero, the first entry should be returned
        (sz[0] + sz[1], 2),  # limit to 2
        (sz[0] + sz[1] + sz[2] // 2, 2),  # limit to 2
        (sz[0] + sz[1] + sz[2] - 1, 2),
        (sz[0] + sz[1] + sz[2], 3),  # all
    ]
    arr = (C.c_uint64 * 3)(*sz)
    for maxsize, want in tests:
        assert lib().orc_limit_size(arr, 3, maxsize) == want, maxsize
    assert lib().orc_limit_size(arr, 0, 0) == 0


@pytest.mark.parametrize("term,index,data_len,etype,has_data", [
    (0, 0, 0, 0, False), (1, 1, 3, 0, True), (4, 4, 0, 0, True), (127, 128, 127, 0, True),
    (300, 70000, 200, 1, True), (2 ** 40, 2 ** 62, 1 << 20, 0, True), (2 ** 64 - 1, 2 ** 63, 0, 1, False)])
def test_entry_size_matches_gogo(term, index, data_len, etype, has_data):
    """Entry.Size() (raft/raftpb/raft.pb.go:1030-1043): 1 + sov(Type) + 1 + sov(Term)
    + 1 + sov(Index) + (Data != nil ? 1 + len + sov(len) : 0), from the oracle, the
    Python mirror and the host library (hbn_entry_size) alike."""
    from oracle.pyoracle import lib
    from etcd_amd.multinode import Entry, entry_size

    def sov(x):
        n = 1
        while x >= 0x80:
            x >>= 7
            n += 1
        return n
    want = 1 + sov(etype) + 1 + sov(term) + 1 + sov(index) + ((1 + data_len + sov(data_len)) if has_data else 0)
    d = abi.hb_ent_desc(data_len, etype, has_data)
    assert lib().orc_entry_size(d, term, index) == want
    assert abi.entry_size(d, term, index) == want
    assert entry_size(Entry(Term=term, Index=index, Type=etype, Data=(b"x" * data_len) if has_data else None)) == want


def test_send_append_cut_by_max_size_per_msg():
    """sendAppend's entries(pr.Next, r.maxMsgSize) (raft/raft.go:265) with a finite
    MaxSizePerMsg: limitSize keeps the first entry and then every entry while the
    running Entry.Size() sum stays <= maxSize; Replicate then records the last
    entry sent (optimisticUpdate + inflights.add, :271-273)."""
    for max_size, want in ((13, 2), (12, 2), (11, 1), (18, 3), (0, 1), (abi.HB_NO_LIMIT, 5)):
        r = Raft(1, [1, 2], ents=[(1, 1), (2, 1), (3, 1), (4, 1)], max_msg_size=max_size)
        if max_size not in (0, abi.HB_NO_LIMIT):
            r.load_sizes([6, 6, 6, 6])  # Entry{Term 1, Index i}.Size() = 6
        r.becomeCandidate()
        r.becomeLeader()  # noop at 5 (Term 2): Size 6
        r.readMessages()
        r.setProgress(2, 0, 1)
        r.pr(2).State = abi.HB_PR_REPLICATE  # becomeReplicate with Match 0: Next = 1
        r.sendAppend(2)
        ms = r.readMessages()
        assert len(ms) == 1 and ms[0].Type == abi.HB_MSG_APP and ms[0].Index == 0
        assert ms[0].nents == want, (max_size, ms[0].nents)
        assert r.pr(2).Next == want + 1 and r.fault == 0


def test_send_append_from_any_depth():
    """With a finite MaxSizePerMsg the engine's log index holds the size of
    every entry of the log (hb_load_entry_sizes + hb_reserve_log), so
    sendAppend cuts entries(Next, maxMsgSize) for a follower at any depth: here
    5,000 entries behind under etcdserver's 1 MiB limit (etcdserver/raft.go:229;
    raft/raft.go:265, raft/util.go:97-110)."""
    n = 6000
    ents = [(i + 1, 1) for i in range(n)]
    r = Raft(1, [1, 2], ents=ents, max_msg_size=1 << 20)
    rng = np.random.default_rng(5)
    data = rng.integers(0, 600, n)
    sizes = [abi.entry_size(abi.hb_ent_desc(int(d), 0, True), 1, i + 1) for i, d in enumerate(data)]
    r.load_sizes(sizes)
    r.becomeCandidate()
    r.becomeLeader()  # noop at n + 1 (Term 2)
    r.readMessages()
    allsz = sizes + [abi.entry_size(0, 2, n + 1)]
    for nxt in (n + 1 - 5000, 2, 1, n - 1):
        r.setProgress(2, nxt - 1, nxt)
        r.pr(2).State = abi.HB_PR_REPLICATE
        r.sendAppend(2)
        ms = r.readMessages()
        tot, k = allsz[nxt - 1], 1
        while nxt - 1 + k < len(allsz) and tot + allsz[nxt - 1 + k] <= (1 << 20):
            tot += allsz[nxt - 1 + k]
            k += 1
        assert r.fault == 0 and len(ms) == 1 and ms[0].Index == nxt - 1 and ms[0].nents == k, (nxt, ms)


def test_send_append_before_loaded_sizes_faults():
    """Engine precondition (not a reference panic): the engine computes
    limitSize from the sizes its caller loaded; a send that starts before them
    faults HB_FAULT_SIZE_WINDOW (oracle and engine alike).  libhbnode always
    loads the whole log, so MultiNode never sees it."""
    r = Raft(1, [1, 2], ents=[(1, 1), (2, 1), (3, 1), (4, 1)], max_msg_size=100)
    r.load_sizes([6, 6])  # only entries 3 and 4 are known: next - 1 >= 2 can be served
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    r.setProgress(2, 0, 3)
    r.sendAppend(2)
    assert r.fault == 0 and r.readMessages()[0].nents == 3
    r.setProgress(2, 0, 2)
    r.sendAppend(2)
    assert r.fault == abi.HB_FAULT_SIZE_WINDOW


# ---------------------------------------------------------------- follower side
APP, APPRESP, HB, HBRESP = abi.HB_MSG_APP, abi.HB_MSG_APP_RESP, abi.HB_MSG_HEARTBEAT, abi.HB_MSG_HEARTBEAT_RESP
VOTE, VOTERESP, SNAP = abi.HB_MSG_VOTE, abi.HB_MSG_VOTE_RESP, abi.HB_MSG_SNAP


def _log_with(ents):
    import ctypes as C
    from oracle.pyoracle import lib, orc_log
    lg = orc_log()
    lib().orc_log_init(C.byref(lg), 1, 0)
    for i, t in ents:
        assert i == lg.last_index + 1
        lib().orc_log_push(C.byref(lg), t, 1)
    return lg


@pytest.mark.parametrize("ents,wconflict", [  # raft/log_test.go:24-57 TestFindConflict
    ([], 0), ([], 0),
    ([(1, 1), (2, 2), (3, 3)], 0), ([(2, 2), (3, 3)], 0), ([(3, 3)], 0),
    ([(1, 1), (2, 2), (3, 3), (4, 4), (5, 4)], 4), ([(2, 2), (3, 3), (4, 4), (5, 4)], 4),
    ([(3, 3), (4, 4), (5, 4)], 4), ([(4, 4), (5, 4)], 4),
    ([(1, 4), (2, 4)], 1), ([(2, 1), (3, 4), (4, 4)], 2), ([(3, 1), (4, 2), (5, 4), (6, 4)], 3)])
def test_find_conflict(ents, wconflict):
    import ctypes as C
    from oracle.pyoracle import lib
    lg = _log_with([(1, 1), (2, 2), (3, 3)])
    terms = (C.c_uint64 * max(1, len(ents)))(*[t for _, t in ents])
    frm = ents[0][0] if ents else 1
    assert lib().orc_log_find_conflict(C.byref(lg), frm, terms, len(ents)) == wconflict


@pytest.mark.parametrize("lasti,term,want", [  # raft/log_test.go:59-88 TestIsUpToDate
    (2, 4, True), (3, 4, True), (4, 4, True), (2, 2, False), (3, 2, False), (4, 2, False),
    (2, 3, False), (3, 3, True), (4, 3, True)])
def test_is_up_to_date(lasti, term, want):
    import ctypes as C
    from oracle.pyoracle import lib
    lg = _log_with([(1, 1), (2, 2), (3, 3)])
    assert bool(lib().orc_log_is_up_to_date(C.byref(lg), lasti, term)) == want


LI, LT, CM = 3, 3, 1


@pytest.mark.parametrize("log_term,index,committed,ents,wlasti,wappend,wcommit,wpanic", [  # log_test.go:152-240
    (LT - 1, LI, LI, [(LI + 1, 4)], 0, False, CM, False),
    (LT, LI + 1, LI, [(LI + 2, 4)], 0, False, CM, False),
    (LT, LI, LI, [], LI, True, LI, False),
    (LT, LI, LI + 1, [], LI, True, LI, False),
    (LT, LI, LI - 1, [], LI, True, LI - 1, False),
    (LT, LI, 0, [], LI, True, CM, False),
    (0, 0, LI, [], 0, True, CM, False),
    (LT, LI, LI, [(LI + 1, 4)], LI + 1, True, LI, False),
    (LT, LI, LI + 1, [(LI + 1, 4)], LI + 1, True, LI + 1, False),
    (LT, LI, LI + 2, [(LI + 1, 4)], LI + 1, True, LI + 1, False),
    (LT, LI, LI + 2, [(LI + 1, 4), (LI + 2, 4)], LI + 2, True, LI + 2, False),
    (LT - 1, LI - 1, LI, [(LI, 4)], LI, True, LI, False),
    (LT - 2, LI - 2, LI, [(LI - 1, 4)], LI - 1, True, LI - 1, False),
    (LT - 3, LI - 3, LI, [(LI - 2, 4)], LI - 2, True, LI - 2, True),
    (LT - 2, LI - 2, LI, [(LI - 1, 4), (LI, 4)], LI, True, LI, False)])
def test_log_maybe_append(log_term, index, committed, ents, wlasti, wappend, wcommit, wpanic):
    import ctypes as C
    from oracle.pyoracle import lib
    lg = _log_with([(1, 1), (2, 2), (3, 3)])
    lg.committed = CM
    terms = (C.c_uint64 * max(1, len(ents)))(*[t for _, t in ents])
    lasti = C.c_uint64()
    rc = lib().orc_log_maybe_append(C.byref(lg), index, log_term, committed, terms, len(ents), C.byref(lasti))
    if wpanic:
        assert rc == -1
        return
    assert (rc == 1) == wappend and lasti.value == wlasti and lg.committed == wcommit
    if wappend and ents:
        assert [lib().orc_log_term(C.byref(lg), i) for i, _ in ents] == [t for _, t in ents]


@pytest.mark.parametrize("m,windex,wcommit,wreject", [  # raft/raft_test.go:803-850 TestHandleMsgApp
    (dict(Term=2, LogTerm=3, Index=2, Commit=3), 2, 0, True),
    (dict(Term=2, LogTerm=3, Index=3, Commit=3), 2, 0, True),
    (dict(Term=2, LogTerm=1, Index=1, Commit=1), 2, 1, False),
    (dict(Term=2, LogTerm=0, Index=0, Commit=1, Entries=[(1, 2)]), 1, 1, False),
    (dict(Term=2, LogTerm=2, Index=2, Commit=3, Entries=[(3, 2), (4, 2)]), 4, 3, False),
    (dict(Term=2, LogTerm=2, Index=2, Commit=4, Entries=[(3, 2)]), 3, 3, False),
    (dict(Term=2, LogTerm=1, Index=1, Commit=4, Entries=[(2, 2)]), 2, 2, False),
    (dict(Term=1, LogTerm=1, Index=1, Commit=3), 2, 1, False),
    (dict(Term=1, LogTerm=1, Index=1, Commit=3, Entries=[(2, 2)]), 2, 2, False),
    (dict(Term=2, LogTerm=2, Index=2, Commit=3), 2, 2, False),
    (dict(Term=2, LogTerm=2, Index=2, Commit=4), 2, 2, False)])
def test_handle_msg_app(m, windex, wcommit, wreject):
    sm = Raft(1, [1], ents=[(1, 1), (2, 2)])
    sm.becomeFollower(2, None_)
    sm.handleAppendEntries(Msg(APP, **m))
    assert sm.lastIndex == windex and sm.committed == wcommit
    ms = sm.readMessages()
    assert len(ms) == 1 and bool(ms[0].Reject) == wreject


@pytest.mark.parametrize("mcommit,wcommit", [(3, 3), (1, 2)])  # raft/raft_test.go:852-882 TestHandleHeartbeat
def test_handle_heartbeat(mcommit, wcommit):
    sm = Raft(1, [1, 2], ents=[(1, 1), (2, 2), (3, 3)], election=5)
    sm.becomeFollower(2, 2)
    sm.commitTo(2)
    sm.handleHeartbeat(Msg(APP, From=2, To=1, Term=2, Commit=mcommit))
    assert sm.committed == wcommit
    ms = sm.readMessages()
    assert len(ms) == 1 and ms[0].Type == HBRESP


@pytest.mark.parametrize("state,i,term,vote_for,wreject", [  # raft/raft_test.go:1004-1066 TestRecvMsgVote
    (F, 0, 0, None_, True), (F, 0, 1, None_, True), (F, 0, 2, None_, True), (F, 0, 3, None_, False),
    (F, 1, 0, None_, True), (F, 1, 1, None_, True), (F, 1, 2, None_, True), (F, 1, 3, None_, False),
    (F, 2, 0, None_, True), (F, 2, 1, None_, True), (F, 2, 2, None_, False), (F, 2, 3, None_, False),
    (F, 3, 0, None_, True), (F, 3, 1, None_, True), (F, 3, 2, None_, False), (F, 3, 3, None_, False),
    (F, 3, 2, 2, False), (F, 3, 2, 1, True),
    (L, 3, 3, 1, True), (Cd, 3, 3, 1, True)])
def test_recv_msg_vote(state, i, term, vote_for, wreject):
    sm = Raft(1, [1], ents=[(1, 2), (2, 2)])  # storage ents {}, 1/2, 2/2; unstable offset 3
    sm.r.state = state
    sm.r.Vote = vote_for
    sm.Step(Msg(VOTE, From=2, Index=i, LogTerm=term))
    ms = sm.readMessages()
    assert len(ms) == 1 and ms[0].Type == VOTERESP and bool(ms[0].Reject) == wreject


@pytest.mark.parametrize("ents,commit", [  # raft/raft_paper_test.go:547-590 TestFollowerCommitEntry
    ([(1, 1)], 1), ([(1, 1), (2, 1)], 2), ([(1, 1), (2, 1)], 2), ([(1, 1), (2, 1)], 1)])
def test_follower_commit_entry(ents, commit):
    r = Raft(1, [1, 2, 3])
    r.becomeFollower(1, 2)
    r.Step(Msg(APP, From=2, To=1, Term=1, Entries=ents, Commit=commit))
    assert r.committed == commit
    # nextEnts = (applied, committed]
    assert list(range(r.r.log.applied + 1, r.committed + 1)) == [i for i, _ in ents[:commit]]


@pytest.mark.parametrize("term,index,windex,wreject,whint", [  # raft_paper_test.go:597-631 TestFollowerCheckMsgApp
    (0, 0, 1, False, 0), (1, 1, 1, False, 0), (2, 2, 2, False, 0), (1, 2, 2, True, 2), (3, 3, 3, True, 2)])
def test_follower_check_msg_app(term, index, windex, wreject, whint):
    r = Raft(1, [1, 2, 3], ents=[(1, 1), (2, 2)], hard=(0, 0, 1))
    r.becomeFollower(2, 2)
    r.Step(Msg(APP, From=2, To=1, Term=2, LogTerm=term, Index=index))
    ms = r.readMessages()
    assert len(ms) == 1
    m = ms[0]
    assert (m.From, m.To, m.Type, m.Term, m.Index, bool(m.Reject), m.RejectHint) == (1, 2, APPRESP, 2, windex,
                                                                                     wreject, whint)


@pytest.mark.parametrize("index,term,ents,wents", [  # raft_paper_test.go:638-681 TestFollowerAppendEntries
    (2, 2, [(3, 3)], [(1, 1), (2, 2), (3, 3)]),
    (1, 1, [(2, 3), (3, 4)], [(1, 1), (2, 3), (3, 4)]),
    (0, 0, [(1, 1)], [(1, 1), (2, 2)]),
    (0, 0, [(1, 3)], [(1, 3)])])
def test_follower_append_entries(index, term, ents, wents):
    # the unstable/stable split (wunstable) is host-side raftLog state: the engine's
    # host half (hbnode) keeps it; the oracle pins the resulting log
    r = Raft(1, [1, 2, 3], ents=[(1, 1), (2, 2)])
    r.becomeFollower(2, 2)
    r.Step(Msg(APP, From=2, To=1, Term=2, LogTerm=term, Index=index, Entries=ents))
    assert r.entries() == wents


@pytest.mark.parametrize("ents,logterm,index,wreject", [  # raft_paper_test.go:821-861 TestVoter
    ([(1, 1)], 1, 1, False), ([(1, 1)], 1, 2, False), ([(1, 1), (2, 1)], 1, 1, True),
    ([(1, 1)], 2, 1, False), ([(1, 1)], 2, 2, False), ([(1, 1), (2, 1)], 2, 1, False),
    ([(1, 2)], 1, 1, True), ([(1, 2)], 1, 2, True), ([(1, 2), (2, 1)], 1, 1, True)])
def test_voter(ents, logterm, index, wreject):
    r = Raft(1, [1, 2], ents=ents)
    r.Step(Msg(VOTE, From=2, To=1, Term=3, LogTerm=logterm, Index=index))
    ms = r.readMessages()
    assert len(ms) == 1 and ms[0].Type == VOTERESP and bool(ms[0].Reject) == wreject


def test_restore_snapshot_via_msg_snap():
    """handleSnapshot + restore (raft/raft.go:671-707, cf. raft/raft_test.go
    TestRestore / TestProvideSnap): a follower behind the snapshot restores it
    (log = the snapshot, Progress reset) and answers MsgAppResp{lastIndex};
    one that already holds the entry fast-forwards its commit; one whose commit
    is past it ignores it and answers MsgAppResp{committed}."""
    r = Raft(1, [1, 2, 3], ents=[(1, 1), (2, 1)])
    r.becomeFollower(2, 2)
    r.Step(Msg(SNAP, From=2, To=1, Term=2, Snapshot=(11, 2)))
    assert (r.lastIndex, r.committed, r.r.log.first_index, r.term(11)) == (11, 11, 12, 2)
    ms = r.readMessages()
    assert [(m.Type, m.To, m.Index, bool(m.Reject)) for m in ms] == [(APPRESP, 2, 11, False)]
    assert r.pr(1).Match == 11 and r.pr(2).Match == 0 and r.pr(2).Next == 12
    # the snapshot's entry is already in the log: commit fast-forwards, no restore
    r2 = Raft(1, [1, 2], ents=[(1, 1), (2, 1), (3, 2)])
    r2.becomeFollower(2, 2)
    r2.Step(Msg(SNAP, From=2, To=1, Term=2, Snapshot=(2, 1)))
    assert (r2.lastIndex, r2.committed, r2.r.log.first_index) == (3, 2, 1)
    assert [(m.Type, m.Index) for m in r2.readMessages()] == [(APPRESP, 2)]
    # commit is past the snapshot: ignored
    r2.Step(Msg(SNAP, From=2, To=1, Term=2, Snapshot=(1, 1)))
    assert [(m.Type, m.Index) for m in r2.readMessages()] == [(APPRESP, 2)]


def test_follower_term_lookup_at_any_depth():
    """raftLog.term(i) for any i of the log (raft/log.go:198-217): with every
    older term run in the engine's log index (hb_load_term_runs), a leader
    probing a follower whose log holds 20 term runs is answered from any of
    them — a matching LogTerm deep in the log is accepted, a wrong one rejected."""
    ents = [(i + 1, i // 3 + 1) for i in range(60)]  # 20 runs of 3 entries
    for idx in (2, 5, 31, 59, 60):
        r = Raft(1, [1, 2], ents=ents)
        r.becomeFollower(25, 2)
        t = ents[idx - 1][1]
        r.Step(Msg(APP, From=2, To=1, Term=25, LogTerm=t, Index=idx, Entries=[(idx + 1, 25)], Commit=0))
        ms = r.readMessages()
        assert r.fault == 0 and [(m.Index, bool(m.Reject)) for m in ms] == [(idx + 1, False)], idx
        r2 = Raft(1, [1, 2], ents=ents)
        r2.becomeFollower(25, 2)
        r2.Step(Msg(APP, From=2, To=1, Term=25, LogTerm=t + 1, Index=idx, Commit=0))
        ms = r2.readMessages()
        assert r2.fault == 0 and [(m.Index, bool(m.Reject)) for m in ms] == [(idx, True)], idx


def test_rcommit_zero_before_first_step():
    """r.Commit (HardState.Commit) is set only by loadState and at the end of a
    Step past the term gate (raft/raft.go:466,488,759); handleAppendEntries
    compares m.Index with it, not with raftLog.committed (:652).
    (a) A MultiNode group bootstrapped with peers [1, 2, 3] (raft/multinode.go:
    197-211: Term 1, committed 3, r.Commit 0): MsgApp{Index 1, LogTerm 1} is
    acked at Index 1 by maybeAppend; after that Step r.Commit = 3 and the same
    MsgApp is answered with Index 3.  (b) A group restored from a snapshot at
    10 with an empty HardState (committed = firstIndex - 1 = 10, raft/log.go:60):
    MsgApp{Index 5, LogTerm 1} meets term(5) = 0 below the dummy index
    (raft/log.go:198-203) and is rejected with RejectHint 10."""
    r = Raft(1, [1, 2, 3], ents=[(1, 1), (2, 1), (3, 1)])
    r.r.Term = 1
    r.r.log.committed = 3
    assert r.Commit == 0
    r.Step(Msg(APP, From=2, To=1, Term=2, LogTerm=1, Index=1, Commit=3))
    ms = r.readMessages()
    assert [(m.Type, m.To, m.Index, bool(m.Reject)) for m in ms] == [(abi.HB_MSG_APP_RESP, 2, 1, False)]
    assert r.Commit == 3 and r.committed == 3
    r.Step(Msg(APP, From=2, To=1, Term=2, LogTerm=1, Index=1, Commit=3))
    assert [(m.Index, bool(m.Reject)) for m in r.readMessages()] == [(3, False)]
    r = Raft(1, [1, 2, 3], snapshot=(10, 1))
    assert r.committed == 10 and r.Commit == 0
    r.Step(Msg(APP, From=2, To=1, Term=2, LogTerm=1, Index=5, Commit=10))
    ms = r.readMessages()
    assert [(m.Type, m.Index, bool(m.Reject), m.RejectHint) for m in ms] == [(abi.HB_MSG_APP_RESP, 5, True, 10)]
    assert r.Commit == 10
    # a lower-term message is ignored before the gate: r.Commit keeps its value
    r = Raft(1, [1, 2, 3], ents=[(1, 1), (2, 1), (3, 1)])
    r.r.Term = 3
    r.r.log.committed = 3
    r.Step(Msg(APP, From=2, To=1, Term=2, LogTerm=1, Index=1, Commit=3))
    assert r.readMessages() == [] and r.Commit == 0
