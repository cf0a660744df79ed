"""The reference's leader-side known-answer tables, run on the DEVICE.

tests/test_oracle_kat.py runs these tables on the C oracle (CPU); here every
Step of them goes through the engine's C ABI (hb_step on the MI355X), so the
device's leader path is pinned by the reference's own tables directly, not only
through the engine <-> oracle chain.

DevRaft mirrors oracle.pyoracle.Raft (newTestRaft, raft/raft_test.go:
1884-1898).  The reference tests set a raft up by calling its internals
(becomeCandidate, becomeLeader, setProgress, appendEntry, bcastAppend,
Progress field writes); DevRaft runs that setup on the oracle raft and, at the
first Step, loads the resulting state (hb_group record + live inflight windows)
into a one-group engine — the same state injection the Go tests perform.  From
then on every Step is stepped on the device and the assertions read the
device's record and its events, materialised as the messages r.msgs would hold
(MsgApp Index / Commit / entry range under noLimit, MsgHeartbeat Commit,
MsgVote, MsgSnap).  Internals a test calls after its first Step are the
message the reference routes to them (bcastHeartbeat = Step(MsgBeat), which is
what stepLeader does, raft/raft.go:496-498).
"""
from types import SimpleNamespace

import numpy as np
import pytest

from etcd_amd import abi
from oracle.pyoracle import Msg, Raft

pytestmark = pytest.mark.gpu

P, R, S = abi.HB_PR_PROBE, abi.HB_PR_REPLICATE, abi.HB_PR_SNAPSHOT
F, Cd, L = abi.HB_STATE_FOLLOWER, abi.HB_STATE_CANDIDATE, abi.HB_STATE_LEADER


class DevRaft:
    """newTestRaft on the device (see the module docstring)."""

    def __init__(self, id, peers, ents=(), snapshot=None, hard=None, max_inflight=256):
        self.o = Raft(id, peers, ents=ents, snapshot=snapshot, hard=hard, max_inflight=max_inflight)
        self.id = id
        self.W = max_inflight
        self.eng = None
        self.msgs = []

    # ---- setup on the oracle raft (before the first Step) ---------------------
    def _host(self):
        assert self.eng is None, "raft internals touched after the state moved to the device"
        return self.o

    def becomeCandidate(self):
        self._host().becomeCandidate()

    def becomeLeader(self):
        self._host().becomeLeader()

    def setProgress(self, id, match, next):
        self._host().setProgress(id, match, next)

    def appendEntry(self, k=1):
        self._host().appendEntry(k)

    def bcastAppend(self):
        self._host().bcastAppend()

    def commitTo(self, i):
        self._host().commitTo(i)

    def bcastHeartbeat(self):
        if self.eng is None:
            self.o.bcastHeartbeat()
        else:  # stepLeader MsgBeat -> bcastHeartbeat (raft/raft.go:496-498)
            self.Step(Msg(abi.HB_MSG_BEAT, From=self.id, To=self.id))

    def set_state(self, state, lead=None):
        self._host().r.state = state
        if lead is not None:
            self.o.r.lead = lead

    # ---- the device --------------------------------------------------------------
    def _ids(self):
        return [self.o.r.ids[i] for i in range(self.o.r.n)]

    def _load(self):
        from etcd_amd.hipbatch import Engine
        rec = np.frombuffer(bytes(self.o.to_group()), dtype=abi.GROUP_DTYPE).copy()
        self.ids = self._ids()
        nmax = len(self.ids)
        self.eng = Engine(1, max_replicas=max(nmax, 1), max_inflight=self.W, max_batch=4096)
        self.eng.load_groups(rec)
        for s in range(nmax):  # live inflight windows (raft/progress.go:172-237)
            p = self.o.r.prs_[s]
            if p.State == R and p.ins.count:
                vals = [p.ins.buffer[(p.ins.start + k) % p.ins.size] for k in range(p.ins.count)]
                self.eng.set_inflights(0, s, p.ins.start, np.array(vals, np.uint64))
        self.eng.reserve_log(np.zeros(1, np.uint32), None, 1024)
        self.rec = self.eng.get_groups()[0]

    def _slot(self, id_):
        return self.ids.index(id_) if id_ in self.ids else abi.HB_SLOT_NONE

    def Step(self, *ms):
        """Step the messages (one device batch, arrival order)."""
        if self.eng is None:  # r.msgs the setup left unread stay in r.msgs
            self.msgs.extend(self.o.readMessages())
            self._load()
        info, term, index, hint = [], [], [], []
        for m in ms:
            info.append(abi.hb_info(m.Type, self._slot(m.From), bool(m.Reject)))
            term.append(m.Term)
            index.append(m.nents if m.Type == abi.HB_MSG_PROP else m.Index)  # MsgProp: its entry count
            hint.append(m.RejectHint)
        before = self.rec
        self.eng.step_batch(dict(group=np.zeros(len(ms), np.uint32), info=np.array(info, np.uint32),
                                 term=np.array(term, np.uint64), index=np.array(index, np.uint64),
                                 hint=np.array(hint, np.uint64), props=None), host=True)
        self._materialize(self.eng.events(), before)
        self.rec = self.eng.get_groups()[0]

    def _materialize(self, ev, before):
        """r.msgs from the device's events (what libhbnode builds, raft/raft.go:227-321)."""
        term, committed, last = int(before["term"]), int(before["committed"]), int(before["last_index"])
        for e in ev:
            t, x, to = int(e["type"]), int(e["x"]), int(e["to"])
            if t == abi.HB_EV_TERM:
                term = x
            elif t == abi.HB_EV_COMMIT:
                committed = x
            elif t == abi.HB_EV_LAST:
                last = x
            elif t == abi.HB_EV_APP:  # entries(Index + 1, noLimit) = (Index, last]
                self.msgs.append(SimpleNamespace(Type=abi.HB_MSG_APP, To=self.ids[to], From=self.id, Term=term,
                                                 Index=x, Commit=committed, nents=max(last - x, 0), ent_lo=x + 1))
            elif t == abi.HB_EV_SNAP:
                self.msgs.append(SimpleNamespace(Type=abi.HB_MSG_SNAP, To=self.ids[to], From=self.id, Term=term,
                                                 Index=0, Commit=0, nents=0, ent_lo=0, snap_index=x))
            elif t == abi.HB_EV_HEARTBEAT:
                self.msgs.append(SimpleNamespace(Type=abi.HB_MSG_HEARTBEAT, To=self.ids[to], From=self.id, Term=term,
                                                 Index=0, LogTerm=0, Commit=x, nents=0, ent_lo=0))
            elif t == abi.HB_EV_VOTE:
                self.msgs.append(SimpleNamespace(Type=abi.HB_MSG_VOTE, To=self.ids[to], From=self.id, Term=term,
                                                 Index=x, Commit=0, nents=0, ent_lo=0))

    def readMessages(self):
        if self.eng is None:
            return self.o.readMessages()
        out, self.msgs = self.msgs, []
        return out

    # ---- what the assertions read -----------------------------------------------
    def pr(self, id_):
        if self.eng is None:
            return self.o.pr(id_)
        p = self.rec["pr"][self.ids.index(id_)]
        return SimpleNamespace(Match=int(p["match"]), Next=int(p["next"]), State=int(p["state"]),
                               Paused=int(p["paused"]), PendingSnapshot=int(p["pending_snapshot"]),
                               ins=SimpleNamespace(count=int(p["ins_count"]), size=self.W))

    def _field(self, name, oname):
        return int(self.rec[name]) if self.eng is not None else getattr(self.o, oname)

    @property
    def committed(self):
        return self._field("committed", "committed")

    @property
    def lastIndex(self):
        return self._field("last_index", "lastIndex")

    @property
    def firstIndex(self):
        return self._field("first_index", "firstIndex")

    @property
    def Term(self):
        return self._field("term", "Term")

    @property
    def state(self):
        return self._field("state", "state")

    @property
    def fault(self):
        return self._field("fault", "fault")


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
    """TestCommit: the reference calls maybeCommit() after setProgress; on the
    device maybeCommit runs after an accepted MsgAppResp (raft/raft.go:514-546),
    so the peer with the highest Match is set one below it and acks it."""
    ids = list(range(1, len(matches) + 1))
    sm = DevRaft(1, ids, ents=[(i + 1, t) for i, t in enumerate(terms)], hard=(smterm, 0, 0))
    j = int(np.argmax(matches))
    for k, m in enumerate(matches):
        sm.setProgress(k + 1, m - 1 if k == j else m, m)
    sm.set_state(L, lead=1)
    sm.o.pr(j + 1).State = R
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=j + 1, To=1, Term=smterm, Index=matches[j]))
    assert sm.committed == w and sm.fault == 0


# ---------------------------------------------------------------- leader responses
@pytest.mark.parametrize("index,reject,wmatch,wnext,wmsgnum,windex,wcommitted", [
    (3, True, 0, 3, 0, 0, 0), (2, True, 0, 2, 1, 1, 0), (2, False, 2, 4, 2, 2, 2),
    (0, False, 0, 3, 0, 0, 0)])
def test_leader_app_resp(index, reject, wmatch, wnext, wmsgnum, windex, wcommitted):
    # raft/raft_test.go:1175-1229 — log {1: term 0, 2: term 1}; becomes leader at term 1
    sm = DevRaft(1, [1, 2, 3], ents=[(1, 0), (2, 1)])
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
    sm = DevRaft(1, [1, 2, 3])
    sm.becomeCandidate()
    sm.becomeLeader()
    sm.bcastAppend()
    sm.readMessages()
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=2, Index=1))
    assert sm.committed == 1
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
    sm = DevRaft(1, [1, 2], ents=[(1, 1), (2, 2), (3, 3)])
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
    r = DevRaft(1, [1, 2], ents=[(1, 1), (2, 1), (3, 1)])
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    p = r.pr(2)
    p.Match = 3
    p.State, p.Next = R, 4  # becomeReplicate + optimisticUpdate(5)
    p.Next = 6
    r.Step(Msg(abi.HB_MSG_UNREACHABLE, From=2, To=1))
    assert (r.pr(2).State, r.pr(2).Next) == (P, r.pr(2).Match + 1)


@pytest.mark.parametrize("state,nxt,wnext", [(R, 2, 3 + 1 + 1 + 1), (P, 2, 2)])
def test_leader_increase_next(state, nxt, wnext):  # raft/raft_test.go:1330-1360
    sm = DevRaft(1, [1, 2], ents=[(1, 1), (2, 1), (3, 1)])
    sm.becomeCandidate()
    sm.becomeLeader()
    sm.pr(2).State = state
    sm.pr(2).Next = nxt
    sm.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
    assert sm.pr(2).Next == wnext


def test_bcast_beat():  # raft/raft_test.go:1231-1284
    offset = 1000
    sm = DevRaft(1, [1, 2, 3], snapshot=(offset, 1))
    sm.o.Term = 1
    sm.becomeCandidate()
    sm.becomeLeader()
    for _ in range(10):
        sm.appendEntry()
    sm.pr(2).Match, sm.pr(2).Next = 5, 6
    sm.pr(3).Match, sm.pr(3).Next = sm.lastIndex, sm.lastIndex + 1
    sm.readMessages()
    sm.Step(Msg(abi.HB_MSG_BEAT))
    msgs = sm.readMessages()
    assert len(msgs) == 2
    want = {2: min(sm.committed, 5), 3: min(sm.committed, sm.lastIndex)}
    for m in msgs:
        assert m.Type == abi.HB_MSG_HEARTBEAT and m.Index == 0 and m.LogTerm == 0 and m.nents == 0
        assert m.Commit == want.pop(m.To)


@pytest.mark.parametrize("state,wmsg", [(L, 2), (Cd, 0), (F, 0)])
def test_recv_msg_beat(state, wmsg):  # raft/raft_test.go:1286-1328
    sm = DevRaft(1, [1, 2, 3], ents=[(1, 0), (2, 1)])
    sm.o.Term = 1
    sm.set_state(state)
    sm.Step(Msg(abi.HB_MSG_BEAT, From=1, To=1))
    msgs = sm.readMessages()
    assert len(msgs) == wmsg
    assert all(m.Type == abi.HB_MSG_HEARTBEAT for m in msgs)


# ---------------------------------------------------------------- flow control
def _leader_with_replicating_2(max_inflight=256):
    r = DevRaft(1, [1, 2], max_inflight=max_inflight)
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
    """The reference's inner loop of stale acks (each checked for a still-full
    window) is stepped as one batch per tt: stale acks change nothing, so the
    window after the batch is the window after each of them."""
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
        r.Step(*[Msg(abi.HB_MSG_APP_RESP, From=2, To=1, Index=i) for i in range(tt)])
        assert r.pr(2).ins.count == r.pr(2).ins.size
        assert r.readMessages() == []


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
def _snap_leader():
    # newTestRaft(1, peers) + restore(testingSnap{Index 11, Term 11, Nodes [1 2]})
    sm = DevRaft(1, [1, 2], snapshot=(11, 11))
    sm.becomeCandidate()
    sm.becomeLeader()
    return sm


def test_sending_snapshot_set_pending_snapshot():  # raft/raft_snap_test.go:33-49
    sm = _snap_leader()
    sm.pr(2).Next = sm.firstIndex
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=2, To=1, Index=sm.pr(2).Next - 1, Reject=True))
    assert sm.pr(2).PendingSnapshot == 11


def test_pending_snapshot_pause_replication():  # raft/raft_snap_test.go:51-66
    sm = _snap_leader()
    p = sm.pr(2)
    p.State, p.PendingSnapshot = S, 11
    sm.readMessages()
    sm.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
    assert len(sm.readMessages()) == 0


def test_snapshot_failure():  # raft/raft_snap_test.go:68-89
    sm = _snap_leader()
    p = sm.pr(2)
    p.Next = 1
    p.State, p.PendingSnapshot = S, 11
    sm.Step(Msg(abi.HB_MSG_SNAP_STATUS, From=2, To=1, Reject=True))
    p = sm.pr(2)
    assert (p.PendingSnapshot, p.Next, p.Paused) == (0, 1, 1)


def test_snapshot_succeed():  # raft/raft_snap_test.go:91-112
    sm = _snap_leader()
    p = sm.pr(2)
    p.Next = 1
    p.State, p.PendingSnapshot = S, 11
    sm.Step(Msg(abi.HB_MSG_SNAP_STATUS, From=2, To=1, Reject=False))
    p = sm.pr(2)
    assert (p.PendingSnapshot, p.Next, p.Paused) == (0, 12, 1)


def test_snapshot_abort():  # raft/raft_snap_test.go:114-134
    sm = _snap_leader()
    p = sm.pr(2)
    p.Next = 1
    p.State, p.PendingSnapshot = S, 11
    sm.Step(Msg(abi.HB_MSG_APP_RESP, From=2, To=1, Index=11))
    p = sm.pr(2)
    assert (p.PendingSnapshot, p.Next) == (0, 12)


# ---------------------------------------------------------------- elections / commit (paper tests)
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
    r = DevRaft(1, list(range(1, size + 1)))
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
    r = DevRaft(1, [1, 2, 3])
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
    r = DevRaft(1, list(range(1, size + 1)))
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
    r = DevRaft(1, [1, 2], ents=[(1, 1), (2, 2)], hard=(2, 0, 0))
    r.becomeCandidate()
    r.becomeLeader()
    r.readMessages()
    r.Step(Msg(abi.HB_MSG_PROP, From=1, To=1, Entries=1))
    r.Step(Msg(abi.HB_MSG_APP_RESP, From=2, To=1, Term=r.Term, Index=index))
    assert r.committed == wcommit


@pytest.mark.parametrize("state,wstate,wterm,windex", [(F, F, 3, 0), (Cd, F, 3, 0), (L, F, 3, 1)])
def test_all_server_stepdown(state, wstate, wterm, windex):  # raft/raft_test.go:1121-1173
    """The leader-side half: a higher-term MsgAppResp / MsgVoteResp steps any
    role down to follower at the message's term (raft/raft.go:474-477); the Go
    test's MsgVote / MsgApp rows take the same gate (their follower side runs
    in tests/test_follower_gpu.py)."""
    for mtype in (abi.HB_MSG_APP_RESP, abi.HB_MSG_VOTE_RESP):
        sm = DevRaft(1, [1, 2, 3])
        if state == F:
            sm.o.becomeFollower(1, 0)
        elif state == Cd:
            sm.becomeCandidate()
        else:
            sm.becomeCandidate()
            sm.becomeLeader()
        sm.Step(Msg(mtype, From=2, Term=wterm, LogTerm=wterm))
        assert (sm.state, sm.Term, sm.lastIndex) == (wstate, wterm, windex)
