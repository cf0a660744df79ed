"""Follower side through the MultiNode API on the GPU.

1. The reference's follower tests at the MultiNode boundary: TestHandleMsgApp
   (raft/raft_test.go:803-850), TestHandleHeartbeat (:852-882), TestRecvMsgVote
   (:1004-1066), TestFollowerAppendEntries (raft/raft_paper_test.go:638-681)
   and a MsgSnap restore (handleSnapshot / restore raft/raft.go:671-707): the
   group's Ready (responses, unstable entries, HardState, Snapshot) equals what
   the reference's raft puts in r.msgs / raftLog.
2. Clusters: three MultiNodes (one device engine each) run many groups of
   peers {1, 2, 3} against each other through Ready / Advance / Step, every
   message of every group stepped by an engine (leader and follower side),
   with ticks (heartbeats, election timeouts), leader changes, dropped and
   reordered messages, log compaction and snapshots.  Checked: Raft's safety
   properties (every node applies the same entry at each index; no two
   leaders in one term) and, without drops, liveness (every proposal commits
   on every node).
"""
import random

import pytest

from etcd_amd import abi
from etcd_amd.multinode import (Config, Entry, HardState, Message, MemoryStorage, Snapshot, StartMultiNode,
                                StateLeader, emptyState)

pytestmark = pytest.mark.gpu

APP, APPRESP, VOTE, VOTERESP = abi.HB_MSG_APP, abi.HB_MSG_APP_RESP, abi.HB_MSG_VOTE, abi.HB_MSG_VOTE_RESP
HB, HBRESP, SNAP = abi.HB_MSG_HEARTBEAT, abi.HB_MSG_HEARTBEAT_RESP, abi.HB_MSG_SNAP


def follower(ents, term, vote=0, commit=0, nodes=(1, 2), id=1):
    """A restarted group whose storage holds `ents` [(index, term)] after an
    empty snapshot with ConfState `nodes`, HardState (term, vote, commit)."""
    st = MemoryStorage()
    st.ApplySnapshot(Snapshot(Index=0, Term=0, Nodes=list(nodes)))
    st.Append([Entry(Term=t, Index=i) for i, t in ents])
    st.SetHardState(HardState(Term=term, Vote=vote, Commit=commit))
    mn = StartMultiNode(id, capacity=8)
    mn.CreateGroup(1, Config(10, 1), st)
    rd = mn.Ready()
    if rd:
        mn.Advance(rd)
    return mn, st


def one_ready(mn, st=None):
    """The group's one Ready; with its storage, handled as an application does
    (ApplySnapshot, Append, SetHardState) before Advance."""
    rds = mn.Ready()
    assert list(rds) == [1]
    rd = rds[1]
    if st is not None:
        if rd.Snapshot.Index:
            st.ApplySnapshot(rd.Snapshot)
        st.Append(rd.Entries)
        if rd.HardState != emptyState:
            st.SetHardState(rd.HardState)
    mn.Advance(rds)
    return rd


@pytest.mark.parametrize("m,windex,wcommit,wreject", [  # raft/raft_test.go:803-850 TestHandleMsgApp
    (dict(LogTerm=3, Index=2, Commit=3), 2, 0, True),
    (dict(LogTerm=3, Index=3, Commit=3), 2, 0, True),
    (dict(LogTerm=1, Index=1, Commit=1), 2, 1, False),
    (dict(LogTerm=0, Index=0, Commit=1, Entries=[(1, 2)]), 1, 1, False),
    (dict(LogTerm=2, Index=2, Commit=3, Entries=[(3, 2), (4, 2)]), 4, 3, False),
    (dict(LogTerm=2, Index=2, Commit=4, Entries=[(3, 2)]), 3, 3, False),
    (dict(LogTerm=1, Index=1, Commit=4, Entries=[(2, 2)]), 2, 2, False),
    (dict(LogTerm=2, Index=2, Commit=3), 2, 2, False),
    (dict(LogTerm=2, Index=2, Commit=4), 2, 2, False)])
def test_handle_msg_app(m, windex, wcommit, wreject):
    mn, st = follower([(1, 1), (2, 2)], term=2)
    ents = [Entry(Term=t, Index=i) for i, t in m.pop("Entries", [])]
    mn.Step(1, Message(Type=APP, From=2, To=1, Term=2, Entries=ents, **m))
    rd = one_ready(mn, st)
    assert st.LastIndex() == windex
    assert rd.HardState.Commit == wcommit or (wcommit == 0 and rd.HardState == emptyState)
    assert len(rd.Messages) == 1
    r = rd.Messages[0]
    assert (r.Type, r.To, r.From, r.Term, r.Reject) == (APPRESP, 2, 1, 2, wreject)
    if wreject:
        assert (r.Index, r.RejectHint) == (m["Index"], 2)
    else:
        assert r.Index == m["Index"] + len(ents)
    mn.Stop()


def test_first_msgapp_of_bootstrapped_group_reads_rcommit_zero():
    """A MultiNode group created with peers [1, 2, 3] (raft/multinode.go:197-211)
    has committed = 3 but r.Commit = 0 until its first Step (raft/raft.go:488).
    Its first MsgApp{Index 1, LogTerm 1} is below committed but not below
    r.Commit, so handleAppendEntries (:651-665) runs maybeAppend and acks Index 1
    (not 3); the Step then sets r.Commit = 3, and the same MsgApp again is
    answered MsgAppResp{Index: r.Commit = 3} (:652-653)."""
    mn = StartMultiNode(1, capacity=8)
    s = MemoryStorage()
    mn.CreateGroup(1, Config(10, 1), s, peers=[1, 2, 3])
    rds = mn.Ready()  # the bootstrap entries
    s.Append(rds[1].Entries)
    mn.Advance(rds)
    mn.Step(1, Message(Type=APP, From=2, To=1, Term=2, Index=1, LogTerm=1, Commit=3))
    rd = one_ready(mn, s)
    assert rd.Messages == [Message(Type=APPRESP, To=2, From=1, Term=2, Index=1)]
    assert rd.HardState == HardState(Term=2, Vote=0, Commit=3)
    assert [e.Index for e in rd.CommittedEntries] == [1, 2, 3]
    mn.Step(1, Message(Type=APP, From=2, To=1, Term=2, Index=1, LogTerm=1, Commit=3))
    rd = one_ready(mn, s)
    assert rd.Messages == [Message(Type=APPRESP, To=2, From=1, Term=2, Index=3)]
    mn.Stop()


def test_first_msgapp_after_snapshot_with_empty_hardstate():
    """A group restored from a snapshot at index 10 with an empty HardState:
    committed = firstIndex - 1 = 10 (raft/log.go:60), r.Commit = 0.  Its first
    MsgApp{Index 5, LogTerm 1} is not below r.Commit, so maybeAppend runs;
    raftLog.term(5) is 0 below the dummy index (raft/log.go:198-203), the terms
    differ, and the reference rejects with RejectHint = lastIndex = 10."""
    st = MemoryStorage()
    st.ApplySnapshot(Snapshot(Index=10, Term=1, Nodes=[1, 2, 3]))
    mn = StartMultiNode(1, capacity=8)
    mn.CreateGroup(1, Config(10, 1), st)
    rds = mn.Ready()
    if rds:
        mn.Advance(rds)
    mn.Step(1, Message(Type=APP, From=2, To=1, Term=2, Index=5, LogTerm=1, Commit=10))
    rd = one_ready(mn, st)
    assert rd.Messages == [Message(Type=APPRESP, To=2, From=1, Term=2, Index=5, Reject=True, RejectHint=10)]
    assert rd.HardState == HardState(Term=2, Vote=0, Commit=10)
    mn.Stop()


@pytest.mark.parametrize("mcommit,wcommit", [(3, 3), (1, 2)])  # raft/raft_test.go:852-882 TestHandleHeartbeat
def test_handle_heartbeat(mcommit, wcommit):
    mn, _ = follower([(1, 1), (2, 2), (3, 3)], term=2, commit=2)
    mn.Step(1, Message(Type=HB, From=2, To=1, Term=2, Commit=mcommit))
    rd = one_ready(mn)
    assert rd.Messages == [Message(Type=HBRESP, To=2, From=1, Term=2)]
    assert rd.HardState == (HardState(Term=2, Commit=wcommit) if wcommit != 2 else emptyState)
    mn.Stop()


@pytest.mark.parametrize("i,term,vote_for,wreject", [  # raft/raft_test.go:1004-1066 TestRecvMsgVote (follower rows)
    (0, 0, 0, True), (0, 1, 0, True), (0, 2, 0, True), (0, 3, 0, False),
    (1, 0, 0, True), (1, 1, 0, True), (1, 2, 0, True), (1, 3, 0, False),
    (2, 0, 0, True), (2, 1, 0, True), (2, 2, 0, False), (2, 3, 0, False),
    (3, 0, 0, True), (3, 1, 0, True), (3, 2, 0, False), (3, 3, 0, False),
    (3, 2, 2, False), (3, 2, 1, True)])
def test_recv_msg_vote(i, term, vote_for, wreject):
    mn, _ = follower([(1, 2), (2, 2)], term=2, vote=vote_for, nodes=(1, 2))
    mn.Step(1, Message(Type=VOTE, From=2, To=1, Term=2, Index=i, LogTerm=term))
    rd = one_ready(mn)
    assert rd.Messages == [Message(Type=VOTERESP, To=2, From=1, Term=2, Reject=wreject)]
    if not wreject and vote_for == 0:
        assert rd.HardState.Vote == 2
    mn.Stop()


@pytest.mark.parametrize("index,term,ents,wents,wunstable", [  # raft_paper_test.go:638-681
    (2, 2, [(3, 3)], [(1, 1), (2, 2), (3, 3)], [(3, 3)]),
    (1, 1, [(2, 3), (3, 4)], [(1, 1), (2, 3), (3, 4)], [(2, 3), (3, 4)]),
    (0, 0, [(1, 1)], [(1, 1), (2, 2)], []),
    (0, 0, [(1, 3)], [(1, 3)], [(1, 3)])])
def test_follower_append_entries(index, term, ents, wents, wunstable):
    mn, st = follower([(1, 1), (2, 2)], term=2, nodes=(1, 2, 3))
    mn.Step(1, Message(Type=APP, From=2, To=1, Term=2, LogTerm=term, Index=index,
                       Entries=[Entry(Term=t, Index=i) for i, t in ents]))
    rd = one_ready(mn, st)
    assert [(e.Index, e.Term) for e in rd.Entries] == wunstable  # raftLog.unstableEntries()
    got, err = st.Entries(st.FirstIndex(), st.LastIndex() + 1)
    assert err is None and [(e.Index, e.Term) for e in got] == wents
    mn.Stop()


def test_follower_restores_snapshot_and_appends_after_it():
    """handleSnapshot -> restore (raft/raft.go:671-707): the Ready carries the
    snapshot, committed = its index, the answer is MsgAppResp{lastIndex}; the
    next MsgApp continues after it."""
    mn, st = follower([(1, 1), (2, 1)], term=2, nodes=(1, 2, 3))
    snap = Snapshot(Index=11, Term=2, Nodes=[1, 2, 3], Data=b"state")
    mn.Step(1, Message(Type=SNAP, From=2, To=1, Term=2, Snapshot=snap))
    rd = one_ready(mn, st)
    assert rd.Snapshot == snap and rd.HardState.Commit == 11
    assert rd.Messages == [Message(Type=APPRESP, To=2, From=1, Term=2, Index=11)]
    mn.Step(1, Message(Type=APP, From=2, To=1, Term=2, LogTerm=2, Index=11, Commit=12,
                       Entries=[Entry(Term=2, Index=12, Data=b"x")]))
    rd = one_ready(mn, st)
    assert [(e.Index, e.Term, e.Data) for e in rd.Entries] == [(12, 2, b"x")]
    assert [(e.Index, e.Data) for e in rd.CommittedEntries] == [(12, b"x")]
    assert rd.Messages == [Message(Type=APPRESP, To=2, From=1, Term=2, Index=12)]
    mn.Stop()


def test_snapshot_with_new_conf_state_reloads_peers():
    """A restore whose ConfState differs from the group's peers: r.prs becomes
    the snapshot's nodes (raft/raft.go:700-705); after winning an election the
    group replicates to exactly those."""
    mn, st = follower([(1, 1)], term=2, nodes=(1, 2, 3))
    snap = Snapshot(Index=5, Term=2, Nodes=[1, 2, 4])
    mn.Step(1, Message(Type=SNAP, From=2, To=1, Term=2, Snapshot=snap))
    one_ready(mn, st)
    mn.Campaign(1)
    rd = one_ready(mn, st)
    assert sorted(m.To for m in rd.Messages if m.Type == VOTE) == [2, 4]
    mn.Step(1, Message(Type=VOTERESP, From=4, To=1, Term=3))
    rd = one_ready(mn, st)
    assert rd.SoftState is not None and rd.SoftState.RaftState == StateLeader
    assert sorted(m.To for m in rd.Messages if m.Type == APP) == [2, 4]
    mn.Stop()


def test_vote_from_sender_outside_prs():
    """MsgVote from a node outside prs: granted once (r.Vote = its id, which
    only the host knows), granted again to the same sender, rejected for
    another (raft/raft.go:636-648)."""
    mn, _ = follower([(1, 1)], term=2, nodes=(1, 2))
    mn.Step(1, Message(Type=VOTE, From=7, To=1, Term=3, Index=1, LogTerm=1))
    rd = one_ready(mn)
    assert rd.HardState == HardState(Term=3, Vote=7, Commit=0)
    assert rd.Messages == [Message(Type=VOTERESP, To=7, From=1, Term=3)]
    mn.Step(1, Message(Type=VOTE, From=7, To=1, Term=3, Index=1, LogTerm=1))
    mn.Step(1, Message(Type=VOTE, From=8, To=1, Term=3, Index=1, LogTerm=1))
    rd = one_ready(mn)
    assert rd.Messages == [Message(Type=VOTERESP, To=7, From=1, Term=3),
                           Message(Type=VOTERESP, To=8, From=1, Term=3, Reject=True)]
    # a leader outside prs: lead = its id
    mn.Step(1, Message(Type=HB, From=7, To=1, Term=3, Commit=0))
    rd = one_ready(mn)
    assert rd.SoftState is not None and rd.SoftState.Lead == 7
    mn.Stop()


# ---------------------------------------------------------------- clusters
class Cluster:
    def __init__(self, G, ids=(1, 2, 3), seed=0, election=10, W=256, max_msg_size=abi.HB_NO_LIMIT):
        self.rng = random.Random(seed)
        self.ids = list(ids)
        self.G = G
        self.seed, self.election, self.W, self.max_msg_size = seed, election, W, max_msg_size
        self.down = set()  # stopped nodes: no Ready, no Tick, messages to them are lost
        self.sent = []  # (group, MsgApp) delivered, when self.record
        self.record = False
        self.nodes = {i: self._start(i) for i in ids}
        self.st = {(i, g): MemoryStorage() for i in ids for g in range(1, G + 1)}
        for i in ids:
            for g in range(1, G + 1):
                self.nodes[i].CreateGroup(g, Config(election, 1), self.st[i, g], peers=self.ids)
        self.applied = {(i, g): [] for i in ids for g in range(1, G + 1)}
        self.leaders = {}  # (group, term) -> node
        self.inbox = []
        self.proposed = {g: set() for g in range(1, G + 1)}

    def _start(self, i):
        mn = StartMultiNode(i, capacity=self.G + 4, max_inflight=self.W, max_msg_size=self.max_msg_size)
        r = random.Random(self.seed * 1000 + i)
        mn.SetRand([r.getrandbits(63) for _ in range(1 << 15)])
        return mn

    def stop_node(self, i):
        """Node i crashes: its MultiNode is gone, its storages stay."""
        self.nodes[i].Stop()
        self.down.add(i)

    def restart_node(self, i):
        """Node i restarts from its storages (raft/multinode_test.go:302-370):
        a snapshot at its applied index carries the ConfState (CreateGroup takes
        the peers from it, raft/raft.go:164-172), Config.Applied = that index."""
        mn = self._start(i)
        for g in range(1, self.G + 1):
            st = self.st[i, g]
            ap = [e for e in self.applied[i, g] if e[0] != "snap"]
            at = ap[-1][0] if ap else 0
            if at > st.Snapshot().Index:
                _, err = st.CreateSnapshot(at, self.ids, b"restart@%d" % at)
                assert err is None
            mn.CreateGroup(g, Config(self.election, 1, applied=st.Snapshot().Index), st)
        self.nodes[i] = mn
        self.down.discard(i)

    def ready_round(self):
        for i in self.ids:
            if i in self.down:
                continue
            rds = self.nodes[i].Ready()
            for g, rd in rds.items():
                assert rd.fault == 0, (i, g, rd.fault)
                st = self.st[i, g]
                if rd.Snapshot.Index:
                    st.ApplySnapshot(rd.Snapshot)
                    self.applied[i, g] = [("snap", rd.Snapshot.Index, rd.Snapshot.Term, rd.Snapshot.Data)]
                st.Append(rd.Entries)
                if rd.HardState != emptyState:
                    st.SetHardState(rd.HardState)
                # the application applies each index once: this reference's commitReady
                # moves applied only from a Ready's non-empty HardState (raft/multinode.go:
                # 137-147), so a bootstrapped follower gets its ConfChange entries again
                ap = self.applied[i, g]
                done = ap[-1][1] if ap and ap[-1][0] == "snap" else (ap[-1][0] if ap else 0)
                for e in rd.CommittedEntries:
                    if e.Index > done:
                        ap.append((e.Index, e.Term, e.Data))
                    else:
                        assert e.Index < self.st[i, g].FirstIndex() or any(
                            x[0] == e.Index and x[1:] == (e.Term, e.Data) for x in ap), "re-delivered entry differs"
                if rd.SoftState is not None and rd.SoftState.RaftState == StateLeader:
                    term = self.nodes[i].Status(g).HardState.Term
                    prev = self.leaders.setdefault((g, term), i)
                    assert prev == i, f"two leaders in group {g} term {term}"  # Election Safety
                self.inbox.extend((g, m) for m in rd.Messages)
            self.nodes[i].Advance(rds)

    def deliver(self, drop=0.0):
        box, self.inbox = self.inbox, []
        self.rng.shuffle(box)
        for g, m in box:
            if self.rng.random() < drop or m.To in self.down:
                continue
            if self.record and m.Type == APP:
                self.sent.append((g, m))
            self.nodes[m.To].Step(g, m)

    def propose(self, k, tag, pad=0):
        for _ in range(k):
            g = self.rng.randint(1, self.G)
            i = self.rng.choice([x for x in self.ids if x not in self.down])
            data = f"{tag}-{g}-{i}-{self.rng.getrandbits(32)}".encode()
            if pad:
                data += b"p" * self.rng.randint(0, pad)
            self.proposed[g].add(data)
            self.nodes[i].Propose(g, data)

    def tick(self):
        for i in self.ids:
            if i not in self.down:
                self.nodes[i].Tick()

    def compact(self, keep=3):
        """The application's CreateSnapshot + Compact at its applied index."""
        for (i, g), st in self.st.items():
            if i in self.down:
                continue
            ents = [e for e in self.applied[i, g] if e[0] != "snap"]
            if len(ents) < keep + 2:
                continue
            at = ents[-keep][0]
            snap, err = st.CreateSnapshot(at, self.ids, b"snap@%d" % at)
            if err is None:
                st.Compact(at)

    def check_safety(self):
        """State Machine Safety: the same entry at every index every node applied."""
        for g in range(1, self.G + 1):
            seen = {}
            for i in self.ids:
                prev = None
                for e in self.applied[i, g]:
                    if e[0] == "snap":
                        prev = e[1]
                        continue
                    idx = e[0]
                    assert prev is None or idx == prev + 1, f"node {i} group {g} applied {idx} after {prev}"
                    prev = idx
                    assert seen.setdefault(idx, e) == e, f"group {g} index {idx}: {seen[idx]} vs {e} on {i}"

    def stop(self):
        for i, n in self.nodes.items():
            if i not in self.down:
                n.Stop()


@pytest.mark.parametrize("G,seed", [(16, 1), (64, 2)])
def test_cluster_replicates_every_proposal(G, seed):
    """No drops: campaigns spread over the three nodes, proposals on random
    nodes (followers forward them), heartbeats each tick; at the end every
    proposal is applied, in the same order, on every node."""
    c = Cluster(G, seed=seed)
    for g in range(1, G + 1):
        c.nodes[c.ids[g % 3]].Campaign(g)
    for r in range(30):
        c.ready_round()
        c.deliver()
        if r >= 4:
            c.propose(2 * G, f"r{r}")
        c.tick()
    for _ in range(12):  # settle
        c.ready_round()
        c.deliver()
    c.check_safety()
    for g in range(1, G + 1):
        for i in c.ids:
            got = {e[2] for e in c.applied[i, g] if e[0] != "snap" and e[2] and e[2].startswith(b"r")}
            assert got == c.proposed[g], f"group {g} node {i}: {len(got)} of {len(c.proposed[g])} applied"
    c.stop()


@pytest.mark.parametrize("G,seed,drop", [(32, 3, 0.1), (32, 4, 0.3)])
def test_cluster_safety_under_loss_and_elections(G, seed, drop):
    """Dropped and reordered messages, election timeouts (new leaders, log
    conflicts and truncation on followers), compaction and snapshots to
    lagging followers: every node applies the same entry at every index and
    no group has two leaders in a term."""
    c = Cluster(G, seed=seed, election=6)
    for g in range(1, G + 1):
        c.nodes[c.ids[g % 3]].Campaign(g)
    for r in range(60):
        c.ready_round()
        c.deliver(drop=drop)
        c.propose(G, f"r{r}")
        c.tick()
        if r % 15 == 14:
            c.compact()
    for _ in range(20):  # heal: no loss, keep ticking so every group elects and catches up
        c.ready_round()
        c.deliver()
        c.tick()
    c.check_safety()
    committed = sum(len(c.applied[1, g]) for g in range(1, G + 1))
    assert committed > G * 10
    c.stop()


def test_probe_into_log_with_twenty_term_runs():
    """raftLog.term(i) at any depth of the log (raft/log.go:198-217): a
    restarted follower whose storage holds 60 entries in 20 term runs (libhbnode
    loads every run into the device's log index) answers a leader probing at
    any index (handleAppendEntries raft/raft.go:651-665, maybeAppend
    raft/log.go:72-88): a matching LogTerm is accepted and the log is cut and
    appended after it, a wrong one is rejected with RejectHint = lastIndex."""
    ents = [(i + 1, i // 3 + 1) for i in range(60)]
    for idx in (1, 2, 4, 17, 31, 44, 58, 60):
        t = ents[idx - 1][1]
        mn, st = follower(ents, 25)
        mn.Step(1, Message(Type=APP, From=2, To=1, Term=25, LogTerm=t, Index=idx,
                           Entries=[Entry(Term=25, Index=idx + 1, Data=b"x")], Commit=0))
        rd = one_ready(mn, st)
        assert rd.fault == 0
        assert [(m.Type, m.Index, m.Reject) for m in rd.Messages] == [(APPRESP, idx + 1, False)], idx
        assert [(e.Index, e.Term) for e in rd.Entries] == [(idx + 1, 25)], idx
        mn.Stop()
        mn, st = follower(ents, 25)
        mn.Step(1, Message(Type=APP, From=2, To=1, Term=25, LogTerm=t + 1, Index=idx, Commit=0))
        rd = one_ready(mn, st)
        assert rd.fault == 0
        assert [(m.Type, m.Index, m.Reject, m.RejectHint) for m in rd.Messages] == [(APPRESP, idx, True, 60)], idx
        mn.Stop()
    # isUpToDate over the 20-run log (raft/log.go:235-237): MsgVote from a
    # candidate whose last entry is one term older is rejected
    mn, st = follower(ents, 25)
    mn.Step(1, Message(Type=VOTE, From=2, To=1, Term=26, LogTerm=19, Index=100))
    rd = one_ready(mn, st)
    assert [(m.Type, m.Reject) for m in rd.Messages] == [(VOTERESP, True)]
    mn.Stop()


def test_restarted_follower_catches_up_5000_behind_under_1mib():
    """etcdserver's MaxSizePerMsg = 1 MiB (etcdserver/raft.go:229): node 3
    crashes, every group commits > 5,000 more entries of random payload sizes
    on nodes 1 and 2, node 3 restarts from its storage.  The leaders probe it
    back (rejections, maybeDecrTo) and send entries(Next, 1 MiB) from more than
    5,000 entries behind (raft/raft.go:265, limitSize raft/util.go:97-110): no
    group faults, every MsgApp is cut exactly by limitSize, and node 3 applies
    every entry in the same order as the others."""
    from etcd_amd.multinode import entry_size
    G, lim = 3, 1 << 20
    c = Cluster(G, seed=11, max_msg_size=lim)
    for g in range(1, G + 1):
        c.nodes[1].Campaign(g)
    for _ in range(4):
        c.ready_round()
        c.deliver()
    c.stop_node(3)
    for r in range(13):  # > 5,000 entries per group while node 3 is down
        for g in range(1, G + 1):
            for _ in range(450):
                c.nodes[1].Propose(g, b"e%d-%d-" % (g, r) + b"z" * c.rng.randint(0, 900))
        c.ready_round()
        c.deliver()
        c.tick()
    for _ in range(6):
        c.ready_round()
        c.deliver()
        c.tick()
    last = {g: c.nodes[1].Status(g).HardState.Commit for g in range(1, G + 1)}
    behind = {g: last[g] - c.st[3, g].LastIndex() for g in range(1, G + 1)}
    assert min(behind.values()) > 5000, behind
    c.restart_node(3)
    c.record = True
    for _ in range(40):
        c.ready_round()
        c.deliver()
        c.tick()
        if all(c.st[3, g].LastIndex() >= last[g] for g in range(1, G + 1)):
            break
    for _ in range(4):
        c.ready_round()
        c.deliver()
    c.check_safety()
    deep = 0
    for g, m in c.sent:
        if m.To != 3 or not m.Entries:
            continue
        sz = [entry_size(e) for e in m.Entries]
        assert len(sz) == 1 or sum(sz) <= lim, (g, m.Index, len(sz), sum(sz))
        deep = max(deep, last[g] - m.Index)
    assert deep > 5000, deep
    for g in range(1, G + 1):
        assert c.st[3, g].LastIndex() >= last[g]
        a1 = [e for e in c.applied[1, g] if e[0] != "snap"]
        a3 = {e[0]: e for e in c.applied[3, g] if e[0] != "snap"}
        assert all(a3[e[0]] == e for e in a1 if e[0] in a3) and max(a3) >= last[g], g
    c.stop()


def test_cluster_with_restarted_follower():
    """A 3-node cluster where node 3 crashes and restarts twice from its
    storage (snapshot ConfState, Config.Applied) while proposals, elections (of
    the groups it led) and compaction go on: safety holds throughout, and once
    the cluster is whole again every later proposal commits on every node and
    node 3 holds every committed index."""
    G = 12
    c = Cluster(G, seed=21, election=8)
    for g in range(1, G + 1):
        c.nodes[c.ids[g % 3]].Campaign(g)
    for r in range(45):
        if r in (8, 26):
            c.stop_node(3)
        if r in (17, 35):
            c.restart_node(3)
        c.ready_round()
        c.deliver()
        c.propose(2 * G, f"r{r}", pad=200)
        c.tick()
        if r == 30:
            c.compact(keep=20)

    def leaders():
        return {g for g in range(1, G + 1) for i in c.ids
                if c.nodes[i].Status(g).SoftState.RaftState == StateLeader}
    # without pre-vote a group can take many election rounds (a candidate with a
    # shorter log loses, raft/log.go:235-237); proposals to a group with no
    # leader are dropped (raft/raft.go:619-621), so the late ones wait for leaders
    for _ in range(80):
        if len(leaders()) == G:
            break
        c.ready_round()
        c.deliver()
        c.tick()
    assert len(leaders()) == G
    for r in range(6):
        c.ready_round()
        c.deliver()
        c.propose(2 * G, f"late{r}", pad=200)
        c.tick()
    for _ in range(25):
        c.ready_round()
        c.deliver()
        c.tick()
    c.check_safety()
    for g in range(1, G + 1):
        late = {d for d in c.proposed[g] if d.startswith(b"late")}
        top = set()
        for i in c.ids:
            ap = [e for e in c.applied[i, g] if e[0] != "snap"]
            got = {e[2] for e in ap if e[2]}
            assert late <= got, f"group {g} node {i}: {len(late - got)} late proposals missing"
            top.add(ap[-1][0])
        assert len(top) == 1, f"group {g}: applied up to {top}"
    c.stop()
