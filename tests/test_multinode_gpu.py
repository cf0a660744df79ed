"""MultiNode host side (etcd_amd/libhbnode.so over libhipbatch.so) on the GPU.

1. The reference's own MultiNode tests, transcribed (raft/multinode_test.go:
   29-412): Start, Restart, RestartFromSnapshot, Advance, Status, Propose,
   ProposeConfig, the Step filter.
2. Randomised parity: many groups driven through the MultiNode API (Campaign,
   Propose, MsgVoteResp / MsgAppResp / MsgHeartbeatResp, ReportUnreachable,
   ReportSnapshot, Tick, Ready / Advance), and beside it one oracle raft per
   group (oracle/raft_oracle.c) stepped with the same messages.  Every Ready is
   checked against the oracle: HardState / SoftState, the messages (type, to,
   term, index, log term, commit, reject, entry count and first index — the
   oracle's r.msgs in order), the unstable entries and the committed entries
   (indices and terms), and every payload against what was proposed.
"""
import numpy as np
import pytest

from etcd_amd import abi
from etcd_amd.multinode import (Config, ConfChangeAddNode, ConfChangeRemoveNode, Entry, EntryConfChange, HardState, Message,
                                MemoryStorage, Ready, Snapshot, SoftState, StartMultiNode, StateLeader, emptyState)

pytestmark = pytest.mark.gpu


def cc_data(node_id, typ=ConfChangeAddNode, id=0):
    """ConfChange{ID, Type, NodeID}.Marshal() (raft/raftpb/raft.pb.go:1402-1426)."""
    def v(x):
        out = bytearray()
        while x >= 0x80:
            out.append((x & 0x7F) | 0x80)
            x >>= 7
        out.append(x)
        return bytes(out)
    return b"\x08" + v(id) + b"\x10" + v(typ) + b"\x18" + v(node_id)


def test_multinode_start():  # raft/multinode_test.go:246-300
    ccdata = cc_data(1)
    wants = [
        Ready(SoftState=SoftState(Lead=1, RaftState=StateLeader), HardState=HardState(Term=2, Commit=2, Vote=1),
              Entries=[Entry(Type=EntryConfChange, Term=1, Index=1, Data=ccdata), Entry(Term=2, Index=2)],
              CommittedEntries=[Entry(Type=EntryConfChange, Term=1, Index=1, Data=ccdata), Entry(Term=2, Index=2)]),
        Ready(HardState=HardState(Term=2, Commit=3, Vote=1), Entries=[Entry(Term=2, Index=3, Data=b"foo")],
              CommittedEntries=[Entry(Term=2, Index=3, Data=b"foo")]),
    ]
    mn = StartMultiNode(1)
    storage = MemoryStorage()
    mn.CreateGroup(1, Config(10, 1), storage, peers=[1])
    mn.Campaign(1)
    gs = mn.Ready()
    assert gs[1] == wants[0]
    storage.Append(gs[1].Entries)
    mn.Advance(gs)
    mn.Propose(1, b"foo")
    gs2 = mn.Ready()
    assert gs2[1] == wants[1]
    storage.Append(gs2[1].Entries)
    mn.Advance(gs2)
    assert mn.Ready() == {}
    mn.Stop()


def test_multinode_restart():  # :302-332
    entries = [Entry(Term=1, Index=1), Entry(Term=1, Index=2, Data=b"foo")]
    st = HardState(Term=1, Commit=1)
    want = Ready(HardState=emptyState, CommittedEntries=entries[:st.Commit])
    storage = MemoryStorage()
    storage.SetHardState(st)
    storage.Append(entries)
    mn = StartMultiNode(1)
    mn.CreateGroup(1, Config(10, 1), storage)
    gs = mn.Ready()
    assert gs[1] == want
    mn.Advance(gs)
    assert mn.Ready() == {}
    mn.Stop()


def test_multinode_restart_from_snapshot():  # :334-370
    snap = Snapshot(Index=2, Term=1, Nodes=[1, 2])
    entries = [Entry(Term=1, Index=3, Data=b"foo")]
    st = HardState(Term=1, Commit=3)
    want = Ready(HardState=emptyState, CommittedEntries=entries)
    s = MemoryStorage()
    s.SetHardState(st)
    s.ApplySnapshot(snap)
    s.Append(entries)
    mn = StartMultiNode(1)
    mn.CreateGroup(1, Config(10, 1), s)
    gs = mn.Ready()
    assert gs[1] == want
    mn.Advance(gs)
    assert mn.Ready() == {}
    # the restarted group is on the device: a campaign sends MsgVote to 2 with the log's last (3, 1)
    mn.Campaign(1)
    rd = mn.Ready()[1]
    assert rd.SoftState == SoftState(0, abi.HB_STATE_CANDIDATE)
    assert rd.HardState == HardState(Term=2, Vote=1, Commit=3)
    assert rd.Messages == [Message(Type=abi.HB_MSG_VOTE, To=2, From=1, Term=2, LogTerm=1, Index=3)]


def test_multinode_advance():  # :372-394
    storage = MemoryStorage()
    mn = StartMultiNode(1)
    mn.CreateGroup(1, Config(10, 1), storage, peers=[1])
    mn.Campaign(1)
    rd1 = mn.Ready()
    mn.Propose(1, b"foo")
    assert mn.Ready() == {}, "unexpected Ready before Advance"
    storage.Append(rd1[1].Entries)
    mn.Advance(rd1)
    assert mn.Ready() != {}, "expect Ready after Advance"


def test_multinode_status():  # :396-412
    storage = MemoryStorage()
    mn = StartMultiNode(1)
    mn.CreateGroup(1, Config(10, 1), storage, peers=[1])
    assert mn.Status(1) is not None
    assert mn.Status(2) is None
    mn.Campaign(1)
    st = mn.Status(1)
    assert st.SoftState == SoftState(1, StateLeader) and st.HardState == HardState(2, 1, 2)
    assert list(st.Progress) == [1] and st.Progress[1].match == 2 and st.Progress[1].next == 3


@pytest.mark.parametrize("conf", [False, True])
def test_multinode_propose(conf):  # :109-155 (Propose) and :157-215 (ProposeConfig)
    mn = StartMultiNode(1)
    s = MemoryStorage()
    mn.CreateGroup(1, Config(10, 1), s, peers=[1])
    mn.Campaign(1)
    proposed = False
    for _ in range(10):
        rds = mn.Ready()
        rd = rds[1]
        s.Append(rd.Entries)
        if not proposed and rd.SoftState and rd.SoftState.Lead == mn.id:
            if conf:
                mn.ProposeConfChange(1, ConfChangeAddNode, 1)
            else:
                mn.Propose(1, b"somedata")
            proposed = True
        mn.Advance(rds)
        if s.LastIndex() >= 3:
            break
    last = s.LastIndex()
    ents, err = s.Entries(last, last + 1)
    assert err is None and len(ents) == 1
    if conf:
        assert ents[0].Type == EntryConfChange and ents[0].Data == cc_data(1)
    else:
        assert ents[0].Data == b"somedata"


def test_multinode_step_ignores_local_messages():  # :29-61 with raft/util.go:49-51
    mn = StartMultiNode(1)
    s = MemoryStorage()
    mn.CreateGroup(1, Config(10, 1), s, peers=[1, 2, 3])
    rd = mn.Ready()  # bootstrap entries
    s.Append(rd[1].Entries)
    mn.Advance(rd)
    for t in (abi.HB_MSG_HUP, abi.HB_MSG_BEAT, abi.HB_MSG_UNREACHABLE, abi.HB_MSG_SNAP_STATUS):
        mn.Step(1, Message(Type=t, From=2))
    # nothing was stepped: the only content is the bootstrap entries, still not
    # applied because prevHardSt.Commit is 0 (raft/multinode.go:145-157)
    rd = mn.Ready()[1]
    assert rd.Messages == [] and rd.SoftState is None and rd.HardState == emptyState and rd.Entries == []
    assert [e.Index for e in rd.CommittedEntries] == [1, 2, 3]
    assert mn.Status(1).SoftState.RaftState == abi.HB_STATE_FOLLOWER


def test_conf_change_add_remove_keeps_progress():
    """ApplyConfChange on a leader (raft/multinode.go:239-262): add a node, its
    progress starts at (0, last+1); remove one; the leader keeps the others'."""
    mn = StartMultiNode(1)
    s = MemoryStorage()
    mn.CreateGroup(7, Config(10, 1), s, peers=[1, 2, 3])
    mn.Campaign(7)
    mn.Step(7, Message(Type=abi.HB_MSG_VOTE_RESP, From=2, Term=2))
    rd = mn.Ready()
    s.Append(rd[7].Entries)
    mn.Advance(rd)
    mn.Step(7, Message(Type=abi.HB_MSG_APP_RESP, From=2, Term=2, Index=4))
    assert mn.ApplyConfChange(7, ConfChangeAddNode, 4) == [1, 2, 3, 4]
    st = mn.Status(7)
    assert (st.Progress[2].match, st.Progress[2].next, st.Progress[2].state) == (4, 5, abi.HB_PR_REPLICATE)
    assert (st.Progress[4].match, st.Progress[4].next) == (0, 5)
    assert mn.ApplyConfChange(7, ConfChangeRemoveNode, 3) == [1, 2, 4]
    st = mn.Status(7)
    assert sorted(st.Progress) == [1, 2, 4] and st.Progress[2].match == 4


# ---------------------------------------------------------------------------------------
# randomised parity against the oracle
# ---------------------------------------------------------------------------------------
def _orc_msgs(o):
    return [(m.Type, m.To, m.From, m.Term, m.LogTerm, m.Index, m.Commit, bool(m.Reject), m.nents,
             m.ent_lo if m.nents else 0) for m in o.readMessages()]


def _dev_msgs(rd):
    out = []
    for m in rd.Messages:
        lo = m.Entries[0].Index if m.Entries else 0
        out.append((m.Type, m.To, m.From, m.Term, m.LogTerm, m.Index, m.Commit, m.Reject, len(m.Entries), lo))
    return out


@pytest.mark.parametrize("seed,n", [(1, 3), (2, 5), (3, 3)])
def test_random_multinode_vs_oracle(seed, n):
    from oracle.pyoracle import Msg, Raft
    rng = np.random.default_rng(seed)
    G, ROUNDS = 96, 60
    seen = dict(app_ents=0, leaders=0, commits=0, votes=0, beats=0)
    peers = list(range(1, n + 1))
    draws = rng.integers(0, 1 << 62, 1 << 14, dtype=np.uint64)
    mn = StartMultiNode(1, capacity=128, max_replicas=n, max_inflight=8)
    mn.SetRand(draws)
    gids = [1000 + 17 * g for g in range(G)]
    st = {}
    for gid in gids:
        s = MemoryStorage()
        mn.CreateGroup(gid, Config(election=3, heartbeat=1), s, peers=peers)
        # the bootstrap of raft/multinode.go:197-211: becomeFollower(1, None), one
        # entry per peer at term 1, committed = len(peers) — and r.Commit
        # (HardState.Commit) still 0 until the group's first Step (raft/raft.go:488)
        o = Raft(1, peers, ents=[(i, 1) for i in range(1, n + 1)], max_inflight=8,
                 election=3, heartbeat=1, draws=draws)
        o.r.Term = 1
        o.r.log.committed = n
        assert o.Commit == 0
        st[gid] = dict(s=s, o=o, data={}, applied=0, prev_hard=(1, 0, 0), prev_soft=(0, 0), seq=0)
    for rnd in range(ROUNDS):
        for gid in gids:
            d, o = st[gid], st[gid]["o"]
            if d.get("dead"):
                continue
            for _ in range(int(rng.integers(0, 4))):
                if o.fault:
                    break
                a = rng.random()
                frm = int(rng.integers(1, n + 2))  # n + 1 is a non-member
                member = frm <= n
                if a < 0.12 and (o.state != abi.HB_STATE_LEADER or rng.random() < 0.05):
                    mn.Campaign(gid)  # a leader's campaign panics (raft/raft.go:396): both report it
                    o.Step(Msg(abi.HB_MSG_HUP))
                elif a < 0.30:
                    d["seq"] += 1
                    data = f"{gid}-{d['seq']}".encode()
                    mn.Propose(gid, data)
                    o.Step(Msg(abi.HB_MSG_PROP, From=1, Entries=1))
                    d.setdefault("props", []).append(data)
                elif a < 0.45:
                    term = o.Term + (1 if rng.random() < 0.03 else 0)
                    rej = bool(rng.random() < 0.3)
                    mn.Step(gid, Message(Type=abi.HB_MSG_VOTE_RESP, From=frm, Term=term, Reject=rej))
                    if member:
                        o.Step(Msg(abi.HB_MSG_VOTE_RESP, From=frm, Term=term, Reject=rej))
                elif a < 0.80:
                    rej = bool(rng.random() < 0.15)
                    idx = int(rng.integers(0, o.lastIndex + 1))
                    hint = int(rng.integers(0, o.lastIndex + 1))
                    mn.Step(gid, Message(Type=abi.HB_MSG_APP_RESP, From=frm, Term=o.Term, Index=idx, Reject=rej,
                                         RejectHint=hint))
                    if member:
                        o.Step(Msg(abi.HB_MSG_APP_RESP, From=frm, Term=o.Term, Index=idx, Reject=rej,
                                   RejectHint=hint))
                elif a < 0.92:
                    mn.Step(gid, Message(Type=abi.HB_MSG_HEARTBEAT_RESP, From=frm, Term=o.Term))
                    if member:
                        o.Step(Msg(abi.HB_MSG_HEARTBEAT_RESP, From=frm, Term=o.Term))
                elif a < 0.97:
                    mn.ReportUnreachable(frm, gid)
                    if member:
                        o.Step(Msg(abi.HB_MSG_UNREACHABLE, From=frm))
                elif member and frm != 1 and o.state == abi.HB_STATE_LEADER and \
                        o.pr(frm).State == abi.HB_PR_SNAPSHOT:
                    fail = bool(rng.random() < 0.5)
                    mn.ReportSnapshot(frm, gid, fail)
                    o.Step(Msg(abi.HB_MSG_SNAP_STATUS, From=frm, Reject=fail))
        if rnd % 5 == 4:
            mn.Tick()
            for gid in gids:
                st[gid]["o"].tick()
        rds = mn.Ready()
        for gid in gids:
            d, o = st[gid], st[gid]["o"]
            if d.get("dead"):
                continue
            if o.fault:
                assert gid in rds and rds[gid].fault == o.fault, f"group {gid}: fault"
                d["dead"] = True
                continue
            om = _orc_msgs(o)
            hard = (o.Term, o.Vote, o.Commit)  # r.HardState: r.Commit, not raftLog.committed
            soft = (o.lead, o.state)
            unstable_lo = d["s"].LastIndex() + 1
            committed_lo = max(d["applied"] + 1, d["s"].FirstIndex())
            want_any = bool(om) or hard != d["prev_hard"] or soft != d["prev_soft"] or \
                o.lastIndex >= unstable_lo or o.committed >= committed_lo
            ctx = f"seed {seed} round {rnd} group {gid}"
            if not want_any:
                assert gid not in rds, ctx
                continue
            rd = rds[gid]
            assert rd.fault == 0, ctx
            assert _dev_msgs(rd) == om, f"{ctx}: messages\n dev {_dev_msgs(rd)}\n ora {om}"
            assert rd.HardState == (HardState(*hard) if hard != d["prev_hard"] else emptyState), ctx
            assert rd.SoftState == (SoftState(*soft) if soft != d["prev_soft"] else None), ctx
            assert [(e.Index, e.Term) for e in rd.Entries] == \
                   [(i, o.term(i)) for i in range(unstable_lo, o.lastIndex + 1)], ctx
            assert [(e.Index, e.Term) for e in rd.CommittedEntries] == \
                   [(i, o.term(i)) for i in range(committed_lo, o.committed + 1)], ctx
            # payloads: proposals in order, noops empty
            for e in rd.Entries:
                if e.Data is not None:
                    d["data"][e.Index] = e.Data
            for m in rd.Messages:
                for e in m.Entries:
                    if m.Type == abi.HB_MSG_APP and e.Data is not None:
                        assert d["data"][e.Index] == e.Data, ctx
            seen["app_ents"] += sum(1 for m in rd.Messages if m.Type == abi.HB_MSG_APP and m.Entries)
            seen["votes"] += sum(1 for m in rd.Messages if m.Type == abi.HB_MSG_VOTE)
            seen["beats"] += sum(1 for m in rd.Messages if m.Type == abi.HB_MSG_HEARTBEAT)
            seen["commits"] += len(rd.CommittedEntries)
            seen["leaders"] += int(rd.SoftState is not None and rd.SoftState.RaftState == StateLeader)
            d["s"].Append(rd.Entries)
            if rd.SoftState is not None:
                d["prev_soft"] = soft
            if rd.HardState != emptyState:
                d["prev_hard"] = hard
            if d["prev_hard"][2]:
                d["applied"] = d["prev_hard"][2]
        mn.Advance(rds)
    assert min(seen.values()) > 0, seen  # every kind of Ready content was compared
    # every accepted proposal's payload reached storage in proposal order
    for gid in gids:
        s = st[gid]["s"]
        ents, err = s.Entries(n + 1, s.LastIndex() + 1) if s.LastIndex() > n else ([], None)
        got = [e.Data for e in (ents or []) if e.Data is not None]
        props = st[gid].get("props", [])
        it = iter(props)
        assert all(any(p == g for p in it) for g in got), f"group {gid}: payload order"


# ---------------------------------------------------------------- storage compaction / snapshots
def _lagging_leader(**kw):
    """Group 1 on node 1 with peers 1, 2, 3: node 1 leads at term 2, follower 2
    acks every entry, follower 3 never answers (Probe, paused, Next 4).  Four
    proposals later the log is 1..8, all committed, all in storage."""
    s = MemoryStorage()
    mn = StartMultiNode(1, **kw)
    mn.CreateGroup(1, Config(10, 1), s, peers=[1, 2, 3])

    def cycle():
        rds = mn.Ready()
        if 1 in rds:
            s.Append(rds[1].Entries)
            mn.Advance(rds)
        return rds.get(1)
    cycle()
    mn.Campaign(1)
    cycle()
    mn.Step(1, Message(Type=abi.HB_MSG_VOTE_RESP, From=2, To=1, Term=2))
    cycle()  # leader: noop 4, MsgApp(3, [4]) to 2 and 3
    mn.Step(1, Message(Type=abi.HB_MSG_APP_RESP, From=2, To=1, Term=2, Index=4))
    cycle()
    for k in range(4):
        mn.Propose(1, b"x%d" % k)
        cycle()
        mn.Step(1, Message(Type=abi.HB_MSG_APP_RESP, From=2, To=1, Term=2, Index=5 + k))
        cycle()
    st = mn.Status(1)
    assert st.HardState.Commit == 8 and st.Progress[3].state == abi.HB_PR_PROBE and st.Progress[3].next == 4
    return mn, s, cycle


def test_compacted_log_sends_snapshot_to_lagging_follower():
    """Compact + CreateSnapshot on the leader's storage after CreateGroup: the
    next sendAppend to the lagging follower needs a snapshot (Next 4 <
    firstIndex 9, raft/raft.go:246-260, 715-717) — a MsgSnap carrying the
    storage's snapshot, and the follower's Progress becomes Snapshot(8)."""
    mn, s, cycle = _lagging_leader()
    snap, err = s.CreateSnapshot(8, [1, 2, 3], b"state@8")
    assert err is None and snap.Index == 8 and snap.Term == 2
    assert s.Compact(8) is None
    mn.Tick()  # MsgBeat -> bcastHeartbeat resumes every peer
    rd = cycle()
    assert [(m.Type, m.To) for m in rd.Messages] == [(abi.HB_MSG_HEARTBEAT, 2), (abi.HB_MSG_HEARTBEAT, 3)]
    mn.Step(1, Message(Type=abi.HB_MSG_HEARTBEAT_RESP, From=3, To=1, Term=2))
    rd = cycle()
    assert rd.Messages == [Message(Type=abi.HB_MSG_SNAP, To=3, From=1, Term=2,
                                   Snapshot=Snapshot(Index=8, Term=2, Nodes=[1, 2, 3], Data=b"state@8"))]
    p3 = mn.Status(1).Progress[3]
    assert p3.state == abi.HB_PR_SNAPSHOT and p3.pending_snapshot == 8
    mn.Stop()


def test_compaction_after_send_keeps_the_sent_entries():
    """A MsgApp is built from the log when the reference sends it (raft.go:265):
    a heartbeat response stepped before Compact makes the leader send entries
    4..8 to the lagging follower; compacting them away before the Ready must not
    change that message.  The follower's next sendAppend is then a MsgSnap."""
    mn, s, cycle = _lagging_leader()
    mn.Tick()
    cycle()
    mn.Step(1, Message(Type=abi.HB_MSG_HEARTBEAT_RESP, From=3, To=1, Term=2))
    snap, err = s.CreateSnapshot(8, [1, 2, 3], None)
    assert err is None
    assert s.Compact(8) is None
    rd = cycle()
    assert len(rd.Messages) == 1
    m = rd.Messages[0]
    assert (m.Type, m.To, m.Index, m.LogTerm, m.Commit) == (abi.HB_MSG_APP, 3, 3, 1, 8)
    assert [(e.Index, e.Term) for e in m.Entries] == [(4, 2), (5, 2), (6, 2), (7, 2), (8, 2)]
    assert [e.Data for e in m.Entries] == [None, b"x0", b"x1", b"x2", b"x3"]
    # Probe: paused after the send; the next heartbeat round resumes it and the
    # response finds Next 4 below firstIndex 9
    mn.Tick()
    cycle()
    mn.Step(1, Message(Type=abi.HB_MSG_HEARTBEAT_RESP, From=3, To=1, Term=2))
    rd = cycle()
    assert [(m.Type, m.To, m.Snapshot.Index) for m in rd.Messages] == [(abi.HB_MSG_SNAP, 3, 8)]
    mn.Stop()


def test_max_size_per_msg_cuts_msgapp_entries():
    """MaxSizePerMsg finite (etcdserver runs with 1 MiB, etcdserver/raft.go:229):
    sendAppend sends entries(pr.Next, maxMsgSize) cut by limitSize
    (raft/raft.go:265, raft/util.go:97-110) — the device decides how far the
    follower's Next moves, the host sends exactly those entries."""
    from etcd_amd.multinode import entry_size
    s = MemoryStorage()
    mn = StartMultiNode(1, max_msg_size=60)
    mn.CreateGroup(1, Config(10, 1), s, peers=[1, 2])

    def cycle():
        rds = mn.Ready()
        if 1 in rds:
            s.Append(rds[1].Entries)
            mn.Advance(rds)
        return rds.get(1)
    cycle()
    mn.Campaign(1)
    cycle()
    mn.Step(1, Message(Type=abi.HB_MSG_VOTE_RESP, From=2, To=1, Term=2))
    rd = cycle()  # leader; noop 3; MsgApp(2, [3]) to 2 (Probe: paused)
    assert [(m.Type, m.Index, len(m.Entries)) for m in rd.Messages] == [(abi.HB_MSG_APP, 2, 1)]
    payloads = [b"a" * 10, b"b" * 20, b"c" * 30, None, b"e" * 40, b"f" * 3]
    for p in payloads:
        mn.Propose(1, p)
        assert cycle().Messages == []  # follower 2 is paused in Probe
    log = [Entry(Term=2, Index=3)] + [Entry(Term=2, Index=4 + i, Data=p) for i, p in enumerate(payloads)]
    # the ack of the noop: Probe -> Replicate, Next = 4; commit 3 -> bcastAppend
    mn.Step(1, Message(Type=abi.HB_MSG_APP_RESP, From=2, To=1, Term=2, Index=3))
    sent = []
    nxt = 4
    for _ in range(6):
        rd = cycle()
        apps = [m for m in rd.Messages if m.Type == abi.HB_MSG_APP] if rd else []
        if not apps:
            break
        m = apps[0]
        assert m.Index == nxt - 1
        ents = log[nxt - 3:]
        if not ents:  # the commit's bcastAppend past the last entry: an empty MsgApp
            assert m.Entries == []
            break
        size, k = entry_size(ents[0]), 1
        while k < len(ents) and size + entry_size(ents[k]) <= 60:
            size += entry_size(ents[k])
            k += 1
        assert [(e.Index, e.Data) for e in m.Entries] == [(e.Index, e.Data) for e in ents[:k]]
        sent.append(k)
        nxt += k
        mn.Step(1, Message(Type=abi.HB_MSG_APP_RESP, From=2, To=1, Term=2, Index=nxt - 1))
    assert sum(sent) == len(payloads) and len(sent) > 1
    st = mn.Status(1)
    assert st.Progress[2].match == 3 + len(payloads)
    mn.Stop()


# ---------------------------------------------------------------- bulk ingestion + host threads
def test_bulk_and_threaded_ready_equal_per_call():
    """hbn_step_many / hbn_propose_many with the node's host threads (event
    replay, Ready assembly and Advance split over workers by group) produce the
    same Ready as one hbn_step / hbn_propose call per message on one thread, on
    every cycle: 6,000 groups (above the parallel thresholds), shuffled acks,
    heartbeat responses, stale and rejected acks, and local / lower-term
    messages that take the single-message path inside the bulk call."""
    import random
    G, ids = 6000, [1, 2, 3]
    a = StartMultiNode(1, capacity=G + 8, max_batch=1 << 16)
    b = StartMultiNode(1, capacity=G + 8, max_batch=1 << 16)
    a.SetThreads(8)
    b.SetThreads(1)
    sa = {g: MemoryStorage() for g in range(1, G + 1)}
    sb = {g: MemoryStorage() for g in range(1, G + 1)}
    for g in range(1, G + 1):
        a.CreateGroup(g, Config(10, 1), sa[g], peers=ids)
        b.CreateGroup(g, Config(10, 1), sb[g], peers=ids)

    def cycle():
        ra, rb = a.Ready(), b.Ready()
        assert ra == rb
        for mn, st, rds in ((a, sa, ra), (b, sb, rb)):
            for g, rd in rds.items():
                st[g].Append(rd.Entries)
            mn.Advance(rds)
        return ra
    cycle()
    for g in range(1, G + 1):
        a.Campaign(g)
        b.Campaign(g)
    cycle()
    votes = [(g, Message(Type=abi.HB_MSG_VOTE_RESP, From=f, To=1, Term=2)) for g in range(1, G + 1) for f in (2, 3)]
    assert a.StepMany(votes) == len(votes)
    for g, m in votes:
        b.Step(g, m)
    cycle()
    rng = random.Random(5)
    for r in range(4):
        props = [(g, b"r%d-%d" % (r, g) if rng.random() < 0.9 else None) for g in range(1, G + 1) if rng.random() < 0.8]
        assert a.ProposeMany(props) == len(props)
        for g, d in props:
            b.Propose(g, d)
        rd = cycle()
        msgs = []
        for g in range(1, G + 1):
            last = sa[g].LastIndex()
            for f in (2, 3):
                u = rng.random()
                if u < 0.7:
                    msgs.append((g, Message(Type=abi.HB_MSG_APP_RESP, From=f, To=1, Term=2, Index=last)))
                elif u < 0.8:
                    msgs.append((g, Message(Type=abi.HB_MSG_HEARTBEAT_RESP, From=f, To=1, Term=2)))
                elif u < 0.88:
                    msgs.append((g, Message(Type=abi.HB_MSG_APP_RESP, From=f, To=1, Term=2, Index=last - 1,
                                            Reject=True, RejectHint=last - 2)))
                elif u < 0.94:
                    msgs.append((g, Message(Type=abi.HB_MSG_APP_RESP, From=f, To=1, Term=1, Index=1)))  # lower term
                else:
                    msgs.append((g, Message(Type=abi.HB_MSG_BEAT, From=f, To=1)))  # local: ignored by Step
        rng.shuffle(msgs)
        assert a.StepMany(msgs) == len(msgs)
        for g, m in msgs:
            b.Step(g, m)
        cycle()
    def st(mn, g):
        x = mn.Status(g)
        return (x.HardState, x.SoftState, x.Applied,
                {k: (p.match, p.next, p.state, p.paused, p.ins_count) for k, p in x.Progress.items()})
    for g in rng.sample(range(1, G + 1), 50):
        assert st(a, g) == st(b, g)
    a.Stop()
    b.Stop()


def test_bulk_step_stops_at_the_first_error():
    """hbn_step_many reports the messages it took before an error, as the same
    sequence of hbn_step calls would have stopped: a message for a missing
    group raises ENOGROUP and nothing after it is taken."""
    from etcd_amd.multinode import HbnError
    mn = StartMultiNode(1, capacity=16)
    s = MemoryStorage()
    mn.CreateGroup(1, Config(10, 1), s, peers=[1, 2, 3])
    items = [(1, Message(Type=abi.HB_MSG_VOTE_RESP, From=2, To=1, Term=1))] * 3 + \
            [(99, Message(Type=abi.HB_MSG_VOTE_RESP, From=2, To=1, Term=1))] + \
            [(1, Message(Type=abi.HB_MSG_VOTE_RESP, From=3, To=1, Term=1))]
    with pytest.raises(HbnError) as ei:
        mn.StepMany(items)
    assert "hbn_step_many" in str(ei.value)
    mn.Stop()


def test_bulk_step_after_a_flush_faults_the_group():
    """A bulk call longer than max_batch: the batch is stepped when it fills, and
    that step can fault a group (here "need non-empty snapshot", raft/raft.go:
    246-256: the leader's storage was compacted without a snapshot and a lagging
    follower's heartbeat response makes it send one).  hbn_step_many must stop
    where the same hbn_step calls stop: the message whose push flushed the batch
    is taken (it was checked before the flush), the next one for the faulted
    group raises HBN_EPANIC, and done counts the messages before it."""
    from etcd_amd.multinode import RaftPanic
    hb2 = lambda: (1, Message(Type=abi.HB_MSG_HEARTBEAT_RESP, From=2, To=1, Term=2))
    items = [(1, Message(Type=abi.HB_MSG_HEARTBEAT_RESP, From=3, To=1, Term=2)), hb2(), hb2(), hb2(), hb2()]
    got = []
    for bulk in (False, True):
        mn, s, cycle = _lagging_leader(max_batch=2)
        assert s.Compact(8) is None  # no CreateSnapshot: the storage's snapshot stays empty
        mn.Tick()  # MsgBeat -> bcastHeartbeat resumes follower 3
        cycle()
        taken = 0
        with pytest.raises(RaftPanic) as ei:
            if bulk:
                mn.StepMany(items)
            else:
                for g, m in items:
                    mn.Step(g, m)
                    taken += 1
        got.append(ei.value.done if bulk else taken)
        rd = mn.Ready()[1]
        assert rd.fault == abi.HB_FAULT_EMPTY_SNAPSHOT
        mn.Stop()
    assert got == [3, 3]


def test_member_limit_is_unsupported_not_invalid():
    """The engine keeps at most max_replicas (<= 7) members per group; the
    reference has no such limit (raft/raft.go:729-738).  CreateGroup with more
    peers, and an ApplyConfChange adding one past the limit, return
    HBN_EUNSUPPORTED and leave the group as it was."""
    from etcd_amd.multinode import HBN_EUNSUPPORTED, HbnError
    mn = StartMultiNode(1, capacity=8, max_replicas=3)
    with pytest.raises(HbnError) as ei:
        mn.CreateGroup(1, Config(10, 1), MemoryStorage(), peers=[1, 2, 3, 4])
    assert ei.value.code == HBN_EUNSUPPORTED
    s = MemoryStorage()
    mn.CreateGroup(2, Config(10, 1), s, peers=[1, 2, 3])
    with pytest.raises(HbnError) as ei:
        mn.ApplyConfChange(2, ConfChangeAddNode, 4)
    assert ei.value.code == HBN_EUNSUPPORTED
    assert mn.ApplyConfChange(2, ConfChangeRemoveNode, 3) == [1, 2]
    assert mn.ApplyConfChange(2, ConfChangeAddNode, 4) == [1, 2, 4]
    mn.Stop()
    mn = StartMultiNode(1, capacity=8)  # max_replicas 7
    with pytest.raises(HbnError) as ei:
        mn.CreateGroup(1, Config(10, 1), MemoryStorage(), peers=list(range(1, 9)))
    assert ei.value.code == HBN_EUNSUPPORTED
    mn.CreateGroup(2, Config(10, 1), MemoryStorage(), peers=list(range(1, 8)))
    with pytest.raises(HbnError) as ei:
        mn.ApplyConfChange(2, ConfChangeAddNode, 8)
    assert ei.value.code == HBN_EUNSUPPORTED
    mn.Stop()
