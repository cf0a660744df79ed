"""Python mirror of raft.MultiNode over the MI355X engine (include/hbnode.h,
etcd_amd/libhbnode.so).

Names, argument meaning and results follow the reference's Go API
(raft/multinode.go:12-49, raft/storage.go, raft/node.go Ready) so the tests
read like the reference's own multinode_test.go / storage_test.go.  The
library is the product path; there is no fallback: a missing library raises.

    storage = MemoryStorage()
    mn = StartMultiNode(1)
    mn.CreateGroup(1, Config(election=10, heartbeat=1), storage, peers=[1])
    mn.Campaign(1)
    rds = mn.Ready()            # {group: Ready}, {} when nothing is ready
    storage.Append(rds[1].Entries)
    mn.Advance(rds)
"""
import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional

from . import abi
from .hipbatch import lib as _engine_lib

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("HBN_LIB", os.path.join(_HERE, "libhbnode.so"))
_lib = None

HBN_ENOGROUP = -10
HBN_EEXIST = -11
HBN_EAGAIN = -12
HBN_EUNSUPPORTED = -13
HBN_EPANIC = -14
HBN_ECOMPACTED = -20
HBN_EUNAVAILABLE = -21
HBN_ESNAPOUTOFDATE = -22
HBN_FAULT_DOUBLE_CONF = 32

EntryNormal, EntryConfChange = 0, 1
ConfChangeAddNode, ConfChangeRemoveNode, ConfChangeUpdateNode = 0, 1, 2
StateFollower, StateCandidate, StateLeader = abi.HB_STATE_FOLLOWER, abi.HB_STATE_CANDIDATE, abi.HB_STATE_LEADER
NO_LIMIT = abi.HB_NO_LIMIT


class hbn_entry(C.Structure):
    _fields_ = [("term", C.c_uint64), ("index", C.c_uint64), ("type", C.c_uint32), ("has_data", C.c_uint32),
                ("data", C.c_void_p), ("data_len", C.c_uint64)]


class hbn_hard_state(C.Structure):
    _fields_ = [("term", C.c_uint64), ("vote", C.c_uint64), ("commit", C.c_uint64)]


class hbn_snapshot(C.Structure):
    _fields_ = [("index", C.c_uint64), ("term", C.c_uint64), ("nodes", C.POINTER(C.c_uint64)),
                ("n_nodes", C.c_uint32), ("has_data", C.c_uint32), ("data", C.c_void_p), ("data_len", C.c_uint64)]


class hbn_message(C.Structure):
    _fields_ = [("type", C.c_uint32), ("reject", C.c_uint32), ("to", C.c_uint64), ("from_", C.c_uint64),
                ("term", C.c_uint64), ("log_term", C.c_uint64), ("index", C.c_uint64), ("commit", C.c_uint64),
                ("reject_hint", C.c_uint64), ("entries", C.POINTER(hbn_entry)), ("n_entries", C.c_uint64),
                ("snapshot", hbn_snapshot)]


class hbn_group_ready(C.Structure):
    _fields_ = [("group", C.c_uint64), ("has_soft_state", C.c_uint32), ("raft_state", C.c_uint32),
                ("lead", C.c_uint64), ("hard_state", hbn_hard_state), ("snapshot", hbn_snapshot),
                ("entries", C.POINTER(hbn_entry)), ("n_entries", C.c_uint64),
                ("committed_entries", C.POINTER(hbn_entry)), ("n_committed", C.c_uint64),
                ("messages", C.POINTER(hbn_message)), ("n_messages", C.c_uint64),
                ("fault", C.c_uint32), ("pad", C.c_uint32)]


class hbn_group_status(C.Structure):
    _fields_ = [("id", C.c_uint64), ("hard_state", hbn_hard_state), ("lead", C.c_uint64),
                ("raft_state", C.c_uint32), ("n_progress", C.c_uint32), ("applied", C.c_uint64),
                ("progress_id", C.c_uint64 * abi.HB_MAX_REPLICAS),
                ("progress", abi.hb_progress * abi.HB_MAX_REPLICAS)]


class hbn_config(C.Structure):
    _fields_ = [("election_tick", C.c_uint32), ("heartbeat_tick", C.c_uint32), ("applied", C.c_uint64)]


class RaftPanic(RuntimeError):
    """The reference panics here (raftLogger.Panicf / a Go runtime panic)."""


class HbnError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__(f"{fn} failed: {code} ({lib().hbn_last_error().decode()})")
        self.code = code


# ---- Go value types ----------------------------------------------------------
@dataclass
class Entry:
    Term: int = 0
    Index: int = 0
    Type: int = EntryNormal
    Data: Optional[bytes] = None  # None = Go's nil


@dataclass
class HardState:
    Term: int = 0
    Vote: int = 0
    Commit: int = 0


emptyState = HardState()


@dataclass
class SoftState:
    Lead: int = 0
    RaftState: int = StateFollower


@dataclass
class Snapshot:
    Index: int = 0
    Term: int = 0
    Nodes: List[int] = field(default_factory=list)
    Data: Optional[bytes] = None


@dataclass
class Message:
    Type: int = 0
    To: int = 0
    From: int = 0
    Term: int = 0
    LogTerm: int = 0
    Index: int = 0
    Entries: List[Entry] = field(default_factory=list)
    Commit: int = 0
    Snapshot: Snapshot = field(default_factory=Snapshot)
    Reject: bool = False
    RejectHint: int = 0


@dataclass
class Ready:
    SoftState: Optional[SoftState] = None
    HardState: HardState = field(default_factory=HardState)
    Entries: List[Entry] = field(default_factory=list)
    Snapshot: Snapshot = field(default_factory=Snapshot)
    CommittedEntries: List[Entry] = field(default_factory=list)
    Messages: List[Message] = field(default_factory=list)
    fault: int = 0


@dataclass
class Config:
    election: int = 10
    heartbeat: int = 1
    applied: int = 0


@dataclass
class Status:
    ID: int
    HardState: HardState
    SoftState: SoftState
    Applied: int
    Progress: dict


# ---- library ----------------------------------------------------------------------
def lib():
    global _lib
    if _lib is None:
        _engine_lib()  # libhipbatch first (same directory, ABI-checked)
        if not os.path.exists(_LIB_PATH):
            raise ImportError(f"{_LIB_PATH} is not built (make -C etcd_amd/csrc)")
        L = C.CDLL(_LIB_PATH)
        P, u64, u32, vp = C.POINTER, C.c_uint64, C.c_uint32, C.c_void_p
        sig = {
            "hbn_last_error": (C.c_char_p, []),
            "hbn_entry_size": (u64, [P(hbn_entry)]),
            "hbn_storage_new": (C.c_int, [P(vp)]),
            "hbn_storage_new_with_entries": (C.c_int, [P(hbn_entry), u64, P(vp)]),
            "hbn_storage_free": (C.c_int, [vp]),
            "hbn_storage_initial_state": (C.c_int, [vp, P(hbn_hard_state), P(u64), u32, P(u32)]),
            "hbn_storage_set_hard_state": (C.c_int, [vp, P(hbn_hard_state)]),
            "hbn_storage_entries": (C.c_int, [vp, u64, u64, u64, P(P(hbn_entry)), P(u64)]),
            "hbn_storage_term": (C.c_int, [vp, u64, P(u64)]),
            "hbn_storage_last_index": (C.c_int, [vp, P(u64)]),
            "hbn_storage_first_index": (C.c_int, [vp, P(u64)]),
            "hbn_storage_snapshot": (C.c_int, [vp, P(hbn_snapshot)]),
            "hbn_storage_apply_snapshot": (C.c_int, [vp, P(hbn_snapshot)]),
            "hbn_storage_create_snapshot": (C.c_int, [vp, u64, P(u64), u32, vp, u64, P(hbn_snapshot)]),
            "hbn_storage_compact": (C.c_int, [vp, u64]),
            "hbn_storage_append": (C.c_int, [vp, P(hbn_entry), u64]),
            "hbn_start": (C.c_int, [C.c_int, u64, u32, u32, u32, u64, u64, P(vp)]),
            "hbn_stop": (C.c_int, [vp]),
            "hbn_create_group": (C.c_int, [vp, u64, P(hbn_config), vp, P(u64), u32]),
            "hbn_remove_group": (C.c_int, [vp, u64]),
            "hbn_tick": (C.c_int, [vp]),
            "hbn_set_rand": (C.c_int, [vp, u64, u64, P(u64)]),
            "hbn_campaign": (C.c_int, [vp, u64]),
            "hbn_propose": (C.c_int, [vp, u64, vp, u64]),
            "hbn_propose_conf_change": (C.c_int, [vp, u64, u64, u32, u64, vp, u64]),
            "hbn_step": (C.c_int, [vp, u64, P(hbn_message)]),
            "hbn_step_many": (C.c_int, [vp, u64, P(u64), P(hbn_message), P(u64)]),
            "hbn_propose_many": (C.c_int, [vp, u64, P(u64), P(vp), P(u64), P(u64)]),
            "hbn_set_threads": (C.c_int, [vp, u32]),
            "hbn_profile": (C.c_int, [vp, P(C.c_double), u32, P(u32)]),
            "hbn_report_unreachable": (C.c_int, [vp, u64, u64]),
            "hbn_report_snapshot": (C.c_int, [vp, u64, u64, C.c_int]),
            "hbn_apply_conf_change": (C.c_int, [vp, u64, u32, u64, P(u64), P(u32)]),
            "hbn_ready": (C.c_int, [vp, P(P(hbn_group_ready)), P(u64)]),
            "hbn_advance": (C.c_int, [vp, P(u64), u64]),
            "hbn_status": (C.c_int, [vp, u64, P(hbn_group_status)]),
            "hbn_engine": (vp, [vp]),
            # include/hbroute.h: owner routing across a node's GPUs (etcd_amd/shard.py NativeRouter)
            "hbn_owner": (u32, [u64, u32]),
            "hbn_router_create": (C.c_int, [vp, u64, u32, u32, P(vp)]),
            "hbn_router_destroy": (C.c_int, [vp]),
            "hbn_router_local_count": (u64, [vp, u32]),
            "hbn_router_local_ids": (C.c_int, [vp, u32, vp]),
            "hbn_route": (C.c_int, [vp, vp, u64, vp, P(u64)]),
            "hbn_route_take": (C.c_int, [vp, vp, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def _check(fn, rc, ok=(0,)):
    if rc in ok:
        return rc
    if rc == HBN_EPANIC:
        raise RaftPanic(lib().hbn_last_error().decode())
    raise HbnError(fn, rc)


def _bytes(p, n):
    return C.string_at(p, n) if n else b""


def _entry_out(e):
    return Entry(Term=e.term, Index=e.index, Type=e.type, Data=_bytes(e.data, e.data_len) if e.has_data else None)


def _entries_out(p, n):
    return [_entry_out(p[i]) for i in range(n)]


def _snap_out(s):
    return Snapshot(Index=s.index, Term=s.term, Nodes=[s.nodes[i] for i in range(s.n_nodes)],
                    Data=_bytes(s.data, s.data_len) if s.has_data else None)


def _snap_in(snap):
    """pb.Snapshot in C layout; returns (struct, buffers to keep alive)."""
    nodes = (C.c_uint64 * max(1, len(snap.Nodes)))(*snap.Nodes)
    s = hbn_snapshot(snap.Index, snap.Term, C.cast(nodes, C.POINTER(C.c_uint64)), len(snap.Nodes),
                     snap.Data is not None, None, 0)
    buf = None
    if snap.Data:
        buf = C.create_string_buffer(bytes(snap.Data), len(snap.Data))
        s.data, s.data_len = C.cast(buf, C.c_void_p), len(snap.Data)
    return s, (nodes, buf)


class _EntryArray:
    """Entries in C layout (payload buffers kept alive with the array)."""

    def __init__(self, ents):
        self.bufs = []
        self.arr = (hbn_entry * max(1, len(ents)))()
        for i, e in enumerate(ents):
            a = self.arr[i]
            a.term, a.index, a.type = e.Term, e.Index, e.Type
            a.has_data = e.Data is not None
            if e.Data:
                b = C.create_string_buffer(bytes(e.Data), len(e.Data))
                self.bufs.append(b)
                a.data, a.data_len = C.cast(b, C.c_void_p), len(e.Data)
        self.n = len(ents)


def entry_size(e):
    """Entry.Size() (gogo)."""
    a = _EntryArray([e])
    return lib().hbn_entry_size(a.arr)


# ---- MemoryStorage -----------------------------------------------------------------
class MemoryStorage:
    """raft.MemoryStorage (raft/storage.go:63-248)."""

    def __init__(self, ents=None):
        self.p = C.c_void_p()
        if ents is None:
            _check("hbn_storage_new", lib().hbn_storage_new(C.byref(self.p)))
        else:  # &MemoryStorage{ents: ents} (the reference tests' literal)
            a = _EntryArray(ents)
            _check("hbn_storage_new_with_entries", lib().hbn_storage_new_with_entries(a.arr, a.n, C.byref(self.p)))

    def __del__(self):
        try:
            if self.p:
                lib().hbn_storage_free(self.p)
        except Exception:
            pass

    def InitialState(self):
        hs, n = hbn_hard_state(), C.c_uint32()
        nodes = (C.c_uint64 * abi.HB_MAX_REPLICAS * 4)()
        _check("hbn_storage_initial_state", lib().hbn_storage_initial_state(
            self.p, C.byref(hs), C.cast(nodes, C.POINTER(C.c_uint64)), len(nodes), C.byref(n)))
        flat = C.cast(nodes, C.POINTER(C.c_uint64))
        return HardState(hs.term, hs.vote, hs.commit), [flat[i] for i in range(n.value)]

    def SetHardState(self, st):
        hs = hbn_hard_state(st.Term, st.Vote, st.Commit)
        _check("hbn_storage_set_hard_state", lib().hbn_storage_set_hard_state(self.p, C.byref(hs)))

    def Entries(self, lo, hi, max_size=NO_LIMIT):
        """Returns (entries, err) with err in {None, 'ErrCompacted', 'ErrUnavailable'}."""
        out, n = C.POINTER(hbn_entry)(), C.c_uint64()
        rc = lib().hbn_storage_entries(self.p, lo, hi, max_size, C.byref(out), C.byref(n))
        err = {HBN_ECOMPACTED: "ErrCompacted", HBN_EUNAVAILABLE: "ErrUnavailable"}.get(rc)
        if err:
            return None, err
        _check("hbn_storage_entries", rc)
        return (_entries_out(out, n.value) if n.value else None), None

    def Term(self, i):
        t = C.c_uint64()
        rc = lib().hbn_storage_term(self.p, i, C.byref(t))
        if rc == HBN_ECOMPACTED:
            return 0, "ErrCompacted"
        _check("hbn_storage_term", rc)
        return t.value, None

    def LastIndex(self):
        v = C.c_uint64()
        _check("hbn_storage_last_index", lib().hbn_storage_last_index(self.p, C.byref(v)))
        return v.value

    def FirstIndex(self):
        v = C.c_uint64()
        _check("hbn_storage_first_index", lib().hbn_storage_first_index(self.p, C.byref(v)))
        return v.value

    def Snapshot(self):
        s = hbn_snapshot()
        _check("hbn_storage_snapshot", lib().hbn_storage_snapshot(self.p, C.byref(s)))
        return _snap_out(s)

    def ApplySnapshot(self, snap):
        s, keep = _snap_in(snap)
        _check("hbn_storage_apply_snapshot", lib().hbn_storage_apply_snapshot(self.p, C.byref(s)))

    def CreateSnapshot(self, i, nodes, data):
        """nodes None = a nil *ConfState.  Returns (Snapshot, err)."""
        arr = (C.c_uint64 * max(1, len(nodes or [])))(*(nodes or []))
        out = hbn_snapshot()
        buf = C.create_string_buffer(bytes(data), len(data)) if data is not None else None
        rc = lib().hbn_storage_create_snapshot(self.p, i, C.cast(arr, C.POINTER(C.c_uint64)) if nodes is not None
                                               else None, len(nodes or []), C.cast(buf, C.c_void_p) if buf else None,
                                               len(data or b""), C.byref(out))
        if rc == HBN_ESNAPOUTOFDATE:
            return Snapshot(), "ErrSnapOutOfDate"
        _check("hbn_storage_create_snapshot", rc)
        return _snap_out(out), None

    def Compact(self, i):
        rc = lib().hbn_storage_compact(self.p, i)
        if rc == HBN_ECOMPACTED:
            return "ErrCompacted"
        _check("hbn_storage_compact", rc)
        return None

    def Append(self, ents):
        a = _EntryArray(ents or [])
        _check("hbn_storage_append", lib().hbn_storage_append(self.p, a.arr, a.n))
        return None


NewMemoryStorage = MemoryStorage


# ---- MultiNode -------------------------------------------------------------------------
class MultiNode:
    """raft.MultiNode (raft/multinode.go:12-49) on one GPU."""

    def __init__(self, id, capacity=1 << 12, max_replicas=abi.HB_MAX_REPLICAS, max_inflight=256,
                 max_msg_size=NO_LIMIT, max_batch=1 << 16, device=0):
        self.id = id
        self.p = C.c_void_p()
        self._storages = {}  # keep the caller's storages alive while their group exists
        _check("hbn_start", lib().hbn_start(device, id, capacity, max_replicas, max_inflight, max_msg_size,
                                            max_batch, C.byref(self.p)))

    def Stop(self):
        if self.p:
            lib().hbn_stop(self.p)
            self.p = C.c_void_p()

    def __del__(self):
        try:
            self.Stop()
        except Exception:
            pass

    def CreateGroup(self, group, config, storage, peers=()):
        cfg = hbn_config(config.election, config.heartbeat, config.applied)
        ids = (C.c_uint64 * max(1, len(peers)))(*peers)
        _check("hbn_create_group", lib().hbn_create_group(self.p, group, C.byref(cfg), storage.p, ids, len(peers)))
        self._storages[group] = storage

    def RemoveGroup(self, group):
        _check("hbn_remove_group", lib().hbn_remove_group(self.p, group))
        self._storages.pop(group, None)

    def Tick(self):
        _check("hbn_tick", lib().hbn_tick(self.p))

    def SetRand(self, draws, first=0):
        """The node's rand.New(rand.NewSource(id)).Int() stream (see hb_set_rand)."""
        arr = (C.c_uint64 * max(1, len(draws)))(*[int(d) for d in draws])
        _check("hbn_set_rand", lib().hbn_set_rand(self.p, first, len(draws), arr))

    def Campaign(self, group):
        _check("hbn_campaign", lib().hbn_campaign(self.p, group))

    def Propose(self, group, data):
        buf = C.create_string_buffer(bytes(data), max(1, len(data))) if data is not None else None
        _check("hbn_propose", lib().hbn_propose(self.p, group, C.cast(buf, C.c_void_p) if buf else None,
                                                len(data or b"")))

    def ProposeConfChange(self, group, Type, NodeID, ID=0, Context=None):
        buf = C.create_string_buffer(bytes(Context), max(1, len(Context))) if Context is not None else None
        _check("hbn_propose_conf_change", lib().hbn_propose_conf_change(
            self.p, group, ID, Type, NodeID, C.cast(buf, C.c_void_p) if buf else None, len(Context or b"")))

    def Step(self, group, m):
        ents = _EntryArray(m.Entries)
        cm = hbn_message()
        cm.type, cm.reject, cm.to, cm.from_ = m.Type, int(m.Reject), m.To, m.From
        cm.term, cm.log_term, cm.index, cm.commit, cm.reject_hint = m.Term, m.LogTerm, m.Index, m.Commit, m.RejectHint
        cm.entries, cm.n_entries = ents.arr, ents.n
        cm.snapshot, keep = _snap_in(m.Snapshot)
        _check("hbn_step", lib().hbn_step(self.p, group, C.byref(cm)))

    def StepMany(self, items):
        """[(group, Message), ...] in order through hbn_step_many (one call);
        returns how many were taken (all of them unless it raises)."""
        n = len(items)
        gs = (C.c_uint64 * max(1, n))(*[g for g, _ in items])
        arr = (hbn_message * max(1, n))()
        keep = []
        for i, (_, m) in enumerate(items):
            ents = _EntryArray(m.Entries)
            cm = arr[i]
            cm.type, cm.reject, cm.to, cm.from_ = m.Type, int(m.Reject), m.To, m.From
            cm.term, cm.log_term, cm.index, cm.commit, cm.reject_hint = m.Term, m.LogTerm, m.Index, m.Commit, \
                m.RejectHint
            cm.entries, cm.n_entries = ents.arr, ents.n
            cm.snapshot, k = _snap_in(m.Snapshot)
            keep.append((ents, k))
        done = C.c_uint64()
        try:
            _check("hbn_step_many", lib().hbn_step_many(self.p, n, gs, arr, C.byref(done)))
        except (RaftPanic, HbnError) as e:
            e.done = done.value  # the messages taken before the one that failed
            raise
        return done.value

    def ProposeMany(self, items):
        """[(group, data or None), ...] in order through hbn_propose_many."""
        n = len(items)
        gs = (C.c_uint64 * max(1, n))(*[g for g, _ in items])
        bufs = [C.create_string_buffer(bytes(d), max(1, len(d))) if d is not None else None for _, d in items]
        ptrs = (C.c_void_p * max(1, n))(*[C.cast(b, C.c_void_p).value if b is not None else None for b in bufs])
        lens = (C.c_uint64 * max(1, n))(*[len(d or b"") for _, d in items])
        done = C.c_uint64()
        try:
            _check("hbn_propose_many", lib().hbn_propose_many(self.p, n, gs, ptrs, lens, C.byref(done)))
        except (RaftPanic, HbnError) as e:
            e.done = done.value
            raise
        return done.value

    def SetThreads(self, k):
        _check("hbn_set_threads", lib().hbn_set_threads(self.p, k))

    def ReportUnreachable(self, id, group):
        _check("hbn_report_unreachable", lib().hbn_report_unreachable(self.p, id, group))

    def ReportSnapshot(self, id, group, failure):
        _check("hbn_report_snapshot", lib().hbn_report_snapshot(self.p, id, group, int(bool(failure))))

    def ApplyConfChange(self, group, Type, NodeID):
        nodes, n = (C.c_uint64 * abi.HB_MAX_REPLICAS)(), C.c_uint32()
        _check("hbn_apply_conf_change", lib().hbn_apply_conf_change(self.p, group, Type, NodeID, nodes, C.byref(n)))
        return [nodes[i] for i in range(n.value)]

    def Ready(self):
        """{group: Ready} for every group whose Ready containsUpdates; {} when the
        reference's readyc would not be selectable (nothing, or not advanced)."""
        out, n = C.POINTER(hbn_group_ready)(), C.c_uint64()
        rc = _check("hbn_ready", lib().hbn_ready(self.p, C.byref(out), C.byref(n)), ok=(0, HBN_EAGAIN))
        if rc == HBN_EAGAIN:
            return {}
        rds = {}
        for i in range(n.value):
            r = out[i]
            rd = Ready()
            if r.has_soft_state:
                rd.SoftState = SoftState(r.lead, r.raft_state)
            rd.HardState = HardState(r.hard_state.term, r.hard_state.vote, r.hard_state.commit)
            rd.Snapshot = _snap_out(r.snapshot)
            rd.Entries = _entries_out(r.entries, r.n_entries)
            rd.CommittedEntries = _entries_out(r.committed_entries, r.n_committed)
            for k in range(r.n_messages):
                m = r.messages[k]
                rd.Messages.append(Message(Type=m.type, To=m.to, From=m.from_, Term=m.term, LogTerm=m.log_term,
                                           Index=m.index, Entries=_entries_out(m.entries, m.n_entries),
                                           Commit=m.commit, Snapshot=_snap_out(m.snapshot), Reject=bool(m.reject),
                                           RejectHint=m.reject_hint))
            rd.fault = r.fault
            rds[r.group] = rd
        return rds

    def Advance(self, rds):
        ids = list(rds)
        arr = (C.c_uint64 * max(1, len(ids)))(*ids)
        _check("hbn_advance", lib().hbn_advance(self.p, arr, len(ids)))

    def Status(self, group):
        s = hbn_group_status()
        rc = lib().hbn_status(self.p, group, C.byref(s))
        if rc == HBN_ENOGROUP:
            return None
        _check("hbn_status", rc)
        prog = {s.progress_id[i]: s.progress[i] for i in range(s.n_progress)}
        return Status(ID=s.id, HardState=HardState(s.hard_state.term, s.hard_state.vote, s.hard_state.commit),
                      SoftState=SoftState(s.lead, s.raft_state), Applied=s.applied, Progress=prog)


def StartMultiNode(id, **kw):
    return MultiNode(id, **kw)
