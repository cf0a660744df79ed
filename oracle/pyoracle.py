"""ctypes bindings of the C parity oracle (oracle/raft_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package (etcd_amd).

`Raft` wraps one orc_raft with the method names of the reference's Go `raft`
struct so the transcribed known-answer tests read like raft/raft_test.go.
`OracleGroups` drives many groups through orc_step_batch in the engine's batch
format for GPU parity tests and the CPU baseline.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from etcd_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("ORC_LIB", os.path.join(_HERE, "build", "liboracle.so"))
_lib = None

ORC_MAX_PEERS = 8
NO_LIMIT = abi.HB_NO_LIMIT


class orc_inflights(C.Structure):
    _fields_ = [("start", C.c_int), ("count", C.c_int), ("size", C.c_int),
                ("buffer", C.POINTER(C.c_uint64))]

    @property
    def buf(self):
        return [self.buffer[i] for i in range(self.size)]


class orc_progress(C.Structure):
    _fields_ = [("Match", C.c_uint64), ("Next", C.c_uint64), ("State", C.c_int),
                ("Paused", C.c_int), ("PendingSnapshot", C.c_uint64), ("ins", orc_inflights)]


class orc_run(C.Structure):
    _fields_ = [("index", C.c_uint64), ("term", C.c_uint64)]


class orc_log(C.Structure):
    _fields_ = [("first_index", C.c_uint64), ("last_index", C.c_uint64),
                ("committed", C.c_uint64), ("applied", C.c_uint64), ("snap_index", C.c_uint64),
                ("nruns", C.c_int), ("cap", C.c_int), ("runs", C.POINTER(orc_run))]


class orc_msg(C.Structure):
    _fields_ = [("Type", C.c_int), ("To", C.c_uint64), ("From", C.c_uint64), ("Term", C.c_uint64),
                ("LogTerm", C.c_uint64), ("Index", C.c_uint64), ("Commit", C.c_uint64),
                ("Reject", C.c_int), ("RejectHint", C.c_uint64), ("nents", C.c_uint64),
                ("ent_lo", C.c_uint64), ("snap_index", C.c_uint64), ("edesc", C.c_void_p), ("eterm", C.c_void_p),
                ("snap_term", C.c_uint64), ("outsider", C.c_int), ("voted", C.c_int)]

    def __repr__(self):
        return (f"Msg(type={self.Type}, to={self.To}, from={self.From}, term={self.Term}, "
                f"logterm={self.LogTerm}, index={self.Index}, commit={self.Commit}, "
                f"reject={self.Reject}, nents={self.nents}, ent_lo={self.ent_lo})")


class orc_wire_msg(C.Structure):
    _fields_ = [("type", C.c_int32), ("to", C.c_uint64), ("from_", C.c_uint64), ("term", C.c_uint64),
                ("log_term", C.c_uint64), ("index", C.c_uint64), ("commit", C.c_uint64),
                ("reject_hint", C.c_uint64), ("reject", C.c_int), ("nentries", C.c_uint32)]


def unmarshal_message(data):
    """Message.Unmarshal (raft/raftpb/raft.pb.go:549-799) -> (rc, orc_wire_msg);
    rc 0 ok, 1 error, 2 Go panic / endless loop, 3 groups nested too deep."""
    m = orc_wire_msg()
    rc = lib().orc_unmarshal_message(bytes(data), len(data), C.byref(m))
    return rc, m


def decode_batch(data, off, length, group, capacity, group_n, peers):
    """hb_decode's contract on the CPU.  Returns dict of batch arrays + status."""
    n = len(off)
    d = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray)
                             else data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    group = np.ascontiguousarray(group, dtype=np.uint32)
    group_n = np.ascontiguousarray(group_n, dtype=np.uint32)
    peers = np.ascontiguousarray(peers, dtype=np.uint64)
    out = dict(group=np.zeros(n, np.uint32), info=np.zeros(n, np.uint32), term=np.zeros(n, np.uint64),
               index=np.zeros(n, np.uint64), hint=np.zeros(n, np.uint64), status=np.zeros(n, np.uint8))
    lib().orc_decode_batch(d.ctypes.data, off.ctypes.data, length.ctypes.data, group.ctypes.data, n, capacity,
                           group_n.ctypes.data, peers.ctypes.data, out["group"].ctypes.data, out["info"].ctypes.data,
                           out["term"].ctypes.data, out["index"].ctypes.data, out["hint"].ctypes.data,
                           out["status"].ctypes.data)
    return out


class orc_raft(C.Structure):
    _fields_ = [
        ("id", C.c_uint64), ("Term", C.c_uint64), ("Vote", C.c_uint64), ("Commit", C.c_uint64),
        ("log", orc_log), ("max_inflight", C.c_int), ("max_msg_size", C.c_uint64),
        ("n", C.c_int), ("ids", C.c_uint64 * ORC_MAX_PEERS), ("prs_", orc_progress * ORC_MAX_PEERS),
        ("state", C.c_int), ("lead", C.c_uint64), ("pending_conf", C.c_int), ("elapsed", C.c_int),
        ("election_timeout", C.c_int), ("heartbeat_timeout", C.c_int), ("rand_pos", C.c_uint64),
        ("nvotes", C.c_int), ("vote_ids", C.c_uint64 * (ORC_MAX_PEERS + 1)),
        ("vote_vals", C.c_int * (ORC_MAX_PEERS + 1)),
        ("msgs", C.POINTER(orc_msg)), ("nmsgs", C.c_int), ("msgs_cap", C.c_int),
        ("ev", C.c_void_p), ("nev", C.c_uint64), ("ev_cap", C.c_uint64), ("group", C.c_uint32),
        ("arrival", C.c_uint64), ("fault", C.c_int), ("n_won", C.c_uint64), ("n_lost", C.c_uint64),
        ("szc", C.c_void_p), ("szc_base", C.c_uint64), ("szc_n", C.c_uint64), ("szc_cap", C.c_uint64),
        ("sz_lo", C.c_uint64), ("tw_lo", C.c_uint64), ("tw_tfirst", C.c_uint64),
    ]


def build():
    """Compile the oracle with its Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.POINTER
        R = P(orc_raft)
        sig = {
            "orc_sizeof_raft": (C.c_size_t, []),
            "orc_ins_init": (None, [P(orc_inflights), C.c_int]),
            "orc_ins_free": (None, [P(orc_inflights)]),
            "orc_ins_add": (C.c_int, [P(orc_inflights), C.c_uint64]),
            "orc_ins_free_to": (None, [P(orc_inflights), C.c_uint64]),
            "orc_ins_free_first_one": (None, [P(orc_inflights)]),
            "orc_ins_full": (C.c_int, [P(orc_inflights)]),
            "orc_pr_become_probe": (None, [P(orc_progress)]),
            "orc_pr_become_replicate": (None, [P(orc_progress)]),
            "orc_pr_become_snapshot": (None, [P(orc_progress), C.c_uint64]),
            "orc_pr_maybe_update": (C.c_int, [P(orc_progress), C.c_uint64]),
            "orc_pr_optimistic_update": (None, [P(orc_progress), C.c_uint64]),
            "orc_pr_maybe_decr_to": (C.c_int, [P(orc_progress), C.c_uint64, C.c_uint64]),
            "orc_pr_is_paused": (C.c_int, [P(orc_progress)]),
            "orc_log_init": (None, [P(orc_log), C.c_uint64, C.c_uint64]),
            "orc_log_push": (None, [P(orc_log), C.c_uint64, C.c_uint64]),
            "orc_log_term": (C.c_uint64, [P(orc_log), C.c_uint64]),
            "orc_raft_init": (None, [R, C.c_uint64, P(C.c_uint64), C.c_int, C.c_int, C.c_uint64]),
            "orc_raft_free": (None, [R]),
            "orc_raft_pr": (P(orc_progress), [R, C.c_uint64]),
            "orc_raft_set_progress": (None, [R, C.c_uint64, C.c_uint64, C.c_uint64]),
            "orc_raft_load_state": (None, [R, C.c_uint64, C.c_uint64, C.c_uint64]),
            "orc_raft_q": (C.c_int, [R]),
            "orc_raft_reset": (None, [R, C.c_uint64]),
            "orc_raft_send_append": (None, [R, C.c_uint64]),
            "orc_raft_bcast_append": (None, [R]),
            "orc_raft_bcast_heartbeat": (None, [R]),
            "orc_raft_maybe_commit": (C.c_int, [R]),
            "orc_raft_append_entry": (None, [R, C.c_uint64, C.c_int]),
            "orc_raft_become_follower": (None, [R, C.c_uint64, C.c_uint64]),
            "orc_raft_become_candidate": (None, [R]),
            "orc_raft_become_leader": (None, [R]),
            "orc_raft_campaign": (None, [R]),
            "orc_raft_poll": (C.c_int, [R, C.c_uint64, C.c_int]),
            "orc_raft_step": (None, [R, P(orc_msg)]),
            "orc_raft_commit_to": (None, [R, C.c_uint64]),
            "orc_raft_read_messages": (C.c_int, [R, P(orc_msg), C.c_int]),
            "orc_raft_from_group": (C.c_int, [R, P(abi.hb_group), P(orc_run), C.c_int, C.c_int, C.c_uint64]),
            "orc_raft_to_group": (None, [R, P(abi.hb_group)]),
            "orc_raft_set_inflights": (C.c_int, [R, C.c_int, C.c_int, C.c_int, P(C.c_uint64)]),
            "orc_raft_get_inflights": (C.c_int, [R, C.c_int, P(C.c_uint64)]),
            "orc_step_batch": (C.c_int, [R, C.c_uint32, P(abi.hb_batch), C.c_void_p, C.c_uint64,
                                         P(C.c_uint64), P(C.c_uint64)]),
            "orc_groups_new": (R, [C.c_uint32]),
            "orc_groups_free": (None, [R, C.c_uint32]),
            "orc_groups_at": (R, [R, C.c_uint32]),
            "orc_groups_load": (C.c_int, [R, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_uint64]),
            "orc_groups_export": (None, [R, C.c_uint32, C.c_void_p]),
            "orc_groups_log_info": (None, [R, C.c_uint32, C.c_void_p]),
            "orc_raft_tick": (C.c_int, [R, P(C.c_uint64), C.c_uint64]),
            "orc_unmarshal_message": (C.c_int, [C.c_char_p, C.c_int64, P(orc_wire_msg)]),
            "orc_decode_batch": (None, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_void_p]),
            "orc_tick_batch": (C.c_int, [R, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                         P(C.c_uint64), P(C.c_uint64)]),
            "orc_groups_load_timers": (None, [R, C.c_uint32, C.c_void_p]),
            "orc_groups_export_timers": (None, [R, C.c_uint32, C.c_void_p]),
            "orc_entry_size": (C.c_uint64, [C.c_uint32, C.c_uint64, C.c_uint64]),
            "orc_limit_size": (C.c_uint64, [P(C.c_uint64), C.c_uint64, C.c_uint64]),
            "orc_raft_load_sizes": (C.c_int, [R, C.c_uint32, P(C.c_uint32)]),
            "orc_raft_load_term_runs": (C.c_int, [R, C.c_uint32, P(C.c_uint64)]),
            "orc_log_find_conflict": (C.c_uint64, [P(orc_log), C.c_uint64, P(C.c_uint64), C.c_uint64]),
            "orc_log_is_up_to_date": (C.c_int, [P(orc_log), C.c_uint64, C.c_uint64]),
            "orc_log_truncate": (None, [P(orc_log), C.c_uint64]),
            "orc_log_maybe_append": (C.c_int, [P(orc_log), C.c_uint64, C.c_uint64, C.c_uint64, P(C.c_uint64),
                                               C.c_uint64, P(C.c_uint64)]),
            "orc_raft_handle_append_entries": (None, [R, P(orc_msg)]),
            "orc_raft_handle_heartbeat": (None, [R, P(orc_msg)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        assert L.orc_sizeof_raft() == C.sizeof(orc_raft), "orc_raft layout drift"
        _lib = L
    return _lib


# ---------------------------------------------------------------------------
# Go-shaped wrappers for the known-answer tests
# ---------------------------------------------------------------------------
class Inflights:
    """newInflights(size) (raft/progress.go:183-188)."""

    def __init__(self, size, start=0):
        self.s = orc_inflights()
        lib().orc_ins_init(C.byref(self.s), size)
        self.s.start = start

    def __del__(self):
        try:
            lib().orc_ins_free(C.byref(self.s))
        except Exception:
            pass

    def add(self, v):
        if lib().orc_ins_add(C.byref(self.s), v) != 0:
            raise RuntimeError("cannot add into a full inflights")

    def freeTo(self, to):
        lib().orc_ins_free_to(C.byref(self.s), to)

    def freeFirstOne(self):
        lib().orc_ins_free_first_one(C.byref(self.s))

    def full(self):
        return bool(lib().orc_ins_full(C.byref(self.s)))

    def as_tuple(self):
        return (self.s.start, self.s.count, self.s.size, self.s.buf)


class Progress:
    """A free-standing Progress (raft/progress.go:37-67) for the table tests."""

    def __init__(self, State=abi.HB_PR_PROBE, Match=0, Next=0, Paused=False, PendingSnapshot=0, ins=256):
        self.p = orc_progress()
        self.p.State, self.p.Match, self.p.Next = State, Match, Next
        self.p.Paused, self.p.PendingSnapshot = int(Paused), PendingSnapshot
        lib().orc_ins_init(C.byref(self.p.ins), ins)

    def __getattr__(self, k):
        if k in ("State", "Match", "Next", "PendingSnapshot"):
            return getattr(self.p, k)
        if k == "Paused":
            return bool(self.p.Paused)
        raise AttributeError(k)

    def becomeProbe(self):
        lib().orc_pr_become_probe(C.byref(self.p))

    def becomeReplicate(self):
        lib().orc_pr_become_replicate(C.byref(self.p))

    def becomeSnapshot(self, i):
        lib().orc_pr_become_snapshot(C.byref(self.p), i)

    def maybeUpdate(self, n):
        return bool(lib().orc_pr_maybe_update(C.byref(self.p), n))

    def maybeDecrTo(self, rejected, last):
        return bool(lib().orc_pr_maybe_decr_to(C.byref(self.p), rejected, last))

    def isPaused(self):
        return bool(lib().orc_pr_is_paused(C.byref(self.p)))


def Msg(Type, From=0, To=0, Term=0, Index=0, LogTerm=0, Commit=0, Reject=False, RejectHint=0, Entries=0,
        Snapshot=None):
    """pb.Message for the oracle.  Entries: a count (MsgProp) or a list of
    (index, term) pairs (MsgApp; indices must follow Index); Snapshot: (index, term)."""
    m = orc_msg()
    m.Type, m.From, m.To, m.Term, m.Index = Type, From, To, Term, Index
    m.LogTerm, m.Commit, m.Reject, m.RejectHint = LogTerm, Commit, int(Reject), RejectHint
    if isinstance(Entries, (list, tuple)):
        for k, (i, _) in enumerate(Entries):
            assert i == Index + 1 + k, "entries must follow Index"
        m._terms = (C.c_uint64 * max(1, len(Entries)))(*[t for _, t in Entries])  # kept alive with m
        m.eterm = C.cast(m._terms, C.c_void_p)
        m.nents = len(Entries)
    else:
        m.nents = Entries
    if Snapshot is not None:
        m.snap_index, m.snap_term = Snapshot
    return m


class Raft:
    """newTestRaft(id, peers, election, heartbeat, storage) (raft/raft_test.go:1884-1898).

    `ents` = list of (index, term) entries appended to a MemoryStorage, `snapshot` =
    (index, term) applied first, `hard` = (term, vote, commit) HardState.
    """

    def __init__(self, id, peers, ents=(), snapshot=None, hard=None, max_inflight=256,
                 max_msg_size=NO_LIMIT, election=10, heartbeat=1, draws=()):
        L = lib()
        self.r = orc_raft()
        # r.rand.Int() stream (rand.New(rand.NewSource(id)) in the reference): supplied
        self.draws = np.ascontiguousarray(draws, dtype=np.uint64)
        if snapshot:
            L.orc_log_init(C.byref(self.r.log), snapshot[0] + 1, snapshot[1])
            self.r.log.snap_index = snapshot[0]
        else:
            L.orc_log_init(C.byref(self.r.log), 1, 0)
        for idx, term in ents:
            assert idx == self.r.log.last_index + 1
            L.orc_log_push(C.byref(self.r.log), term, 1)
        arr = (C.c_uint64 * max(1, len(peers)))(*peers)
        L.orc_raft_init(C.byref(self.r), id, arr, len(peers), max_inflight, max_msg_size)
        if hard and any(hard):
            L.orc_raft_load_state(C.byref(self.r), *hard)
        self.r.election_timeout, self.r.heartbeat_timeout = election, heartbeat

    def load_sizes(self, sizes):
        """Entry.Size() of the last len(sizes) entries (finite max_msg_size, hb_load_entry_sizes)."""
        a = (C.c_uint32 * max(1, len(sizes)))(*sizes)
        if lib().orc_raft_load_sizes(C.byref(self.r), len(sizes), a) != 0:
            raise ValueError("orc_raft_load_sizes failed")

    def __del__(self):
        try:
            lib().orc_raft_free(C.byref(self.r))
        except Exception:
            pass

    # -- fields ------------------------------------------------------------
    @property
    def Term(self):
        return self.r.Term

    @Term.setter
    def Term(self, v):
        self.r.Term = v

    @property
    def Commit(self):
        return self.r.Commit

    @property
    def state(self):
        return self.r.state

    @property
    def lead(self):
        return self.r.lead

    @property
    def Vote(self):
        return self.r.Vote

    @property
    def committed(self):
        return self.r.log.committed

    @property
    def lastIndex(self):
        return self.r.log.last_index

    @property
    def firstIndex(self):
        return self.r.log.first_index

    @property
    def fault(self):
        return self.r.fault

    def pr(self, id):
        p = lib().orc_raft_pr(C.byref(self.r), id)
        if not p:
            return None
        return p.contents

    def nodes(self):
        return sorted(self.r.ids[i] for i in range(self.r.n))

    def term(self, i):
        return lib().orc_log_term(C.byref(self.r.log), i)

    # -- methods -----------------------------------------------------------
    def handleAppendEntries(self, m):
        lib().orc_raft_handle_append_entries(C.byref(self.r), C.byref(m))

    def handleHeartbeat(self, m):
        lib().orc_raft_handle_heartbeat(C.byref(self.r), C.byref(m))

    def entries(self):
        """(index, term) of every entry in [firstIndex, lastIndex] (allEntries)."""
        lo = self.r.log.first_index
        return [(i, self.term(i)) for i in range(lo, self.r.log.last_index + 1)]

    def Step(self, m):
        lib().orc_raft_step(C.byref(self.r), C.byref(m))

    def readMessages(self):
        n = self.r.nmsgs
        out = (orc_msg * max(1, n))()
        lib().orc_raft_read_messages(C.byref(self.r), out, n)
        return [out[i] for i in range(n)]

    @property
    def elapsed(self):
        return self.r.elapsed

    def tick(self):
        """r.tick(): tickHeartbeat / tickElection with the supplied draw stream."""
        d = self.draws
        return lib().orc_raft_tick(C.byref(self.r), d.ctypes.data_as(C.POINTER(C.c_uint64)), len(d))

    def becomeFollower(self, term, lead):
        lib().orc_raft_become_follower(C.byref(self.r), term, lead)

    def becomeCandidate(self):
        lib().orc_raft_become_candidate(C.byref(self.r))

    def becomeLeader(self):
        lib().orc_raft_become_leader(C.byref(self.r))

    def setProgress(self, id, match, next):
        lib().orc_raft_set_progress(C.byref(self.r), id, match, next)

    def maybeCommit(self):
        return bool(lib().orc_raft_maybe_commit(C.byref(self.r)))

    def appendEntry(self, k=1):
        lib().orc_raft_append_entry(C.byref(self.r), k, 0)

    def sendAppend(self, to):
        lib().orc_raft_send_append(C.byref(self.r), to)

    def bcastAppend(self):
        lib().orc_raft_bcast_append(C.byref(self.r))

    def bcastHeartbeat(self):
        lib().orc_raft_bcast_heartbeat(C.byref(self.r))

    def commitTo(self, i):
        lib().orc_raft_commit_to(C.byref(self.r), i)

    def reset(self, term):
        lib().orc_raft_reset(C.byref(self.r), term)

    def q(self):
        return lib().orc_raft_q(C.byref(self.r))

    def to_group(self):
        g = abi.hb_group()
        lib().orc_raft_to_group(C.byref(self.r), C.byref(g))
        return g


# ---------------------------------------------------------------------------
# batch driver (engine format)
# ---------------------------------------------------------------------------
def flat_runs(runs):
    """Log term runs per group as (flat [R, 2] u64 (index, term), offsets [G+1] u64).
    Accepts the list-of-lists form or an already flat (flat, off) tuple."""
    if isinstance(runs, tuple):
        flat, off = runs
        return np.ascontiguousarray(flat, dtype=np.uint64), np.ascontiguousarray(off, dtype=np.uint64)
    off = np.zeros(len(runs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r) for r in runs])
    flat = np.array([x for r in runs for x in r], dtype=np.uint64).reshape(-1, 2)
    return np.ascontiguousarray(flat), off


class OracleGroups:
    """ngroups oracle rafts stepped with orc_step_batch (the engine's batch format)."""

    def __init__(self, groups, runs, max_inflight, max_msg_size=NO_LIMIT, inflights=None):
        """groups: numpy GROUP_DTYPE [G]; runs: list of [(index, term), ...] per group;
        inflights: optional dict {(g, slot): np.uint64 array of the live window}."""
        L = lib()
        self.G = len(groups)
        self.max_inflight = max_inflight
        self.ptr = L.orc_groups_new(self.G)
        gbuf = np.ascontiguousarray(groups, dtype=abi.GROUP_DTYPE)
        flat, off = flat_runs(runs)
        rc = L.orc_groups_load(self.ptr, self.G, gbuf.ctypes.data, flat.ctypes.data, off.ctypes.data,
                               max_inflight, max_msg_size)
        if rc != 0:
            raise ValueError(f"orc_raft_from_group({-rc - 1}) failed")
        for (g, s), vals in (inflights or {}).items():
            v = np.ascontiguousarray(vals, dtype=np.uint64)
            start = int(gbuf[g]["pr"][s]["ins_start"])
            L.orc_raft_set_inflights(L.orc_groups_at(self.ptr, g), s, start, len(v),
                                     v.ctypes.data_as(C.POINTER(C.c_uint64)))

    def __del__(self):
        try:
            lib().orc_groups_free(self.ptr, self.G)
        except Exception:
            pass

    def step(self, batch_arrays, ev_cap=None):
        """batch_arrays: dict of numpy arrays group/info/term/index/hint/props.
        Returns (events ndarray EVENT_DTYPE, stats ndarray u64)."""
        L = lib()
        b = abi.hb_batch()
        n = len(batch_arrays["group"])
        keep = {}
        for k, dt in (("group", np.uint32), ("info", np.uint32), ("term", np.uint64),
                      ("index", np.uint64), ("hint", np.uint64), ("props", np.uint32),
                      ("edesc", np.uint32), ("eoff", np.uint64), ("peoff", np.uint64), ("commit", np.uint64),
                      ("eterm", np.uint64)):
            a = batch_arrays.get(k)
            if a is None:
                setattr(b, k, None)
                continue
            a = np.ascontiguousarray(a, dtype=dt)
            keep[k] = a
            setattr(b, k, a.ctypes.data)
        b.n = n
        b.n_edesc = len(keep["edesc"]) if "edesc" in keep else (len(keep["eterm"]) if "eterm" in keep else 0)
        if ev_cap is None:
            ev_cap = (n + self.G) * (abi.HB_MAX_REPLICAS + 6) + 64
        if getattr(self, "_ev", None) is None or len(self._ev) < ev_cap:
            self._ev = np.empty(ev_cap, dtype=abi.EVENT_DTYPE)  # reused: the oracle writes what it reports
        ev = self._ev
        nev = C.c_uint64()
        stats = (C.c_uint64 * abi.HB_STAT_COUNT)()
        rc = L.orc_step_batch(self.ptr, self.G, C.byref(b), ev.ctypes.data, ev_cap, C.byref(nev), stats)
        if rc != 0:
            raise RuntimeError("oracle event buffer too small")
        return ev[: nev.value].copy(), np.array(stats[:], dtype=np.uint64)

    def tick(self, draws, ev_cap=None):
        """One MultiNode.Tick over all groups; draws = the r.rand.Int() stream."""
        L = lib()
        d = np.ascontiguousarray(draws, dtype=np.uint64)
        if ev_cap is None:
            ev_cap = self.G * (abi.HB_MAX_REPLICAS + 6) + 64
        ev = np.empty(ev_cap, dtype=abi.EVENT_DTYPE)
        nev = C.c_uint64()
        stats = (C.c_uint64 * abi.HB_STAT_COUNT)()
        rc = L.orc_tick_batch(self.ptr, self.G, d.ctypes.data if len(d) else None, len(d), ev.ctypes.data, ev_cap,
                              C.byref(nev), stats)
        if rc != 0:
            raise RuntimeError("oracle event buffer too small")
        return ev[: nev.value].copy(), np.array(stats[:], dtype=np.uint64)

    def load_timers(self, timers):
        t = np.ascontiguousarray(timers, dtype=abi.TIMER_DTYPE)
        assert len(t) == self.G
        lib().orc_groups_load_timers(self.ptr, self.G, t.ctypes.data)

    def timers(self):
        out = np.zeros(self.G, dtype=abi.TIMER_DTYPE)
        lib().orc_groups_export_timers(self.ptr, self.G, out.ctypes.data)
        return out

    def groups(self):
        out = np.zeros(self.G, dtype=abi.GROUP_DTYPE)
        lib().orc_groups_export(self.ptr, self.G, out.ctypes.data)
        return out

    def log_info(self):
        """Per group [G, 4] u64: term runs of its log (covering [firstIndex-1, lastIndex]),
        the oldest index whose size is loaded (sz_lo), firstIndex, lastIndex — what a
        caller of the engine reserves its log index from (hb_reserve_log)."""
        out = np.zeros((self.G, 4), dtype=np.uint64)
        lib().orc_groups_log_info(self.ptr, self.G, out.ctypes.data)
        return out

    def load_sizes(self, sizes):
        """Finite max_msg_size: {group: Entry.Size() of its last n entries} (hb_load_entry_sizes)."""
        L = lib()
        for g, z in sizes.items():
            a = np.ascontiguousarray(z, dtype=np.uint32)
            rc = L.orc_raft_load_sizes(L.orc_groups_at(self.ptr, g), len(a), a.ctypes.data_as(C.POINTER(C.c_uint32)))
            if rc != 0:
                raise ValueError(f"orc_raft_load_sizes(group {g}) failed")

    def load_term_runs(self, runs):
        """Follower side: {group: [(start, term), ...] older term runs} (hb_load_term_runs)."""
        L = lib()
        for g, rr in runs.items():
            a = (C.c_uint64 * max(1, 2 * len(rr)))(*[x for r in rr for x in r])
            if L.orc_raft_load_term_runs(L.orc_groups_at(self.ptr, g), len(rr), a) != 0:
                raise ValueError(f"orc_raft_load_term_runs(group {g}) failed")

    def term(self, g, i):
        """raftLog.term(i) of group g (the oracle's whole log)."""
        L = lib()
        return L.orc_log_term(C.byref(L.orc_groups_at(self.ptr, g).contents.log), i)

    def inflights(self, g, slot):
        L = lib()
        buf = (C.c_uint64 * max(1, self.max_inflight))()
        n = L.orc_raft_get_inflights(L.orc_groups_at(self.ptr, g), slot, buf)
        return np.array(buf[: max(n, 0)], dtype=np.uint64)

    def raft(self, g):
        return lib().orc_groups_at(self.ptr, g).contents


class ShardedOracleGroups:
    """The same groups as OracleGroups, split into `shards` contiguous ranges
    that are stepped concurrently (one thread per shard; ctypes releases the
    GIL inside the C oracle).  Groups are independent (raft/multinode.go:125-131)
    and each shard steps its groups' messages in their arrival order, so the
    result equals one OracleGroups over the whole batch: events are mapped
    back to global group ids and global arrival positions, statistics summed.
    Used for the full-size BASELINE configurations, where one core would take
    minutes.  Supports the batch fields group / info / term / index / hint /
    props / commit / eoff + eterm (a message's entries re-based per shard), not
    the entry descriptors of a finite MaxSizePerMsg."""

    def __init__(self, groups, runs, max_inflight, max_msg_size=NO_LIMIT, shards=16):
        G = len(groups)
        self.G = G
        self.max_inflight = max_inflight
        per = -(-G // shards)
        self.bounds = [(lo, min(G, lo + per)) for lo in range(0, G, per)]
        flat, off = flat_runs(runs)
        self.parts = []
        for lo, hi in self.bounds:
            o = off[lo:hi + 1]
            sub_flat = flat[int(o[0]):int(o[-1])]
            self.parts.append(OracleGroups(groups[lo:hi], (sub_flat, o - o[0]), max_inflight, max_msg_size))

    def _map(self, fn):
        import threading
        out = [None] * len(self.parts)

        def run(i):
            out[i] = fn(i, self.parts[i])
        th = [threading.Thread(target=run, args=(i,)) for i in range(len(self.parts))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return out

    def step(self, b):
        for k in ("edesc", "peoff"):
            assert b.get(k) is None, f"ShardedOracleGroups: batch field {k} not supported"
        ne = None
        if b.get("eoff") is not None:  # entries per message (eoff / eterm in arrival order)
            eoff = np.asarray(b["eoff"], dtype=np.int64)
            eterm = np.asarray(b["eterm"], dtype=np.uint64)
            ne = np.diff(np.append(eoff, len(eterm)))
        grp = np.asarray(b["group"], dtype=np.uint32)
        per = self.bounds[0][1] - self.bounds[0][0]
        sid = np.minimum(grp // np.uint32(per), np.uint32(len(self.parts)))  # out-of-range ids: dropped below
        order = np.argsort(sid, kind="stable")
        cuts = np.searchsorted(sid[order], np.arange(len(self.parts) + 1))
        drop_stats = np.zeros(abi.HB_STAT_COUNT, np.uint64)
        assert np.all(grp < self.G), "ShardedOracleGroups: out-of-range group ids"

        def run(i, og):
            lo, hi = self.bounds[i]
            idx = order[cuts[i]:cuts[i + 1]]
            sub = {"group": grp[idx] - np.uint32(lo), "info": np.asarray(b["info"])[idx],
                   "term": np.asarray(b["term"])[idx], "index": np.asarray(b["index"])[idx]}
            if b.get("hint") is not None:
                sub["hint"] = np.asarray(b["hint"])[idx]
            if b.get("props") is not None:
                sub["props"] = np.asarray(b["props"])[lo:hi]
            if b.get("commit") is not None:
                sub["commit"] = np.asarray(b["commit"])[idx]
            if ne is not None:
                k = ne[idx]
                sub["eoff"] = np.concatenate([[0], np.cumsum(k)[:-1]]).astype(np.uint64)
                pos = np.repeat(eoff[idx] - sub["eoff"].astype(np.int64), k) + np.arange(int(k.sum()))
                sub["eterm"] = eterm[pos]
            ev, st = og.step(sub)
            ev["group"] += np.uint32(lo)
            # events that name an arrival position: back to the global batch
            arr = np.isin(ev["type"], [abi.HB_EV_PROP_FWD, abi.HB_EV_PROP_DROP, abi.HB_EV_FAULT, abi.HB_EV_FOLLOW]) & \
                (ev["x"] != np.uint64(abi.HB_NO_INDEX))
            ev["x"][arr] = idx[ev["x"][arr].astype(np.int64)].astype(np.uint64)
            return ev, st
        res = self._map(run)
        return np.concatenate([r[0] for r in res]), sum((r[1] for r in res), drop_stats)

    def tick(self, draws, ev_cap=None):
        """One MultiNode.Tick over every shard (each group reads the shared
        r.rand stream at its own position, so the shards are independent)."""
        def run(i, og):
            ev, st = og.tick(draws)
            ev["group"] += np.uint32(self.bounds[i][0])
            return ev, st
        res = self._map(run)
        return np.concatenate([r[0] for r in res]), sum((r[1] for r in res), np.zeros(abi.HB_STAT_COUNT, np.uint64))

    def load_timers(self, timers):
        for (lo, hi), og in zip(self.bounds, self.parts):
            og.load_timers(timers[lo:hi])

    def timers(self):
        return np.concatenate(self._map(lambda i, og: og.timers()))

    def groups(self):
        return np.concatenate(self._map(lambda i, og: og.groups()))

    def log_info(self):
        return np.concatenate(self._map(lambda i, og: og.log_info()))

    def inflights(self, g, slot):
        for (lo, hi), og in zip(self.bounds, self.parts):
            if lo <= g < hi:
                return og.inflights(g - lo, slot)
        raise IndexError(g)
