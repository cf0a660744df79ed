"""ctypes mirror of include/hipbatch.h (records, enums, constants).

Shared by the product bindings (etcd_amd.hipbatch) and the test harness.
tests/test_abi.py checks every constant and record layout here against the
header text, so the two cannot drift apart.
"""
import ctypes as C

import numpy as np

HB_ABI_VERSION = 5

HB_OK = 0
HB_EINVAL = -1
HB_ENOMEM = -2
HB_EDEVICE = -3
HB_EINVARIANT = -4

HB_MAX_REPLICAS = 7
HB_MAX_INFLIGHT = 1024
HB_NO_LIMIT = (1 << 64) - 1
HB_NO_INDEX = (1 << 64) - 1
HB_SIZE_RING_MIN = 16
HB_TERM_RING_MIN = 8
HB_INFO_VOTED = 0x200
HB_ENT_MAX_DATA = 0x3FFFFFFF

# StateType raft/raft.go:35-39
HB_STATE_FOLLOWER = 0
HB_STATE_CANDIDATE = 1
HB_STATE_LEADER = 2
# ProgressStateType raft/progress.go:19-23
HB_PR_PROBE = 0
HB_PR_REPLICATE = 1
HB_PR_SNAPSHOT = 2
# MessageType raft/raftpb/raft.proto:34-47
HB_MSG_HUP = 0
HB_MSG_BEAT = 1
HB_MSG_PROP = 2
HB_MSG_APP = 3
HB_MSG_APP_RESP = 4
HB_MSG_VOTE = 5
HB_MSG_VOTE_RESP = 6
HB_MSG_SNAP = 7
HB_MSG_HEARTBEAT = 8
HB_MSG_HEARTBEAT_RESP = 9
HB_MSG_UNREACHABLE = 10
HB_MSG_SNAP_STATUS = 11

HB_REF_SLOT_MAX = 6
HB_REF_OTHER = 0xD
HB_REF_SELF = 0xE
HB_REF_NONE = 0xF
HB_SLOT_NONE = 0xF

HB_STEP_HOST_PTRS = 0x1
HB_STEP_PROFILE = 0x2
HB_STEP_PROFILE_APPLY = 0x4
HB_STEP_MSG_PROPS = 0x8

HB_FAULT_NONE = 0
HB_FAULT_LEADER_CAMPAIGN = 1
HB_FAULT_EMPTY_PROP = 2
HB_FAULT_EMPTY_SNAPSHOT = 3
HB_FAULT_INFLIGHTS_FULL = 4
HB_FAULT_NIL_PROGRESS = 5
HB_FAULT_COMMIT_RANGE = 6
HB_FAULT_NO_SELF = 7
HB_FAULT_FOLLOWER_LEADER = 8
HB_FAULT_RAND_EXHAUSTED = 9
HB_FAULT_SIZE_WINDOW = 10
HB_FAULT_TERM_WINDOW = 11
HB_FAULT_CONFLICT_COMMITTED = 12

HB_EV_TERM = 1
HB_EV_STATE = 2
HB_EV_COMMIT = 3
HB_EV_LAST = 4
HB_EV_APP = 5
HB_EV_SNAP = 6
HB_EV_HEARTBEAT = 7
HB_EV_VOTE = 8
HB_EV_PROP_FWD = 9
HB_EV_PROP_DROP = 10
HB_EV_FAULT = 11
HB_STATE_OTH_LEAD = 1
HB_STATE_OTH_VOTE = 2
HB_EV_RESP = 13
HB_EV_FOLLOW = 14
HB_RESP_APP = 0
HB_RESP_HEARTBEAT = 1
HB_RESP_VOTE = 2
HB_RESP_REJECT = 8
HB_FOLLOW_STEP = 0
HB_FOLLOW_APPEND = 1
HB_FOLLOW_RESTORE = 2
HB_EVW_BCAST = 12  # device event word: HB_EV_APP to every slot of a mask
HB_EVW_VBCAST = 0  # device event word: HB_EV_VOTE to every slot of a mask
HB_EVW_CONT = 15  # device event word: continuation (x bits 40..63)

# wire ingestion record status (hb_decode)
HB_WIRE_OK = 0
HB_WIRE_LOCAL = 1
HB_WIRE_HOST = 2
HB_WIRE_ERROR = 3
HB_WIRE_PANIC = 4
HB_WIRE_BADGROUP = 5

HB_STAT_MSGS = 0
HB_STAT_APPRESP = 1
HB_STAT_VOTERESP = 2
HB_STAT_DROPPED = 3
HB_STAT_COMMITS = 4
HB_STAT_WON = 5
HB_STAT_LOST = 6
HB_STAT_EVENTS = 7
HB_STAT_FAULTS = 8
HB_STAT_ENTRIES = 9
HB_STAT_COUNT = 10

HB_PHASE_PARTITION = 0
HB_PHASE_APPLY = 1
HB_PHASE_GENERAL = 2
HB_PHASE_FINISH = 3
HB_PHASE_COUNT = 4
HB_KERN_ROUTE_FAST = 1  # hb_step_kernels: k_route_fast ran the route and the fast lane
HB_KERN_ROUTE_ELECT = 2  # hb_step_kernels: k_route closed storm partitions and ran the election lane

STAT_NAMES = ["msgs", "appresp", "voteresp", "dropped", "commits", "won", "lost",
              "events", "faults", "entries"]


def hb_info(mtype, from_slot, reject=False):
    return (mtype & 0xF) | ((from_slot & 0xF) << 4) | ((1 if reject else 0) << 8)


def hb_ent_desc(data_len, etype=0, has_data=True):
    """Entry descriptor (HB_ENT_DESC): len(Data) | Type << 30 | (Data != nil) << 31."""
    return (int(data_len) & HB_ENT_MAX_DATA) | ((int(etype) & 1) << 30) | ((1 if has_data else 0) << 31)


def _sov(x):
    n = 1
    while x >= 0x80:
        x >>= 7
        n += 1
    return n


def entry_size(desc, term, index):
    """gogo Entry.Size() (raft/raftpb/raft.pb.go:1030-1043) of the entry a descriptor describes."""
    n = 1 + _sov((desc >> 30) & 1) + 1 + _sov(term) + 1 + _sov(index)
    if desc >> 31:
        ln = desc & HB_ENT_MAX_DATA
        n += 1 + ln + _sov(ln)
    return n


class hb_progress(C.Structure):
    _fields_ = [
        ("match", C.c_uint64),
        ("next", C.c_uint64),
        ("pending_snapshot", C.c_uint64),
        ("state", C.c_uint32),
        ("paused", C.c_uint32),
        ("ins_start", C.c_uint32),
        ("ins_count", C.c_uint32),
    ]


class hb_group(C.Structure):
    _fields_ = [
        ("term", C.c_uint64),
        ("committed", C.c_uint64),
        ("first_index", C.c_uint64),
        ("last_index", C.c_uint64),
        ("term_first", C.c_uint64),
        ("term_last", C.c_uint64),
        ("snap_index", C.c_uint64),
        ("state", C.c_uint32),
        ("n", C.c_uint32),
        ("self_slot", C.c_uint32),
        ("lead", C.c_uint32),
        ("vote", C.c_uint32),
        ("votes_resp", C.c_uint32),
        ("votes_grant", C.c_uint32),
        ("fault", C.c_uint32),
        ("commit_zero", C.c_uint32),
        ("pad", C.c_uint32),
        ("pr", hb_progress * HB_MAX_REPLICAS),
    ]


class hb_event(C.Structure):
    _fields_ = [
        ("x", C.c_uint64),
        ("group", C.c_uint32),
        ("type", C.c_uint8),
        ("to", C.c_uint8),
        ("aux", C.c_uint16),
    ]


class hb_timer(C.Structure):
    _fields_ = [
        ("elapsed", C.c_uint32),
        ("rand_pos", C.c_uint32),
        ("election_tick", C.c_uint16),
        ("heartbeat_tick", C.c_uint16),
        ("pad", C.c_uint32),
    ]


class hb_batch(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("group", C.c_void_p),
        ("info", C.c_void_p),
        ("term", C.c_void_p),
        ("index", C.c_void_p),
        ("hint", C.c_void_p),
        ("props", C.c_void_p),
        ("n_edesc", C.c_uint64),
        ("edesc", C.c_void_p),
        ("eoff", C.c_void_p),
        ("peoff", C.c_void_p),
        ("commit", C.c_void_p),
        ("eterm", C.c_void_p),
    ]


# numpy views of the records (same layout as the ctypes structs)
PROGRESS_DTYPE = np.dtype([
    ("match", "<u8"), ("next", "<u8"), ("pending_snapshot", "<u8"),
    ("state", "<u4"), ("paused", "<u4"), ("ins_start", "<u4"), ("ins_count", "<u4"),
])
GROUP_DTYPE = np.dtype([
    ("term", "<u8"), ("committed", "<u8"), ("first_index", "<u8"), ("last_index", "<u8"),
    ("term_first", "<u8"), ("term_last", "<u8"), ("snap_index", "<u8"),
    ("state", "<u4"), ("n", "<u4"), ("self_slot", "<u4"), ("lead", "<u4"), ("vote", "<u4"),
    ("votes_resp", "<u4"), ("votes_grant", "<u4"), ("fault", "<u4"), ("commit_zero", "<u4"), ("pad", "<u4"),
    ("pr", PROGRESS_DTYPE, (HB_MAX_REPLICAS,)),
])
TIMER_DTYPE = np.dtype([("elapsed", "<u4"), ("rand_pos", "<u4"), ("election_tick", "<u2"),
                        ("heartbeat_tick", "<u2"), ("pad", "<u4")])
EVENT_DTYPE = np.dtype([("x", "<u8"), ("group", "<u4"), ("type", "u1"), ("to", "u1"), ("aux", "<u2")])

assert GROUP_DTYPE.itemsize == C.sizeof(hb_group)
assert EVENT_DTYPE.itemsize == C.sizeof(hb_event) == 16
assert TIMER_DTYPE.itemsize == C.sizeof(hb_timer) == 16
assert PROGRESS_DTYPE.itemsize == C.sizeof(hb_progress)
