/*
 * hipbatch.h — C ABI of the MI355X batched Raft leader-bookkeeping engine.
 *
 * This is the drop-in boundary that a Go `raft/hipbatch` package binds through
 * cgo.  It replaces the per-group CPU loop that
 * `raft.MultiNode` runs in its single `run` goroutine
 * (reference: raft/multinode.go:166-322) for the leader-side bookkeeping:
 *
 *   - MsgAppResp progress updates    raft/raft.go:514-546, raft/progress.go:100-166
 *   - inflight flow control          raft/progress.go:172-237
 *   - quorum commit                  raft/raft.go:323-332, raft/log.go:241-247
 *   - vote tally / campaign          raft/raft.go:429-460, 585-614
 *   - the Step term gate             raft/raft.go:462-490
 *   - MultiNode dispatch filters     raft/multinode.go:233-237, raft/util.go:49-55
 *
 * Design rules:
 *   - Group state lives on the device as structure-of-arrays in HBM; one
 *     handle owns one GPU's shard of groups.  A handle is single-owner and not
 *     thread-safe, mirroring the single `run` goroutine that owns all group
 *     state in the reference (raft/multinode.go:166-168).
 *   - Every export returns an int: 0 = OK, negative = HB_E*.  Invariant
 *     violations that make the reference panic are reported per group as an
 *     HB_EV_FAULT event (the host then panics with the reference message); they
 *     never unwind across this ABI.
 *   - No torch types, no C++ types: plain pointers and sizes only.
 */
#ifndef HIPBATCH_H_
#define HIPBATCH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HB_ABI_VERSION 5

/* ---- error codes -------------------------------------------------------- */
#define HB_OK          0
#define HB_EINVAL     -1   /* bad argument (range, size, unsupported config)   */
#define HB_ENOMEM     -2   /* device or pinned allocation failed               */
#define HB_EDEVICE    -3   /* HIP runtime error / no device                    */
#define HB_EINVARIANT -4   /* a device-side capacity invariant was violated    */

/* ---- limits -------------------------------------------------------------- */
#define HB_MAX_REPLICAS   7      /* n = len(r.prs) per group, 1..7 (north star: 3/5/7) */
#define HB_MAX_INFLIGHT   1024   /* Config.MaxInflightMsgs upper bound on device       */
#define HB_NO_LIMIT       UINT64_MAX  /* raft noLimit (raft/raft.go:30)                */
#define HB_NO_INDEX       UINT64_MAX
/* The log index (hb_reserve_log): per group, the cumulative Entry.Size() of
 * its log (finite MaxSizePerMsg) and its older term runs (follower side), in
 * rings of any power-of-two capacity; these are the capacities hb_create
 * starts every group with (128 bytes per ring). */
#define HB_SIZE_RING_MIN  16
#define HB_TERM_RING_MIN  8

/* ---- raft enums (values equal the reference's) --------------------------- */
/* StateType raft/raft.go:35-39 */
#define HB_STATE_FOLLOWER  0
#define HB_STATE_CANDIDATE 1
#define HB_STATE_LEADER    2
/* ProgressStateType raft/progress.go:19-23 */
#define HB_PR_PROBE     0
#define HB_PR_REPLICATE 1
#define HB_PR_SNAPSHOT  2
/* MessageType raft/raftpb/raft.proto:34-47 */
#define HB_MSG_HUP            0
#define HB_MSG_BEAT           1
#define HB_MSG_PROP           2
#define HB_MSG_APP            3
#define HB_MSG_APP_RESP       4
#define HB_MSG_VOTE           5
#define HB_MSG_VOTE_RESP      6
#define HB_MSG_SNAP           7
#define HB_MSG_HEARTBEAT      8
#define HB_MSG_HEARTBEAT_RESP 9
#define HB_MSG_UNREACHABLE    10
#define HB_MSG_SNAP_STATUS    11

/* ---- node references ------------------------------------------------------
 * Peers of a group are addressed by their slot in the group's peer list
 * (the host keeps slot -> node id).  lead / vote are encoded as:           */
#define HB_REF_SLOT_MAX   6      /* 0..6 = slot in the peer list              */
#define HB_REF_OTHER      0xD    /* an id that is not in prs (host keeps it)   */
#define HB_REF_SELF       0xE    /* r.id while r.id is not in prs              */
#define HB_REF_NONE       0xF    /* raft.None (raft/raft.go:29)                */
#define HB_SLOT_NONE      0xF    /* from_slot of a non-member / self not in prs*/

/* ---- messages (structure-of-arrays batch) --------------------------------
 * One batch = messages in arrival order, as the `run` goroutine would receive
 * them on recvc/propc.  Only the relative order of messages of the same group
 * is significant (groups are independent, raft/multinode.go:125-131).
 *
 * info[i] = type | from_slot << 4 | reject << 8 | voted << 9
 *   type      : HB_MSG_* of m.Type.  Device types: HUP, BEAT, PROP, APP_RESP,
 *               VOTE_RESP, HEARTBEAT_RESP, UNREACHABLE, SNAP_STATUS and the
 *               follower side: APP, HEARTBEAT, SNAP, VOTE.
 *   from_slot : slot of m.From in the group's prs, HB_SLOT_NONE if absent.
 *   reject    : m.Reject.
 *   voted     : only for from_slot == HB_SLOT_NONE: m.From is the node the
 *               group voted for (its Vote is HB_REF_OTHER), read by MsgVote's
 *               `r.Vote == m.From` (raft/raft.go:641).
 * term[i]  = m.Term (0 = local message, no term gate, raft/raft.go:471-472)
 * index[i] = m.Index; for HB_MSG_PROP the number of entries (>0); for
 *            HB_MSG_SNAP the snapshot's Metadata.Index.
 * hint[i]  = m.RejectHint of a rejected MsgAppResp; m.LogTerm of MsgApp /
 *            MsgVote; the snapshot's Metadata.Term of MsgSnap (may be NULL
 *            when the batch holds none of these).
 * commit[i]= m.Commit of MsgApp / MsgHeartbeat (may be NULL when it holds none).
 * MsgApp entries: message i's entries are k = eoff[i]..eoff[i+1] (the last
 *            message's run ends at n_edesc); eterm[k] = their terms (Index =
 *            m.Index + 1 + position), edesc[k] their descriptors (finite
 *            max_msg_size).
 * props    = optional dense [capacity] entry counts: group g first steps one
 *            MsgProp carrying props[g] entries (if > 0), before its messages
 *            in this batch.  NULL = none.
 *
 * Entry descriptors — read only when the handle's max_msg_size is finite
 * (neither HB_NO_LIMIT nor 0): sendAppend then sends entries(Next,
 * maxMsgSize) cut by limitSize (raft/raft.go:265, raft/util.go:97-110), which
 * needs every appended entry's protobuf size (raft/raftpb/raft.pb.go:1030-
 * 1043).  The device computes Entry.Size() from the descriptor plus the Term
 * and Index it assigns (appendEntry, raft/raft.go:351-360):
 *   edesc[k] = HB_ENT_DESC(len(Data), Type, Data != nil)
 *   eoff[i]  = first descriptor of MsgProp message i (its index[i] entries)
 *   peoff[g] = first descriptor of the dense proposal props[g]
 * n_edesc = number of descriptors (bytes copied with HB_STEP_HOST_PTRS).
 */
#define HB_INFO(type, from_slot, reject) \
  ((uint32_t)(type) | ((uint32_t)(from_slot) << 4) | ((uint32_t)((reject) ? 1 : 0) << 8))
#define HB_INFO_VOTED     0x200u
#define HB_ENT_MAX_DATA   0x3FFFFFFF
#define HB_ENT_DESC(data_len, type, has_data) \
  ((uint32_t)(data_len) | ((uint32_t)(type) << 30) | ((uint32_t)((has_data) ? 1 : 0) << 31))

typedef struct hb_batch {
  uint64_t        n;
  const uint32_t* group;
  const uint32_t* info;
  const uint64_t* term;
  const uint64_t* index;
  const uint64_t* hint;
  const uint32_t* props;
  uint64_t        n_edesc;   /* entries described by edesc / eterm */
  const uint32_t* edesc;
  const uint64_t* eoff;
  const uint64_t* peoff;
  const uint64_t* commit;
  const uint64_t* eterm;
} hb_batch;

/* hb_step flags */
#define HB_STEP_HOST_PTRS 0x1u   /* batch arrays are host pointers (copied H2D; up to 8 MiB in all
                                    they are packed into one pinned block during the call and sent
                                    with one copy, so the arrays may be reused once hb_step returns) */
#define HB_STEP_PROFILE   0x2u   /* record per-phase HIP events (hb_phase_ms)   */
#define HB_STEP_PROFILE_APPLY 0x4u  /* only the HB_PHASE_APPLY events (two, on the apply stream) */
#define HB_STEP_MSG_PROPS 0x8u   /* the batch carries MsgProp messages (no dense props): groups of
                                    3 keep a third route slot, so a leader's two MsgAppResp and its
                                    proposal stay on the fast path (a hint: results are the same) */

/* ---- per-group state (host view, array-of-structures) --------------------
 * Device keeps this as SoA.  Field meanings follow the reference:
 *   term/vote/commit : pb.HardState (raft/raft.go:126; vote is a node ref)
 *   lead, state      : SoftState (raft/node.go:40-43)
 *   committed        : raftLog.committed
 *   first_index      : raftLog.firstIndex()   (raft/log.go:150-159)
 *   last_index       : raftLog.lastIndex()    (raft/log.go:161-170)
 *   term_first..term_last : the maximal run of indices i in
 *        [first_index-1, last_index] with raftLog.term(i) == term.  Exact
 *        because log terms never decrease with the index and never exceed the
 *        current Term.  Empty run: term_first = HB_NO_INDEX, term_last = 0.
 *   snap_index       : raftLog.snapshot().Metadata.Index (0 = empty snapshot)
 *   votes_resp/grant : r.votes (raft/raft.go:139) as slot bitmasks; bit 7 =
 *                      r.id when r.id is not in prs.
 *   fault            : non-zero once the group hit a reference panic; the
 *                      device ignores the group until it is reloaded.
 *   commit_zero      : r.Commit (= HardState.Commit) is 0 although committed
 *                      is not.  The reference sets r.Commit = raftLog.committed
 *                      only in loadState and at the end of every Step that
 *                      passes the term gate (raft/raft.go:466,488,759), so a
 *                      group created with an empty HardState keeps r.Commit = 0
 *                      until its first Step: a bootstrapped MultiNode group
 *                      (committed = len(peers), raft/multinode.go:197-211) or
 *                      one restored from a snapshot (committed = firstIndex - 1,
 *                      raft/log.go:60).  handleAppendEntries tests m.Index <
 *                      r.Commit (raft/raft.go:652), not committed.  These are
 *                      the only values r.Commit takes (r.Commit == committed,
 *                      or 0 before the first Step); 0 = r.Commit == committed.
 *                      The device clears it when the group steps a message
 *                      past the term gate.
 */
typedef struct hb_progress {
  uint64_t match;
  uint64_t next;
  uint64_t pending_snapshot;  /* valid in HB_PR_SNAPSHOT, else 0 */
  uint32_t state;             /* HB_PR_* */
  uint32_t paused;
  uint32_t ins_start;         /* inflights.start */
  uint32_t ins_count;         /* inflights.count */
} hb_progress;

typedef struct hb_group {
  uint64_t term;
  uint64_t committed;
  uint64_t first_index;
  uint64_t last_index;
  uint64_t term_first;
  uint64_t term_last;
  uint64_t snap_index;
  uint32_t state;
  uint32_t n;
  uint32_t self_slot;         /* slot of r.id or HB_SLOT_NONE */
  uint32_t lead;              /* node ref */
  uint32_t vote;              /* node ref */
  uint32_t votes_resp;
  uint32_t votes_grant;
  uint32_t fault;             /* HB_FAULT_* */
  uint32_t commit_zero;       /* r.Commit == 0 != committed (no Step since an empty HardState) */
  uint32_t pad;
  hb_progress pr[HB_MAX_REPLICAS];
} hb_group;

/* fault codes: the reference panic each one stands for */
#define HB_FAULT_NONE            0
#define HB_FAULT_LEADER_CAMPAIGN 1  /* "invalid transition [leader -> candidate]" raft/raft.go:396 */
#define HB_FAULT_EMPTY_PROP      2  /* "%x stepped empty MsgProp" raft/raft.go:502               */
#define HB_FAULT_EMPTY_SNAPSHOT  3  /* "need non-empty snapshot" raft/raft.go:252-254            */
#define HB_FAULT_INFLIGHTS_FULL  4  /* "cannot add into a full inflights" raft/progress.go:192  */
#define HB_FAULT_NIL_PROGRESS    5  /* nil *Progress dereference (local msg from non-member)    */
#define HB_FAULT_COMMIT_RANGE    6  /* "tocommit(%d) is out of range" raft/log.go:175-177       */
#define HB_FAULT_NO_SELF         7  /* appendEntry with r.id not in prs (nil deref raft.go:358) */
#define HB_FAULT_FOLLOWER_LEADER 8  /* "invalid transition [follower -> leader]" raft/raft.go:409 (oracle KATs only) */
#define HB_FAULT_RAND_EXHAUSTED  9  /* engine-defined, no reference panic: hb_tick needed draw
                                       rand_pos of the group but hb_set_rand supplied fewer */
#define HB_FAULT_SIZE_WINDOW    10  /* engine precondition, no reference panic: with a finite
                                       max_msg_size, sendAppend needed the size of an entry the
                                       caller never loaded into the log index
                                       (hb_load_entry_sizes), or one a ring smaller than the
                                       log dropped (hb_reserve_log).  libhbnode loads and
                                       reserves both, so it never sees this code. */
#define HB_FAULT_TERM_WINDOW    11  /* engine precondition, no reference panic: the follower side
                                       needed the term of an entry the caller never loaded
                                       (hb_load_term_runs) or a too-small ring dropped; as above,
                                       unreachable through libhbnode */
#define HB_FAULT_CONFLICT_COMMITTED 12  /* "entry %d conflict with committed entry" raft/log.go:79 */

/* ---- events (the sparse delta list) ---------------------------------------
 * One ordered stream of 16-byte records per group describes everything the
 * host needs to build `Ready` (raft/node.go:447-463) for the groups that
 * changed: HardState/SoftState marks and the messages raft.send appended to
 * r.msgs (raft/raft.go:227-236), in the order the reference produced them.
 * Groups with no event did not change.  Marks are emitted eagerly at the
 * point the reference changes the value.
 *
 *   HB_EV_TERM      x = new Term                   (raft.reset, raft/raft.go:334-338)
 *   HB_EV_STATE     x = state | lead<<8 | vote<<16 (becomeFollower/Candidate/Leader,
 *                   and the follower side's r.lead / r.Vote = m.From); aux =
 *                   HB_STATE_OTH_LEAD / _VOTE when that lead / vote was just
 *                   set to the sender of the message being stepped and the
 *                   sender is outside prs (ref HB_REF_OTHER: its id is that
 *                   message's m.From); such an event is emitted even when the
 *                   packed refs did not change
 *   HB_EV_COMMIT    x = new committed              (raftLog.commitTo, raft/log.go:172-180)
 *   HB_EV_LAST      x = new lastIndex, aux = 1 for the becomeLeader noop entry,
 *                   0 for proposal entries        (raft.appendEntry, raft/raft.go:351-360)
 *   HB_EV_APP       to, x = m.Index (= Next-1).  Entries are (x, L] where L is
 *                   the current lastIndex (max_msg_size noLimit), x+1
 *                   (max_msg_size 0), or limitSize's cut of (x, lastIndex]
 *                   (finite max_msg_size); none if x+1 > lastIndex.  m.Commit =
 *                   current committed, m.Term = current term, m.LogTerm = term(x);
 *                   aux = 1 when term(x) == m.Term (the host then needs no log
 *                   lookup for LogTerm), else 0.
 *                   (raft.sendAppend, raft/raft.go:261-281)
 *   HB_EV_SNAP      to, x = snapshot index         (raft/raft.go:246-260)
 *   HB_EV_HEARTBEAT to, x = m.Commit              (raft.sendHeartbeat, raft/raft.go:285-299)
 *   HB_EV_VOTE      to, x = m.Index (lastIndex); m.LogTerm = lastTerm (raft/raft.go:435-442)
 *   HB_EV_PROP_FWD  to = lead ref, x = arrival index of the MsgProp (HB_NO_INDEX
 *                   for a dense props[] proposal)  (stepFollower, raft/raft.go:618-624)
 *   HB_EV_PROP_DROP x = arrival index (HB_NO_INDEX for props[]): proposal dropped
 *                   (raft/raft.go:587-589, 619-621)
 *   HB_EV_FAULT     aux = HB_FAULT_*, x = arrival index of the message
 *   HB_EV_RESP      a response the follower side sends to `to` (m.From of the
 *                   message being stepped: slot, or HB_REF_OTHER for a sender
 *                   outside prs): aux = HB_RESP_APP (MsgAppResp, x = m.Index),
 *                   HB_RESP_HEARTBEAT (MsgHeartbeatResp), HB_RESP_VOTE
 *                   (MsgVoteResp), | HB_RESP_REJECT; a rejecting MsgAppResp's
 *                   RejectHint is lastIndex at that point (raft/raft.go:651-682)
 *   HB_EV_FOLLOW    aux = HB_FOLLOW_STEP: the follower-side message at arrival
 *                   x (MsgApp / MsgHeartbeat / MsgSnap / MsgVote) is stepped
 *                   (it is not of a lower term; emitted before the term gate's
 *                   becomeFollower): the events up to the next one belong to it.
 *                   aux = HB_FOLLOW_APPEND: raftLog.maybeAppend appended that
 *                   MsgApp's entries from its first conflict (raft/log.go:72-88).
 *                   aux = HB_FOLLOW_RESTORE: that MsgSnap's snapshot was
 *                   restored (raft/raft.go:684-707): log = the snapshot, every
 *                   peer slot's Progress reset; a caller whose snapshot
 *                   ConfState differs from the group's peers reloads the group.
 */
#define HB_EV_TERM      1
#define HB_EV_STATE     2
#define HB_EV_COMMIT    3
#define HB_STATE_OTH_LEAD  1
#define HB_STATE_OTH_VOTE  2
#define HB_EV_LAST      4
#define HB_EV_APP       5
#define HB_EV_SNAP      6
#define HB_EV_HEARTBEAT 7
#define HB_EV_VOTE      8
#define HB_EV_PROP_FWD  9
#define HB_EV_PROP_DROP 10
#define HB_EV_FAULT     11
#define HB_EV_RESP      13
#define HB_EV_FOLLOW    14
#define HB_RESP_APP        0
#define HB_RESP_HEARTBEAT  1
#define HB_RESP_VOTE       2
#define HB_RESP_REJECT     8
#define HB_FOLLOW_STEP     0
#define HB_FOLLOW_APPEND   1
#define HB_FOLLOW_RESTORE  2

typedef struct hb_event {
  uint64_t x;
  uint32_t group;
  uint8_t  type;
  uint8_t  to;
  uint16_t aux;
} hb_event;

/* ---- step statistics (reduced over the batch; RCCL-reducible u64s) ------- */
#define HB_STAT_MSGS       0  /* messages stepped (after the membership filter)     */
#define HB_STAT_APPRESP    1  /* MsgAppResp stepped (incl. stale / ignored ones)     */
#define HB_STAT_VOTERESP   2  /* MsgVoteResp stepped                                 */
#define HB_STAT_DROPPED    3  /* responses from non-members (raft/multinode.go:235)  */
#define HB_STAT_COMMITS    4  /* groups whose committed advanced in this batch       */
#define HB_STAT_WON        5  /* elections won (candidate -> leader)                 */
#define HB_STAT_LOST       6  /* elections lost by poll (candidate -> follower)      */
#define HB_STAT_EVENTS     7  /* events emitted                                      */
#define HB_STAT_FAULTS     8  /* groups that faulted in this batch                   */
#define HB_STAT_ENTRIES    9  /* log entries appended (proposals + noops)            */
#define HB_STAT_COUNT      10

/* ---- phases (HB_STEP_PROFILE) -------------------------------------------- */
#define HB_PHASE_PARTITION 0  /* bucket radix sort + per-partition routing to lanes */
#define HB_PHASE_APPLY     1  /* steady-state fast path (the dominant kernel)      */
#define HB_PHASE_GENERAL   2  /* general state machine for handed-over groups      */
#define HB_PHASE_FINISH    3  /* statistics reduction                              */
#define HB_PHASE_COUNT     4

typedef struct hb_handle hb_handle;

/* ---- lifecycle ------------------------------------------------------------ */
/* Create a handle on `device` holding up to `capacity` groups of at most
 * `max_replicas` peers, MaxInflightMsgs = max_inflight (Config.MaxInflightMsgs,
 * raft/raft.go:98) and MaxSizePerMsg = max_msg_size (raft/raft.go:93; any
 * value: HB_NO_LIMIT, 0, or a finite size, for which the device keeps the
 * cumulative sizes of each group's log, see hb_load_entry_sizes /
 * hb_reserve_log).  `max_batch` bounds hb_step's n.
 * Device memory: per group ~100 B + nmax x (28 + 8 max_inflight) B of state,
 * 16 B + a 128-byte term-run ring, and for a finite max_msg_size 16 B + a
 * 128-byte size ring (rings grow with hb_reserve_log: 8 B per log entry,
 * 16 B per term run).
 * A step of at most 16,384 messages on a handle of at most 1M groups
 * partitions in one workgroup (one launch), and hb_events_to_host compacts at
 * most 1,024 chunks in one; HB_SMALL_STEP=0 in the environment at hb_create
 * keeps the tiled kernels for such steps (the same results). */
int  hb_create(int device, uint32_t capacity, uint32_t max_replicas,
               uint32_t max_inflight, uint64_t max_msg_size, uint64_t max_batch,
               hb_handle** out);
int  hb_destroy(hb_handle* h);
/* Launch on this HIP stream (hipStream_t as void*); NULL = the null stream.
 * This is the apply stream: the group state, the events and the statistics
 * are produced on it, in hb_step order. */
int  hb_set_stream(hb_handle* h, void* hip_stream);
/* Each hb_step runs in two stages: prep (sort the batch by bucket and route
 * every group's messages to it; a library-owned stream, double-buffered) and
 * apply (the raft bookkeeping; the apply stream).  Prep only reads the batch,
 * so the prep of step k+1 may run while step k applies.  Prep waits for the
 * work enqueued so far on the INPUT stream, the one that produces the batch
 * arrays: by default the apply stream (prep k+1 then starts after apply k);
 * a caller whose batches are ready earlier, or produced on a stream of their
 * own, names that stream here to let the two stages overlap.  NULL stream
 * pointer = the null stream.  The caller must keep a batch's arrays intact
 * until hb_step for it has been followed by hb_sync or by the next hb_step
 * returning. */
int  hb_set_input_stream(hb_handle* h, void* hip_stream);
int  hb_sync(hb_handle* h);   /* waits for both stages of every step so far */
int  hb_abi_version(void);
const char* hb_strerror(int code);

/* ---- group state (CreateGroup / RemoveGroup / Status) ---------------------
 * Load `count` groups into slots [first, first+count) from host records
 * (CreateGroup, raft/multinode.go:181-217; inflight windows start empty
 * unless set with hb_set_inflights).  Gather them back for Status
 * (raft/status.go:34-49). */
int  hb_load_groups(hb_handle* h, uint32_t first, uint32_t count, const hb_group* groups);
int  hb_get_groups(hb_handle* h, uint32_t first, uint32_t count, hb_group* out);
/* RemoveGroup (raft/multinode.go:219-222): mark slots empty (all messages to
 * them are ignored until reloaded). */
int  hb_remove_groups(hb_handle* h, uint32_t first, uint32_t count);
/* The application changed a group's Storage (MemoryStorage.Compact /
 * CreateSnapshot / ApplySnapshot, raft/storage.go:150-214): refresh the
 * device copies of raftLog.firstIndex() and raftLog.snapshot().Metadata.Index
 * that sendAppend reads (needSnapshot, raft/raft.go:246-260, 715-717) for
 * `count` group slots (host arrays). */
int  hb_set_log_bounds(hb_handle* h, uint32_t count, const uint32_t* groups,
                       const uint64_t* first_index, const uint64_t* snap_index);
/* ---- the log index ---------------------------------------------------------
 * What the device needs of a group's log besides its current-term run: the
 * entries' protobuf sizes (a finite MaxSizePerMsg: sendAppend cuts
 * entries(Next, maxMsgSize) with limitSize, raft/raft.go:265,
 * raft/log.go:219-224, raft/util.go:97-110, for ANY Next in the log) and the
 * terms below the current-term run (follower side: raftLog.term(i) for any i,
 * raft/log.go:198-217).  The host owns the log (it holds the payloads and
 * Storage) and loads both once per group; the device keeps them up to date as
 * it appends, truncates and restores.  Each lives in a per-group ring whose
 * capacity the host reserves: the ring drops its oldest element only when it
 * is full, so a capacity covering [firstIndex - 1, lastIndex] plus what the
 * next step can append (entries of MsgProp / props / MsgApp, one noop per
 * election) means nothing the reference can read is ever missing.
 *
 * Finite max_msg_size only: the Entry.Size() of the entries (last_index -
 * n_sizes[i], last_index] of group groups[i] (any n_sizes[i] <= last_index;
 * normally the whole log from first_index), in index order, concatenated over
 * i in `sizes` (host arrays); the ring grows to hold them.  hb_load_groups
 * leaves a group with none (only a follower at Next = last_index + 1 can be
 * served); a send that needs an entry never loaded faults HB_FAULT_SIZE_WINDOW. */
int  hb_load_entry_sizes(hb_handle* h, uint32_t count, const uint32_t* groups,
                         const uint32_t* n_sizes, const uint32_t* sizes);
/* Follower side: the terms of a loaded group's log below its current-term run
 * (term_first), which raftLog.term() lookups of MsgApp / MsgVote / MsgSnap
 * need (matchTerm, findConflict, isUpToDate; raft/log.go:72-123, 249-251).
 * groups[i] takes n_runs[i] runs (start index, term), oldest first, the pairs
 * of all groups concatenated in `runs` (host arrays): run k covers [start_k,
 * start_k+1) and the last one reaches term_first - 1 (or last_index when
 * term_first = HB_NO_INDEX); normally every run down to first_index - 1.  The
 * ring grows to hold them plus one.  hb_load_groups leaves a group with none:
 * a lookup below term_first then faults HB_FAULT_TERM_WINDOW. */
int  hb_load_term_runs(hb_handle* h, uint32_t count, const uint32_t* groups,
                       const uint32_t* n_runs, const uint64_t* runs);
/* Grow the rings of groups[i] to hold at least size_cap[i] cumulative sizes
 * (the span [oldest needed index, lastIndex] including firstIndex - 1; ignored
 * unless max_msg_size is finite) and run_cap[i] term runs (every run of the log
 * plus the runs the next step can start); a NULL array or 0 leaves that ring
 * as is.  Capacities round up to a power of two and never shrink; the content
 * is kept.  Synchronous (one copy kernel for the groups that grow).  Call it
 * before an hb_step / hb_tick that could outgrow a ring. */
int  hb_reserve_log(hb_handle* h, uint32_t count, const uint32_t* groups,
                    const uint64_t* size_cap, const uint64_t* run_cap);
/* The current ring capacities of one group (0 sizes: max_msg_size not finite). */
int  hb_log_capacity(hb_handle* h, uint32_t group, uint64_t* size_cap, uint64_t* run_cap);
/* Inflight window of (group, slot): buffer[(start + i) % max_inflight] = vals[i]. */
int  hb_set_inflights(hb_handle* h, uint32_t group, uint32_t slot,
                      uint32_t start, uint32_t count, const uint64_t* vals);
int  hb_get_inflights(hb_handle* h, uint32_t group, uint32_t slot,
                      uint32_t* start, uint32_t* count, uint64_t* vals /* [max_inflight] */);

/* ---- timers (MultiNode.Tick) ---------------------------------------------
 * Per group: r.elapsed, Config.ElectionTick / HeartbeatTick, and how many
 * values the group's r.rand has produced.  Every group of a MultiNode owns a
 * rand.Rand seeded with the same node id (raft/raft.go:189 with
 * config.ID = mn.id, raft/multinode.go:182), so all groups read one stream,
 * each at its own position.  The host supplies that stream (the outputs of
 * rand.New(rand.NewSource(id)).Int(), in order) with hb_set_rand and keeps it
 * longer than any group's rand_pos + 1 (one draw per group per tick at most).
 * hb_create sets election_tick 10, heartbeat_tick 1 (the reference tests'
 * defaults, raft/raft_test.go:1884-1894); hb_load_groups zeroes elapsed and
 * rand_pos of the loaded groups (newRaft: fresh rand, becomeFollower -> reset).
 * Follower-side receipts that reset r.elapsed (MsgApp / MsgHeartbeat /
 * MsgSnap / granted MsgVote, raft/raft.go:625-640) are handled by the host;
 * it reports them with hb_load_timers. */
typedef struct hb_timer {
  uint32_t elapsed;          /* r.elapsed */
  uint32_t rand_pos;         /* r.rand.Int() values taken so far */
  uint16_t election_tick;    /* r.electionTimeout (>= 1) */
  uint16_t heartbeat_tick;   /* r.heartbeatTimeout */
  uint32_t pad;
} hb_timer;
int  hb_load_timers(hb_handle* h, uint32_t first, uint32_t count, const hb_timer* timers);
int  hb_get_timers(hb_handle* h, uint32_t first, uint32_t count, hb_timer* out);
/* draws[i] = the (first + i)-th r.rand.Int() value (0 <= v < 2^63); the table
 * grows to first + count, earlier entries are kept.  Host memory. */
int  hb_set_rand(hb_handle* h, uint64_t first, uint64_t count, const uint64_t* draws);
/* One MultiNode.Tick (raft/multinode.go:264-275): every live group ticks
 * once, tickHeartbeat for leaders, tickElection otherwise (raft/raft.go:
 * 362-382, isElectionTimeout :765-771); a due MsgBeat / MsgHup is stepped at
 * once.  Events and statistics as for hb_step (the stepped MsgBeat / MsgHup
 * count in HB_STAT_MSGS).  flags: 0. */
int  hb_tick(hb_handle* h, uint32_t flags);

/* ---- wire ingestion ------------------------------------------------------
 * Decode raftpb.Message records (protobuf, raft/raftpb/raft.pb.go:549-799
 * Message.Unmarshal with its Entry / Snapshot / SnapshotMetadata / ConfState
 * sub-messages and gogo proto.Skip) straight into a device batch, as
 * multiNode.Step receives them (raft/multinode.go:432-439).  Record i is
 * bytes[off[i], off[i] + len[i]) for group slot group[i]; m.From becomes the
 * group's slot through the node ids set with hb_load_peers (HB_SLOT_NONE when
 * absent, so hb_step's membership filter applies).  bytes / off / len / group
 * and every array of `out` are device memory; out->props is ignored.  Record
 * i of `out` is the batch record (group = 0xFFFFFFFF unless HB_WIRE_OK, so
 * hb_step drops it); status[i] says what became of it:                      */
#define HB_WIRE_OK       0  /* MsgAppResp / MsgVoteResp / MsgHeartbeatResp: in the batch      */
#define HB_WIRE_LOCAL    1  /* local type from the network, dropped by Step (IsLocalMsg)      */
#define HB_WIRE_HOST     2  /* well-formed, not for the device batch (other types, or unknown
                               fields nesting groups deeper than 16): the host steps it        */
#define HB_WIRE_ERROR    3  /* Unmarshal returns an error (truncated, wrong / illegal wire type) */
#define HB_WIRE_PANIC    4  /* the reference would panic or never return (negative lengths)  */
#define HB_WIRE_BADGROUP 5  /* group[i] >= capacity                                          */
/* ids[i * HB_MAX_REPLICAS + s] = node id of slot s of group first + i (host memory). */
int  hb_load_peers(hb_handle* h, uint32_t first, uint32_t count, const uint64_t* ids);
int  hb_decode(hb_handle* h, const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
               const uint32_t* group, uint64_t n, const hb_batch* out, uint8_t* status);

/* ---- the hot path ----------------------------------------------------------
 * Step one batch (all messages of the batch, per group in arrival order).
 * Asynchronous on the handle's stream.  Events and statistics of the step
 * are read with the functions below. */
int  hb_step(hb_handle* h, const hb_batch* b, uint32_t flags);

/* Events of the last step, as written by the device (zero-copy access for a
 * consumer on the GPU): `n_chunks` chunks, two per 256-group partition p
 * (chunk 2p: the events of the dense props[] proposals, chunk 2p+1: the
 * events of the partition's messages); chunk c holds counts[c] 8-byte words
 * at base + chunk_off[c].  A group's events are its words in chunk 2p, then
 * in chunk 2p+1, each in order.  Word format (bit ranges):
 *   [0:4)   type: HB_EV_*; 12 = an HB_EV_APP to every slot of the mask in
 *           `to` (same x and aux), in slot order; 0 = an HB_EV_VOTE to every
 *           slot of the mask (same x, aux 0: campaign's MsgVotes), in slot
 *           order; 15 = continuation word
 *   [4:11)  to (slot / node ref), or the slot mask of types 12 and 0
 *   [11]    x needs 64 bits: the next word is a continuation holding
 *           x bits 40..63 in its bits [4:28)
 *   [12:16) aux
 *   [16:24) group - 256 p
 *   [24:64) x bits 0..39
 * hb_copy_events expands them into hb_event records.  Device pointers; valid
 * until the next hb_step. */
#define HB_EVW_BCAST 12
#define HB_EVW_VBCAST 0
#define HB_EVW_CONT  15
int  hb_events_device(hb_handle* h, const uint64_t** base, const uint64_t** chunk_off,
                      const uint32_t** counts, uint32_t* n_chunks);
/* Gather the last step's events densely into host memory (synchronizes).
 * *n = number of events; returns HB_EINVAL if cap is too small. */
int  hb_copy_events(hb_handle* h, hb_event* out, uint64_t cap, uint64_t* n);
/* The compact delta list for a host consumer: the last
 * step's event words exactly as the device wrote them (format above), densely
 * in chunk order, written by the device into pinned host memory from
 * hb_alloc_pinned: words[0 .. *total) when *total <= cap (else only counts and
 * total are written: call again with a larger buffer, the step's events stay
 * valid until the next hb_step / hb_tick), counts[c] = the words of chunk c for
 * every chunk (hb_event_words_chunks).  Asynchronous on the handle's stream
 * (8 bytes per word over PCIe instead of hb_copy_events' 16 per event, one
 * word per bcastAppend): the host reads the buffers after hb_sync.  A group's
 * events are its words in chunk 2p, then chunk 2p + 1, in order, p = group /
 * groups_per_chunk; hb_expand_event_words turns them into hb_event records. */
int  hb_events_to_host(hb_handle* h, uint64_t* words, uint64_t cap, uint32_t* counts, uint64_t* total);
int  hb_event_words_chunks(hb_handle* h, uint32_t* n_chunks, uint32_t* groups_per_chunk);
/* Host-side expansion of hb_events_to_host's output into hb_event records
 * (*n_out = the number of records; HB_EINVAL if cap is too small; out NULL
 * only counts).  Pure CPU, no handle. */
int  hb_expand_event_words(const uint64_t* words, uint64_t n_words, const uint32_t* counts, uint32_t n_chunks,
                           hb_event* out, uint64_t cap, uint64_t* n_out);
/* Statistics of the last step: device pointer to HB_STAT_COUNT u64 (for an
 * RCCL all-reduce on the same stream) or a synchronous host copy. */
int  hb_stats_device(hb_handle* h, uint64_t** dev_stats);
int  hb_stats(hb_handle* h, uint64_t* out);
/* Asynchronous device-to-device copy of the last step's statistics (on the
 * handle's stream), e.g. into a buffer that an RCCL all-reduce then sums. */
int  hb_stats_to(hb_handle* h, uint64_t* dev_dst /* [HB_STAT_COUNT] */);
/* Optional device accumulator: every later hb_step also adds its statistics
 * into dev_accum[HB_STAT_COUNT] in its finish phase (no extra launch).
 * NULL turns it off.  The buffer must outlive its use. */
int  hb_set_stats_accum(hb_handle* h, uint64_t* dev_accum);
/* Per-phase device time (ms) averaged over the HB_STEP_PROFILE steps since
 * hb_phase_reset (the last 256 of them); *steps = how many (synchronizes). */
int  hb_phase_ms(hb_handle* h, float* out /* [HB_PHASE_COUNT] */, uint32_t* steps);
int  hb_phase_reset(hb_handle* h);
/* Which apply kernels the last hb_step launched (for profiles and rooflines):
 * HB_KERN_ROUTE_FAST = the route and the n = 3 fast lane ran as one kernel
 * (k_route_fast; HB_PHASE_APPLY then brackets it), else k_route and
 * k_apply_fast / k_apply_lead separately.  HB_KERN_ROUTE_ELECT = (n >= 5,
 * batches without dense proposals) the route closed the partitions whose
 * groups k_apply_lead would only hand over and ran the election lane there
 * (k_route<8, false, n>; HB_STORM=0/1 at hb_create turns it off / keeps only
 * the hand-over). */
#define HB_KERN_ROUTE_FAST 1u
#define HB_KERN_ROUTE_ELECT 2u
int  hb_step_kernels(hb_handle* h, uint32_t* mask);

/* ---- pinned host memory for cgo callers (Go must not hand Go memory to C
 * that C retains; raft/hipbatch packs batches into these buffers). -------- */
int  hb_alloc_pinned(size_t bytes, void** out);
int  hb_free_pinned(void* p);

#ifdef __cplusplus
}
#endif
#endif /* HIPBATCH_H_ */
