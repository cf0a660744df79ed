/*
 * hbnode.h — C ABI of the host side of raft.MultiNode over the MI355X engine.
 *
 * libhipbatch (include/hipbatch.h) owns the per-group leader bookkeeping on
 * the device and returns a sparse event stream.  This library is the host
 * half of the reference's `multiNode.run` loop (raft/multinode.go:166-322):
 * it keeps what the reference keeps in `raftLog` on the host — entry payloads,
 * the unstable tail, committed/applied (raft/log.go, raft/log_unstable.go) —
 * and the application's `MemoryStorage` (raft/storage.go), batches every
 * Step / Propose / Campaign / Report* of a Ready cycle into one hb_step, and
 * assembles `Ready` (raft/node.go:447-463) for exactly the groups that
 * changed, materialising `pb.Message`s (MsgApp with its entries, MsgVote,
 * MsgHeartbeat, MsgSnap, forwarded MsgProp) from the device's send intents.
 *
 * A Go `raft/hipbatch` package binds this header through cgo the way
 * INTEGRATION.md shows for hipbatch.h; the Python mirror is
 * etcd_amd/multinode.py.
 *
 * Rules: one hbn_node = one MultiNode = one hb_handle (one GPU); single-owner,
 * not thread-safe (the reference serialises everything on its run goroutine).
 * Every export returns 0 or a negative code.  Where the reference panics
 * (raftLogger.Panicf / a Go runtime panic) the call returns HBN_EPANIC and
 * hbn_last_error() holds the reference's message; nothing unwinds across the
 * ABI.  Pointers returned by hbn_ready / hbn_storage_entries stay valid until
 * the next call on the same node / storage.
 */
#ifndef HBNODE_H_
#define HBNODE_H_

#include <stddef.h>
#include <stdint.h>

#include "hipbatch.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes (hb codes plus these) ------------------------------------ */
#define HBN_ENOGROUP       -10  /* no group with this id (the reference dereferences nil)  */
#define HBN_EEXIST         -11  /* CreateGroup for an id that exists                        */
#define HBN_EAGAIN         -12  /* Ready: nothing to report, or the last Ready is not
                                   advanced yet (the reference's readyc is nil then)        */
#define HBN_EUNSUPPORTED   -13  /* outside the engine's limits, where the reference proceeds:
                                   a group with more members than hbn_start's max_replicas
                                   (at most HB_MAX_REPLICAS = 7: CreateGroup, or an
                                   ApplyConfChange / snapshot restore adding one), or a group
                                   whose prs is empty receiving a message the device would
                                   have to step (MsgHup, MsgProp, MsgApp, MsgVote ...)      */
#define HBN_EPANIC         -14  /* the reference panics here; see hbn_last_error()          */
/* MemoryStorage errors (raft/storage.go:25-31) */
#define HBN_ECOMPACTED     -20  /* ErrCompacted */
#define HBN_EUNAVAILABLE   -21  /* ErrUnavailable */
#define HBN_ESNAPOUTOFDATE -22  /* ErrSnapOutOfDate */

/* host-detected panics, reported like HB_FAULT_* in hbn_ready.fault */
#define HBN_FAULT_DOUBLE_CONF 32  /* "unexpected double uncommitted config entry" raft/raft.go:421 */

/* EntryType raft/raftpb/raft.pb.go:36-40; ConfChangeType :131-136 */
#define HBN_ENTRY_NORMAL      0
#define HBN_ENTRY_CONF_CHANGE 1
#define HBN_CC_ADD_NODE    0
#define HBN_CC_REMOVE_NODE 1
#define HBN_CC_UPDATE_NODE 2

/* pb.Entry.  has_data = 0 is Go's nil Data (distinct from an empty slice). */
typedef struct hbn_entry {
  uint64_t term;
  uint64_t index;
  uint32_t type;
  uint32_t has_data;
  const uint8_t* data;
  uint64_t data_len;
} hbn_entry;

typedef struct hbn_hard_state {
  uint64_t term, vote, commit;
} hbn_hard_state;

/* pb.Snapshot (Metadata.Index == 0 is IsEmptySnap, raft/node.go:76-78) */
typedef struct hbn_snapshot {
  uint64_t index, term;
  const uint64_t* nodes;  /* Metadata.ConfState.Nodes */
  uint32_t n_nodes;
  uint32_t has_data;
  const uint8_t* data;
  uint64_t data_len;
} hbn_snapshot;

/* pb.Message (raft/raftpb/raft.pb.go:200-213) */
typedef struct hbn_message {
  uint32_t type;        /* HB_MSG_* */
  uint32_t reject;
  uint64_t to, from, term, log_term, index, commit, reject_hint;
  const hbn_entry* entries;
  uint64_t n_entries;
  hbn_snapshot snapshot;
} hbn_message;

/* One group's Ready (raft/node.go:45-70).  has_soft_state = 0 is a nil
 * *SoftState; an all-zero hard_state is emptyState.  fault != 0: the group hit
 * a reference panic (HB_FAULT_* from the device, HBN_FAULT_* from the host);
 * it is frozen and the binding panics with the reference's message. */
typedef struct hbn_group_ready {
  uint64_t group;
  uint32_t has_soft_state;
  uint32_t raft_state;  /* HB_STATE_* */
  uint64_t lead;
  hbn_hard_state hard_state;
  hbn_snapshot snapshot;
  const hbn_entry* entries;
  uint64_t n_entries;
  const hbn_entry* committed_entries;
  uint64_t n_committed;
  const hbn_message* messages;
  uint64_t n_messages;
  uint32_t fault;
  uint32_t pad;
} hbn_group_ready;

/* Status (raft/status.go:22-49); progress only while leader. */
typedef struct hbn_group_status {
  uint64_t id;
  hbn_hard_state hard_state;
  uint64_t lead;
  uint32_t raft_state;
  uint32_t n_progress;
  uint64_t applied;
  uint64_t progress_id[HB_MAX_REPLICAS];
  hb_progress progress[HB_MAX_REPLICAS];
} hbn_group_status;

/* Config fields a group is created with (raft/raft.go:62-110); ID is the
 * MultiNode's id (raft/multinode.go:182), Storage is passed separately. */
typedef struct hbn_config {
  uint32_t election_tick;
  uint32_t heartbeat_tick;
  uint64_t applied;
} hbn_config;

typedef struct hbn_storage hbn_storage;
typedef struct hbn_node hbn_node;

const char* hbn_last_error(void);

/* ---- MemoryStorage (raft/storage.go:63-248) ------------------------------- */
int hbn_storage_new(hbn_storage** out);                       /* NewMemoryStorage :75-80 */
/* &MemoryStorage{ents: ents} as the reference's tests build it (ents[0] is the dummy). */
int hbn_storage_new_with_entries(const hbn_entry* ents, uint64_t n, hbn_storage** out);
/* Memory: the entries of every storage (and of every node's unstable log) live
 * in 512- and 64-byte blocks from process-wide block pools (1 GiB MAP_NORESERVE
 * regions carved into 2 MiB chunks).  A freed block returns to the pool's free
 * lists, not to the system: hbn_storage_free / hbn_stop / Compact make the
 * memory reusable by later storages in the same process, while the process
 * keeps its peak entry memory mapped for its lifetime. */
int hbn_storage_free(hbn_storage* s);
int hbn_storage_initial_state(hbn_storage* s, hbn_hard_state* hs, uint64_t* nodes, uint32_t cap, uint32_t* n_nodes);
int hbn_storage_set_hard_state(hbn_storage* s, const hbn_hard_state* hs);
int hbn_storage_entries(hbn_storage* s, uint64_t lo, uint64_t hi, uint64_t max_size,
                        const hbn_entry** out, uint64_t* n);
int hbn_storage_term(hbn_storage* s, uint64_t i, uint64_t* term);
int hbn_storage_last_index(hbn_storage* s, uint64_t* out);
int hbn_storage_first_index(hbn_storage* s, uint64_t* out);
int hbn_storage_snapshot(hbn_storage* s, hbn_snapshot* out);
int hbn_storage_apply_snapshot(hbn_storage* s, const hbn_snapshot* snap);
/* nodes == NULL is a nil *ConfState (keeps the stored one). */
int hbn_storage_create_snapshot(hbn_storage* s, uint64_t i, const uint64_t* nodes, uint32_t n_nodes,
                                const uint8_t* data, uint64_t data_len, hbn_snapshot* out);
int hbn_storage_compact(hbn_storage* s, uint64_t i);
int hbn_storage_append(hbn_storage* s, const hbn_entry* ents, uint64_t n);
/* Entry.Size() (gogo, raft/raftpb/raft.pb.go) — what limitSize sums. */
uint64_t hbn_entry_size(const hbn_entry* e);

/* ---- MultiNode (raft/multinode.go:12-49) ---------------------------------- */
/* StartMultiNode(id) on `device`: up to `capacity` groups of <= max_replicas
 * peers, Config.MaxInflightMsgs = max_inflight, MaxSizePerMsg = max_msg_size
 *
 * Engine limits (the reference has none of these: raft/raft.go:101-123 only
 * requires MaxInflightMsgs > 0, addNode raft/raft.go:729-738 takes any id):
 *   max_replicas <= HB_MAX_REPLICAS (7): a group's prs (self included) is at
 *     most max_replicas; CreateGroup with more peers, or an ApplyConfChange /
 *     snapshot restore that would add one, returns HBN_EUNSUPPORTED and leaves
 *     the group unchanged;
 *   1 <= max_inflight <= HB_MAX_INFLIGHT (1024), capacity <= 2^24 groups,
 *   max_batch < 2^31 messages per device step: hbn_start returns HB_EINVAL.
 * Within them every result is the reference's, bit for bit.
 * (any value: HB_NO_LIMIT, 0 or finite; the device's log index then holds
 * every entry's size, loaded and reserved by this library), at most max_batch
 * messages per device step (the batch is flushed early when it fills). */
int hbn_start(int device, uint64_t id, uint32_t capacity, uint32_t max_replicas, uint32_t max_inflight,
              uint64_t max_msg_size, uint64_t max_batch, hbn_node** out);
int hbn_stop(hbn_node* n);
/* CreateGroup (:181-217).  `storage` stays owned by the caller and must outlive
 * the group.  Empty storage: bootstrap with ConfChangeAddNode entries for
 * peer_ids (nil Context).  Otherwise restart from the storage (peers from the
 * snapshot's ConfState). */
int hbn_create_group(hbn_node* n, uint64_t group, const hbn_config* cfg, hbn_storage* storage,
                     const uint64_t* peer_ids, uint32_t n_peers);
int hbn_remove_group(hbn_node* n, uint64_t group);                    /* :219-222 */
int hbn_tick(hbn_node* n);                                            /* :264-275 */
int hbn_set_rand(hbn_node* n, uint64_t first, uint64_t count, const uint64_t* draws);
int hbn_campaign(hbn_node* n, uint64_t group);                        /* :369-375 */
int hbn_propose(hbn_node* n, uint64_t group, const uint8_t* data, uint64_t len);  /* :377-385 */
/* ProposeConfChange (:387-399); cc_context == NULL is a nil Context. */
int hbn_propose_conf_change(hbn_node* n, uint64_t group, uint64_t cc_id, uint32_t cc_type, uint64_t node_id,
                            const uint8_t* cc_context, uint64_t context_len);
/* Step (:431-439): local types are ignored, MsgProp goes the Propose way,
 * responses, reports and the follower side (MsgApp with its entries, whose
 * Index must run m.index+1, +2, ...; MsgHeartbeat; MsgSnap with its snapshot;
 * MsgVote) go to the device batch.  A MsgSnap whose ConfState differs from the
 * group's peers ends the batch (the restore reloads the group's prs). */
int hbn_step(hbn_node* n, uint64_t group, const hbn_message* m);
/* Bulk ingestion: exactly count calls of hbn_step(n, groups[i], &msgs[i]) /
 * hbn_propose(n, groups[i], data[i], len[i]) in order (data[i] NULL = nil
 * Data), in one call.  The reference hands each message to its run goroutine
 * over a channel (raft/multinode.go:401-415), and a cgo call costs ~100 ns, so
 * a binding collects a Ready cycle's network input and proposals and passes
 * them together; responses and proposals are laid into the device batch by the
 * node's host threads.  On an error, *done = the messages taken before the one
 * that failed (its error is returned, as hbn_step would). */
int hbn_step_many(hbn_node* n, uint64_t count, const uint64_t* groups, const hbn_message* msgs, uint64_t* done);
int hbn_propose_many(hbn_node* n, uint64_t count, const uint64_t* groups, const uint8_t* const* data,
                     const uint64_t* len, uint64_t* done);
/* Host threads for the per-group work of a Ready cycle (event replay, Ready
 * assembly, Advance, bulk ingestion); groups are independent, each worker owns
 * a disjoint set.  Default min(16, cores), or the HBN_THREADS environment
 * variable.  The calling thread is one of them.  Phases below a few thousand
 * groups run on the caller alone, except the event replay, the Ready assembly,
 * Advance and bulk ingestion, which take up to HBN_SMALL_WAYS workers (default
 * 4; 1 = the caller alone) from 512 groups / messages (2,048 event words) on.
 * Those partner workers are pinned, one physical core each, to the L3 domain
 * (CCD) of the thread that starts the node or sets its threads (HBN_PIN_L3=0:
 * not pinned), are woken when hbn_ready launches the device step and spin for
 * up to HBN_SPIN_US microseconds (default 150) after a job before blocking;
 * the other workers may run on any CPU of the container's cpuset. */
int hbn_set_threads(hbn_node* n, uint32_t threads);
/* Seconds the node's host side spent per phase since hbn_start (diagnostics;
 * out[0..min(cap, *count)), order: load sync, log-index reserve, hb_step call,
 * event fetch, event replay, stepped marks, Ready assembly, Ready merge,
 * Advance, bulk lookup, bulk responses, bulk proposals, batch reset). */
int hbn_profile(hbn_node* n, double* out, uint32_t cap, uint32_t* count);
int hbn_report_unreachable(hbn_node* n, uint64_t id, uint64_t group);           /* :461-469 */
int hbn_report_snapshot(hbn_node* n, uint64_t id, uint64_t group, int failure); /* :471-481 */
/* ApplyConfChange (:401-430, run :239-262): node_id 0 only resets pendingConf.
 * nodes_out (sorted, <= HB_MAX_REPLICAS) may be NULL. */
int hbn_apply_conf_change(hbn_node* n, uint64_t group, uint32_t cc_type, uint64_t node_id,
                          uint64_t* nodes_out, uint32_t* n_nodes);
/* Ready (:276-282): runs the pending device step and returns one hbn_ready per
 * group whose Ready containsUpdates (raft/node.go:96-100).  HBN_EAGAIN when
 * there is none or the previous Ready has not been advanced. */
int hbn_ready(hbn_node* n, const hbn_group_ready** out, uint64_t* count);
/* Advance (:284-299) for these groups of the last Ready (commitReady :137-164). */
int hbn_advance(hbn_node* n, const uint64_t* groups, uint64_t count);
int hbn_status(hbn_node* n, uint64_t group, hbn_group_status* out);         /* :302-309 */
/* The device handle underneath (statistics, profiling). */
hb_handle* hbn_engine(hbn_node* n);

#ifdef __cplusplus
}
#endif
#endif /* HBNODE_H_ */
