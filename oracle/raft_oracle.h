/*
 * raft_oracle.h — CPU restatement of the reference's raft leader bookkeeping.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle for the MI355X engine
 * (etcd_amd/csrc).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / CPU baseline; the
 * product path never calls it.
 *
 * It restates, sequentially and per group, the Go functions of the reference
 * (holandes22/etcd @ 2.1.0-alpha, package raft) that the engine replaces:
 *   raft/progress.go:69-237    Progress state machine + inflights ring
 *   raft/raft.go:215-490       q, send, sendAppend, bcast*, maybeCommit, reset,
 *                              appendEntry, become*, campaign, poll, Step
 *   raft/raft.go:494-649       stepLeader / stepCandidate / stepFollower (the
 *                              branches on the leader-bookkeeping path)
 *   raft/log.go:172-247        commitTo, term, maybeCommit
 *   raft/multinode.go:233-237  recvc membership filter
 * Each function below cites the lines it follows.  Go's map iteration order in
 * bcastAppend / bcastHeartbeat / campaign is unspecified; the oracle iterates
 * prs in slot order and parity on emitted messages is per-(group, peer).
 *
 * Parity status: pinned by transcriptions of the reference's own known-answer
 * tests (tests/test_oracle_kat.py).  The Go reference cannot be
 * built in this image (no Go toolchain), so there is no oracle/_ref build.
 */
#ifndef RAFT_ORACLE_H_
#define RAFT_ORACLE_H_

#include <stdint.h>
#include "../include/hipbatch.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_PEERS 8
#define ORC_NONE 0ull   /* raft.None, raft/raft.go:29 */

/* inflights, raft/progress.go:172-181 */
typedef struct orc_inflights {
  int start;
  int count;
  int size;
  uint64_t* buffer;
} orc_inflights;

/* Progress, raft/progress.go:37-67 */
typedef struct orc_progress {
  uint64_t match, next;
  int state;
  int paused;
  uint64_t pending_snapshot;
  orc_inflights ins;
} orc_progress;

/* Log term metadata.  raftLog.term(i) (raft/log.go:198-217) is 0 outside
 * [first_index-1, last_index] and otherwise the term of entry i (the dummy
 * entry first_index-1 carries the snapshot term).  Entry terms are stored
 * run-length encoded: run k covers [runs[k].index, runs[k+1].index). */
typedef struct orc_run {
  uint64_t index;
  uint64_t term;
} orc_run;

typedef struct orc_log {
  uint64_t first_index;
  uint64_t last_index;
  uint64_t committed;
  uint64_t applied;
  uint64_t snap_index;  /* raftLog.snapshot().Metadata.Index */
  int nruns, cap;
  orc_run* runs;
} orc_log;

/* pb.Message fields on this path (raft/raftpb/raft.pb.go:200-213).
 * Entries are represented by their index range [ent_lo, ent_hi]. */
typedef struct orc_msg {
  int type;
  uint64_t to, from, term, log_term, index, commit;
  int reject;
  uint64_t reject_hint;
  uint64_t nents;       /* len(m.Entries) */
  uint64_t ent_lo;      /* index of first entry (MsgApp) */
  uint64_t snap_index;  /* MsgSnap snapshot metadata index */
  const uint32_t* edesc;  /* MsgProp / MsgApp: descriptors of its nents entries (HB_ENT_DESC), or NULL */
  const uint64_t* eterm;  /* MsgApp: terms of its nents entries (Index = index + 1 + k) */
  uint64_t snap_term;     /* MsgSnap snapshot metadata term */
  int outsider;           /* batch path: the sender is outside prs (from = ORC_OUTSIDER) ... */
  int voted;              /* ... and HB_INFO_VOTED says it is the node this group voted for */
} orc_msg;

#define ORC_OUTSIDER 0xFFFFFFFFFFFFFFF0ull  /* id of a batch message's sender outside prs */

typedef struct orc_raft {
  /* pb.HardState + id, raft/raft.go:125-155 */
  uint64_t id;
  uint64_t term, vote, commit;
  orc_log log;
  int max_inflight;
  uint64_t max_msg_size;
  int n;                          /* len(prs) */
  uint64_t ids[ORC_MAX_PEERS];    /* prs keys, slot order */
  orc_progress prs[ORC_MAX_PEERS];
  int state;
  uint64_t lead;
  int pending_conf;
  int elapsed;
  int election_timeout;           /* r.electionTimeout (Config.ElectionTick) */
  int heartbeat_timeout;          /* r.heartbeatTimeout (Config.HeartbeatTick) */
  uint64_t rand_pos;              /* r.rand.Int() values taken so far */
  int nvotes;                     /* r.votes map */
  uint64_t vote_ids[ORC_MAX_PEERS + 1];
  int vote_vals[ORC_MAX_PEERS + 1];
  /* r.msgs */
  orc_msg* msgs;
  int nmsgs, msgs_cap;
  /* event sink (the engine's delta format, include/hipbatch.h) */
  hb_event* ev;
  uint64_t nev, ev_cap;
  uint32_t group;
  uint64_t arrival;               /* arrival index of the message being stepped */
  int fault;                      /* HB_FAULT_* once a reference panic happened */
  uint64_t n_won, n_lost;         /* elections won (-> leader) / lost by poll (-> follower) */
  /* Entry.Size() of the log's entries, as cumulative sums (finite
   * max_msg_size): szc[i - szc_base] = sum of sizes of (szc_base, i].  sz_lo
   * = the oldest index whose size the caller loaded into the engine's log
   * index (hb_load_entry_sizes), mirrored so that the engine precondition
   * HB_FAULT_SIZE_WINDOW is checked too; the harness reserves ring capacity
   * (hb_reserve_log), so the engine drops nothing the oracle keeps. */
  uint64_t* szc;
  uint64_t szc_base, szc_n, szc_cap, sz_lo;
  /* What the engine's log index knows of the terms (follower side; the terms
   * themselves come from `log`): the oldest older-run start it holds (tw_lo,
   * HB_NO_INDEX: none) plus the current-term run [tw_tfirst, last_index];
   * a lookup below both is the engine precondition HB_FAULT_TERM_WINDOW. */
  uint64_t tw_lo;
  uint64_t tw_tfirst;
} orc_raft;

/* ---- inflights (raft/progress.go:183-237) ---- */
void orc_ins_init(orc_inflights* in, int size);
void orc_ins_free(orc_inflights* in);
int  orc_ins_add(orc_inflights* in, uint64_t inflight);  /* -1 = panic (full) */
void orc_ins_free_to(orc_inflights* in, uint64_t to);
void orc_ins_free_first_one(orc_inflights* in);
int  orc_ins_full(const orc_inflights* in);
void orc_ins_reset(orc_inflights* in);

/* ---- Progress (raft/progress.go:69-166) ---- */
void orc_pr_reset_state(orc_progress* pr, int state);
void orc_pr_become_probe(orc_progress* pr);
void orc_pr_become_replicate(orc_progress* pr);
void orc_pr_become_snapshot(orc_progress* pr, uint64_t snapshoti);
int  orc_pr_maybe_update(orc_progress* pr, uint64_t n);
void orc_pr_optimistic_update(orc_progress* pr, uint64_t n);
int  orc_pr_maybe_decr_to(orc_progress* pr, uint64_t rejected, uint64_t last);
void orc_pr_pause(orc_progress* pr);
void orc_pr_resume(orc_progress* pr);
int  orc_pr_is_paused(const orc_progress* pr);
void orc_pr_snapshot_failure(orc_progress* pr);
int  orc_pr_maybe_snapshot_abort(const orc_progress* pr);

/* ---- log (raft/log.go) ---- */
void     orc_log_init(orc_log* l, uint64_t first_index, uint64_t dummy_term);
void     orc_log_free(orc_log* l);
void     orc_log_push(orc_log* l, uint64_t term, uint64_t k);    /* append k entries of term */
uint64_t orc_log_term(const orc_log* l, uint64_t i);
uint64_t orc_log_last_term(const orc_log* l);

/* ---- raft ---- */
/* newRaft (raft/raft.go:157-209) with Config peers; the log must be set up
 * with orc_raft_log() first (or left empty = NewMemoryStorage()). */
void orc_raft_init(orc_raft* r, uint64_t id, const uint64_t* peers, int npeers,
                   int max_inflight, uint64_t max_msg_size);
void orc_raft_free(orc_raft* r);
orc_log* orc_raft_log(orc_raft* r);
int  orc_raft_slot(const orc_raft* r, uint64_t id);  /* -1 if id not in prs */
orc_progress* orc_raft_pr(orc_raft* r, uint64_t id);
void orc_raft_set_progress(orc_raft* r, uint64_t id, uint64_t match, uint64_t next);
void orc_raft_load_state(orc_raft* r, uint64_t term, uint64_t vote, uint64_t commit);
int  orc_raft_q(const orc_raft* r);
void orc_raft_reset(orc_raft* r, uint64_t term);
void orc_raft_send_append(orc_raft* r, uint64_t to);
void orc_raft_bcast_append(orc_raft* r);
void orc_raft_bcast_heartbeat(orc_raft* r);
int  orc_raft_maybe_commit(orc_raft* r);
void orc_raft_append_entry(orc_raft* r, uint64_t k, int noop);
/* entry sizes (finite MaxSizePerMsg): gogo Entry.Size() (raft/raftpb/raft.pb.go:
 * 1030-1043) of a descriptor's entry, limitSize (raft/util.go:97-110) over
 * entry sizes (how many entries it keeps), and the sizes of a loaded group's
 * last n entries (hb_load_entry_sizes' contract) */
uint64_t orc_entry_size(uint32_t desc, uint64_t term, uint64_t index);
uint64_t orc_limit_size(const uint64_t* sizes, uint64_t n, uint64_t max_size);
int  orc_raft_load_sizes(orc_raft* r, uint32_t n, const uint32_t* sizes);
/* follower side (raft/raft.go:616-707, raft/log.go:72-123, 235-239) */
void orc_log_truncate(orc_log* l, uint64_t after);       /* keep entries <= after */
uint64_t orc_log_find_conflict(const orc_log* l, uint64_t from, const uint64_t* terms, uint64_t n);
int  orc_log_is_up_to_date(const orc_log* l, uint64_t lasti, uint64_t term);
/* the engine's older term runs of a loaded group (hb_load_term_runs' contract) */
int  orc_raft_load_term_runs(orc_raft* r, uint32_t n, const uint64_t* runs);
/* raftLog.maybeAppend (raft/log.go:72-88) on a bare log: 1 appended (*lastnewi
 * set), 0 no match, -1 the reference's "conflict with committed entry" panic */
int  orc_log_maybe_append(orc_log* l, uint64_t index, uint64_t log_term, uint64_t committed,
                          const uint64_t* terms, uint64_t n, uint64_t* lastnewi);
void orc_raft_handle_append_entries(orc_raft* r, const orc_msg* m);  /* raft/raft.go:651-665 */
void orc_raft_handle_heartbeat(orc_raft* r, const orc_msg* m);       /* raft/raft.go:666-669 */
void orc_raft_become_follower(orc_raft* r, uint64_t term, uint64_t lead);
void orc_raft_become_candidate(orc_raft* r);
void orc_raft_become_leader(orc_raft* r);
void orc_raft_campaign(orc_raft* r);
int  orc_raft_poll(orc_raft* r, uint64_t id, int v);
void orc_raft_step(orc_raft* r, const orc_msg* m);
void orc_raft_commit_to(orc_raft* r, uint64_t tocommit);
/* readMessages (raft/raft_test.go:44-49): copies up to cap, clears, returns count */
int  orc_raft_read_messages(orc_raft* r, orc_msg* out, int cap);

/* ---- engine-format conversion + batch driver (parity harness) ---- */
uint32_t orc_raft_ref(const orc_raft* r, uint64_t id);   /* node id -> HB_REF_* */
/* Build a group from the engine record plus its log term runs (runs[0].index
 * must be first_index-1; terms non-decreasing).  Node ids are slot+1 and the
 * local id is self_slot+1 (or 100 when HB_SLOT_NONE); lead/vote refs of
 * HB_REF_OTHER become id 99. */
int  orc_raft_from_group(orc_raft* r, const hb_group* g, const orc_run* runs, int nruns,
                         int max_inflight, uint64_t max_msg_size);
/* Export to the engine record (term_first/term_last derived from the runs). */
void orc_raft_to_group(const orc_raft* r, hb_group* g);
/* Inflight window of prs[slot]: buffer[(start+i) % size] = vals[i]. */
int  orc_raft_set_inflights(orc_raft* r, int slot, int start, int count, const uint64_t* vals);
int  orc_raft_get_inflights(const orc_raft* r, int slot, uint64_t* vals /* [count] */);

/* Step one engine batch over `ngroups` groups exactly as MultiNode.run would
 * (props first per group, then messages in arrival order).  Events go to
 * ev[0..*nev).  Returns 0, or -1 if ev_cap was too small. */
int orc_step_batch(orc_raft* groups, uint32_t ngroups, const hb_batch* b,
                   hb_event* ev, uint64_t ev_cap, uint64_t* nev,
                   uint64_t stats[HB_STAT_COUNT]);

/* Tick (raft/raft.go:362-382, isElectionTimeout :765-771); r.rand.Int() is
 * draws[r->rand_pos++] (the shared rand.NewSource(id) stream).  Returns the
 * local message type stepped (HB_MSG_BEAT / HB_MSG_HUP) or -1. */
int orc_raft_tick(orc_raft* r, const uint64_t* draws, uint64_t ndraws);
/* MultiNode.Tick over all groups (raft/multinode.go:264-275), events and
 * statistics as orc_step_batch. */
int orc_tick_batch(orc_raft* groups, uint32_t ngroups, const uint64_t* draws, uint64_t ndraws,
                   hb_event* ev, uint64_t ev_cap, uint64_t* nev, uint64_t stats[HB_STAT_COUNT]);
void orc_groups_load_timers(orc_raft* gs, uint32_t n, const hb_timer* t);
void orc_groups_export_timers(const orc_raft* gs, uint32_t n, hb_timer* out);

/* ---- wire decoding (wire_oracle.c: raft/raftpb/raft.pb.go Unmarshal) ---- */
typedef struct orc_wire_msg {
  int32_t type;
  uint64_t to, from, term, log_term, index, commit, reject_hint;
  int reject;
  uint32_t nentries;
} orc_wire_msg;
/* 0 = ok, 1 = Unmarshal error, 2 = Go panic / endless loop, 3 = groups nested too deep */
int  orc_unmarshal_message(const uint8_t* data, int64_t len, orc_wire_msg* m);
/* hb_decode's contract on the CPU; peers [capacity][HB_MAX_REPLICAS], group_n [capacity] */
void orc_decode_batch(const uint8_t* bytes, const uint64_t* off, const uint32_t* len, const uint32_t* group,
                      uint64_t n, uint32_t capacity, const uint32_t* group_n, const uint64_t* peers,
                      uint32_t* o_group, uint32_t* o_info, uint64_t* o_term, uint64_t* o_index, uint64_t* o_hint,
                      uint8_t* status);

/* Flat-array helpers so the Python harness can drive many groups via ctypes. */
orc_raft* orc_groups_new(uint32_t ngroups);
void      orc_groups_free(orc_raft* g, uint32_t ngroups);
int       orc_groups_load(orc_raft* gs, uint32_t n, const hb_group* recs, const orc_run* runs,
                          const uint64_t* run_off, int max_inflight, uint64_t max_msg_size);
void      orc_groups_export(const orc_raft* gs, uint32_t n, hb_group* out);
/* per group out[4i..4i+3] = log term runs, sz_lo (oldest loaded size), first_index, last_index */
void      orc_groups_log_info(const orc_raft* gs, uint32_t n, uint64_t* out);
orc_raft* orc_groups_at(orc_raft* g, uint32_t i);
size_t    orc_sizeof_raft(void);

#ifdef __cplusplus
}
#endif
#endif
