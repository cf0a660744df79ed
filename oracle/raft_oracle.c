/*
 * raft_oracle.c — CPU restatement of the reference raft leader bookkeeping.
 * TEST INFRASTRUCTURE ONLY (see raft_oracle.h).  Every function cites the
 * reference Go it restates (paths relative to holandes22/etcd).
 */
#include "raft_oracle.h"

#include <stdlib.h>
#include <string.h>

static inline uint64_t umin(uint64_t a, uint64_t b) { return a > b ? b : a; }  /* raft/util.go:35-40 */
static inline uint64_t umax(uint64_t a, uint64_t b) { return a > b ? a : b; }  /* raft/util.go:42-47 */

/* ========================================================================
 * inflights — raft/progress.go:172-237
 * ======================================================================== */
void orc_ins_init(orc_inflights* in, int size) {          /* newInflights :183-188 */
  in->start = 0;
  in->count = 0;
  in->size = size;
  in->buffer = (uint64_t*)calloc((size_t)(size > 0 ? size : 1), sizeof(uint64_t));
}

void orc_ins_free(orc_inflights* in) {
  free(in->buffer);
  in->buffer = NULL;
}

int orc_ins_full(const orc_inflights* in) { return in->count == in->size; }  /* :229-231 */

int orc_ins_add(orc_inflights* in, uint64_t inflight) {   /* add :191-201 */
  if (orc_ins_full(in)) return -1;                        /* panic "cannot add into a full inflights" */
  int next = in->start + in->count;
  if (next >= in->size) next -= in->size;
  in->buffer[next] = inflight;
  in->count++;
  return 0;
}

void orc_ins_free_to(orc_inflights* in, uint64_t to) {    /* freeTo :204-224 */
  if (in->count == 0 || to < in->buffer[in->start]) return;
  int i, idx = in->start;
  for (i = 0; i < in->count; i++) {
    if (to < in->buffer[idx]) break;
    if (++idx >= in->size) idx -= in->size;
  }
  in->count -= i;
  in->start = idx;
}

void orc_ins_free_first_one(orc_inflights* in) {          /* :226 */
  orc_ins_free_to(in, in->buffer[in->start]);
}

void orc_ins_reset(orc_inflights* in) {                   /* :234-237 */
  in->count = 0;
  in->start = 0;
}

/* ========================================================================
 * Progress — raft/progress.go:69-166
 * ======================================================================== */
void orc_pr_reset_state(orc_progress* pr, int state) {    /* resetState :69-74 */
  pr->paused = 0;
  pr->pending_snapshot = 0;
  pr->state = state;
  orc_ins_reset(&pr->ins);
}

void orc_pr_become_probe(orc_progress* pr) {              /* :76-88 */
  if (pr->state == HB_PR_SNAPSHOT) {
    uint64_t pending = pr->pending_snapshot;
    orc_pr_reset_state(pr, HB_PR_PROBE);
    pr->next = umax(pr->match + 1, pending + 1);
  } else {
    orc_pr_reset_state(pr, HB_PR_PROBE);
    pr->next = pr->match + 1;
  }
}

void orc_pr_become_replicate(orc_progress* pr) {          /* :90-93 */
  orc_pr_reset_state(pr, HB_PR_REPLICATE);
  pr->next = pr->match + 1;
}

void orc_pr_become_snapshot(orc_progress* pr, uint64_t snapshoti) {  /* :95-98 */
  orc_pr_reset_state(pr, HB_PR_SNAPSHOT);
  pr->pending_snapshot = snapshoti;
}

void orc_pr_pause(orc_progress* pr) { pr->paused = 1; }   /* :143 */
void orc_pr_resume(orc_progress* pr) { pr->paused = 0; }  /* :144 */

int orc_pr_maybe_update(orc_progress* pr, uint64_t n) {   /* :102-113 */
  int updated = 0;
  if (pr->match < n) {
    pr->match = n;
    updated = 1;
    orc_pr_resume(pr);
  }
  if (pr->next < n + 1) pr->next = n + 1;
  return updated;
}

void orc_pr_optimistic_update(orc_progress* pr, uint64_t n) { pr->next = n + 1; }  /* :115 */

int orc_pr_maybe_decr_to(orc_progress* pr, uint64_t rejected, uint64_t last) {  /* :119-141 */
  if (pr->state == HB_PR_REPLICATE) {
    if (rejected <= pr->match) return 0;
    pr->next = pr->match + 1;
    return 1;
  }
  if (pr->next - 1 != rejected) return 0;
  pr->next = umin(rejected, last + 1);
  if (pr->next < 1) pr->next = 1;
  orc_pr_resume(pr);
  return 1;
}

int orc_pr_is_paused(const orc_progress* pr) {            /* :147-158 */
  switch (pr->state) {
    case HB_PR_PROBE: return pr->paused;
    case HB_PR_REPLICATE: return orc_ins_full(&pr->ins);
    default: return 1;                                    /* ProgressStateSnapshot */
  }
}

void orc_pr_snapshot_failure(orc_progress* pr) { pr->pending_snapshot = 0; }  /* :160 */

int orc_pr_maybe_snapshot_abort(const orc_progress* pr) { /* :164-166 */
  return pr->state == HB_PR_SNAPSHOT && pr->match >= pr->pending_snapshot;
}

/* ========================================================================
 * log metadata — raft/log.go, raft/log_unstable.go
 * ======================================================================== */
void orc_log_init(orc_log* l, uint64_t first_index, uint64_t dummy_term) {
  /* newLog (raft/log.go:43-64): committed = applied = firstIndex-1 */
  memset(l, 0, sizeof(*l));
  l->first_index = first_index;
  l->last_index = first_index - 1;
  l->committed = first_index - 1;
  l->applied = first_index - 1;
  l->cap = 4;
  l->runs = (orc_run*)malloc(sizeof(orc_run) * (size_t)l->cap);
  l->runs[0].index = first_index - 1;  /* dummy entry (snapshot index) */
  l->runs[0].term = dummy_term;
  l->nruns = 1;
}

void orc_log_free(orc_log* l) {
  free(l->runs);
  l->runs = NULL;
  l->nruns = l->cap = 0;
}

void orc_log_push(orc_log* l, uint64_t term, uint64_t k) {
  if (k == 0) return;
  if (l->runs[l->nruns - 1].term != term) {
    if (l->nruns == l->cap) {
      l->cap *= 2;
      l->runs = (orc_run*)realloc(l->runs, sizeof(orc_run) * (size_t)l->cap);
    }
    l->runs[l->nruns].index = l->last_index + 1;
    l->runs[l->nruns].term = term;
    l->nruns++;
  }
  l->last_index += k;
}

uint64_t orc_log_term(const orc_log* l, uint64_t i) {     /* term raft/log.go:198-217 */
  uint64_t dummy = l->first_index - 1;
  if (i < dummy || i > l->last_index) return 0;
  int lo = 0, hi = l->nruns - 1;                          /* last run with index <= i */
  while (lo < hi) {
    int mid = (lo + hi + 1) / 2;
    if (l->runs[mid].index <= i) lo = mid; else hi = mid - 1;
  }
  return l->runs[lo].term;
}

uint64_t orc_log_last_term(const orc_log* l) {            /* lastTerm raft/log.go:196 */
  return orc_log_term(l, l->last_index);
}

void orc_log_truncate(orc_log* l, uint64_t after) {      /* unstable.truncateAndAppend's cut */
  while (l->nruns > 1 && l->runs[l->nruns - 1].index > after) l->nruns--;
  l->last_index = after;
}

uint64_t orc_log_find_conflict(const orc_log* l, uint64_t from, const uint64_t* terms, uint64_t n) {
  /* findConflict raft/log.go:112-123: first entry whose term does not match */
  for (uint64_t k = 0; k < n; k++)
    if (orc_log_term(l, from + k) != terms[k]) return from + k;
  return 0;
}

int orc_log_is_up_to_date(const orc_log* l, uint64_t lasti, uint64_t term) {  /* :235-237 */
  uint64_t lt = orc_log_last_term(l);
  return term > lt || (term == lt && lasti >= l->last_index);
}

/* ========================================================================
 * raft — raft/raft.go
 * ======================================================================== */
static void fault(orc_raft* r, int code);
static void tw_push(orc_raft* r, uint64_t start, uint64_t term);

static void emit(orc_raft* r, int type, int to, uint64_t x, int aux) {
  if (r->ev) {
    if (r->nev < r->ev_cap) {
      hb_event* e = &r->ev[r->nev];
      e->x = x;
      e->group = r->group;
      e->type = (uint8_t)type;
      e->to = (uint8_t)to;
      e->aux = (uint16_t)aux;
    }
    r->nev++;
  }
}

static void fault(orc_raft* r, int code) {
  if (r->fault) return;
  r->fault = code;
  emit(r, HB_EV_FAULT, 0, r->arrival, code);
}

int orc_raft_slot(const orc_raft* r, uint64_t id) {
  for (int i = 0; i < r->n; i++)
    if (r->ids[i] == id) return i;
  return -1;
}

orc_progress* orc_raft_pr(orc_raft* r, uint64_t id) {
  int s = orc_raft_slot(r, id);
  return s < 0 ? NULL : &r->prs[s];
}

uint32_t orc_raft_ref(const orc_raft* r, uint64_t id) {
  if (id == ORC_NONE) return HB_REF_NONE;
  int s = orc_raft_slot(r, id);
  if (s >= 0) return (uint32_t)s;
  if (id == r->id) return HB_REF_SELF;
  return HB_REF_OTHER;
}

static uint64_t soft_pack(const orc_raft* r) {
  return (uint64_t)r->state | ((uint64_t)orc_raft_ref(r, r->lead) << 8) |
         ((uint64_t)orc_raft_ref(r, r->vote) << 16);
}

orc_log* orc_raft_log(orc_raft* r) { return &r->log; }

void orc_raft_init(orc_raft* r, uint64_t id, const uint64_t* peers, int npeers,
                   int max_inflight, uint64_t max_msg_size) {
  /* newRaft (raft/raft.go:157-209).  The caller set up r->log beforehand
   * (zeroed struct => empty MemoryStorage: firstIndex 1, lastIndex 0). */
  orc_log saved = r->log;
  memset(r, 0, sizeof(*r));
  if (saved.runs) r->log = saved; else orc_log_init(&r->log, 1, 0);
  r->id = id;
  r->max_inflight = max_inflight;
  r->max_msg_size = max_msg_size;
  r->election_timeout = 10;                               /* engine defaults (hb_create) */
  r->heartbeat_timeout = 1;
  r->n = 0;
  for (int i = 0; i < npeers && i < ORC_MAX_PEERS; i++) {
    r->ids[r->n] = peers[i];
    memset(&r->prs[r->n], 0, sizeof(orc_progress));
    r->prs[r->n].next = 1;                                /* :190-192 */
    orc_ins_init(&r->prs[r->n].ins, max_inflight);
    r->n++;
  }
  r->state = HB_STATE_FOLLOWER;
  r->tw_tfirst = HB_NO_INDEX;                             /* KAT rafts: the engine would know every run */
  r->tw_lo = HB_NO_INDEX;
  for (int k = 0; k < r->log.nruns; k++) tw_push(r, r->log.runs[k].index, r->log.runs[k].term);
  orc_raft_become_follower(r, r->term, ORC_NONE);         /* :199 */
}

void orc_raft_free(orc_raft* r) {
  for (int i = 0; i < r->n; i++) orc_ins_free(&r->prs[i].ins);
  orc_log_free(&r->log);
  free(r->msgs);
  r->msgs = NULL;
  free(r->szc);
  r->szc = NULL;
  r->n = 0;
}

void orc_raft_set_progress(orc_raft* r, uint64_t id, uint64_t match, uint64_t next) {
  /* setProgress raft/raft.go:744-746 (adds the id when absent) */
  int s = orc_raft_slot(r, id);
  if (s < 0) {
    if (r->n >= ORC_MAX_PEERS) return;
    s = r->n++;
    r->ids[s] = id;
  } else {
    orc_ins_free(&r->prs[s].ins);
  }
  memset(&r->prs[s], 0, sizeof(orc_progress));
  r->prs[s].match = match;
  r->prs[s].next = next;
  orc_ins_init(&r->prs[s].ins, r->max_inflight);
}

void orc_raft_load_state(orc_raft* r, uint64_t term, uint64_t vote, uint64_t commit) {
  /* loadState raft/raft.go:752-760 */
  r->log.committed = commit;
  r->term = term;
  r->vote = vote;
  r->commit = commit;
}

int orc_raft_q(const orc_raft* r) { return r->n / 2 + 1; }  /* q raft/raft.go:215 */

static void send(orc_raft* r, orc_msg m) {                /* send raft/raft.go:227-236 */
  m.from = r->id;
  if (m.type != HB_MSG_PROP) m.term = r->term;
  if (r->nmsgs == r->msgs_cap) {
    r->msgs_cap = r->msgs_cap ? r->msgs_cap * 2 : 8;
    r->msgs = (orc_msg*)realloc(r->msgs, sizeof(orc_msg) * (size_t)r->msgs_cap);
  }
  r->msgs[r->nmsgs++] = m;
  int to = (int)orc_raft_ref(r, m.to);
  switch (m.type) {
    case HB_MSG_APP: emit(r, HB_EV_APP, to, m.index, m.log_term == r->term ? 1 : 0); break;  /* aux: LogTerm == Term */
    case HB_MSG_SNAP: emit(r, HB_EV_SNAP, to, m.snap_index, 0); break;
    case HB_MSG_HEARTBEAT: emit(r, HB_EV_HEARTBEAT, to, m.commit, 0); break;
    case HB_MSG_VOTE: emit(r, HB_EV_VOTE, to, m.index, 0); break;
    case HB_MSG_PROP: emit(r, HB_EV_PROP_FWD, to, r->arrival, 0); break;
    case HB_MSG_APP_RESP: emit(r, HB_EV_RESP, to, m.index, HB_RESP_APP | (m.reject ? HB_RESP_REJECT : 0)); break;
    case HB_MSG_HEARTBEAT_RESP: emit(r, HB_EV_RESP, to, 0, HB_RESP_HEARTBEAT); break;
    case HB_MSG_VOTE_RESP: emit(r, HB_EV_RESP, to, 0, HB_RESP_VOTE | (m.reject ? HB_RESP_REJECT : 0)); break;
    default: break;
  }
}

int orc_raft_read_messages(orc_raft* r, orc_msg* out, int cap) {
  int n = r->nmsgs;
  const int k = n < cap ? n : cap;
  if (out && k > 0) memcpy(out, r->msgs, sizeof(orc_msg) * (size_t)k);
  r->nmsgs = 0;
  return n;
}

void orc_raft_commit_to(orc_raft* r, uint64_t tocommit) { /* commitTo raft/log.go:172-180 */
  if (r->log.committed < tocommit) {
    if (r->log.last_index < tocommit) {
      fault(r, HB_FAULT_COMMIT_RANGE);
      return;
    }
    r->log.committed = tocommit;
    emit(r, HB_EV_COMMIT, 0, tocommit, 0);
  }
}

/* ---- what the engine's log index knows of the terms (follower side) ----
 * The engine's term runs hold every run the caller loaded (hb_load_term_runs)
 * plus the ones its own appends / resets started; the harness reserves ring
 * capacity so none is dropped (hb_reserve_log).  All the oracle tracks is
 * the oldest run start the engine knows (tw_lo) and its current-term run; the
 * terms themselves come from `log`. */
static void tw_push(orc_raft* r, uint64_t start, uint64_t term) {
  (void)term;
  if (r->tw_lo == HB_NO_INDEX) r->tw_lo = start;
}

static void tw_term_change(orc_raft* r, uint64_t old_term) {  /* reset to a new Term */
  if (r->tw_tfirst != HB_NO_INDEX) tw_push(r, r->tw_tfirst, old_term);
  r->tw_tfirst = HB_NO_INDEX;
}

static void tw_leader_append(orc_raft* r, uint64_t first_new) {  /* entries at Term */
  if (r->tw_tfirst == HB_NO_INDEX) r->tw_tfirst = first_new;
}

/* the engine knows term(i) for every i >= this in [first-1, last] */
static uint64_t tw_known_lo(const orc_raft* r) {
  if (r->tw_lo != HB_NO_INDEX) return r->tw_lo;
  if (r->tw_tfirst != HB_NO_INDEX) return r->tw_tfirst;
  return r->log.last_index + 1;
}

/* raftLog.term(i) on the follower side; sets the engine-defined fault when
 * the engine could not answer (returns 0 then) */
static uint64_t f_term(orc_raft* r, uint64_t i) {
  if (i + 1 < r->log.first_index || i > r->log.last_index) return 0;
  if (i < tw_known_lo(r)) {
    fault(r, HB_FAULT_TERM_WINDOW);
    return 0;
  }
  return orc_log_term(&r->log, i);
}

int orc_raft_load_term_runs(orc_raft* r, uint32_t n, const uint64_t* runs) {
  r->tw_lo = n > 0 ? runs[0] : HB_NO_INDEX;
  return 0;
}

/* ---- entry sizes (finite MaxSizePerMsg) ---- */
static uint64_t sov_raft(uint64_t x) {                    /* sovRaft raft/raftpb/raft.pb.go */
  uint64_t n = 0;
  for (;;) {
    n++;
    x >>= 7;
    if (x == 0) break;
  }
  return n;
}

uint64_t orc_entry_size(uint32_t desc, uint64_t term, uint64_t index) {  /* Entry.Size() :1030-1043 */
  uint64_t n = 0;
  n += 1 + sov_raft((desc >> 30) & 1u);                   /* Type */
  n += 1 + sov_raft(term);
  n += 1 + sov_raft(index);
  if (desc >> 31) {                                       /* Data != nil */
    uint64_t l = desc & HB_ENT_MAX_DATA;
    n += 1 + l + sov_raft(l);
  }
  return n;
}

uint64_t orc_limit_size(const uint64_t* sizes, uint64_t n, uint64_t max_size) {  /* limitSize raft/util.go:97-110 */
  if (n == 0) return 0;
  uint64_t size = sizes[0];
  uint64_t limit;
  for (limit = 1; limit < n; limit++) {
    size += sizes[limit];
    if (size > max_size) break;
  }
  return limit;
}

static int sized(const orc_raft* r) { return r->max_msg_size != 0 && r->max_msg_size != HB_NO_LIMIT; }

static void szc_push(orc_raft* r, uint64_t v) {
  if (r->szc_n == r->szc_cap) {
    r->szc_cap = r->szc_cap ? 2 * r->szc_cap : 16;
    r->szc = (uint64_t*)realloc(r->szc, sizeof(uint64_t) * (size_t)r->szc_cap);
  }
  r->szc[r->szc_n++] = v;
}

static void szc_reset(orc_raft* r, uint64_t base) {      /* no entry size known: szc = {base: 0} */
  r->szc_n = 0;
  r->szc_base = base;
  r->sz_lo = base;
  szc_push(r, 0);
}

int orc_raft_load_sizes(orc_raft* r, uint32_t n, const uint32_t* sizes) {
  if (!sized(r) || n > r->log.last_index) return -1;
  szc_reset(r, r->log.last_index - n);
  uint64_t acc = 0;
  for (uint32_t j = 0; j < n; j++) szc_push(r, acc += sizes[j]);
  return 0;
}

/* entries (last0, last0 + k] appended at the current Term (appendEntry) */
static void szc_append(orc_raft* r, uint64_t last0, uint64_t k, const uint32_t* desc) {
  if (!sized(r)) return;
  if (r->szc_n == 0) szc_reset(r, last0);                 /* a raft built by orc_raft_init */
  uint64_t acc = r->szc[last0 - r->szc_base];
  for (uint64_t j = 1; j <= k; j++) szc_push(r, acc += orc_entry_size(desc ? desc[j - 1] : 0u, r->term, last0 + j));
}

/* the last index of entries(next, maxMsgSize) (raft/log.go:219-224 + limitSize);
 * -1 when the engine would not hold the sizes it needs */
static int64_t entries_last(orc_raft* r, uint64_t next) {
  uint64_t last = r->log.last_index;
  if (r->max_msg_size == HB_NO_LIMIT) return (int64_t)last;
  if (r->max_msg_size == 0) return (int64_t)next;
  if (r->szc_n == 0) szc_reset(r, last);                  /* a raft built by orc_raft_init */
  if (next - 1 < r->sz_lo) return -1;
  uint64_t n = last - next + 1;
  uint64_t* sz = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
  for (uint64_t i = 0; i < n; i++) {
    uint64_t idx = next + i;
    sz[i] = r->szc[idx - r->szc_base] - r->szc[idx - 1 - r->szc_base];
  }
  uint64_t k = orc_limit_size(sz, n, r->max_msg_size);
  free(sz);
  return (int64_t)(next + k - 1);
}

void orc_raft_send_append(orc_raft* r, uint64_t to) {     /* sendAppend raft/raft.go:239-282 */
  orc_progress* pr = orc_raft_pr(r, to);
  if (!pr) { fault(r, HB_FAULT_NIL_PROGRESS); return; }
  if (orc_pr_is_paused(pr)) return;
  orc_msg m;
  memset(&m, 0, sizeof(m));
  m.to = to;
  if (pr->next < r->log.first_index) {                    /* needSnapshot :715-717 */
    m.type = HB_MSG_SNAP;
    if (r->log.snap_index == 0) { fault(r, HB_FAULT_EMPTY_SNAPSHOT); return; }  /* :252-254 */
    m.snap_index = r->log.snap_index;
    orc_pr_become_snapshot(pr, r->log.snap_index);
  } else {
    m.type = HB_MSG_APP;
    m.index = pr->next - 1;
    m.log_term = orc_log_term(&r->log, pr->next - 1);
    /* entries(Next, maxMsgSize) raft/log.go:219-224 + limitSize raft/util.go:97-110:
     * noLimit -> through lastIndex; 0 -> exactly one entry; finite -> limitSize */
    if (pr->next <= r->log.last_index) {
      int64_t last = entries_last(r, pr->next);
      if (last < 0) { fault(r, HB_FAULT_SIZE_WINDOW); return; }
      m.nents = (uint64_t)last - pr->next + 1;
      m.ent_lo = pr->next;
    }
    m.commit = r->log.committed;
    if (m.nents != 0) {
      uint64_t last = m.ent_lo + m.nents - 1;
      switch (pr->state) {
        case HB_PR_REPLICATE:
          orc_pr_optimistic_update(pr, last);
          if (orc_ins_add(&pr->ins, last) < 0) { fault(r, HB_FAULT_INFLIGHTS_FULL); return; }
          break;
        case HB_PR_PROBE:
          orc_pr_pause(pr);
          break;
        default:
          break;  /* unreachable: isPaused() is true in Snapshot */
      }
    }
  }
  send(r, m);
}

static void send_heartbeat(orc_raft* r, int slot) {       /* sendHeartbeat raft/raft.go:285-299 */
  orc_msg m;
  memset(&m, 0, sizeof(m));
  m.to = r->ids[slot];
  m.type = HB_MSG_HEARTBEAT;
  m.commit = umin(r->prs[slot].match, r->log.committed);
  send(r, m);
}

void orc_raft_bcast_append(orc_raft* r) {                 /* bcastAppend raft/raft.go:303-310 */
  for (int i = 0; i < r->n && !r->fault; i++) {
    if (r->ids[i] == r->id) continue;
    orc_raft_send_append(r, r->ids[i]);
  }
}

void orc_raft_bcast_heartbeat(orc_raft* r) {              /* bcastHeartbeat raft/raft.go:313-321 */
  for (int i = 0; i < r->n; i++) {
    if (r->ids[i] == r->id) continue;
    send_heartbeat(r, i);
    orc_pr_resume(&r->prs[i]);
  }
}

static int cmp_desc(const void* a, const void* b) {
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? 1 : (x > y ? -1 : 0);
}

int orc_raft_maybe_commit(orc_raft* r) {                  /* maybeCommit raft/raft.go:323-332 */
  uint64_t mis[ORC_MAX_PEERS];
  for (int i = 0; i < r->n; i++) mis[i] = r->prs[i].match;
  qsort(mis, (size_t)r->n, sizeof(uint64_t), cmp_desc);   /* sort.Sort(sort.Reverse(mis)) */
  uint64_t mci = mis[orc_raft_q(r) - 1];
  /* raftLog.maybeCommit raft/log.go:241-247 */
  if (mci > r->log.committed && orc_log_term(&r->log, mci) == r->term) {
    orc_raft_commit_to(r, mci);
    return !r->fault;
  }
  return 0;
}

void orc_raft_reset(orc_raft* r, uint64_t term) {         /* reset raft/raft.go:334-349 */
  if (r->term != term) {
    tw_term_change(r, r->term);
    r->term = term;
    r->vote = ORC_NONE;
    emit(r, HB_EV_TERM, 0, term, 0);
  }
  r->lead = ORC_NONE;
  r->elapsed = 0;
  r->nvotes = 0;
  for (int i = 0; i < r->n; i++) {
    orc_progress* pr = &r->prs[i];
    orc_ins_free(&pr->ins);
    memset(pr, 0, sizeof(*pr));
    pr->next = r->log.last_index + 1;
    orc_ins_init(&pr->ins, r->max_inflight);
    if (r->ids[i] == r->id) pr->match = r->log.last_index;
  }
  r->pending_conf = 0;
}

static void append_entries(orc_raft* r, uint64_t k, int noop, const uint32_t* desc) {  /* appendEntry raft/raft.go:351-360 */
  /* entries get Term = r.Term, Index = li+1..; raftLog.append (raft/log.go:90-99) */
  szc_append(r, r->log.last_index, k, noop ? NULL : desc);
  if (k) tw_leader_append(r, r->log.last_index + 1);
  orc_log_push(&r->log, r->term, k);
  emit(r, HB_EV_LAST, 0, r->log.last_index, noop);
  orc_progress* self = orc_raft_pr(r, r->id);
  if (!self) { fault(r, HB_FAULT_NO_SELF); return; }     /* r.prs[r.id] is nil */
  orc_pr_maybe_update(self, r->log.last_index);
  orc_raft_maybe_commit(r);
}

void orc_raft_append_entry(orc_raft* r, uint64_t k, int noop) { append_entries(r, k, noop, NULL); }

/* oth: HB_STATE_OTH_* of the fields just set to a batch sender outside prs
 * (the event names the assignment even when the packed refs did not change) */
static void emit_state_oth(orc_raft* r, uint64_t before, uint32_t oth) {
  uint64_t now = soft_pack(r);
  if (now != before || oth) emit(r, HB_EV_STATE, 0, now, oth);
}
static void emit_state_if_changed(orc_raft* r, uint64_t before) { emit_state_oth(r, before, 0); }

void orc_raft_become_follower(orc_raft* r, uint64_t term, uint64_t lead) {  /* :384-391 */
  uint64_t before = soft_pack(r);
  orc_raft_reset(r, term);
  r->lead = lead;
  r->state = HB_STATE_FOLLOWER;
  emit_state_oth(r, before, lead == ORC_OUTSIDER ? HB_STATE_OTH_LEAD : 0);
}

void orc_raft_become_candidate(orc_raft* r) {             /* :393-404 */
  if (r->state == HB_STATE_LEADER) { fault(r, HB_FAULT_LEADER_CAMPAIGN); return; }
  uint64_t before = soft_pack(r);
  orc_raft_reset(r, r->term + 1);
  r->vote = r->id;
  r->state = HB_STATE_CANDIDATE;
  emit_state_if_changed(r, before);
}

void orc_raft_become_leader(orc_raft* r) {                /* :406-427 */
  /* unreachable on the engine's paths (only poll/campaign promote, both from
   * candidate); kept for the TestStateTransition KAT. */
  if (r->state == HB_STATE_FOLLOWER) { fault(r, HB_FAULT_FOLLOWER_LEADER); return; }
  uint64_t before = soft_pack(r);
  orc_raft_reset(r, r->term);
  r->lead = r->id;
  r->state = HB_STATE_LEADER;
  emit_state_if_changed(r, before);
  /* pendingConf scan of (committed, last] entries: host side (entry types) */
  orc_raft_append_entry(r, 1, 1);                         /* appendEntry(pb.Entry{Data: nil}) */
}

int orc_raft_poll(orc_raft* r, uint64_t id, int v) {      /* poll raft/raft.go:445-460 */
  int found = 0;
  for (int i = 0; i < r->nvotes; i++)
    if (r->vote_ids[i] == id) found = 1;
  if (!found && r->nvotes < ORC_MAX_PEERS + 1) {
    r->vote_ids[r->nvotes] = id;
    r->vote_vals[r->nvotes] = v;
    r->nvotes++;
  }
  int granted = 0;
  for (int i = 0; i < r->nvotes; i++) granted += r->vote_vals[i] ? 1 : 0;
  return granted;
}

void orc_raft_campaign(orc_raft* r) {                     /* campaign raft/raft.go:429-443 */
  orc_raft_become_candidate(r);
  if (r->fault) return;
  if (orc_raft_q(r) == orc_raft_poll(r, r->id, 1)) {
    r->n_won++;
    orc_raft_become_leader(r);
    return;
  }
  for (int i = 0; i < r->n; i++) {
    if (r->ids[i] == r->id) continue;
    orc_msg m;
    memset(&m, 0, sizeof(m));
    m.to = r->ids[i];
    m.type = HB_MSG_VOTE;
    m.index = r->log.last_index;
    m.log_term = orc_log_last_term(&r->log);
    send(r, m);
  }
}

/* ======================================================================
 * follower side — raft/raft.go:616-707, raft/log.go:72-123
 * ====================================================================== */

/* maybeAppend's raftLog.append of ents[ci-offset:] (raft/log.go:80-85, 90-98) */
static void follower_append(orc_raft* r, const orc_msg* m, uint64_t ci) {
  const uint64_t off = m->index + 1;
  orc_log_truncate(&r->log, ci - 1);                      /* unstable.truncateAndAppend */
  /* the engine's term runs: those from ci on are gone (starts increase, so the
   * oldest survives iff it starts below ci) */
  if (r->tw_lo != HB_NO_INDEX && r->tw_lo >= ci) r->tw_lo = HB_NO_INDEX;
  if (r->tw_tfirst != HB_NO_INDEX && r->tw_tfirst >= ci) r->tw_tfirst = HB_NO_INDEX;
  if (sized(r)) {                                         /* and its entry sizes */
    if (r->szc_n == 0 || ci - 1 < r->sz_lo) szc_reset(r, ci - 1);
    else r->szc_n = ci - r->szc_base;
  }
  for (uint64_t j = ci; j < off + m->nents; j++) {
    const uint64_t t = m->eterm[j - off];
    if (t == r->term) {
      if (r->tw_tfirst == HB_NO_INDEX) r->tw_tfirst = j;
    } else {
      if (r->tw_tfirst != HB_NO_INDEX) {                  /* a lower term after Term entries */
        tw_push(r, r->tw_tfirst, r->term);
        r->tw_tfirst = HB_NO_INDEX;
      }
      tw_push(r, j, t);
    }
    if (sized(r)) {
      const uint64_t acc = r->szc[r->szc_n - 1];
      szc_push(r, acc + orc_entry_size(m->edesc ? m->edesc[j - off] : 0u, t, j));
    }
    orc_log_push(&r->log, t, 1);
  }
  emit(r, HB_EV_FOLLOW, 0, r->arrival, HB_FOLLOW_APPEND);
}

static void handle_append_entries(orc_raft* r, const orc_msg* m) {  /* raft/raft.go:651-665 */
  orc_msg resp;
  memset(&resp, 0, sizeof(resp));
  resp.to = m->from;
  resp.type = HB_MSG_APP_RESP;
  if (m->index < r->commit) {
    resp.index = r->commit;
    send(r, resp);
    return;
  }
  /* maybeAppend raft/log.go:72-88 */
  const uint64_t lastnewi = m->index + m->nents;
  const uint64_t t = f_term(r, m->index);                 /* matchTerm(index, logTerm) */
  if (r->fault) return;
  if (t == m->log_term) {
    uint64_t ci = 0;                                      /* findConflict :112-123 */
    for (uint64_t k = 0; k < m->nents; k++) {
      const uint64_t et = f_term(r, m->index + 1 + k);
      if (r->fault) return;
      if (et != m->eterm[k]) {
        ci = m->index + 1 + k;
        break;
      }
    }
    if (ci != 0) {
      if (ci <= r->log.committed) {                       /* "entry %d conflict with committed entry" */
        fault(r, HB_FAULT_CONFLICT_COMMITTED);
        return;
      }
      follower_append(r, m, ci);
    }
    orc_raft_commit_to(r, lastnewi < m->commit ? lastnewi : m->commit);
    if (r->fault) return;
    resp.index = lastnewi;
  } else {
    resp.index = m->index;
    resp.reject = 1;
    resp.reject_hint = r->log.last_index;
  }
  send(r, resp);
}

static void handle_heartbeat(orc_raft* r, const orc_msg* m) {  /* raft/raft.go:666-669 */
  orc_raft_commit_to(r, m->commit);
  if (r->fault) return;
  orc_msg resp;
  memset(&resp, 0, sizeof(resp));
  resp.to = m->from;
  resp.type = HB_MSG_HEARTBEAT_RESP;
  send(r, resp);
}

static int restore(orc_raft* r, uint64_t sindex, uint64_t sterm) {  /* raft/raft.go:684-707 */
  if (sindex <= r->log.committed) return 0;
  const uint64_t t = f_term(r, sindex);                   /* matchTerm */
  if (r->fault) return 0;
  if (t == sterm) {
    orc_raft_commit_to(r, sindex);
    return 0;
  }
  /* raftLog.restore (raft/log.go:249-253): committed = index, unstable = the snapshot */
  const uint64_t applied = r->log.applied;
  orc_log_free(&r->log);
  orc_log_init(&r->log, sindex + 1, sterm);
  r->log.applied = applied;
  r->log.snap_index = sindex;
  /* prs from the snapshot's ConfState: the engine resets the group's peers */
  const uint64_t last = r->log.last_index;
  for (int i = 0; i < r->n; i++) {
    orc_progress* pr = &r->prs[i];
    orc_ins_free(&pr->ins);
    memset(pr, 0, sizeof(*pr));
    pr->next = last + 1;
    pr->match = r->ids[i] == r->id ? last : 0;
    orc_ins_init(&pr->ins, r->max_inflight);
  }
  r->tw_lo = HB_NO_INDEX;
  r->tw_tfirst = HB_NO_INDEX;
  if (sterm == r->term) r->tw_tfirst = sindex;
  else tw_push(r, sindex, sterm);
  if (sized(r)) szc_reset(r, sindex);
  emit(r, HB_EV_FOLLOW, 0, r->arrival, HB_FOLLOW_RESTORE);
  return 1;
}

static void handle_snapshot(orc_raft* r, const orc_msg* m) {  /* raft/raft.go:671-682 */
  const int ok = restore(r, m->snap_index, m->snap_term);
  if (r->fault) return;
  orc_msg resp;
  memset(&resp, 0, sizeof(resp));
  resp.to = m->from;
  resp.type = HB_MSG_APP_RESP;
  resp.index = ok ? r->log.last_index : r->log.committed;
  send(r, resp);
}

void orc_raft_handle_append_entries(orc_raft* r, const orc_msg* m) { handle_append_entries(r, m); }
void orc_raft_handle_heartbeat(orc_raft* r, const orc_msg* m) { handle_heartbeat(r, m); }

int orc_log_maybe_append(orc_log* l, uint64_t index, uint64_t log_term, uint64_t committed,
                         const uint64_t* terms, uint64_t n, uint64_t* lastnewi) {
  *lastnewi = index + n;
  if (orc_log_term(l, index) != log_term) {              /* matchTerm */
    *lastnewi = 0;
    return 0;
  }
  const uint64_t ci = orc_log_find_conflict(l, index + 1, terms, n);
  if (ci != 0 && ci <= l->committed) return -1;           /* Panicf: conflict with committed entry */
  if (ci != 0) {
    orc_log_truncate(l, ci - 1);
    for (uint64_t j = ci; j <= index + n; j++) orc_log_push(l, terms[j - index - 1], 1);
  }
  const uint64_t to = committed < *lastnewi ? committed : *lastnewi;
  if (l->committed < to) {                                /* commitTo */
    if (l->last_index < to) return -1;
    l->committed = to;
  }
  return 1;
}

static void reject_vote(orc_raft* r, const orc_msg* m) {
  orc_msg resp;
  memset(&resp, 0, sizeof(resp));
  resp.to = m->from;
  resp.type = HB_MSG_VOTE_RESP;
  resp.reject = 1;
  send(r, resp);
}

static void step_leader(orc_raft* r, const orc_msg* m) {  /* stepLeader raft/raft.go:494-583 */
  orc_progress* pr = orc_raft_pr(r, m->from);
  switch (m->type) {
    case HB_MSG_BEAT:
      orc_raft_bcast_heartbeat(r);
      break;
    case HB_MSG_PROP:
      if (m->nents == 0) { fault(r, HB_FAULT_EMPTY_PROP); return; }
      /* EntryConfChange / pendingConf rewriting (:504-511) acts on entry
       * payloads, which stay on the host. */
      append_entries(r, m->nents, 0, m->edesc);
      if (r->fault) return;
      orc_raft_bcast_append(r);
      break;
    case HB_MSG_APP_RESP:
      if (!pr) { fault(r, HB_FAULT_NIL_PROGRESS); return; }
      if (m->reject) {
        if (orc_pr_maybe_decr_to(pr, m->index, m->reject_hint)) {
          if (pr->state == HB_PR_REPLICATE) orc_pr_become_probe(pr);
          orc_raft_send_append(r, m->from);
        }
      } else {
        int old_paused = orc_pr_is_paused(pr);
        if (orc_pr_maybe_update(pr, m->index)) {
          if (pr->state == HB_PR_PROBE) {
            orc_pr_become_replicate(pr);
          } else if (pr->state == HB_PR_SNAPSHOT && orc_pr_maybe_snapshot_abort(pr)) {
            orc_pr_become_probe(pr);
          } else if (pr->state == HB_PR_REPLICATE) {
            orc_ins_free_to(&pr->ins, m->index);
          }
          if (orc_raft_maybe_commit(r)) {
            orc_raft_bcast_append(r);
          } else if (old_paused && !r->fault) {
            orc_raft_send_append(r, m->from);
          }
        }
      }
      break;
    case HB_MSG_HEARTBEAT_RESP:
      if (!pr) { fault(r, HB_FAULT_NIL_PROGRESS); return; }
      if (pr->state == HB_PR_REPLICATE && orc_ins_full(&pr->ins)) orc_ins_free_first_one(&pr->ins);
      if (pr->match < r->log.last_index) orc_raft_send_append(r, m->from);
      break;
    case HB_MSG_VOTE: {
      orc_msg resp;
      memset(&resp, 0, sizeof(resp));
      resp.to = m->from;
      resp.type = HB_MSG_VOTE_RESP;
      resp.reject = 1;
      send(r, resp);
      break;
    }
    case HB_MSG_SNAP_STATUS:
      if (!pr) { fault(r, HB_FAULT_NIL_PROGRESS); return; }
      if (pr->state != HB_PR_SNAPSHOT) return;
      if (!m->reject) {
        orc_pr_become_probe(pr);
      } else {
        orc_pr_snapshot_failure(pr);
        orc_pr_become_probe(pr);
      }
      orc_pr_pause(pr);
      break;
    case HB_MSG_UNREACHABLE:
      if (!pr) { fault(r, HB_FAULT_NIL_PROGRESS); return; }
      if (pr->state == HB_PR_REPLICATE) orc_pr_become_probe(pr);
      break;
    default:
      break;
  }
}

static void step_candidate(orc_raft* r, const orc_msg* m) {  /* stepCandidate raft/raft.go:585-614 */
  switch (m->type) {
    case HB_MSG_PROP:
      emit(r, HB_EV_PROP_DROP, 0, r->arrival, 0);          /* "no leader ... dropping proposal" */
      return;
    case HB_MSG_VOTE: {
      orc_msg resp;
      memset(&resp, 0, sizeof(resp));
      resp.to = m->from;
      resp.type = HB_MSG_VOTE_RESP;
      resp.reject = 1;
      send(r, resp);
      break;
    }
    case HB_MSG_APP:                                      /* :591-593 */
      orc_raft_become_follower(r, r->term, m->from);
      if (!r->fault) handle_append_entries(r, m);
      break;
    case HB_MSG_HEARTBEAT:                                /* :594-596 */
      orc_raft_become_follower(r, r->term, m->from);
      if (!r->fault) handle_heartbeat(r, m);
      break;
    case HB_MSG_SNAP:                                     /* :597-599 */
      orc_raft_become_follower(r, m->term, m->from);
      if (!r->fault) handle_snapshot(r, m);
      break;
    case HB_MSG_VOTE_RESP: {
      int gr = orc_raft_poll(r, m->from, !m->reject);
      int q = orc_raft_q(r);
      if (q == gr) {
        r->n_won++;
        orc_raft_become_leader(r);
        if (!r->fault) orc_raft_bcast_append(r);
      } else if (q == r->nvotes - gr) {
        r->n_lost++;
        orc_raft_become_follower(r, r->term, ORC_NONE);
      }
      break;
    }
    default:
      break;
  }
}

static void step_follower(orc_raft* r, const orc_msg* m) {   /* stepFollower raft/raft.go:616-649 */
  switch (m->type) {
    case HB_MSG_PROP:
      if (r->lead == ORC_NONE) {
        emit(r, HB_EV_PROP_DROP, 0, r->arrival, 0);
        return;
      } else {
        orc_msg fwd = *m;
        fwd.to = r->lead;
        send(r, fwd);
      }
      break;
    case HB_MSG_APP: {                                    /* :625-628 */
      uint64_t before = soft_pack(r);
      r->elapsed = 0;
      r->lead = m->from;
      emit_state_oth(r, before, m->from == ORC_OUTSIDER ? HB_STATE_OTH_LEAD : 0);
      handle_append_entries(r, m);
      break;
    }
    case HB_MSG_HEARTBEAT: {                              /* :629-632 */
      uint64_t before = soft_pack(r);
      r->elapsed = 0;
      r->lead = m->from;
      emit_state_oth(r, before, m->from == ORC_OUTSIDER ? HB_STATE_OTH_LEAD : 0);
      handle_heartbeat(r, m);
      break;
    }
    case HB_MSG_SNAP:                                     /* :633-635 */
      r->elapsed = 0;
      handle_snapshot(r, m);
      break;
    case HB_MSG_VOTE: {                                   /* :636-648 */
      int grant = 0;
      /* r.Vote == m.From: for a batch sender outside prs the host says (HB_INFO_VOTED) */
      const int same = m->outsider ? m->voted : r->vote == m->from;
      if (r->vote == ORC_NONE || same) {
        const uint64_t lt = f_term(r, r->log.last_index); /* isUpToDate (raft/log.go:235-237) */
        if (r->fault) return;
        grant = m->log_term > lt || (m->log_term == lt && m->index >= r->log.last_index);
      }
      if (grant) {
        uint64_t before = soft_pack(r);
        r->elapsed = 0;
        r->vote = m->from;
        emit_state_oth(r, before, m->from == ORC_OUTSIDER ? HB_STATE_OTH_VOTE : 0);
        orc_msg resp;
        memset(&resp, 0, sizeof(resp));
        resp.to = m->from;
        resp.type = HB_MSG_VOTE_RESP;
        send(r, resp);
      } else {
        reject_vote(r, m);
      }
      break;
    }
    default:
      break;
  }
}

void orc_raft_step(orc_raft* r, const orc_msg* m) {       /* Step raft/raft.go:462-490 */
  if (r->fault) return;
  if (m->type == HB_MSG_HUP) {
    orc_raft_campaign(r);
    r->commit = r->log.committed;
    return;
  }
  if (m->term != 0 && m->term < r->term) return;          /* ignore */
  if (m->type == HB_MSG_APP || m->type == HB_MSG_HEARTBEAT || m->type == HB_MSG_SNAP || m->type == HB_MSG_VOTE)
    emit(r, HB_EV_FOLLOW, 0, r->arrival, HB_FOLLOW_STEP);  /* the events that follow belong to it */
  if (m->term > r->term) {                                /* (m.Term == 0: local message, no gate) */
    uint64_t lead = m->from;
    if (m->type == HB_MSG_VOTE) lead = ORC_NONE;
    orc_raft_become_follower(r, m->term, lead);
  }
  if (r->fault) return;
  switch (r->state) {
    case HB_STATE_LEADER: step_leader(r, m); break;
    case HB_STATE_CANDIDATE: step_candidate(r, m); break;
    default: step_follower(r, m); break;
  }
  r->commit = r->log.committed;
}

/* ========================================================================
 * engine-format conversion + batch driver
 * ======================================================================== */
static uint64_t slot_id(const hb_group* g, uint32_t ref) {
  if (ref == HB_REF_NONE) return ORC_NONE;
  if (ref == HB_REF_SELF) return 100;
  if (ref == HB_REF_OTHER) return 99;
  (void)g;
  return (uint64_t)ref + 1;
}

int orc_raft_from_group(orc_raft* r, const hb_group* g, const orc_run* runs, int nruns,
                        int max_inflight, uint64_t max_msg_size) {
  if (g->n < 1 || g->n > HB_MAX_REPLICAS || nruns < 1) return -1;
  memset(r, 0, sizeof(*r));
  orc_log_init(&r->log, g->first_index, runs[0].term);
  for (int k = 1; k < nruns; k++) {
    orc_log_push(&r->log, runs[k - 1].term, runs[k].index - (r->log.last_index + 1));
  }
  /* last run extends to last_index */
  if (g->last_index >= r->log.last_index + 1)
    orc_log_push(&r->log, runs[nruns - 1].term, g->last_index - r->log.last_index);
  if (r->log.last_index != g->last_index) return -2;
  r->log.committed = g->committed;
  r->log.applied = g->committed;
  r->log.snap_index = g->snap_index;
  r->id = g->self_slot == HB_SLOT_NONE ? 100 : (uint64_t)g->self_slot + 1;
  r->max_inflight = max_inflight;
  r->max_msg_size = max_msg_size;
  r->election_timeout = 10;
  r->heartbeat_timeout = 1;
  r->term = g->term;
  /* r.Commit: committed, or 0 before the first Step of a group created with an
     empty HardState (newRaft raft/raft.go:157-209 leaves it 0; loadState :759
     and every Step past the term gate :466,488 set it) */
  r->commit = g->commit_zero ? 0 : g->committed;
  r->vote = slot_id(g, g->vote);
  r->lead = slot_id(g, g->lead);
  r->state = (int)g->state;
  r->n = (int)g->n;
  for (int i = 0; i < r->n; i++) {
    r->ids[i] = (uint64_t)i + 1;
    orc_progress* pr = &r->prs[i];
    pr->match = g->pr[i].match;
    pr->next = g->pr[i].next;
    pr->state = (int)g->pr[i].state;
    pr->paused = (int)g->pr[i].paused;
    pr->pending_snapshot = g->pr[i].pending_snapshot;
    orc_ins_init(&pr->ins, max_inflight);
    pr->ins.start = (int)g->pr[i].ins_start;
    pr->ins.count = (int)g->pr[i].ins_count;
  }
  r->nvotes = 0;
  for (int i = 0; i < 8; i++) {
    if (!(g->votes_resp & (1u << i))) continue;
    r->vote_ids[r->nvotes] = i == 7 ? r->id : (uint64_t)i + 1;
    r->vote_vals[r->nvotes] = (g->votes_grant >> i) & 1u;
    r->nvotes++;
  }
  r->fault = (int)g->fault;
  if (sized(r)) szc_reset(r, r->log.last_index);            /* hb_load_groups: no entry size yet */
  r->tw_lo = HB_NO_INDEX;                                   /* hb_load_groups: no older term run yet */
  r->tw_tfirst = HB_NO_INDEX;
  for (int k = 0; k < r->log.nruns; k++)                    /* the current-term run (term_first) */
    if (r->log.runs[k].term == r->term) {
      r->tw_tfirst = r->log.runs[k].index;
      break;
    }
  if (r->tw_tfirst != HB_NO_INDEX && r->tw_tfirst > r->log.last_index) r->tw_tfirst = HB_NO_INDEX;
  return 0;
}

void orc_raft_to_group(const orc_raft* r, hb_group* g) {
  memset(g, 0, sizeof(*g));
  g->term = r->term;
  g->committed = r->log.committed;
  g->first_index = r->log.first_index;
  g->last_index = r->log.last_index;
  g->snap_index = r->log.snap_index;
  /* maximal run of indices in [first-1, last] whose term == r->term */
  g->term_first = HB_NO_INDEX;
  g->term_last = 0;
  for (int k = 0; k < r->log.nruns; k++) {
    if (r->log.runs[k].term != r->term) continue;
    uint64_t lo = r->log.runs[k].index;
    uint64_t hi = (k + 1 < r->log.nruns) ? r->log.runs[k + 1].index - 1 : r->log.last_index;
    if (lo > hi) continue;
    if (g->term_first == HB_NO_INDEX) g->term_first = lo;
    g->term_last = hi;
  }
  g->state = (uint32_t)r->state;
  g->n = (uint32_t)r->n;
  int self = orc_raft_slot(r, r->id);
  g->self_slot = self < 0 ? HB_SLOT_NONE : (uint32_t)self;
  g->lead = orc_raft_ref(r, r->lead);
  g->vote = orc_raft_ref(r, r->vote);
  for (int i = 0; i < r->nvotes; i++) {
    int s = orc_raft_slot(r, r->vote_ids[i]);
    uint32_t bit = s < 0 ? 7u : (uint32_t)s;
    g->votes_resp |= 1u << bit;
    if (r->vote_vals[i]) g->votes_grant |= 1u << bit;
  }
  g->fault = (uint32_t)r->fault;
  g->commit_zero = (r->commit == 0 && r->log.committed != 0) ? 1u : 0u;
  for (int i = 0; i < r->n && i < HB_MAX_REPLICAS; i++) {
    const orc_progress* pr = &r->prs[i];
    g->pr[i].match = pr->match;
    g->pr[i].next = pr->next;
    g->pr[i].state = (uint32_t)pr->state;
    g->pr[i].paused = (uint32_t)pr->paused;
    g->pr[i].pending_snapshot = pr->state == HB_PR_SNAPSHOT ? pr->pending_snapshot : 0;
    g->pr[i].ins_start = (uint32_t)pr->ins.start;
    g->pr[i].ins_count = (uint32_t)pr->ins.count;
  }
}

int orc_raft_set_inflights(orc_raft* r, int slot, int start, int count, const uint64_t* vals) {
  if (slot < 0 || slot >= r->n) return -1;
  orc_inflights* in = &r->prs[slot].ins;
  if (start < 0 || start >= in->size || count < 0 || count > in->size) return -1;
  in->start = start;
  in->count = count;
  for (int i = 0; i < count; i++) in->buffer[(start + i) % in->size] = vals[i];
  return 0;
}

int orc_raft_get_inflights(const orc_raft* r, int slot, uint64_t* vals) {
  if (slot < 0 || slot >= r->n) return -1;
  const orc_inflights* in = &r->prs[slot].ins;
  for (int i = 0; i < in->count; i++) vals[i] = in->buffer[(in->start + i) % in->size];
  return in->count;
}

static int is_response(int type) {                        /* IsResponseMsg raft/util.go:53-55 */
  return type == HB_MSG_APP_RESP || type == HB_MSG_VOTE_RESP ||
         type == HB_MSG_HEARTBEAT_RESP || type == HB_MSG_UNREACHABLE;
}

/* per-batch bookkeeping shared by orc_step_batch and orc_tick_batch */
typedef struct {
  uint64_t *commit0, *last0;
  int* fault0;
  uint64_t won0, lost0;
} batch_ctx;

static void batch_begin(batch_ctx* c, orc_raft* groups, uint32_t ngroups, uint64_t stats[HB_STAT_COUNT]) {
  memset(stats, 0, sizeof(uint64_t) * HB_STAT_COUNT);
  c->commit0 = (uint64_t*)malloc(sizeof(uint64_t) * (ngroups ? ngroups : 1));
  c->last0 = (uint64_t*)malloc(sizeof(uint64_t) * (ngroups ? ngroups : 1));
  c->fault0 = (int*)malloc(sizeof(int) * (ngroups ? ngroups : 1));
  c->won0 = c->lost0 = 0;
  for (uint32_t g = 0; g < ngroups; g++) {
    c->won0 += groups[g].n_won;
    c->lost0 += groups[g].n_lost;
    c->commit0[g] = groups[g].log.committed;
    c->last0[g] = groups[g].log.last_index;
    c->fault0[g] = groups[g].fault;
    groups[g].group = g;
  }
}

static void batch_end(batch_ctx* c, orc_raft* groups, uint32_t ngroups, uint64_t stats[HB_STAT_COUNT],
                      uint64_t total) {
  uint64_t won1 = 0, lost1 = 0;
  for (uint32_t g = 0; g < ngroups; g++) {
    orc_raft* r = &groups[g];
    if (r->log.committed > c->commit0[g]) stats[HB_STAT_COMMITS]++;
    if (r->fault && !c->fault0[g]) stats[HB_STAT_FAULTS]++;
    stats[HB_STAT_ENTRIES] += r->log.last_index - c->last0[g];
    r->nmsgs = 0;                                          /* msgs handed to the app via Ready */
    won1 += r->n_won;
    lost1 += r->n_lost;
  }
  stats[HB_STAT_WON] = won1 - c->won0;
  stats[HB_STAT_LOST] = lost1 - c->lost0;
  stats[HB_STAT_EVENTS] = total;
  free(c->commit0);
  free(c->last0);
  free(c->fault0);
}

static void account(orc_raft* r, int type, uint64_t stats[HB_STAT_COUNT]) {
  stats[HB_STAT_MSGS]++;
  if (type == HB_MSG_APP_RESP) stats[HB_STAT_APPRESP]++;
  if (type == HB_MSG_VOTE_RESP) stats[HB_STAT_VOTERESP]++;
  (void)r;
}

int orc_step_batch(orc_raft* groups, uint32_t ngroups, const hb_batch* b,
                   hb_event* ev, uint64_t ev_cap, uint64_t* nev,
                   uint64_t stats[HB_STAT_COUNT]) {
  batch_ctx cx;
  batch_begin(&cx, groups, ngroups, stats);
  uint64_t total = 0;
  /* one sink shared by all groups, appended in processing order */
  #define BIND(r) do { (r)->ev = ev; (r)->ev_cap = ev_cap; (r)->nev = total; } while (0)
  #define UNBIND(r) do { total = (r)->nev; (r)->ev = NULL; } while (0)

  /* dense proposals: one MsgProp{Entries: props[g]} per group, stepped first */
  if (b->props) {
    for (uint32_t g = 0; g < ngroups; g++) {
      if (b->props[g] == 0) continue;
      orc_raft* r = &groups[g];
      if (r->fault || r->n == 0) continue;
      BIND(r);
      r->arrival = HB_NO_INDEX;
      orc_msg m;
      memset(&m, 0, sizeof(m));
      m.type = HB_MSG_PROP;
      m.from = r->id;                                     /* raft/multinode.go:229 */
      m.nents = b->props[g];
      m.edesc = (b->edesc && b->peoff) ? b->edesc + b->peoff[g] : NULL;
      orc_raft_step(r, &m);
      UNBIND(r);
    }
  }
  for (uint64_t i = 0; i < b->n; i++) {
    uint32_t g = b->group[i];
    if (g >= ngroups) continue;
    orc_raft* r = &groups[g];
    if (r->n == 0) continue;                              /* removed group */
    uint32_t info = b->info[i];
    int type = (int)(info & 0xF);
    uint32_t from_slot = (info >> 4) & 0xF;
    int reject = (int)((info >> 8) & 1);
    if (r->fault) continue;
    uint64_t from = from_slot < (uint32_t)r->n ? r->ids[from_slot] : 0xFFFFFFFFull;
    /* MultiNode recvc filter raft/multinode.go:235 */
    if (from_slot >= (uint32_t)r->n && is_response(type)) {
      stats[HB_STAT_DROPPED]++;
      continue;
    }
    if (from_slot >= (uint32_t)r->n && (type == HB_MSG_HUP || type == HB_MSG_BEAT || type == HB_MSG_PROP))
      from = r->id;
    else if (from_slot >= (uint32_t)r->n)                 /* a sender outside prs (its id is the host's) */
      from = ORC_OUTSIDER;
    BIND(r);
    r->arrival = i;
    orc_msg m;
    memset(&m, 0, sizeof(m));
    m.type = type;
    m.from = from;
    m.to = r->id;
    m.term = b->term[i];
    m.index = b->index[i];
    m.reject = reject;
    m.outsider = from_slot >= (uint32_t)r->n;
    m.voted = (info & HB_INFO_VOTED) != 0;
    m.reject_hint = (reject && type == HB_MSG_APP_RESP && b->hint) ? b->hint[i] : 0;
    if (type == HB_MSG_APP || type == HB_MSG_VOTE) m.log_term = b->hint ? b->hint[i] : 0;
    if (type == HB_MSG_APP || type == HB_MSG_HEARTBEAT) m.commit = b->commit ? b->commit[i] : 0;
    if (type == HB_MSG_SNAP) {
      m.snap_index = b->index[i];
      m.snap_term = b->hint ? b->hint[i] : 0;
      m.index = 0;
    }
    if (type == HB_MSG_APP && b->eoff) {                  /* entries eoff[i] .. eoff[i+1] */
      const uint64_t e0 = b->eoff[i], e1 = i + 1 < b->n ? b->eoff[i + 1] : b->n_edesc;
      m.nents = e1 - e0;
      m.eterm = b->eterm ? b->eterm + e0 : NULL;
      m.edesc = b->edesc ? b->edesc + e0 : NULL;
      if (!m.eterm) m.nents = 0;
    }
    if (type == HB_MSG_PROP) {
      m.nents = b->index[i];
      m.index = 0;
      m.edesc = (b->edesc && b->eoff) ? b->edesc + b->eoff[i] : NULL;
    }
    orc_raft_step(r, &m);
    account(r, type, stats);
    UNBIND(r);
  }
  batch_end(&cx, groups, ngroups, stats, total);
  *nev = total;
  #undef BIND
  #undef UNBIND
  return total <= ev_cap ? 0 : -1;
}

/* ---- tick (raft/raft.go:362-382, 765-771; raft/multinode.go:264-275) ---- */
static int is_election_timeout(orc_raft* r, const uint64_t* draws, uint64_t ndraws) {
  int64_t d = (int64_t)r->elapsed - r->election_timeout;
  if (d < 0) return 0;
  if (r->rand_pos >= ndraws) {          /* the host's stream is too short (engine-defined) */
    fault(r, HB_FAULT_RAND_EXHAUSTED);
    return 0;
  }
  uint64_t v = draws[r->rand_pos++];    /* r.rand.Int() */
  return d > (int64_t)(v % (uint64_t)r->election_timeout);
}

static void step_local(orc_raft* r, int type) {
  orc_msg m;
  memset(&m, 0, sizeof(m));
  m.type = type;
  m.from = r->id;
  m.to = r->id;
  orc_raft_step(r, &m);
}

int orc_raft_tick(orc_raft* r, const uint64_t* draws, uint64_t ndraws) {
  if (r->state == HB_STATE_LEADER) {    /* tickHeartbeat */
    r->elapsed++;
    if (r->elapsed >= r->heartbeat_timeout) {
      r->elapsed = 0;
      step_local(r, HB_MSG_BEAT);
      return HB_MSG_BEAT;
    }
    return -1;
  }
  if (orc_raft_slot(r, r->id) < 0) {    /* tickElection: !promotable() */
    r->elapsed = 0;
    return -1;
  }
  r->elapsed++;
  if (is_election_timeout(r, draws, ndraws)) {
    r->elapsed = 0;
    step_local(r, HB_MSG_HUP);
    return HB_MSG_HUP;
  }
  return -1;
}

int orc_tick_batch(orc_raft* groups, uint32_t ngroups, const uint64_t* draws, uint64_t ndraws,
                   hb_event* ev, uint64_t ev_cap, uint64_t* nev, uint64_t stats[HB_STAT_COUNT]) {
  batch_ctx cx;
  batch_begin(&cx, groups, ngroups, stats);
  uint64_t total = 0;
  for (uint32_t g = 0; g < ngroups; g++) {
    orc_raft* r = &groups[g];
    if (r->n == 0 || r->fault) continue;
    r->ev = ev;
    r->ev_cap = ev_cap;
    r->nev = total;
    r->arrival = HB_NO_INDEX;
    int t = orc_raft_tick(r, draws, ndraws);
    if (t >= 0) account(r, t, stats);
    total = r->nev;
    r->ev = NULL;
  }
  batch_end(&cx, groups, ngroups, stats, total);
  *nev = total;
  return total <= ev_cap ? 0 : -1;
}

void orc_groups_load_timers(orc_raft* gs, uint32_t n, const hb_timer* t) {
  for (uint32_t i = 0; i < n; i++) {
    gs[i].elapsed = (int)t[i].elapsed;
    gs[i].rand_pos = t[i].rand_pos;
    gs[i].election_timeout = t[i].election_tick;
    gs[i].heartbeat_timeout = t[i].heartbeat_tick;
  }
}

void orc_groups_export_timers(const orc_raft* gs, uint32_t n, hb_timer* out) {
  for (uint32_t i = 0; i < n; i++) {
    memset(&out[i], 0, sizeof(out[i]));
    out[i].elapsed = (uint32_t)gs[i].elapsed;
    out[i].rand_pos = (uint32_t)gs[i].rand_pos;
    out[i].election_tick = (uint16_t)gs[i].election_timeout;
    out[i].heartbeat_tick = (uint16_t)gs[i].heartbeat_timeout;
  }
}

orc_raft* orc_groups_new(uint32_t ngroups) {
  return (orc_raft*)calloc(ngroups ? ngroups : 1, sizeof(orc_raft));
}

void orc_groups_free(orc_raft* g, uint32_t ngroups) {
  for (uint32_t i = 0; i < ngroups; i++) orc_raft_free(&g[i]);
  free(g);
}

orc_raft* orc_groups_at(orc_raft* g, uint32_t i) { return &g[i]; }

size_t orc_sizeof_raft(void) { return sizeof(orc_raft); }

/* Bulk CreateGroup / Status for n groups (test infrastructure: lets the
 * Python harness load and read back a million groups without a per-group
 * ctypes call).  Group i's log term runs are runs[run_off[i], run_off[i+1]). */
int orc_groups_load(orc_raft* gs, uint32_t n, const hb_group* recs, const orc_run* runs, const uint64_t* run_off,
                    int max_inflight, uint64_t max_msg_size) {
  for (uint32_t i = 0; i < n; i++) {
    int rc = orc_raft_from_group(&gs[i], &recs[i], runs + run_off[i], (int)(run_off[i + 1] - run_off[i]),
                                 max_inflight, max_msg_size);
    if (rc != 0) return -(int)i - 1;
  }
  return 0;
}

void orc_groups_export(const orc_raft* gs, uint32_t n, hb_group* out) {
  for (uint32_t i = 0; i < n; i++) orc_raft_to_group(&gs[i], &out[i]);
}

void orc_groups_log_info(const orc_raft* gs, uint32_t n, uint64_t* out) {
  for (uint32_t i = 0; i < n; i++) {
    const orc_raft* r = &gs[i];
    out[4 * i] = (uint64_t)r->log.nruns;
    out[4 * i + 1] = r->szc_n ? r->sz_lo : r->log.last_index;
    out[4 * i + 2] = r->log.first_index;
    out[4 * i + 3] = r->log.last_index;
  }
}
