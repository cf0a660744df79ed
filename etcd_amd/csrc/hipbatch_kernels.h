// hipbatch_kernels.h — device-side layout and per-group logic of the engine.
//
// Group state lives in HBM as structure-of-arrays (one array per field, group
// index fastest) so that a wave of 64 lanes, one lane per group, reads every
// field with one coalesced 256/512-byte access.  Per-peer progress is
// replica-major ([slot][group]) for the same reason; the inflight rings are
// [slot][ring index][group] so that lanes whose rings advance in lockstep
// (steady-state replication) touch adjacent words.
//
// The per-group logic below is the device restatement of the reference's
// leader bookkeeping; each function cites the Go it mirrors and the oracle
// (oracle/raft_oracle.c) restates the same lines sequentially.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hipbatch.h"

namespace hb {

#ifndef HB_PART_LOG
#define HB_PART_LOG 8
#endif
constexpr int PART_LOG = HB_PART_LOG;        // groups per partition = apply workgroup
constexpr uint32_t PART = 1u << PART_LOG;    // lanes of the apply workgroup, one group each
#ifndef HB_APPLY_WAVES3
#define HB_APPLY_WAVES3 3
#endif
constexpr uint32_t CHUNK = 4 * PART;         // messages staged in LDS per round (4 per lane)

// ---- packed group meta (u64) ------------------------------------------------
//  [0:2) state  [2:5) n  [5:9) self slot  [9:13) lead ref  [13:17) vote ref
//  [17:21) fault  [21] M_TL  [22] M_SM  [23] M_RS  [24] M_NC
//  [32:40) votes granted  [40:48) votes responded
//  (the flags every lane tests sit in the low word, which the fast lanes load
//  and store alone; the vote tally, read only by the election lanes, is above)
//  M_TL: tlast == last — the tlast array is then not kept (a leader's current-
//  term run always ends at its last entry).  M_SM: the self slot's Match ==
//  last and Next == last + 1 — its match / next arrays are then not kept (a
//  leader's own progress after every append).  The steady-state fast path
//  neither reads nor writes those 48 bytes per group; every other reader
//  materializes them from `last`.
constexpr int M_GRANT_SHIFT = 32;
constexpr int M_RESP_SHIFT = 40;
__host__ __device__ inline uint64_t meta_make(uint32_t state, uint32_t n, uint32_t self, uint32_t lead,
                                              uint32_t vote, uint32_t fault, uint32_t resp, uint32_t grant) {
  return (uint64_t)(state & 3) | ((uint64_t)(n & 7) << 2) | ((uint64_t)(self & 0xF) << 5) |
         ((uint64_t)(lead & 0xF) << 9) | ((uint64_t)(vote & 0xF) << 13) | ((uint64_t)(fault & 0xF) << 17) |
         ((uint64_t)(resp & 0xFF) << M_RESP_SHIFT) | ((uint64_t)(grant & 0xFF) << M_GRANT_SHIFT);
}
constexpr uint64_t M_TL = 1ull << 21;
constexpr uint64_t M_SM = 1ull << 22;
// M_RS: every Progress is in the form an election leaves it (k_elect does not
// write the n entries): reset (raft/raft.go:334-349) at lastIndex rl — Match 0,
// Next rl + 1, Probe, an empty window; the self slot Match = lastIndex, Next =
// lastIndex + 1 (M_SM) — plus, for a leader, becomeLeader's noop at rl + 1 (so
// rl = tfirst - 1) and bcastAppend's pause of every peer (:406-427, :239-282).
// A non-leader's rl is its lastIndex (anything that moves a follower's
// lastIndex loads its Progress first).  Readers materialize it (rs_progress),
// writers of Progress clear it.
constexpr uint64_t M_RS = 1ull << 23;
// M_NC: r.Commit (HardState.Commit) is 0 while raftLog.committed is not — a
// group created with an empty HardState that has not stepped a message yet
// (hb_group.commit_zero).  The reference sets r.Commit = committed at the end
// of every Step past the term gate (raft/raft.go:466,488), and only
// handleAppendEntries reads it (`m.Index < r.Commit`, :652).  Only the general
// lane (Lane::step) steps such a group: every specialised lane hands it over,
// and Lane::step clears the flag once the message passes the gate.
constexpr uint64_t M_NC = 1ull << 24;
__host__ __device__ inline uint32_t m_state(uint64_t m) { return (uint32_t)(m & 3); }
__host__ __device__ inline uint32_t m_n(uint64_t m) { return (uint32_t)((m >> 2) & 7); }
__host__ __device__ inline uint32_t m_self(uint64_t m) { return (uint32_t)((m >> 5) & 0xF); }
__host__ __device__ inline uint32_t m_lead(uint64_t m) { return (uint32_t)((m >> 9) & 0xF); }
__host__ __device__ inline uint32_t m_vote(uint64_t m) { return (uint32_t)((m >> 13) & 0xF); }
__host__ __device__ inline uint32_t m_fault(uint64_t m) { return (uint32_t)((m >> 17) & 0xF); }
__host__ __device__ inline uint32_t m_resp(uint64_t m) { return (uint32_t)((m >> M_RESP_SHIFT) & 0xFF); }
__host__ __device__ inline uint32_t m_grant(uint64_t m) { return (uint32_t)((m >> M_GRANT_SHIFT) & 0xFF); }

// ---- packed progress meta (u32) ----------------------------------------------
//  [0:2) ProgressState  [2] Paused  [3:13) inflights.start  [13:24) inflights.count
__host__ __device__ inline uint32_t pm_make(uint32_t st, uint32_t paused, uint32_t start, uint32_t count) {
  return (st & 3) | ((paused & 1) << 2) | ((start & 0x3FF) << 3) | ((count & 0x7FF) << 13);
}
__host__ __device__ inline uint32_t pm_state(uint32_t p) { return p & 3; }
__host__ __device__ inline uint32_t pm_paused(uint32_t p) { return (p >> 2) & 1; }
__host__ __device__ inline uint32_t pm_start(uint32_t p) { return (p >> 3) & 0x3FF; }
__host__ __device__ inline uint32_t pm_count(uint32_t p) { return (p >> 13) & 0x7FF; }
constexpr uint32_t PM_PAUSED = 1u << 2;

// Slot s's Progress under M_RS (meta m, the group's lastIndex and term_first).
__device__ __forceinline__ void rs_progress(uint64_t m, uint32_t s, uint64_t last, uint64_t tfirst, uint64_t* match,
                                            uint64_t* next, uint32_t* pm) {
  const bool leader = m_state(m) == HB_STATE_LEADER;
  const uint64_t rl = leader ? tfirst - 1 : last;
  const bool me = s == m_self(m);
  *match = me ? last : 0ull;
  *next = me ? last + 1 : rl + 1;
  *pm = pm_make(HB_PR_PROBE, (!me && leader) ? 1u : 0u, 0, 0);
}

// ---- device state (SoA in HBM) -------------------------------------------------
struct DevState {
  uint32_t G;                 // group capacity
  uint32_t W;                 // MaxInflightMsgs
  uint32_t nmax;              // max replicas of this handle
  uint32_t pad;
  uint64_t max_msg_size;      // HB_NO_LIMIT or 0
  uint64_t* term;             // [G] HardState.Term
  uint64_t* commit;           // [G] raftLog.committed
  uint64_t* first;            // [G] raftLog.firstIndex()
  uint64_t* last;             // [G] raftLog.lastIndex()
  uint64_t* tfirst;           // [G] first index of the current-term run
  uint64_t* tlast;            // [G] last index of the current-term run
  uint64_t* snap;             // [G] snapshot index (read only for MsgSnap)
  uint64_t* meta;             // [G] packed meta
  uint64_t* match;            // [nmax][G]
  uint64_t* next;             // [nmax][G]
  uint64_t* pending;          // [nmax][G] PendingSnapshot (valid in Snapshot state)
  uint32_t* pm;               // [nmax][G] packed progress meta
  uint64_t* ring;             // [nmax][W][G] inflight ring
  uint32_t* elapsed;          // [G] r.elapsed
  uint32_t* rpos;             // [G] r.rand.Int() values taken so far
  uint32_t* tcfg;             // [G] ElectionTick | HeartbeatTick << 16
  const uint64_t* rnd;        // [nrnd] the node's r.rand.Int() stream (host supplied)
  uint64_t nrnd;
  // The log index (§3.12 of DESIGN.md): per group, two rings in extents of the
  // handle's log pool whose capacities the host reserves (hb_reserve_log).
  // An extent word is the extent's address (128-byte aligned) | log2(capacity).
  // finite max_msg_size only (sz_on): the cumulative Entry.Size() of the log, for limitSize
  uint64_t* szx;              // [G] extent of u64 cum[i & (cap-1)] = sum of Entry.Size() of (szlo, i]
  uint64_t* szlo;             // [G] oldest index i whose cum(i) is kept (cum(szlo) = the base)
  const uint32_t* edesc;      // this step's entry descriptors (hb_batch.edesc / eoff / peoff)
  const uint64_t* eoff;
  const uint64_t* peoff;
  // the log's term runs below the current-term run (follower side lookups)
  uint64_t* trx;              // [G] extent of {start, term} u64 pairs (a ring, oldest at head)
  uint64_t* trc;              // [G] runs kept | ring head << 32
  const uint64_t* bcommit;    // this step's hb_batch.commit (m.Commit of MsgApp / MsgHeartbeat)
  const uint64_t* eterm;      // hb_batch.eterm (MsgApp entry terms)
  uint64_t n_ent;             // hb_batch.n_edesc
  uint64_t bn;                // hb_batch.n
};

// Element i of a device array addressed by a 32-bit byte offset from the
// array's (uniform) base: one global_load / global_store with an SGPR base and a
// 32-bit VGPR offset instead of a 64-bit address per lane.  For the [G] and
// [slot][G] arrays (at most 8 x 2^24 x 8 B = 1 GiB, hb_create caps capacity at
// 2^24), not for the inflight rings.
template <class T>
__device__ __forceinline__ T& at32(T* base, uint32_t i) {
  return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + i * (uint32_t)sizeof(T));
}
template <class T>
__device__ __forceinline__ const T& at32(const T* base, uint32_t i) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + i * (uint32_t)sizeof(T));
}

// ---- log-pool extents ------------------------------------------------------------
constexpr uint64_t LX_TAG = 0x3F;  // low bits of an extent word: log2(capacity)
__host__ __device__ inline uint64_t lx_word(uint64_t addr, uint32_t log2cap) { return addr | log2cap; }
__device__ __forceinline__ uint64_t* lx_base(uint64_t x) { return reinterpret_cast<uint64_t*>(x & ~LX_TAG); }
__device__ __forceinline__ uint64_t lx_cap(uint64_t x) { return 1ull << (x & LX_TAG); }

// ---- entry sizes (finite MaxSizePerMsg) -----------------------------------------
__host__ __device__ inline bool sz_on(uint64_t max_msg_size) { return max_msg_size != 0 && max_msg_size != HB_NO_LIMIT; }
// sovRaft: varint length (raft/raftpb/raft.pb.go)
__device__ __forceinline__ uint64_t sov(uint64_t x) { return x ? (uint64_t)(70 - __clzll(x)) / 7 : 1; }
// Entry.Size() raft/raftpb/raft.pb.go:1030-1043 of the entry a descriptor (HB_ENT_DESC) describes
__device__ __forceinline__ uint64_t ent_size(uint32_t desc, uint64_t term, uint64_t index) {
  uint64_t n = 1 + sov((desc >> 30) & 1u) + 1 + sov(term) + 1 + sov(index);
  if (desc >> 31) {
    const uint64_t l = desc & HB_ENT_MAX_DATA;
    n += 1 + l + sov(l);
  }
  return n;
}
// the cumulative size of entry i in the group's ring (extent word x)
__device__ __forceinline__ uint64_t* cum_at(uint64_t x, uint64_t i) { return lx_base(x) + (i & (lx_cap(x) - 1)); }
// The ring keeps cum(i) for i in [szlo, last] as long as that span fits its
// capacity; appending past it drops the oldest (szlo moves up).  The host
// reserves a capacity that covers [firstIndex - 1, lastIndex] plus what a batch
// can append (hb_reserve_log), so only entries below firstIndex - 1 ever leave.
__device__ __forceinline__ void sz_keep(const DevState& S, uint32_t g, uint64_t x, uint64_t last) {
  const uint64_t cap = lx_cap(x);
  if (last >= cap && S.szlo[g] < last - (cap - 1)) S.szlo[g] = last - (cap - 1);
}
// appendEntry's entries (last0, last0 + k] at Term `term`: their sizes enter the
// ring (d = their descriptors; null = the becomeLeader noop, pb.Entry{})
__device__ __forceinline__ void sz_append(const DevState& S, uint32_t g, uint64_t last0, uint64_t k, uint64_t term,
                                          const uint32_t* d) {
  if (!sz_on(S.max_msg_size)) return;
  const uint64_t x = S.szx[g];
  const uint64_t cap = lx_cap(x);
  uint64_t acc = *cum_at(x, last0);
  for (uint64_t j = 1; j <= k; ++j) {
    acc += ent_size(d ? d[j - 1] : 0u, term, last0 + j);
    if (j + cap > k) *cum_at(x, last0 + j) = acc;
  }
  sz_keep(S, g, x, last0 + k);
}
// sendAppend's entries(next, maxMsgSize) (raft/raft.go:265, raft/log.go:219-224)
// cut by limitSize (raft/util.go:97-110): the last index sent, next <= last.
// The first entry always goes; each further one while the running sum of
// Entry.Size() stays <= maxSize (a binary search over the cumulative sizes).
// *ok = false when the ring does not reach back to next - 1 (the caller did
// not load the group's sizes: hb_load_entry_sizes / hb_reserve_log).
__device__ __forceinline__ uint64_t sz_limit(const DevState& S, uint32_t g, uint64_t next, uint64_t last, bool* ok) {
  if (S.max_msg_size == 0) return next;
  if (S.max_msg_size == HB_NO_LIMIT) return last;
  if (next - 1 < S.szlo[g]) {
    *ok = false;
    return next;
  }
  const uint64_t x = S.szx[g];
  const uint64_t base = *cum_at(x, next - 1);
  uint64_t lo = next, hi = last;
  while (lo < hi) {
    const uint64_t mid = lo + (hi - lo + 1) / 2;
    if (*cum_at(x, mid) - base <= S.max_msg_size) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// ---- term runs (follower side) ---------------------------------------------------
// The log's runs below the current-term run, oldest first, as a ring of
// {start index, term} pairs: run k covers [start_k, start_k+1).  push adds a
// newer run (a full ring drops its oldest; the host reserves enough that only
// runs wholly below firstIndex - 1 can leave), cut drops the runs starting at
// or after an index, find returns the newest run starting at or before i.
struct Runs {
  uint64_t* R;
  uint64_t mask;
  uint32_t n, h;
  __device__ __forceinline__ void open(const DevState& S, uint32_t g) {
    const uint64_t x = S.trx[g], c = S.trc[g];
    R = lx_base(x);
    mask = lx_cap(x) - 1;
    n = (uint32_t)c;
    h = (uint32_t)(c >> 32);
  }
  __device__ __forceinline__ uint64_t* at(uint32_t k) const { return R + 2 * ((h + k) & mask); }
  __device__ __forceinline__ void close(const DevState& S, uint32_t g) const {
    S.trc[g] = (uint64_t)n | ((uint64_t)h << 32);
  }
  __device__ __forceinline__ void push(uint64_t start, uint64_t t) {
    if (n > 0 && at(n - 1)[1] == t) return;  // the run goes on
    if ((uint64_t)n == mask + 1) {           // full: the oldest run leaves
      h = (uint32_t)((h + 1) & mask);
      --n;
    }
    uint64_t* r = at(n);
    r[0] = start;
    r[1] = t;
    ++n;
  }
  __device__ __forceinline__ void cut(uint64_t ci) {
    while (n > 0 && at(n - 1)[0] >= ci) --n;
  }
  // the term of index i (binary search; starts increase), *ok = false below the oldest run
  __device__ __forceinline__ uint64_t find(uint64_t i, bool* ok) const {
    if (n == 0 || at(0)[0] > i) {
      *ok = false;
      return 0;
    }
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo + 1) / 2;
      if (at(mid)[0] <= i) lo = mid;
      else hi = mid - 1;
    }
    return at(lo)[1];
  }
};
// reset of a group whose term changes: its current-term run becomes an older run
__device__ __forceinline__ void tr_push(const DevState& S, uint32_t g, uint64_t start, uint64_t t) {
  Runs r;
  r.open(S, g);
  const uint32_t n0 = r.n, h0 = r.h;
  r.push(start, t);
  if (r.n != n0 || r.h != h0) r.close(S, g);
}

// ---- event sink ---------------------------------------------------------------
// Device event records are compact 8-byte words (the public 16-byte hb_event
// stream is expanded from them by hb_copy_events, see hipbatch.hip):
//
//   [0:4)   type: HB_EV_*, or EVC_BCAST (an HB_EV_APP to every slot in the
//           mask, same x), or EVC_VBCAST (an HB_EV_VOTE to every slot in the
//           mask, same x), or EVC_CONT (second word of a long record)
//   [4:11)  to (slot / node ref), or the slot mask of EVC_BCAST
//   [11]    long: x >= 2^40, its high 24 bits follow in an EVC_CONT word
//   [12:16) aux (LAST noop flag, FAULT code)
//   [16:24) the group's lane in its partition (the chunk names the partition)
//   [24:64) x bits 0..39
//   EVC_CONT word: [0:4) = EVC_CONT, [4:28) = x bits 40..63
//
// A workgroup appends its words to its own chunk: the chunk base is computed
// by every lane from kernel arguments (a global-address-space pointer, so the
// stores are global_store, not flat) and the fill cursor is one LDS word.
constexpr uint32_t EVC_BCAST = HB_EVW_BCAST;
constexpr uint32_t EVC_VBCAST = HB_EVW_VBCAST;  // an HB_EV_VOTE to every slot in the mask, same x
constexpr uint32_t EVC_CONT = HB_EVW_CONT;
constexpr uint32_t EVC_WORDS_MAX = 2;  // words per event (long records)

struct EvSink {
  uint64_t* chunk;            // this workgroup's chunk (global)
  uint32_t* fill;             // words written by the workgroup (LDS)
};
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a > b ? b : a; }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__host__ __device__ constexpr uint64_t evc_word(uint32_t type, uint32_t to, uint32_t aux, uint32_t lane, uint64_t x,
                                                bool lng) {
  return (uint64_t)(type & 0xF) | ((uint64_t)(to & 0x7F) << 4) | ((uint64_t)lng << 11) | ((uint64_t)(aux & 0xF) << 12) |
         ((uint64_t)(lane & 0xFF) << 16) | ((x & 0xFFFFFFFFFFull) << 24);
}

// Append one event.  One LDS atomic per active lane (the compiler's atomic
// optimizer makes it one ds_add per wave plus mbcnt), so the lanes of a wave
// write side by side; a lane's events keep their order.  Values of x that
// need more than 40 bits take a second word (rare path).
__device__ __forceinline__ void emit_ev(const EvSink& sink, uint32_t lane, uint32_t type, uint32_t to, uint32_t aux,
                                        uint64_t x) {
  if (__builtin_expect((x >> 40) == 0, 1)) {
    const uint32_t pos = atomicAdd(sink.fill, 1u);
    sink.chunk[pos] = evc_word(type, to, aux, lane, x, false);
  } else {
    const uint32_t pos = atomicAdd(sink.fill, 2u);
    sink.chunk[pos] = evc_word(type, to, aux, lane, x, true);
    sink.chunk[pos + 1] = (uint64_t)EVC_CONT | ((x >> 40) << 4);
  }
}

template <int N>
__device__ __forceinline__ uint64_t sel64(const uint64_t (&a)[N], uint32_t s) {
  uint64_t v = a[0];
#pragma unroll
  for (int i = 1; i < N; ++i) v = (s == (uint32_t)i) ? a[i] : v;
  return v;
}
template <int N>
__device__ __forceinline__ uint32_t sel32(const uint32_t (&a)[N], uint32_t s) {
  uint32_t v = a[0];
#pragma unroll
  for (int i = 1; i < N; ++i) v = (s == (uint32_t)i) ? a[i] : v;
  return v;
}

// dirty bits
constexpr uint32_t D_META = 1u << 0;
constexpr uint32_t D_TERM = 1u << 1;
constexpr uint32_t D_COMMIT = 1u << 2;
constexpr uint32_t D_LAST = 1u << 3;
constexpr uint32_t D_TRUN = 1u << 4;
constexpr uint32_t D_ELAPSED = 1u << 5;  // reset zeroed r.elapsed
constexpr uint32_t D_FIRST = 1u << 6;    // a restored snapshot moved firstIndex (and the snapshot index)
constexpr uint32_t D_SLOT0 = 8;  // bit D_SLOT0 + s: slot s (match, next, pm)

struct Pr {
  uint64_t match, next;
  uint64_t head;  // inflights.buffer[start] (valid while count > 0)
  uint32_t pm;
};

// Per-slot state is held in vector registers: a runtime slot index becomes a
// register-indexed extract/insert instead of a private-memory array access
// (which would push the whole lane state to scratch).
template <int NMAX> struct SlotVec;
template <> struct SlotVec<3> {
  typedef uint64_t u64 __attribute__((ext_vector_type(4)));
  typedef uint32_t u32 __attribute__((ext_vector_type(4)));
};
template <> struct SlotVec<5> {
  typedef uint64_t u64 __attribute__((ext_vector_type(8)));
  typedef uint32_t u32 __attribute__((ext_vector_type(8)));
};
template <> struct SlotVec<7> {
  typedef uint64_t u64 __attribute__((ext_vector_type(8)));
  typedef uint32_t u32 __attribute__((ext_vector_type(8)));
};

// One lane = one raft group.  All state of the group is held in registers
// between load() and store().
__device__ __forceinline__ bool is_follower_type(uint32_t t) {  // the follower side of Step
  return t == HB_MSG_APP || t == HB_MSG_HEARTBEAT || t == HB_MSG_SNAP || t == HB_MSG_VOTE;
}

// FOLLOW: the variant that also steps the follower side (MsgApp / MsgHeartbeat
// / MsgSnap / MsgVote, raft/raft.go:585-707); the other one never sees those
// types (its kernels hand such a group over to k_follow).
template <int NMAX, bool FOLLOW = false>
struct Lane {
  DevState S;
  EvSink E;
  uint32_t g;
  uint32_t arrival;  // batch position of the message; 0xFFFFFFFF: props[] proposal
  uint64_t term, committed, first, last, tfirst, tlast, meta;
  uint64_t meta0;  // meta as loaded (which arrays are stale: M_TL / M_SM)
  typename SlotVec<NMAX>::u64 match, next;
  typename SlotVec<NMAX>::u64 head;  // register copy of each ring's head entry
  typename SlotVec<NMAX>::u32 pm;
  uint32_t dirty;
  uint32_t won, lost;
  uint32_t nev;  // events emitted
  bool prog;     // match / next / pm / head hold the group's progress (loaded or reset)
  bool rc_zero;  // r.Commit was 0 when the message being stepped arrived (M_NC)
  bool voted;    // the message's HB_INFO_VOTED bit (follower side)

  // ---------------------------------------------------------------- meta
  __device__ __forceinline__ uint32_t n() const { return m_n(meta); }
  __device__ __forceinline__ uint32_t state() const { return m_state(meta); }
  __device__ __forceinline__ uint32_t self() const { return m_self(meta); }
  __device__ __forceinline__ uint32_t lead() const { return m_lead(meta); }
  __device__ __forceinline__ uint32_t vote() const { return m_vote(meta); }
  __device__ __forceinline__ uint32_t faulted() const { return m_fault(meta); }
  __device__ __forceinline__ uint32_t self_ref() const { return self() == HB_SLOT_NONE ? HB_REF_SELF : self(); }
  __device__ __forceinline__ uint64_t soft() const {
    return (uint64_t)state() | ((uint64_t)lead() << 8) | ((uint64_t)vote() << 16);
  }
  __device__ __forceinline__ void set_field(int shift, uint64_t mask, uint64_t v) {
    meta = (meta & ~(mask << shift)) | ((v & mask) << shift);
    dirty |= D_META;
  }
  __device__ __forceinline__ void set_state(uint32_t v) { set_field(0, 3, v); }
  __device__ __forceinline__ void set_lead(uint32_t v) { set_field(9, 0xF, v); }
  __device__ __forceinline__ void set_vote(uint32_t v) { set_field(13, 0xF, v); }
  __device__ __forceinline__ void set_votes(uint32_t resp, uint32_t grant) {
    set_field(M_RESP_SHIFT, 0xFF, resp);
    set_field(M_GRANT_SHIFT, 0xFF, grant);
  }

  __device__ __forceinline__ uint64_t arrival_x() const {
    return arrival == 0xFFFFFFFFu ? HB_NO_INDEX : (uint64_t)arrival;
  }
  __device__ __forceinline__ void ev(uint32_t type, uint32_t to, uint32_t aux, uint64_t x) {
    emit_ev(E, g & (PART - 1), type, to, aux, x);
    nev++;
  }
  // A reference panic: the group stops; the FAULT event is emitted once, at
  // the end of the message (nothing else is emitted after a fault).
  __device__ __forceinline__ void fault(uint32_t code) {
    if (faulted()) return;
    set_field(17, 0xF, code);
  }

  // ---------------------------------------------------------------- memory
  __device__ __forceinline__ uint64_t* ring_at(uint32_t s, uint32_t idx) const {
    return S.ring + ((size_t)s * S.W + idx) * S.G + g;
  }
  __device__ __forceinline__ Pr get(uint32_t s) const {
    Pr p;
    p.match = match[s];
    p.next = next[s];
    p.pm = pm[s];
    p.head = head[s];
    return p;
  }
  __device__ __forceinline__ void put(uint32_t s, const Pr& p) {
    match[s] = p.match;
    next[s] = p.next;
    pm[s] = p.pm;
    head[s] = p.head;
    dirty |= 1u << (D_SLOT0 + s);
  }

  // Load every field of the group (all NMAX slots, independent of meta, so all
  // loads of a lane are in flight together); slots >= n hold zeros (k_load).
  // A ring head is read only for a non-empty ring.
  __device__ __forceinline__ void load_all() {
    load_group();
    load_progress();
  }
  // The per-group fields only; step() loads the progress when a leader first
  // steps a message.  A vote tally reads none, and an election or a higher
  // term re-initialises every Progress (raft/raft.go:334-349), so a storm
  // never loads it.
  __device__ __forceinline__ void load_group() {
    term = S.term[g];
    committed = S.commit[g];
    first = S.first[g];
    last = S.last[g];
    tfirst = S.tfirst[g];
    tlast = S.tlast[g];
    meta0 = meta;
    if (meta & M_TL) tlast = last;
    dirty = 0;
    prog = false;
  }
  __device__ __forceinline__ void load_progress() {
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      match[s] = S.match[(size_t)s * S.G + g];
      next[s] = S.next[(size_t)s * S.G + g];
      pm[s] = S.pm[(size_t)s * S.G + g];
    }
    if (meta & M_RS) {  // the reset form (every slot rewritten by store)
      const uint32_t nn = n();
#pragma unroll
      for (int s = 0; s < NMAX; ++s) {
        if ((uint32_t)s < nn) {
          uint64_t mt, nx;
          uint32_t p;
          rs_progress(meta, (uint32_t)s, last, tfirst, &mt, &nx, &p);
          match[s] = mt;
          next[s] = nx;
          pm[s] = p;
          dirty |= 1u << (D_SLOT0 + s);
        }
      }
      meta &= ~M_RS;
      dirty |= D_META;
    }
#pragma unroll
    for (int s = 0; s < NMAX; ++s) head[s] = pm_count(pm[s]) ? *ring_at(s, pm_start(pm[s])) : 0;
    if (meta0 & M_SM) {  // as loaded: the self arrays are stale, last (unchanged so far) is their value
      const uint32_t sf = m_self(meta0);
#pragma unroll
      for (int s = 0; s < NMAX; ++s) {
        if ((uint32_t)s == sf) {
          match[s] = last;
          next[s] = last + 1;
        }
      }
    }
    prog = true;
  }

  __device__ __forceinline__ void store() {
    if (dirty & D_FIRST) S.first[g] = first;  // a restored snapshot
    {  // re-derive M_TL / M_SM; an array that was stale and no longer may be is written
      const uint32_t sf = self(), nn = n();
      const bool tl = tlast == last;
      bool sm = (meta0 & M_SM) != 0;  // progress never loaded: nothing (incl. last) changed it
      if (prog) {
        sm = false;
#pragma unroll
        for (int s = 0; s < NMAX; ++s)
          if ((uint32_t)s == sf && (uint32_t)s < nn) sm = match[s] == last && next[s] == last + 1;
      }
      const uint64_t m2 = (meta & ~(M_TL | M_SM)) | (tl ? M_TL : 0ull) | (sm ? M_SM : 0ull);
      if (m2 != meta) {
        meta = m2;
        dirty |= D_META;
      }
      if (!tl && (meta0 & M_TL)) dirty |= D_TRUN;
      if (!sm && (meta0 & M_SM) && sf < (uint32_t)NMAX) dirty |= 1u << (D_SLOT0 + sf);
    }
    if (dirty & D_META) S.meta[g] = meta;
    if (dirty & D_TERM) S.term[g] = term;
    if (dirty & D_COMMIT) S.commit[g] = committed;
    if (dirty & D_LAST) S.last[g] = last;
    if (dirty & D_TRUN) {
      S.tfirst[g] = tfirst;
      S.tlast[g] = tlast;
    }
    if (dirty & D_ELAPSED) S.elapsed[g] = 0;
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      if (dirty & (1u << (D_SLOT0 + s))) {
        S.match[(size_t)s * S.G + g] = match[s];
        S.next[(size_t)s * S.G + g] = next[s];
        S.pm[(size_t)s * S.G + g] = pm[s];
      }
    }
  }

  // ---------------------------------------------------------------- Progress
  // raft/progress.go:147-158
  __device__ __forceinline__ bool is_paused(uint32_t p) const {
    const uint32_t st = pm_state(p);
    if (st == HB_PR_PROBE) return pm_paused(p) != 0;
    if (st == HB_PR_REPLICATE) return pm_count(p) == S.W;
    return true;
  }
  // becomeProbe raft/progress.go:76-88
  __device__ __forceinline__ void become_probe(uint32_t s, Pr& p) const {
    if (pm_state(p.pm) == HB_PR_SNAPSHOT) {
      const uint64_t pending = S.pending[(size_t)s * S.G + g];
      p.pm = pm_make(HB_PR_PROBE, 0, 0, 0);
      p.next = umax64(p.match + 1, pending + 1);
    } else {
      p.pm = pm_make(HB_PR_PROBE, 0, 0, 0);
      p.next = p.match + 1;
    }
  }
  // becomeReplicate raft/progress.go:90-93
  __device__ __forceinline__ void become_replicate(Pr& p) const {
    p.pm = pm_make(HB_PR_REPLICATE, 0, 0, 0);
    p.next = p.match + 1;
  }
  // maybeUpdate raft/progress.go:102-113
  __device__ __forceinline__ bool maybe_update(Pr& p, uint64_t nidx) const {
    bool updated = false;
    if (p.match < nidx) {
      p.match = nidx;
      updated = true;
      p.pm &= ~PM_PAUSED;
    }
    if (p.next < nidx + 1) p.next = nidx + 1;
    return updated;
  }
  // maybeDecrTo raft/progress.go:119-141
  __device__ __forceinline__ bool maybe_decr_to(Pr& p, uint64_t rejected, uint64_t lasthint) const {
    if (pm_state(p.pm) == HB_PR_REPLICATE) {
      if (rejected <= p.match) return false;
      p.next = p.match + 1;
      return true;
    }
    if (p.next - 1 != rejected) return false;
    p.next = umin64(rejected, lasthint + 1);
    if (p.next < 1) p.next = 1;
    p.pm &= ~PM_PAUSED;
    return true;
  }
  // inflights.freeTo raft/progress.go:204-224
  // (the head entry comes from the register copy; only entries behind it are read)
  __device__ __forceinline__ void free_to(uint32_t s, Pr& p, uint64_t to) const {
    const uint32_t cnt = pm_count(p.pm);
    if (cnt == 0) return;
    uint64_t v = p.head;
    if (to < v) return;
    uint32_t idx = pm_start(p.pm);
    const uint32_t W = S.W;
    uint32_t i = 0;
    while (true) {
      ++i;
      if (++idx >= W) idx -= W;
      if (i == cnt) break;
      v = *ring_at(s, idx);
      if (to < v) break;
    }
    p.pm = pm_make(pm_state(p.pm), pm_paused(p.pm), idx, cnt - i);
    p.head = v;
  }

  // ---------------------------------------------------------------- log
  // raftLog.term(i) == Term, restated over the current-term run (raft/log.go:198-217)
  __device__ __forceinline__ bool term_eq(uint64_t i) const {
    if (i + 1 < first || i > last) return term == 0;
    return tfirst <= i && i <= tlast;
  }
  // commitTo raft/log.go:172-180
  __device__ __forceinline__ void commit_to(uint64_t to) {
    if (committed < to) {
      if (last < to) {
        fault(HB_FAULT_COMMIT_RANGE);
        return;
      }
      committed = to;
      dirty |= D_COMMIT;
      ev(HB_EV_COMMIT, 0, 0, to);
    }
  }
  // maybeCommit raft/raft.go:323-332 + raftLog.maybeCommit raft/log.go:241-247:
  // the q-th largest Match by a register sorting network.
  __device__ __forceinline__ bool maybe_commit() {
    typename SlotVec<NMAX>::u64 v;
    const uint32_t nn = n();
#pragma unroll
    for (int s = 0; s < NMAX; ++s) v[s] = ((uint32_t)s < nn) ? match[s] : 0;
#pragma unroll
    for (int r = 0; r < NMAX; ++r) {
#pragma unroll
      for (int j = (r & 1); j + 1 < NMAX; j += 2) {
        const uint64_t a = v[j], b = v[j + 1];
        v[j] = a > b ? a : b;
        v[j + 1] = a > b ? b : a;
      }
    }
    const uint64_t mci = v[nn / 2];  // q-1 with q = n/2+1
    if (mci > committed && term_eq(mci)) {
      commit_to(mci);
      return faulted() == 0;
    }
    return false;
  }

  // ---------------------------------------------------------------- sends
  // sendAppend raft/raft.go:239-282 for the progress p of slot s
  __device__ __forceinline__ void send_append(uint32_t s, Pr& p) {
    if (is_paused(p.pm)) return;
    if (p.next < first) {  // needSnapshot raft/raft.go:715-717
      const uint64_t snapi = S.snap[g];
      if (snapi == 0) {
        fault(HB_FAULT_EMPTY_SNAPSHOT);
        return;
      }
      p.pm = pm_make(HB_PR_SNAPSHOT, 0, 0, 0);  // becomeSnapshot
      S.pending[(size_t)s * S.G + g] = snapi;
      ev(HB_EV_SNAP, s, 0, snapi);
      return;
    }
    const uint64_t x = p.next - 1;
    if (p.next <= last) {
      bool ok = true;
      const uint64_t lastsent = sz_limit(S, g, p.next, last, &ok);
      if (!ok) {
        fault(HB_FAULT_SIZE_WINDOW);
        return;
      }
      const uint32_t st = pm_state(p.pm);
      if (st == HB_PR_REPLICATE) {
        const uint32_t cnt = pm_count(p.pm), start = pm_start(p.pm);
        if (cnt == S.W) {
          fault(HB_FAULT_INFLIGHTS_FULL);
          return;
        }
        uint32_t idx = start + cnt;
        if (idx >= S.W) idx -= S.W;
        *ring_at(s, idx) = lastsent;                    // inflights.add
        if (cnt == 0) p.head = lastsent;
        p.next = lastsent + 1;                          // optimisticUpdate
        p.pm = pm_make(HB_PR_REPLICATE, pm_paused(p.pm), start, cnt + 1);
      } else if (st == HB_PR_PROBE) {
        p.pm |= PM_PAUSED;                              // pause
      }
    }
    ev(HB_EV_APP, s, (tfirst <= x && x <= tlast) ? 1u : 0u, x);  // aux: term(x) == Term (m.LogTerm)
  }

  // ---------------------------------------------------------------- transitions
  // reset raft/raft.go:334-349.  The log's terms as the device keeps them: the
  // current-term run [tfirst, last] (tfirst = HB_NO_INDEX: none) plus the
  // older runs (Runs, the log index).
  __device__ __forceinline__ void reset(uint64_t t) {
    if (term != t) {
      if (tfirst != HB_NO_INDEX) tr_push(S, g, tfirst, term);  // the old current-term run becomes an older run
      term = t;
      set_vote(HB_REF_NONE);
      tfirst = HB_NO_INDEX;  // no entry carries a term newer than the old Term
      tlast = 0;
      dirty |= D_TERM | D_TRUN;
      ev(HB_EV_TERM, 0, 0, t);
    }
    set_lead(HB_REF_NONE);
    dirty |= D_ELAPSED;  // r.elapsed = 0
    set_votes(0, 0);
    const uint32_t nn = n(), sf = self();
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      if ((uint32_t)s < nn) {
        match[s] = ((uint32_t)s == sf) ? last : 0;
        next[s] = last + 1;
        pm[s] = pm_make(HB_PR_PROBE, 0, 0, 0);
        dirty |= 1u << (D_SLOT0 + s);
      }
    }
    if (meta & M_RS) set_field(23, 1, 0);  // every slot is written
    prog = true;
  }
  // becomeFollower :384-391 / becomeCandidate :393-404 / becomeLeader :406-427.
  // Returns true when the transition happened (false on a reference panic).
  // oth: HB_STATE_OTH_LEAD when ld is the stepped message's sender outside prs.
  __device__ __forceinline__ bool transition(uint32_t kind, uint64_t t, uint32_t ld, uint32_t oth = 0) {
    if (kind == HB_STATE_CANDIDATE && state() == HB_STATE_LEADER) {
      fault(HB_FAULT_LEADER_CAMPAIGN);
      return false;
    }
    if (kind == HB_STATE_LEADER && state() == HB_STATE_FOLLOWER) {
      fault(HB_FAULT_FOLLOWER_LEADER);
      return false;
    }
    const uint64_t before = soft();
    reset(kind == HB_STATE_CANDIDATE ? term + 1 : (kind == HB_STATE_FOLLOWER ? t : term));
    set_lead(kind == HB_STATE_LEADER ? self_ref() : (kind == HB_STATE_FOLLOWER ? ld : (uint32_t)HB_REF_NONE));
    if (kind == HB_STATE_CANDIDATE) set_vote(self_ref());
    set_state(kind);
    if (soft() != before || oth) ev(HB_EV_STATE, 0, oth, soft());
    return true;
  }
  // poll raft/raft.go:445-460 (votes map as responded/granted bitmasks)
  __device__ __forceinline__ uint32_t poll(uint32_t bit, bool v) {
    uint32_t resp = m_resp(meta), grant = m_grant(meta);
    if (!((resp >> bit) & 1u)) {
      resp |= 1u << bit;
      if (v) grant |= 1u << bit;
      set_votes(resp, grant);
    }
    return (uint32_t)__popc(grant);
  }

  // ---------------------------------------------------------------- follower side
  // raftLog.term(i) from what the device keeps: 0 outside [first-1, last]
  // (raft/log.go:198-203), Term in the current-term run, else the newest older
  // run starting at or before i; *ok = false when the loaded runs do not reach
  // back (the caller did not load the group's runs: hb_load_term_runs).
  __device__ __forceinline__ uint64_t fterm(uint64_t i, bool* ok) const {
    if (i + 1 < first || i > last) return 0;
    if (tfirst != HB_NO_INDEX && i >= tfirst) return term;
    Runs r;
    r.open(S, g);
    return r.find(i, ok);
  }
  __device__ __forceinline__ void resp(uint32_t to, uint32_t kind, uint64_t x) { ev(HB_EV_RESP, to, kind, x); }

  // raftLog.append of the MsgApp's entries from the first conflict ci
  // (maybeAppend raft/log.go:80-85 -> unstable.truncateAndAppend): the log is
  // cut at ci - 1 and takes entries ci .. index + ne (terms eterm[e0 ..]).
  __device__ __forceinline__ void follower_append(uint64_t ci, uint64_t index, uint64_t e0, uint64_t ne) {
    if (!prog) load_progress();  // M_SM derives the self Match from last: pin it before last moves
    Runs rr;
    rr.open(S, g);
    rr.cut(ci);
    if (tfirst != HB_NO_INDEX && tfirst >= ci) tfirst = HB_NO_INDEX;
    const bool sized = sz_on(S.max_msg_size);
    uint64_t acc = 0, x = 0;
    if (sized) {
      x = S.szx[g];
      if (ci - 1 < S.szlo[g]) {  // the log (and its sizes) restart at ci - 1
        S.szlo[g] = ci - 1;
        *cum_at(x, ci - 1) = 0;
      }
      acc = *cum_at(x, ci - 1);
    }
    const uint64_t lastnewi = index + ne;
#pragma nounroll
    for (uint64_t j = ci; j <= lastnewi; ++j) {
      const uint64_t k = e0 + (j - index - 1);
      const uint64_t t = S.eterm[k];
      if (t == term) {
        if (tfirst == HB_NO_INDEX) tfirst = j;
      } else {
        if (tfirst != HB_NO_INDEX) {  // a lower term after Term entries
          rr.push(tfirst, term);
          tfirst = HB_NO_INDEX;
        }
        rr.push(j, t);
      }
      if (sized) {
        acc += ent_size(S.edesc ? S.edesc[k] : 0u, t, j);
        *cum_at(x, j) = acc;
      }
    }
    rr.close(S, g);
    last = lastnewi;
    tlast = tfirst != HB_NO_INDEX ? last : 0;
    dirty |= D_LAST | D_TRUN;
    if (sized) sz_keep(S, g, x, last);
    ev(HB_EV_FOLLOW, 0, HB_FOLLOW_APPEND, arrival_x());
  }

  // handleAppendEntries raft/raft.go:651-665 + maybeAppend raft/log.go:72-88
  __device__ __forceinline__ void handle_append(uint64_t index, uint64_t lterm, uint32_t fref) {
    const uint64_t mcommit = S.bcommit ? S.bcommit[arrival] : 0;
    uint64_t e0 = 0, ne = 0;
    if (S.eoff && S.eterm) {
      e0 = S.eoff[arrival];
      ne = (arrival + 1 < S.bn ? S.eoff[arrival + 1] : S.n_ent) - e0;
    }
    // r.Commit: committed at a Step boundary, or 0 before the group's first Step (M_NC)
    if (!rc_zero && index < committed) {
      resp(fref, HB_RESP_APP, committed);
      return;
    }
    const uint64_t lastnewi = index + ne;
    bool ok = true;
    const uint64_t t = fterm(index, &ok);
    if (!ok) {
      fault(HB_FAULT_TERM_WINDOW);
      return;
    }
    if (t != lterm) {  // reject; RejectHint = lastIndex (the host reads it from its log)
      resp(fref, HB_RESP_APP | HB_RESP_REJECT, index);
      return;
    }
    uint64_t ci = 0;  // findConflict raft/log.go:112-123
#pragma nounroll
    for (uint64_t k = 0; k < ne; ++k) {
      const uint64_t et = fterm(index + 1 + k, &ok);
      if (!ok) {
        fault(HB_FAULT_TERM_WINDOW);
        return;
      }
      if (et != S.eterm[e0 + k]) {
        ci = index + 1 + k;
        break;
      }
    }
    if (ci) {
      if (ci <= committed) {  // "entry %d conflict with committed entry" raft/log.go:79
        fault(HB_FAULT_CONFLICT_COMMITTED);
        return;
      }
      follower_append(ci, index, e0, ne);
    }
    commit_to(umin64(mcommit, lastnewi));
    if (faulted()) return;
    resp(fref, HB_RESP_APP, lastnewi);
  }

  // restore raft/raft.go:684-707 + handleSnapshot :671-682
  __device__ __forceinline__ void handle_snapshot(uint64_t sidx, uint64_t sterm, uint32_t fref) {
    bool restored = false;
    if (sidx > committed) {
      bool ok = true;
      const uint64_t t = fterm(sidx, &ok);
      if (!ok) {
        fault(HB_FAULT_TERM_WINDOW);
        return;
      }
      if (t == sterm) {  // matchTerm: fast-forward the commit
        commit_to(sidx);
        if (faulted()) return;
      } else {  // raftLog.restore: committed = index, the log = the snapshot
        restored = true;
        first = sidx + 1;
        last = sidx;
        committed = sidx;
        S.snap[g] = sidx;
        dirty |= D_FIRST | D_LAST | D_COMMIT | D_TRUN;
        tfirst = HB_NO_INDEX;
        tlast = 0;
        Runs rr;
        rr.open(S, g);
        rr.n = 0;
        rr.h = 0;
        if (sterm == term) {
          tfirst = sidx;
          tlast = sidx;
        } else {
          rr.push(sidx, sterm);
        }
        rr.close(S, g);
        const uint32_t nn = n(), sf = self();
#pragma unroll
        for (int s = 0; s < NMAX; ++s) {  // setProgress for every peer of the ConfState
          if ((uint32_t)s < nn) {
            match[s] = ((uint32_t)s == sf) ? last : 0;
            next[s] = last + 1;
            pm[s] = pm_make(HB_PR_PROBE, 0, 0, 0);
            dirty |= 1u << (D_SLOT0 + s);
          }
        }
        if (meta & M_RS) set_field(23, 1, 0);  // every slot is written
        prog = true;
        if (sz_on(S.max_msg_size)) {
          S.szlo[g] = sidx;
          *cum_at(S.szx[g], sidx) = 0;
        }
        ev(HB_EV_FOLLOW, 0, HB_FOLLOW_RESTORE, arrival_x());
      }
    }
    resp(fref, HB_RESP_APP, restored ? last : committed);
  }

  // The follower-side message types after the term gate: stepLeader /
  // stepCandidate / stepFollower (raft/raft.go:494-649); lterm = m.LogTerm
  // (MsgApp / MsgVote) or the snapshot's term (MsgSnap).
  __device__ __forceinline__ void follow(uint32_t type, uint32_t from, uint64_t mterm, uint64_t index,
                                         uint64_t lterm) {
    const uint32_t fref = from < n() ? from : (uint32_t)HB_REF_OTHER;
    const uint32_t oth = fref == HB_REF_OTHER ? (uint32_t)HB_STATE_OTH_LEAD : 0u;
    const uint32_t st = state();
    if (st == HB_STATE_LEADER || (st == HB_STATE_CANDIDATE && type == HB_MSG_VOTE)) {
      if (type == HB_MSG_VOTE) resp(fref, HB_RESP_VOTE | HB_RESP_REJECT, 0);  // :555-558, :600-602
      return;
    }
    if (st == HB_STATE_CANDIDATE) {  // :591-599: becomeFollower, then handle
      if (!transition(HB_STATE_FOLLOWER, type == HB_MSG_SNAP ? mterm : term, fref, oth)) return;
    } else if (type == HB_MSG_VOTE) {  // stepFollower :636-648
      const bool can = vote() == HB_REF_NONE || (from < n() ? vote() == from : voted);
      bool grant = false;
      if (can) {
        bool ok = true;
        const uint64_t lt = fterm(last, &ok);  // isUpToDate raft/log.go:235-237
        if (!ok) {
          fault(HB_FAULT_TERM_WINDOW);
          return;
        }
        grant = lterm > lt || (lterm == lt && index >= last);
      }
      if (grant) {
        dirty |= D_ELAPSED;
        const uint64_t before = soft();
        set_vote(fref);
        if (soft() != before || oth) ev(HB_EV_STATE, 0, oth ? (uint32_t)HB_STATE_OTH_VOTE : 0u, soft());
        resp(fref, HB_RESP_VOTE, 0);
      } else {
        resp(fref, HB_RESP_VOTE | HB_RESP_REJECT, 0);
      }
      return;
    } else {  // stepFollower :625-635: r.elapsed = 0; lead = m.From (not for MsgSnap)
      dirty |= D_ELAPSED;
      if (type != HB_MSG_SNAP) {
        const uint64_t before = soft();
        set_lead(fref);
        if (soft() != before || oth) ev(HB_EV_STATE, 0, oth, soft());
      }
    }
    if (type == HB_MSG_APP) {
      handle_append(index, lterm, fref);
    } else if (type == HB_MSG_HEARTBEAT) {  // handleHeartbeat :666-669
      commit_to(S.bcommit ? S.bcommit[arrival] : 0);
      if (!faulted()) resp(fref, HB_RESP_HEARTBEAT, 0);
    } else {
      handle_snapshot(index, lterm, fref);
    }
  }

  // ---------------------------------------------------------------- step
  // Step (raft/raft.go:462-490) + stepLeader/stepCandidate/stepFollower
  // (:494-649) for the engine's message types, as one straight-line pipeline
  // so that each primitive (and each event site) exists once in the code:
  //   gate -> transition 1 -> progress / poll -> transition 2 -> append ->
  //   maybeCommit -> sends.
  // The order of effects (and events) equals the reference's call order.
  enum : uint32_t { SEND_NONE = 0, SEND_ONE, SEND_BCAST, SEND_VOTES, SEND_BEATS };

  __device__ __forceinline__ void step(uint32_t type, uint32_t from, uint64_t mterm, uint64_t index, bool reject,
                                       uint64_t lasthint) {
    uint32_t t1 = 0xFF, t2 = 0xFF, ld1 = HB_REF_NONE;
    uint64_t tt1 = 0;
    // ---- gate (raft/raft.go:462-486)
    if (type == HB_MSG_HUP) {
      t1 = HB_STATE_CANDIDATE;                                   // campaign -> becomeCandidate
    } else if (mterm != 0) {
      if (mterm < term) return;                                  // ignore lower term
      if (mterm > term) {
        t1 = HB_STATE_FOLLOWER;
        tt1 = mterm;
        if (type == HB_MSG_VOTE) ld1 = HB_REF_NONE;             // lead = None for MsgVote (:476-478)
        else if (from < n()) ld1 = from;
        else if (type == HB_MSG_BEAT || type == HB_MSG_PROP) ld1 = self_ref();
        else ld1 = HB_REF_OTHER;
      }
    }
    // past the gate: this Step ends with r.Commit = committed (raft/raft.go:466,488)
    rc_zero = (meta & M_NC) != 0;
    if (rc_zero) set_field(24, 1, 0);
    if constexpr (FOLLOW) {  // the events up to the next marker belong to this message
      if (is_follower_type(type)) ev(HB_EV_FOLLOW, 0, HB_FOLLOW_STEP, arrival_x());
    }
    if (t1 != 0xFF) transition(t1, tt1, ld1, ld1 == HB_REF_OTHER ? (uint32_t)HB_STATE_OTH_LEAD : 0u);
    if constexpr (FOLLOW) {
      if (is_follower_type(type)) {
        if (!faulted()) follow(type, from, mterm, index, lasthint);
        if (faulted()) ev(HB_EV_FAULT, 0, faulted(), arrival_x());
        return;
      }
    }
    // Only a leader reads its progress without resetting it first: a candidate
    // or follower polls, and becomeCandidate / becomeLeader / becomeFollower
    // reset every Progress before a send or an append touches one.
    if (!prog && state() == HB_STATE_LEADER) load_progress();

    uint32_t send = SEND_NONE, send_to = 0;
    uint64_t append_k = 0;
    uint32_t noop = 0;
    bool resolve_accept = false, old_paused = false;
    if (!faulted()) {
      const uint32_t st = state();
      const uint32_t nn = n();
      const uint32_t q = nn / 2 + 1;
      if (type == HB_MSG_HUP) {
        // campaign raft/raft.go:429-443 (after becomeCandidate)
        const uint32_t sf = self();
        if (q == poll(sf == HB_SLOT_NONE ? 7u : sf, true)) {
          won++;
          t2 = HB_STATE_LEADER;
        } else {
          send = SEND_VOTES;
        }
      } else if (st == HB_STATE_LEADER) {
        if (type == HB_MSG_BEAT) {
          send = SEND_BEATS;                                     // bcastHeartbeat
        } else if (type == HB_MSG_PROP) {
          if (index == 0) fault(HB_FAULT_EMPTY_PROP);
          else {
            append_k = index;                                    // appendEntry + bcastAppend
            send = SEND_BCAST;
          }
        } else if (type == HB_MSG_APP_RESP || type == HB_MSG_HEARTBEAT_RESP || type == HB_MSG_SNAP_STATUS ||
                   type == HB_MSG_UNREACHABLE) {
          if (from >= nn) {
            fault(HB_FAULT_NIL_PROGRESS);                        // r.prs[m.From] == nil
          } else {
            Pr p = get(from);
            const uint32_t ps = pm_state(p.pm);
            if (type == HB_MSG_APP_RESP) {                       // :514-546
              if (reject) {
                if (maybe_decr_to(p, index, lasthint)) {
                  if (ps == HB_PR_REPLICATE) become_probe(from, p);
                  send = SEND_ONE;
                  send_to = from;
                }
              } else {
                old_paused = is_paused(p.pm);
                if (maybe_update(p, index)) {
                  if (ps == HB_PR_PROBE) {
                    become_replicate(p);
                  } else if (ps == HB_PR_SNAPSHOT) {
                    if (p.match >= S.pending[(size_t)from * S.G + g]) become_probe(from, p);  // maybeSnapshotAbort
                  } else {
                    free_to(from, p, index);
                  }
                  resolve_accept = true;
                }
              }
            } else if (type == HB_MSG_HEARTBEAT_RESP) {          // :547-554
              if (ps == HB_PR_REPLICATE && pm_count(p.pm) == S.W)
                free_to(from, p, p.head);                        // freeFirstOne
              if (p.match < last) {
                send = SEND_ONE;
                send_to = from;
              }
            } else if (type == HB_MSG_SNAP_STATUS) {             // :559-574
              if (ps == HB_PR_SNAPSHOT) {
                if (!reject) become_probe(from, p);
                else {                                           // snapshotFailure, becomeProbe
                  p.pm = pm_make(HB_PR_PROBE, 0, 0, 0);
                  p.next = p.match + 1;
                }
                p.pm |= PM_PAUSED;
              }
            } else {                                             // MsgUnreachable :575-581
              if (ps == HB_PR_REPLICATE) become_probe(from, p);
            }
            put(from, p);
          }
        }
      } else if (st == HB_STATE_CANDIDATE) {
        if (type == HB_MSG_PROP) {
          ev(HB_EV_PROP_DROP, 0, 0, arrival_x());                    // :587-589
        } else if (type == HB_MSG_VOTE_RESP) {                   // :603-612
          const uint32_t gr = poll(from < nn ? from : 7u, !reject);
          if (q == gr) {
            won++;
            t2 = HB_STATE_LEADER;
            send = SEND_BCAST;
          } else if (q == (uint32_t)__popc(m_resp(meta)) - gr) {
            lost++;
            t2 = HB_STATE_FOLLOWER;
          }
        }
      } else if (type == HB_MSG_PROP) {                          // stepFollower :618-624
        if (lead() == HB_REF_NONE) ev(HB_EV_PROP_DROP, 0, 0, arrival_x());
        else ev(HB_EV_PROP_FWD, lead(), 0, arrival_x());
      }
    }
    // ---- transition 2: becomeLeader (+ noop entry) or becomeFollower(Term, None)
    if (t2 != 0xFF && !faulted()) {
      if (transition(t2, term, HB_REF_NONE) && t2 == HB_STATE_LEADER) {
        append_k = 1;
        noop = 1;
      }
    }
    // ---- appendEntry raft/raft.go:351-360
    bool check_commit = resolve_accept;
    if (append_k && !faulted()) {
      const uint64_t old = last;
      if (sz_on(S.max_msg_size))  // the entries' sizes: noop, dense proposal, or MsgProp message
        sz_append(S, g, old, append_k, term, noop ? nullptr
                                                  : (arrival == 0xFFFFFFFFu ? S.edesc + S.peoff[g]
                                                                            : S.edesc + S.eoff[arrival]));
      last += append_k;
      if (tfirst == HB_NO_INDEX) tfirst = old + 1;
      tlast = last;
      dirty |= D_LAST | D_TRUN;
      ev(HB_EV_LAST, 0, noop, last);
      const uint32_t sf = self();
      if (sf == HB_SLOT_NONE) {
        fault(HB_FAULT_NO_SELF);
      } else {
        Pr p = get(sf);
        maybe_update(p, last);
        put(sf, p);
        check_commit = true;
      }
    }
    // ---- maybeCommit
    if (check_commit && !faulted()) {
      const bool c = maybe_commit();
      if (resolve_accept) {
        if (c) send = SEND_BCAST;
        else if (old_paused) {
          send = SEND_ONE;
          send_to = from;
        }
      }
    }
    // ---- sends: bcastAppend / sendAppend / MsgVote / bcastHeartbeat (slot order)
    if (send != SEND_NONE) {
      const uint32_t nn = n(), sf = self();
#pragma nounroll
      for (uint32_t s = 0; s < nn; ++s) {
        if (faulted()) break;
        if (send == SEND_ONE ? s != send_to : s == sf) continue;
        Pr p = get(s);
        if (send == SEND_VOTES) {
          ev(HB_EV_VOTE, s, 0, last);
          continue;
        }
        if (send == SEND_BEATS) {
          ev(HB_EV_HEARTBEAT, s, 0, umin64(p.match, committed));
          p.pm &= ~PM_PAUSED;
        } else {
          send_append(s, p);
        }
        put(s, p);
      }
    }
    if (faulted()) ev(HB_EV_FAULT, 0, faulted(), arrival_x());  // faulted groups are never stepped
  }
};

}  // namespace hb
