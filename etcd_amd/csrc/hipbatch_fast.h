// hipbatch_fast.h — the steady-state leader fast path of the apply phase.
//
// k_apply_fast steps, per group (one lane), exactly the two operations that
// make up steady-state replication (BASELINE.json cfg2):
//
//   * MsgProp on a leader whose own id is in prs
//       stepLeader raft/raft.go:500-513 -> appendEntry :351-360 ->
//       maybeCommit :323-332 -> bcastAppend :303-310
//   * MsgAppResp, Reject = false, from a member whose Progress is Replicate,
//     on a leader, m.Term == 0 or == Term (the Step gate raft/raft.go:462-490
//     passes without a transition)
//       stepLeader raft/raft.go:514-546 (maybeUpdate, freeTo, maybeCommit,
//       bcastAppend / sendAppend)
//
// Every other message (and everything after it for that group) is handed to
// k_apply<NMAX> (the general state machine in hipbatch_kernels.h) through a
// per-group resume word, so the two kernels together step every group's
// messages once, in arrival order.  FastLane is the specialization of
// Lane::step for these preconditions; the parity tests run both paths
// against the oracle.
//
// Why a separate lane type: the general pipeline is ~4k instructions of
// mostly-skipped branches and register-indexed slot access.  Here every slot
// access uses a compile-time slot index (runtime slots become predicated
// unrolled loops), so the hot lane is a few hundred instructions and needs
// few registers.
#pragma once

#include "hipbatch_kernels.h"

namespace hb {

template <int NMAX>
struct FastLane {
  DevState S;
  EvSink E;
  uint32_t g;
  uint32_t arrival;  // batch position of the message; 0xFFFFFFFF: props[] proposal
  uint64_t term, committed, first, last, tfirst, tlast;
  uint32_t mlo;      // meta bits [0, 32): state, n, self, lead, vote, fault
  uint64_t match[NMAX], next[NMAX], head[NMAX];
  uint32_t pm[NMAX];
  uint32_t dirty;
  uint32_t hv;       // bit s: head[s] holds inflights.buffer[start] of slot s (read lazily)
  // n = 7 keeps no head copies: the leader lane's 7 x 3 Progress words plus its
  // 8 route slots otherwise spill (132 B/lane); a head is then read when needed
  static constexpr bool HEADS = NMAX <= 5;
  uint32_t nev;      // public events emitted (an EVC_BCAST word counts once per slot)

  __device__ __forceinline__ uint32_t n() const { return (mlo >> 2) & 7; }
  __device__ __forceinline__ uint32_t state() const { return mlo & 3; }
  __device__ __forceinline__ uint32_t self() const { return (mlo >> 5) & 0xF; }
  __device__ __forceinline__ uint32_t faulted() const { return (mlo >> 17) & 0xF; }
  __device__ __forceinline__ uint64_t arrival_x() const {
    return arrival == 0xFFFFFFFFu ? HB_NO_INDEX : (uint64_t)arrival;
  }
  __device__ __forceinline__ void ev(uint32_t type, uint32_t to, uint32_t aux, uint64_t x) {
    emit_ev(E, g & (PART - 1), type, to, aux, x);
    nev++;
  }
  __device__ __forceinline__ void fault(uint32_t code) {
    if (faulted()) return;
    mlo = (mlo & ~(0xFu << 17)) | (code << 17);
    dirty |= D_META;
  }
  __device__ __forceinline__ uint64_t* ring_at(uint32_t s, uint32_t idx) const {
    return S.ring + ((size_t)s * S.W + idx) * S.G + g;
  }

  // All state loads of the lane are independent, so they are in flight together.
  __device__ __forceinline__ void load() {
    load_head();
    load_rest();
  }
  // The loads that depend on nothing the lane reads (k_apply_fast issues them
  // with meta itself, in its first round trip) ...
  __device__ __forceinline__ void load_head() {
    load_state_head();
    load_pm();
  }
  // (the per-group fields, which every role steps with, and the packed
  // Progress states, which only a leader reads)
  __device__ __forceinline__ void load_state_head() {
    term = at32(S.term, g);
    committed = at32(S.commit, g);
    first = at32(S.first, g);
    last = at32(S.last, g);
    tfirst = at32(S.tfirst, g);
  }
  __device__ __forceinline__ void load_pm() {
#pragma unroll
    for (int s = 0; s < NMAX; ++s) pm[s] = at32(S.pm, s * S.G + g);
  }
  // ... and those that wait for meta (which arrays are kept) and pm (the ring
  // heads): the second round trip.
  __device__ __forceinline__ void load_rest() {
    // arrays the meta flags mark as not kept are not read (M_TL / M_SM,
    // hipbatch_kernels.h); these loads issue once meta is in, beside the
    // ring heads, which wait for pm anyway
    tlast = (mlo & (uint32_t)M_TL) ? last : at32(S.tlast, g);
    const uint32_t sf = (mlo & (uint32_t)M_SM) ? self() : 0xFFu;
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      match[s] = ((uint32_t)s == sf) ? last : at32(S.match, s * S.G + g);
      next[s] = ((uint32_t)s == sf) ? last + 1 : at32(S.next, s * S.G + g);
    }
    if (mlo & (uint32_t)M_RS) {  // a group k_elect left in the reset form: every slot written back
      const uint32_t nn = n();
#pragma unroll
      for (int s = 0; s < NMAX; ++s) {
        if ((uint32_t)s < nn) {
          uint64_t mt, nx;
          uint32_t p;
          rs_progress(mlo, (uint32_t)s, last, tfirst, &mt, &nx, &p);
          match[s] = mt;
          next[s] = nx;
          pm[s] = p;
        }
      }
    }
    // The ring heads are loaded with the state (one more round trip, beside
    // nothing else); free_to reads one lazily if a lane has none.  (Loading
    // them only on demand — an ack at or past Next - 1 frees the whole window
    // unread — measured 1-3 % slower on cfg2 / cfg3 / cfg5.)
#pragma unroll
    for (int s = 0; s < NMAX; ++s) head[s] = (HEADS && pm_count(pm[s])) ? *ring_at(s, pm_start(pm[s])) : 0;
    hv = HEADS ? (1u << NMAX) - 1 : 0u;
    dirty = 0;
    if (mlo & (uint32_t)M_RS) {
      mlo &= ~(uint32_t)M_RS;
      dirty |= D_META;
#pragma unroll
      for (int s = 0; s < NMAX; ++s)
        if ((uint32_t)s < n()) dirty |= (1u << (D_SLOT0 + s)) | (1u << (D_PM0 + s));
    }
  }
  // Dirty bits (hipbatch_kernels.h) plus, lane-local to the fast path:
  // D_TFIRST (tfirst alone; D_TRUN then means tlast) and per-slot D_PM0 + s
  // (pm alone; D_SLOT0 + s then means match / next).
  static constexpr uint32_t D_TFIRST = 1u << 5;
  static constexpr uint32_t D_PM0 = 16;
  __device__ __forceinline__ void store() {
    // keep M_TL / M_SM only while they still hold; a cleared flag makes its
    // array live again, so it is written
    const bool tl = (mlo & (uint32_t)M_TL) && tlast == last;
    if ((mlo & (uint32_t)M_TL) && !tl) {
      mlo &= ~(uint32_t)M_TL;
      dirty |= D_META | D_TRUN;
    }
    uint32_t sf = 0xFFu;
    if (mlo & (uint32_t)M_SM) {
      const uint32_t s0 = self();
      bool ok = false;
#pragma unroll
      for (int s = 0; s < NMAX; ++s)
        if ((uint32_t)s == s0) ok = match[s] == last && next[s] == last + 1;
      if (ok) {
        sf = s0;
      } else {
        mlo &= ~(uint32_t)M_SM;
        dirty |= D_META | (1u << (D_SLOT0 + s0));
      }
    }
    if (dirty & D_META) at32(reinterpret_cast<uint32_t*>(S.meta), 2 * g) = mlo;  // little-endian low word
    if (dirty & D_COMMIT) at32(S.commit, g) = committed;
    if (dirty & D_LAST) at32(S.last, g) = last;
    if (dirty & D_TFIRST) at32(S.tfirst, g) = tfirst;
    if ((dirty & D_TRUN) && !tl) at32(S.tlast, g) = tlast;
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      if ((dirty & (1u << (D_SLOT0 + s))) && (uint32_t)s != sf) {
        at32(S.match, s * S.G + g) = match[s];
        at32(S.next, s * S.G + g) = next[s];
      }
      if (dirty & (1u << (D_PM0 + s))) at32(S.pm, s * S.G + g) = pm[s];
    }
  }
  __device__ __forceinline__ void set_pm(int s, uint32_t v) {
    if (v != pm[s]) dirty |= 1u << (D_PM0 + s);
    pm[s] = v;
  }

  // isPaused raft/progress.go:147-158
  __device__ __forceinline__ bool is_paused(uint32_t p) const {
    const uint32_t st = pm_state(p);
    if (st == HB_PR_PROBE) return pm_paused(p) != 0;
    if (st == HB_PR_REPLICATE) return pm_count(p) == S.W;
    return true;
  }
  // inflights.freeTo raft/progress.go:204-224 (s is a compile-time constant
  // after the callers' unrolled slot loops).  nx0 = Next before the ack: in
  // Replicate every entry is below Next (inflights.add of the last index sent,
  // then Next = that + 1, raft/raft.go:270-273; Next only grows until the
  // window is reset), so to >= nx0 - 1 pops the whole window without reading
  // it; otherwise the head entry comes from the register copy, read once.
  __device__ __forceinline__ void free_to(int s, uint64_t to, uint64_t nx0) {
    const uint32_t p = pm[s];
    const uint32_t cnt = pm_count(p);
    if (cnt == 0) return;
    uint32_t idx = pm_start(p);
    const uint32_t W = S.W;
    if (nx0 != 0 && to >= nx0 - 1) {
      idx += cnt;
      if (idx >= W) idx -= W;
      set_pm(s, pm_make(pm_state(p), pm_paused(p), idx, 0));
      return;
    }
    if (!((hv >> s) & 1u)) {
      head[s] = *ring_at(s, idx);
      hv |= 1u << s;
    }
    uint64_t v = head[s];
    if (to < v) return;
    uint32_t i = 0;
    while (true) {
      ++i;
      if (++idx >= W) idx -= W;
      if (i == cnt) break;
      v = *ring_at(s, idx);
      if (to < v) break;
    }
    set_pm(s, pm_make(pm_state(p), pm_paused(p), idx, cnt - i));
    head[s] = v;
  }
  // an HB_EV_APP's aux: the entry at x (the MsgApp's Index) has the current Term
  // (m.LogTerm == m.Term), so the host need not look it up
  __device__ __forceinline__ uint32_t lt_cur(uint64_t x) const { return (tfirst <= x && x <= tlast) ? 1u : 0u; }
  // raftLog.term(i) == Term over the current-term run (raft/log.go:198-217)
  __device__ __forceinline__ bool term_eq(uint64_t i) const {
    if (i + 1 < first || i > last) return term == 0;
    return tfirst <= i && i <= tlast;
  }
  // maybeCommit raft/raft.go:323-332 + raftLog.maybeCommit raft/log.go:241-247 +
  // commitTo :172-180.  The q-th largest Match by an odd-even transposition
  // network over the NMAX registers (absent slots read as 0).
  __device__ __forceinline__ bool maybe_commit() {
    uint64_t v[NMAX];
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
    uint64_t mci = v[0];
#pragma unroll
    for (int s = 1; s < NMAX; ++s) mci = ((uint32_t)s == nn / 2) ? v[s] : mci;  // q-1, q = n/2+1
    if (mci > committed && term_eq(mci)) {
      if (last < mci) {
        fault(HB_FAULT_COMMIT_RANGE);
        return false;
      }
      committed = mci;
      dirty |= D_COMMIT;
      ev(HB_EV_COMMIT, 0, 0, mci);
      return true;
    }
    return false;
  }
  // sendAppend raft/raft.go:239-282 to slot s: the progress side effects;
  // returns the message it sends (SEND_NONE / SEND_APP / SEND_SNAP, index *x)
  // for the caller to emit.
  enum : uint32_t { SEND_NONE = 0, SEND_APP = 1, SEND_SNAP = 2 };
  __device__ __forceinline__ uint32_t send_decide(int s, uint64_t* xo) {
    const uint32_t p = pm[s];
    if (is_paused(p)) return SEND_NONE;
    if (next[s] < first) {  // needSnapshot raft/raft.go:715-717
      const uint64_t snapi = S.snap[g];
      if (snapi == 0) {
        fault(HB_FAULT_EMPTY_SNAPSHOT);
        return SEND_NONE;
      }
      set_pm(s, pm_make(HB_PR_SNAPSHOT, 0, 0, 0));  // becomeSnapshot
      S.pending[(size_t)s * S.G + g] = snapi;
      *xo = snapi;
      return SEND_SNAP;
    }
    const uint64_t x = next[s] - 1;
    if (next[s] <= last) {
      bool ok = true;
      const uint64_t lastsent = sz_limit(S, g, next[s], last, &ok);
      if (!ok) {
        fault(HB_FAULT_SIZE_WINDOW);
        return SEND_NONE;
      }
      const uint32_t st = pm_state(p);
      if (st == HB_PR_REPLICATE) {
        const uint32_t cnt = pm_count(p), start = pm_start(p);
        if (cnt == S.W) {
          fault(HB_FAULT_INFLIGHTS_FULL);
          return SEND_NONE;
        }
        uint32_t idx = start + cnt;
        if (idx >= S.W) idx -= S.W;
        *ring_at(s, idx) = lastsent;              // inflights.add
        if (cnt == 0) {
          head[s] = lastsent;
          hv |= 1u << s;
        }
        next[s] = lastsent + 1;                   // optimisticUpdate
        dirty |= 1u << (D_SLOT0 + s);
        set_pm(s, pm_make(HB_PR_REPLICATE, pm_paused(p), start, cnt + 1));
      } else if (st == HB_PR_PROBE) {
        set_pm(s, p | PM_PAUSED);                 // pause
      }
    }
    *xo = x;
    return SEND_APP;
  }
  __device__ __forceinline__ void send_append(int s) {
    uint64_t x = 0;
    const uint32_t k = send_decide(s, &x);
    if (k != SEND_NONE) ev(k == SEND_APP ? HB_EV_APP : HB_EV_SNAP, s, k == SEND_APP ? lt_cur(x) : 0u, x);
  }
  // bcastAppend raft/raft.go:303-310 (slot order, self skipped).  When every
  // message it sends is a MsgApp with the same Index (steady state), the sends
  // are recorded as one EVC_BCAST word; otherwise one event per send, in slot
  // order.  Nothing else is emitted between the sends, so the order holds.
  __device__ __forceinline__ void bcast_append() {
    const uint32_t nn = n(), sf = self();
    uint32_t kind[NMAX];
    uint64_t xs[NMAX];
    uint32_t mask = 0;
    uint64_t x0 = 0;
    bool same = true;
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      kind[s] = SEND_NONE;
      xs[s] = 0;
      if ((uint32_t)s < nn && (uint32_t)s != sf && !faulted()) kind[s] = send_decide(s, &xs[s]);
      if (kind[s] != SEND_NONE) {
        if (mask == 0) x0 = xs[s];
        same = same && kind[s] == SEND_APP && xs[s] == x0;
        mask |= 1u << s;
      }
    }
    if (mask == 0) return;
    if (same && (mask & (mask - 1))) {
      emit_ev(E, g & (PART - 1), EVC_BCAST, mask, lt_cur(x0), x0);
      nev += __popc(mask);
      return;
    }
#pragma unroll
    for (int s = 0; s < NMAX; ++s)
      if (kind[s] != SEND_NONE)
        ev(kind[s] == SEND_APP ? HB_EV_APP : HB_EV_SNAP, s, kind[s] == SEND_APP ? lt_cur(xs[s]) : 0u, xs[s]);
  }

  // ---- preconditions (checked per message by the kernel)
  __device__ __forceinline__ bool prop_ok(uint32_t k) const {
    return k != 0 && state() == HB_STATE_LEADER && self() != HB_SLOT_NONE;
  }
  __device__ __forceinline__ bool accept_ok(uint32_t type, uint32_t from, uint64_t mterm, bool reject) const {
    bool rep = false;
#pragma unroll
    for (int s = 0; s < NMAX; ++s) rep = ((uint32_t)s == from) ? (pm_state(pm[s]) == HB_PR_REPLICATE) : rep;
    return type == HB_MSG_APP_RESP && !reject && state() == HB_STATE_LEADER && (mterm == 0 || mterm == term) &&
           from < n() && rep;
  }

  // ---- MsgProp with k entries on a leader (prop_ok)
  __device__ __forceinline__ void prop(uint32_t k) {
    const uint64_t old = last;
    if (sz_on(S.max_msg_size))  // the entries' descriptors: the dense proposal's, or the MsgProp message's
      sz_append(S, g, old, k, term, S.edesc + (arrival == 0xFFFFFFFFu ? S.peoff[g] : S.eoff[arrival]));
    last += k;
    if (tfirst == HB_NO_INDEX) {
      tfirst = old + 1;
      dirty |= D_TFIRST;
    }
    tlast = last;
    dirty |= D_LAST | D_TRUN;
    ev(HB_EV_LAST, 0, 0, last);
    const uint32_t sf = self();
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      if ((uint32_t)s == sf) {  // self maybeUpdate(lastIndex) raft/raft.go:358
        if (match[s] < last) {
          match[s] = last;
          set_pm(s, pm[s] & ~PM_PAUSED);
        }
        if (next[s] < last + 1) next[s] = last + 1;
        dirty |= 1u << (D_SLOT0 + s);
      }
    }
    maybe_commit();
    bcast_append();
    if (faulted()) ev(HB_EV_FAULT, 0, faulted(), arrival_x());
  }

  // ---- accepted MsgAppResp from a Replicate member (accept_ok)
  __device__ __forceinline__ void accept(uint32_t from, uint64_t index) {
    bool updated = false, old_paused = false;
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      if ((uint32_t)s == from) {
        old_paused = pm_count(pm[s]) == S.W;      // isPaused() in Replicate, before maybeUpdate
        const uint64_t nx0 = next[s];
        if (next[s] < index + 1) next[s] = index + 1;
        if (match[s] < index) {                   // maybeUpdate raft/progress.go:102-113
          match[s] = index;
          set_pm(s, pm[s] & ~PM_PAUSED);
          updated = true;
          free_to(s, index, nx0);                 // Replicate: ins.freeTo(m.Index)
        }
        dirty |= 1u << (D_SLOT0 + s);
      }
    }
    if (!updated) return;
    if (maybe_commit()) {
      bcast_append();
    } else if (old_paused && !faulted()) {
#pragma unroll
      for (int s = 0; s < NMAX; ++s)
        if ((uint32_t)s == from) send_append(s);
    }
    if (faulted()) ev(HB_EV_FAULT, 0, faulted(), arrival_x());
  }
};

}  // namespace hb
