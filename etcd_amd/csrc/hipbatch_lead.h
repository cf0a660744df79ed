// hipbatch_lead.h — the leader lane: Lane::step (hipbatch_kernels.h)
// restricted to what a leader steps at its own term, with its Progress in
// registers.  It runs in k_apply_lead, the n >= 5 apply kernel.
//
// FastLane (k_apply_fast, n = 3) takes only proposals and accepted MsgAppResp
// from Replicate followers; any other response on a leader would hand the group
// to the general kernel, which carries every role and message type and needs
// all 256 VGPRs plus scratch.  On BASELINE.json cfg3 (1M groups x 5, lagging
// followers) that is most groups: rejected MsgAppResp (maybeDecrTo +
// becomeProbe + sendAppend), accepts from Probe / Snapshot followers
// (becomeReplicate, maybeSnapshotAbort), stale and lagging acks that pause or
// unpause a full window, MsgHeartbeatResp (freeFirstOne + sendAppend),
// MsgUnreachable and MsgSnapStatus.  LeadLane is FastLane (its loads and
// store, maybeCommit network, limitSize) plus exactly those transitions, with
// one code path for every slot: the sender's Progress is selected into
// scalars, stepped once and put back, and bcastAppend is a rolled loop whose
// consecutive equal-Index MsgApps become one EVC_BCAST word.
//
// It steps a message when the group is a leader, the sender is a member and
// the message's term is not higher than the group's (stepLeader
// raft/raft.go:514-583; a lower non-zero term is ignored by the gate, :479-486).
// Anything else — a higher term (step-down), MsgProp messages, MsgHup /
// MsgBeat, follower-side types, a non-member MsgSnapStatus — hands the group
// over, at that message, to k_elect / k_apply.  Every event and state write is
// the one Lane::step makes, in the same order; the GPU parity tests compare
// the kernels with the oracle.
#pragma once

#include "hipbatch_fast.h"

namespace hb {

template <int NMAX>
struct LeadLane : FastLane<NMAX> {
  using B = FastLane<NMAX>;
  using B::S;
  using B::g;
  using B::term;
  using B::first;
  using B::last;
  using B::match;
  using B::next;
  using B::head;
  using B::pm;
  using B::dirty;
  using B::faulted;

  // Whether this lane steps the message (false: hand the group over here).
  // The caller has dropped non-member responses (raft/multinode.go:235).
  __device__ __forceinline__ bool takes(uint32_t type, uint32_t from, uint64_t mterm) const {
    if (this->state() != HB_STATE_LEADER || from >= this->n() || mterm > term) return false;
    return type == HB_MSG_APP_RESP || type == HB_MSG_HEARTBEAT_RESP || type == HB_MSG_UNREACHABLE ||
           type == HB_MSG_SNAP_STATUS || type == HB_MSG_VOTE_RESP;
  }
  // head: the per-group fields were loaded already (load_state_head)
  __device__ __forceinline__ void load(bool head = false) {
    if (!head) B::load_state_head();
    B::load_pm();
    B::load_rest();
  }

  // One slot's Progress as scalars (a runtime slot: one select per slot and
  // field, so the transitions below exist once in the code, not once per slot).
  __device__ __forceinline__ Pr get(uint32_t s) const {
    Pr p{match[0], next[0], B::HEADS ? head[0] : 0ull, pm[0]};
#pragma unroll
    for (int k = 1; k < NMAX; ++k) {
      const bool h = (uint32_t)k == s;
      p.match = h ? match[k] : p.match;
      p.next = h ? next[k] : p.next;
      if (B::HEADS) p.head = h ? head[k] : p.head;
      p.pm = h ? pm[k] : p.pm;
    }
    return p;
  }
  __device__ __forceinline__ void put(uint32_t s, const Pr& p) {
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {
      const bool h = (uint32_t)k == s;
      if (h && (p.match != match[k] || p.next != next[k])) dirty |= 1u << (D_SLOT0 + k);
      if (h && p.pm != pm[k]) dirty |= 1u << (B::D_PM0 + k);
      match[k] = h ? p.match : match[k];
      next[k] = h ? p.next : next[k];
      if (B::HEADS) head[k] = h ? p.head : head[k];
      pm[k] = h ? p.pm : pm[k];
    }
  }
  __device__ __forceinline__ uint64_t pending_of(uint32_t s) const { return S.pending[(size_t)s * S.G + g]; }
  __device__ __forceinline__ uint64_t* ring_at(uint32_t s, uint32_t idx) const {
    return S.ring + ((size_t)s * S.W + idx) * S.G + g;
  }

  // inflights.freeTo raft/progress.go:204-224; nx0 = Next before the ack
  // (FastLane::free_to: to >= nx0 - 1 pops the whole window unread; else the
  // head entry is read once into the register copy)
  __device__ __forceinline__ void free_to(uint32_t s, Pr& p, uint64_t to, uint64_t nx0) {
    const uint32_t cnt = pm_count(p.pm);
    if (cnt == 0) return;
    uint32_t idx = pm_start(p.pm);
    const uint32_t W = S.W;
    if (nx0 != 0 && to >= nx0 - 1) {
      idx += cnt;
      if (idx >= W) idx -= W;
      p.pm = pm_make(pm_state(p.pm), pm_paused(p.pm), idx, 0);
      return;
    }
    if (!((this->hv >> s) & 1u)) {
      p.head = *ring_at(s, idx);
      if (B::HEADS) this->hv |= 1u << s;
    }
    uint64_t v = p.head;
    if (to < v) return;
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

  // sendAppend raft/raft.go:239-282 to slot s: the progress side effects;
  // returns what it sends (FastLane::SEND_*), its index in *xo.
  __device__ __forceinline__ uint32_t send_decide(uint32_t s, Pr& p, uint64_t* xo) {
    if (B::is_paused(p.pm)) return B::SEND_NONE;
    if (p.next < first) {  // needSnapshot raft/raft.go:715-717
      const uint64_t snapi = S.snap[g];
      if (snapi == 0) {
        this->fault(HB_FAULT_EMPTY_SNAPSHOT);
        return B::SEND_NONE;
      }
      p.pm = pm_make(HB_PR_SNAPSHOT, 0, 0, 0);  // becomeSnapshot
      S.pending[(size_t)s * S.G + g] = snapi;
      *xo = snapi;
      return B::SEND_SNAP;
    }
    const uint64_t x = p.next - 1;
    if (p.next <= last) {
      bool ok = true;
      const uint64_t lastsent = sz_limit(S, g, p.next, last, &ok);
      if (!ok) {
        this->fault(HB_FAULT_SIZE_WINDOW);
        return B::SEND_NONE;
      }
      const uint32_t st = pm_state(p.pm);
      if (st == HB_PR_REPLICATE) {
        const uint32_t cnt = pm_count(p.pm), start = pm_start(p.pm);
        if (cnt == S.W) {
          this->fault(HB_FAULT_INFLIGHTS_FULL);
          return B::SEND_NONE;
        }
        uint32_t idx = start + cnt;
        if (idx >= S.W) idx -= S.W;
        *ring_at(s, idx) = lastsent;  // inflights.add
        if (cnt == 0 && B::HEADS) {
          p.head = lastsent;
          this->hv |= 1u << s;
        }
        p.next = lastsent + 1;        // optimisticUpdate
        p.pm = pm_make(HB_PR_REPLICATE, pm_paused(p.pm), start, cnt + 1);
      } else if (st == HB_PR_PROBE) {
        p.pm |= PM_PAUSED;            // pause
      }
    }
    *xo = x;
    return B::SEND_APP;
  }

  // The sends of a bcastAppend (raft/raft.go:303-310, slot order, self
  // skipped) or of one sendAppend, as runs: consecutive MsgApps with the same
  // Index become one EVC_BCAST word (the same records once expanded).
  uint32_t run_mask;
  uint64_t run_x;
  __device__ __forceinline__ void run_flush() {
    if (run_mask & (run_mask - 1)) {
      emit_ev(this->E, g & (PART - 1), EVC_BCAST, run_mask, this->lt_cur(run_x), run_x);
      this->nev += __popc(run_mask);
    } else if (run_mask) {
      this->ev(HB_EV_APP, __ffs(run_mask) - 1, this->lt_cur(run_x), run_x);
    }
    run_mask = 0;
  }
  __device__ __forceinline__ void send(uint32_t s) {
    Pr p = get(s);
    uint64_t x = 0;
    const uint32_t k = send_decide(s, p, &x);
    put(s, p);
    if (k == B::SEND_APP) {
      if (run_mask && x != run_x) run_flush();
      run_mask |= 1u << s;
      run_x = x;
    } else if (k == B::SEND_SNAP) {
      run_flush();
      this->ev(HB_EV_SNAP, s, 0, x);
    }
  }
  __device__ __forceinline__ void bcast() {
    const uint32_t nn = this->n(), sf = this->self();
    run_mask = 0;
    // (rolled: unrolling the sends at compile-time slots measured cfg3 -1.3 %,
    // cfg4 neutral, at 20 / 52 B of scratch for n = 5 / 7 — not kept)
#pragma nounroll
    for (uint32_t s = 0; s < nn; ++s) {
      if (faulted()) break;
      if (s != sf) send(s);
    }
    run_flush();
  }

  // MsgProp with k entries on a leader (FastLane::prop with the rolled
  // bcastAppend): stepLeader raft/raft.go:500-513 -> appendEntry :351-360 ->
  // maybeCommit :323-332 -> bcastAppend :303-310
  __device__ __forceinline__ void prop(uint32_t k) {
    const uint64_t old = last;
    if (sz_on(S.max_msg_size)) sz_append(S, g, old, k, term, S.edesc + S.peoff[g]);  // dense proposal entries
    last += k;
    if (this->tfirst == HB_NO_INDEX) {
      this->tfirst = old + 1;
      dirty |= B::D_TFIRST;
    }
    this->tlast = last;
    dirty |= D_LAST | D_TRUN;
    this->ev(HB_EV_LAST, 0, 0, last);
    const uint32_t sf = this->self();  // self maybeUpdate(lastIndex) raft/raft.go:358
    Pr p = get(sf);
    if (p.match < last) {
      p.match = last;
      p.pm &= ~PM_PAUSED;
    }
    if (p.next < last + 1) p.next = last + 1;
    put(sf, p);
    this->maybe_commit();
    bcast();
    if (faulted()) this->ev(HB_EV_FAULT, 0, faulted(), this->arrival_x());
  }

  // stepLeader (raft/raft.go:514-583) for the messages takes() accepts.
  __device__ __forceinline__ void step(uint32_t type, uint32_t from, uint64_t mterm, uint64_t index, bool reject,
                                       uint64_t hint) {
    if (mterm != 0 && mterm < term) return;  // the gate ignores a lower term (:483-486)
    bool updated = false, old_paused = false, send_one = false;
    Pr p = get(from);
    const uint32_t ps = pm_state(p.pm);
    if (type == HB_MSG_APP_RESP) {  // :514-546
      if (reject) {
        bool dec = false;  // maybeDecrTo raft/progress.go:119-141
        if (ps == HB_PR_REPLICATE) {
          if (index > p.match) {
            p.next = p.match + 1;
            dec = true;
          }
        } else if (p.next - 1 == index) {
          p.next = umin64(index, hint + 1);
          if (p.next < 1) p.next = 1;
          p.pm &= ~PM_PAUSED;
          dec = true;
        }
        if (dec && ps == HB_PR_REPLICATE) {  // becomeProbe from Replicate raft/progress.go:76-88
          p.pm = pm_make(HB_PR_PROBE, 0, 0, 0);
          p.next = p.match + 1;
        }
        send_one = dec;
      } else {
        old_paused = B::is_paused(p.pm);
        const uint64_t nx0 = p.next;
        if (p.match < index) {  // maybeUpdate raft/progress.go:102-113
          p.match = index;
          p.pm &= ~PM_PAUSED;
          updated = true;
        }
        if (p.next < index + 1) p.next = index + 1;
        if (updated) {
          if (ps == HB_PR_PROBE) {  // becomeReplicate :90-93
            p.pm = pm_make(HB_PR_REPLICATE, 0, 0, 0);
            p.next = p.match + 1;
          } else if (ps == HB_PR_SNAPSHOT) {  // maybeSnapshotAbort -> becomeProbe
            const uint64_t pend = pending_of(from);
            if (p.match >= pend) {
              p.pm = pm_make(HB_PR_PROBE, 0, 0, 0);
              p.next = umax64(p.match + 1, pend + 1);
            }
          } else {  // ins.freeTo(m.Index)
            free_to(from, p, index, nx0);
          }
        }
      }
    } else if (type == HB_MSG_HEARTBEAT_RESP) {  // :547-554
      if (ps == HB_PR_REPLICATE && pm_count(p.pm) == S.W) {  // freeFirstOne: entries increase, so one pops
        uint32_t idx = pm_start(p.pm) + 1;
        if (idx >= S.W) idx -= S.W;
        p.pm = pm_make(HB_PR_REPLICATE, pm_paused(p.pm), idx, S.W - 1);
        this->hv &= ~(1u << from);
      }
      send_one = p.match < last;
    } else if (type == HB_MSG_SNAP_STATUS) {  // :559-574
      if (ps == HB_PR_SNAPSHOT) {
        p.next = reject ? p.match + 1                                 // snapshotFailure, becomeProbe
                        : umax64(p.match + 1, pending_of(from) + 1);  // becomeProbe from Snapshot
        p.pm = pm_make(HB_PR_PROBE, 1, 0, 0);                         // ... and pause
      }
    } else if (type == HB_MSG_UNREACHABLE) {  // :575-581
      if (ps == HB_PR_REPLICATE) {
        p.pm = pm_make(HB_PR_PROBE, 0, 0, 0);
        p.next = p.match + 1;
      }
    }  // MsgVoteResp: a leader ignores it
    put(from, p);
    if (updated) {  // maybeCommit -> bcastAppend, else a paused follower gets sendAppend
      if (this->maybe_commit()) bcast();
      else if (old_paused) send_one = true;
    }
    if (send_one && !faulted()) {
      run_mask = 0;
      send(from);
      run_flush();
    }
    if (faulted()) this->ev(HB_EV_FAULT, 0, faulted(), this->arrival_x());
  }
};

}  // namespace hb

namespace hb {

// LeadLaneL: LeadLane with each lane's Match / Next in LDS ([slot][lane],
// 16 bytes per slot) instead of registers.  A runtime slot (the sender of a
// response, a bcastAppend's peer) is then one indexed LDS access instead of
// an NMAX-way select per field — on cfg3 (1M x 5) the register lane spent
// most of its VALU issue on those selects under divergence (accept / lag /
// reject / heartbeat lanes in one wave).  The packed Progress
// states stay in registers (32-bit selects are cheap); the inflight ring
// heads are not cached (a partial freeTo reads its head from the ring).
// Same transitions, events and state writes as LeadLane, line for line.
template <int NMAX>
struct LeadLaneL : FastLane<NMAX> {
  using B = FastLane<NMAX>;
  using B::S;
  using B::g;
  using B::term;
  using B::first;
  using B::last;
  using B::dirty;
  using B::faulted;
  // this lane's {Match, Next} of slot s at lp[s * PART] (LDS, one 16-byte word:
  // lanes of a wave are adjacent, a get is one ds_read_b128)
  uint4* lp;
  // the packed Progress states as a vector (a runtime slot is a register-indexed
  // extract; an array indexed through selects is folded into a private-memory
  // access, which put the whole lane in scratch)
  typename SlotVec<NMAX>::u32 pm;

  __device__ __forceinline__ uint64_t mt(uint32_t s) const {
    const uint4 w = lp[s * PART];
    return (uint64_t)w.x | ((uint64_t)w.y << 32);
  }
  __device__ __forceinline__ uint64_t nx(uint32_t s) const {
    const uint4 w = lp[s * PART];
    return (uint64_t)w.z | ((uint64_t)w.w << 32);
  }
  __device__ __forceinline__ void set_mn(uint32_t s, uint64_t m, uint64_t x) {
    lp[s * PART] = make_uint4((uint32_t)m, (uint32_t)(m >> 32), (uint32_t)x, (uint32_t)(x >> 32));
  }

  __device__ __forceinline__ bool takes(uint32_t type, uint32_t from, uint64_t mterm) const {
    if (this->state() != HB_STATE_LEADER || from >= this->n() || mterm > term) return false;
    return type == HB_MSG_APP_RESP || type == HB_MSG_HEARTBEAT_RESP || type == HB_MSG_UNREACHABLE ||
           type == HB_MSG_SNAP_STATUS || type == HB_MSG_VOTE_RESP;
  }

  // FastLane::load_rest with Match / Next into LDS (ring heads not cached);
  // head: the per-group fields were loaded already (load_state_head)
  __device__ __forceinline__ void load(bool head = false) {
    if (!head) B::load_state_head();
    B::load_pm();
#pragma unroll
    for (int s = 0; s < NMAX; ++s) pm[s] = B::pm[s];
    this->tlast = (this->mlo & (uint32_t)M_TL) ? last : at32(S.tlast, g);
    const uint32_t sf = (this->mlo & (uint32_t)M_SM) ? this->self() : 0xFFu;
    uint64_t m[NMAX], x[NMAX];
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      m[s] = ((uint32_t)s == sf) ? last : at32(S.match, s * S.G + g);
      x[s] = ((uint32_t)s == sf) ? last + 1 : at32(S.next, s * S.G + g);
    }
    dirty = 0;
    if (this->mlo & (uint32_t)M_RS) {  // a group k_elect left in the reset form: every slot written back
      const uint32_t nn = this->n();
#pragma unroll
      for (int s = 0; s < NMAX; ++s) {
        if ((uint32_t)s < nn) {
          uint32_t p;
          rs_progress(this->mlo, (uint32_t)s, last, this->tfirst, &m[s], &x[s], &p);
          pm[s] = p;
          dirty |= (1u << (D_SLOT0 + s)) | (1u << (B::D_PM0 + s));
        }
      }
      this->mlo &= ~(uint32_t)M_RS;
      dirty |= D_META;
    }
#pragma unroll
    for (int s = 0; s < NMAX; ++s) set_mn((uint32_t)s, m[s], x[s]);
    this->hv = 0;
  }
  // FastLane::store reading Match / Next from LDS
  __device__ __forceinline__ void store() {
    const bool tl = (this->mlo & (uint32_t)M_TL) && this->tlast == last;
    if ((this->mlo & (uint32_t)M_TL) && !tl) {
      this->mlo &= ~(uint32_t)M_TL;
      dirty |= D_META | D_TRUN;
    }
    uint32_t sf = 0xFFu;
    if (this->mlo & (uint32_t)M_SM) {
      const uint32_t s0 = this->self();
      if (mt(s0) == last && nx(s0) == last + 1) {
        sf = s0;
      } else {
        this->mlo &= ~(uint32_t)M_SM;
        dirty |= D_META | (1u << (D_SLOT0 + s0));
      }
    }
    if (dirty & D_META) at32(reinterpret_cast<uint32_t*>(S.meta), 2 * g) = this->mlo;  // little-endian low word
    if (dirty & D_COMMIT) at32(S.commit, g) = this->committed;
    if (dirty & D_LAST) at32(S.last, g) = last;
    if (dirty & B::D_TFIRST) at32(S.tfirst, g) = this->tfirst;
    if ((dirty & D_TRUN) && !tl) at32(S.tlast, g) = this->tlast;
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      if ((dirty & (1u << (D_SLOT0 + s))) && (uint32_t)s != sf) {
        const uint4 w = lp[s * PART];
        at32(S.match, s * S.G + g) = (uint64_t)w.x | ((uint64_t)w.y << 32);
        at32(S.next, s * S.G + g) = (uint64_t)w.z | ((uint64_t)w.w << 32);
      }
      if (dirty & (1u << (B::D_PM0 + s))) at32(S.pm, s * S.G + g) = pm[s];
    }
  }

  // maybeCommit raft/raft.go:323-332 + raftLog.maybeCommit raft/log.go:241-247 +
  // commitTo :172-180 (FastLane::maybe_commit over the LDS Match)
  __device__ __forceinline__ bool maybe_commit() {
    uint64_t v[NMAX];
    const uint32_t nn = this->n();
#pragma unroll
    for (int s = 0; s < NMAX; ++s) v[s] = ((uint32_t)s < nn) ? mt(s) : 0;
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
    if (mci > this->committed && this->term_eq(mci)) {
      if (last < mci) {
        this->fault(HB_FAULT_COMMIT_RANGE);
        return false;
      }
      this->committed = mci;
      dirty |= D_COMMIT;
      this->ev(HB_EV_COMMIT, 0, 0, mci);
      return true;
    }
    return false;
  }

  // The Progress of slot s: Match / Next from LDS, the state word by select
  __device__ __forceinline__ Pr get(uint32_t s) const {
    const uint4 w = lp[s * PART];
    return Pr{(uint64_t)w.x | ((uint64_t)w.y << 32), (uint64_t)w.z | ((uint64_t)w.w << 32), 0ull, pm[s]};
  }
  // write back what changed against p0 (the value get() returned)
  __device__ __forceinline__ void put(uint32_t s, const Pr& p, const Pr& p0) {
    if (p.match != p0.match || p.next != p0.next) {
      set_mn(s, p.match, p.next);
      dirty |= 1u << (D_SLOT0 + s);
    }
    if (p.pm != p0.pm) {
      dirty |= 1u << (B::D_PM0 + s);
      pm[s] = p.pm;
    }
  }
  __device__ __forceinline__ uint64_t pending_of(uint32_t s) const { return S.pending[(size_t)s * S.G + g]; }
  __device__ __forceinline__ uint64_t* ring_at(uint32_t s, uint32_t idx) const {
    return S.ring + ((size_t)s * S.W + idx) * S.G + g;
  }

  // inflights.freeTo raft/progress.go:204-224; nx0 = Next before the ack
  // (to >= nx0 - 1 pops the whole window unread; else the entries are read
  // from the ring, head first)
  __device__ __forceinline__ void free_to(uint32_t s, Pr& p, uint64_t to, uint64_t nx0) const {
    const uint32_t cnt = pm_count(p.pm);
    if (cnt == 0) return;
    uint32_t idx = pm_start(p.pm);
    const uint32_t W = S.W;
    if (nx0 != 0 && to >= nx0 - 1) {
      idx += cnt;
      if (idx >= W) idx -= W;
      p.pm = pm_make(pm_state(p.pm), pm_paused(p.pm), idx, 0);
      return;
    }
    uint64_t v = *ring_at(s, idx);
    if (to < v) return;
    uint32_t i = 0;
    while (true) {
      ++i;
      if (++idx >= W) idx -= W;
      if (i == cnt) break;
      v = *ring_at(s, idx);
      if (to < v) break;
    }
    p.pm = pm_make(pm_state(p.pm), pm_paused(p.pm), idx, cnt - i);
  }

  // sendAppend raft/raft.go:239-282 to slot s: the progress side effects;
  // returns what it sends (FastLane::SEND_*), its index in *xo.
  __device__ __forceinline__ uint32_t send_decide(uint32_t s, Pr& p, uint64_t* xo) {
    if (B::is_paused(p.pm)) return B::SEND_NONE;
    if (p.next < first) {  // needSnapshot raft/raft.go:715-717
      const uint64_t snapi = S.snap[g];
      if (snapi == 0) {
        this->fault(HB_FAULT_EMPTY_SNAPSHOT);
        return B::SEND_NONE;
      }
      p.pm = pm_make(HB_PR_SNAPSHOT, 0, 0, 0);  // becomeSnapshot
      S.pending[(size_t)s * S.G + g] = snapi;
      *xo = snapi;
      return B::SEND_SNAP;
    }
    const uint64_t x = p.next - 1;
    if (p.next <= last) {
      bool ok = true;
      const uint64_t lastsent = sz_limit(S, g, p.next, last, &ok);
      if (!ok) {
        this->fault(HB_FAULT_SIZE_WINDOW);
        return B::SEND_NONE;
      }
      const uint32_t st = pm_state(p.pm);
      if (st == HB_PR_REPLICATE) {
        const uint32_t cnt = pm_count(p.pm), start = pm_start(p.pm);
        if (cnt == S.W) {
          this->fault(HB_FAULT_INFLIGHTS_FULL);
          return B::SEND_NONE;
        }
        uint32_t idx = start + cnt;
        if (idx >= S.W) idx -= S.W;
        *ring_at(s, idx) = lastsent;  // inflights.add
        p.next = lastsent + 1;        // optimisticUpdate
        p.pm = pm_make(HB_PR_REPLICATE, pm_paused(p.pm), start, cnt + 1);
      } else if (st == HB_PR_PROBE) {
        p.pm |= PM_PAUSED;            // pause
      }
    }
    *xo = x;
    return B::SEND_APP;
  }

  // The sends of a bcastAppend (raft/raft.go:303-310, slot order, self
  // skipped) or of one sendAppend, as runs: consecutive MsgApps with the same
  // Index become one EVC_BCAST word (the same records once expanded).
  uint32_t run_mask;
  uint64_t run_x;
  __device__ __forceinline__ void run_flush() {
    if (run_mask & (run_mask - 1)) {
      emit_ev(this->E, g & (PART - 1), EVC_BCAST, run_mask, this->lt_cur(run_x), run_x);
      this->nev += __popc(run_mask);
    } else if (run_mask) {
      this->ev(HB_EV_APP, __ffs(run_mask) - 1, this->lt_cur(run_x), run_x);
    }
    run_mask = 0;
  }
  __device__ __forceinline__ void send(uint32_t s) {
    Pr p = get(s);
    const Pr p0 = p;
    uint64_t x = 0;
    const uint32_t k = send_decide(s, p, &x);
    put(s, p, p0);
    if (k == B::SEND_APP) {
      if (run_mask && x != run_x) run_flush();
      run_mask |= 1u << s;
      run_x = x;
    } else if (k == B::SEND_SNAP) {
      run_flush();
      this->ev(HB_EV_SNAP, s, 0, x);
    }
  }
  // The sends to the slots of `mask` in slot order — bcastAppend (every peer
  // but self) or one sendAppend — at compile-time slots: every decision first
  // (each slot's {Match, Next} at a constant LDS offset, its state word a
  // constant register), then the events in slot order (a send emits nothing
  // itself, so deferring them keeps the order).  A fault stops the slots after
  // it, as the rolled loop did.
  __device__ __forceinline__ void sends(uint32_t mask) {
    uint32_t kind[NMAX];
    uint64_t xs[NMAX];
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      kind[s] = B::SEND_NONE;
      xs[s] = 0;
      if (((mask >> s) & 1u) && !faulted()) {
        Pr p = get((uint32_t)s);
        const Pr p0 = p;
        kind[s] = send_decide((uint32_t)s, p, &xs[s]);
        put((uint32_t)s, p, p0);
      }
    }
    run_mask = 0;
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      if (kind[s] == B::SEND_APP) {
        if (run_mask && xs[s] != run_x) run_flush();
        run_mask |= 1u << s;
        run_x = xs[s];
      } else if (kind[s] == B::SEND_SNAP) {
        run_flush();
        this->ev(HB_EV_SNAP, s, 0, xs[s]);
      }
    }
    run_flush();
  }
  __device__ __forceinline__ void bcast() {
    const uint32_t nn = this->n(), sf = this->self();
    sends(((1u << nn) - 1) & ~(1u << sf));
  }

  // MsgProp with k entries on a leader: stepLeader raft/raft.go:500-513 ->
  // appendEntry :351-360 -> maybeCommit :323-332 -> bcastAppend :303-310
  __device__ __forceinline__ void prop(uint32_t k) {
    const uint64_t old = last;
    if (sz_on(S.max_msg_size)) sz_append(S, g, old, k, term, S.edesc + S.peoff[g]);  // dense proposal entries
    last += k;
    if (this->tfirst == HB_NO_INDEX) {
      this->tfirst = old + 1;
      dirty |= B::D_TFIRST;
    }
    this->tlast = last;
    dirty |= D_LAST | D_TRUN;
    this->ev(HB_EV_LAST, 0, 0, last);
    const uint32_t sf = this->self();  // self maybeUpdate(lastIndex) raft/raft.go:358
    Pr p = get(sf);
    const Pr p0 = p;
    if (p.match < last) {
      p.match = last;
      p.pm &= ~PM_PAUSED;
    }
    if (p.next < last + 1) p.next = last + 1;
    put(sf, p, p0);
    maybe_commit();
    bcast();
    if (faulted()) this->ev(HB_EV_FAULT, 0, faulted(), this->arrival_x());
  }

  // stepLeader (raft/raft.go:514-583) for the messages takes() accepts.
  __device__ __forceinline__ void step(uint32_t type, uint32_t from, uint64_t mterm, uint64_t index, bool reject,
                                       uint64_t hint) {
    if (mterm != 0 && mterm < term) return;  // the gate ignores a lower term (:483-486)
    bool updated = false, old_paused = false, send_one = false;
    Pr p = get(from);
    const Pr p0 = p;
    const uint32_t ps = pm_state(p.pm);
    if (type == HB_MSG_APP_RESP) {  // :514-546
      if (reject) {
        bool dec = false;  // maybeDecrTo raft/progress.go:119-141
        if (ps == HB_PR_REPLICATE) {
          if (index > p.match) {
            p.next = p.match + 1;
            dec = true;
          }
        } else if (p.next - 1 == index) {
          p.next = umin64(index, hint + 1);
          if (p.next < 1) p.next = 1;
          p.pm &= ~PM_PAUSED;
          dec = true;
        }
        if (dec && ps == HB_PR_REPLICATE) {  // becomeProbe from Replicate raft/progress.go:76-88
          p.pm = pm_make(HB_PR_PROBE, 0, 0, 0);
          p.next = p.match + 1;
        }
        send_one = dec;
      } else {
        old_paused = B::is_paused(p.pm);
        const uint64_t nx0 = p.next;
        if (p.match < index) {  // maybeUpdate raft/progress.go:102-113
          p.match = index;
          p.pm &= ~PM_PAUSED;
          updated = true;
        }
        if (p.next < index + 1) p.next = index + 1;
        if (updated) {
          if (ps == HB_PR_PROBE) {  // becomeReplicate :90-93
            p.pm = pm_make(HB_PR_REPLICATE, 0, 0, 0);
            p.next = p.match + 1;
          } else if (ps == HB_PR_SNAPSHOT) {  // maybeSnapshotAbort -> becomeProbe
            const uint64_t pend = pending_of(from);
            if (p.match >= pend) {
              p.pm = pm_make(HB_PR_PROBE, 0, 0, 0);
              p.next = umax64(p.match + 1, pend + 1);
            }
          } else {  // ins.freeTo(m.Index)
            free_to(from, p, index, nx0);
          }
        }
      }
    } else if (type == HB_MSG_HEARTBEAT_RESP) {  // :547-554
      if (ps == HB_PR_REPLICATE && pm_count(p.pm) == S.W) {  // freeFirstOne: entries increase, so one pops
        uint32_t idx = pm_start(p.pm) + 1;
        if (idx >= S.W) idx -= S.W;
        p.pm = pm_make(HB_PR_REPLICATE, pm_paused(p.pm), idx, S.W - 1);
      }
      send_one = p.match < last;
    } else if (type == HB_MSG_SNAP_STATUS) {  // :559-574
      if (ps == HB_PR_SNAPSHOT) {
        p.next = reject ? p.match + 1                                 // snapshotFailure, becomeProbe
                        : umax64(p.match + 1, pending_of(from) + 1);  // becomeProbe from Snapshot
        p.pm = pm_make(HB_PR_PROBE, 1, 0, 0);                         // ... and pause
      }
    } else if (type == HB_MSG_UNREACHABLE) {  // :575-581
      if (ps == HB_PR_REPLICATE) {
        p.pm = pm_make(HB_PR_PROBE, 0, 0, 0);
        p.next = p.match + 1;
      }
    }  // MsgVoteResp: a leader ignores it
    put(from, p, p0);
    // maybeCommit -> bcastAppend, else a paused follower gets sendAppend: one
    // send pass either way
    uint32_t mask = send_one ? 1u << from : 0u;
    if (updated) {
      if (maybe_commit()) mask = ((1u << this->n()) - 1) & ~(1u << this->self());
      else if (old_paused) mask = 1u << from;
    }
    if (mask && !faulted()) sends(mask);
    if (faulted()) this->ev(HB_EV_FAULT, 0, faulted(), this->arrival_x());
  }
};

}  // namespace hb
