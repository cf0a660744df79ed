// hipbatch_elect.h — the election lane: Lane::step (hipbatch_kernels.h)
// restricted to what an election storm steps on groups that are not (yet)
// leaders — campaign on MsgHup, the term gate's step-down on a higher-term
// response, the vote tally of MsgVoteResp, becomeLeader with its noop entry
// and bcastAppend, becomeFollower on a lost election — and the responses a
// follower or candidate ignores.
//
// Why a lane of its own: every Progress an election touches is in the form
// reset() leaves it (raft/raft.go:334-349: Match = 0 except self, Next =
// lastIndex + 1, Probe) plus, after becomeLeader, the noop append and the
// sendAppend pause (raft/raft.go:406-427, :239-282).  The lane keeps that as
// two words (the lastIndex at the reset, whether the peers were sent to)
// instead of n Progress entries in registers, so its kernel (k_elect) runs at
// several waves per SIMD where the general kernel needs all 256 VGPRs.
//
// Anything else hands the group over, at that message and with nothing of it
// stepped, to the general kernel (k_apply): a leader that must read its
// Progress (a response at its own term, or any message to a leader that was
// one at batch start), MsgHup to a leader (the reference's panic), proposals,
// follower-side types, a non-member sender, a group without a self slot.
// Every event and every state write below is the one Lane::step makes, in the
// same order; the GPU parity tests compare both paths with the oracle.
#pragma once

#include "hipbatch_kernels.h"

namespace hb {

template <int NMAX>
struct ElectLane {
  DevState S;
  EvSink E;
  uint32_t g;
  uint64_t term, committed, last, tfirst, tlast, meta, meta0;
  uint64_t rlast;   // lastIndex when the last reset() ran
  uint32_t dirty;
  uint32_t won, lost, nev;
  bool rst;         // reset() ran: Progress = the reset form of rlast (+ the leader's noop / sends)
  bool sent;        // becomeLeader's bcastAppend paused every peer after that reset

  __device__ __forceinline__ uint32_t n() const { return m_n(meta); }
  __device__ __forceinline__ uint32_t state() const { return m_state(meta); }
  __device__ __forceinline__ uint32_t self() const { return m_self(meta); }
  __device__ __forceinline__ uint32_t lead() const { return m_lead(meta); }
  __device__ __forceinline__ uint32_t vote() const { return m_vote(meta); }
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
  __device__ __forceinline__ void ev(uint32_t type, uint32_t to, uint32_t aux, uint64_t x) {
    emit_ev(E, g & (PART - 1), type, to, aux, x);
    nev++;
  }

  // the per-group fields (Lane::load_group); meta is set by the caller
  __device__ __forceinline__ void load() {
    term = S.term[g];
    committed = S.commit[g];
    last = S.last[g];
    tfirst = S.tfirst[g];
    tlast = S.tlast[g];
    meta0 = meta;
    if (meta & M_TL) tlast = last;
    dirty = 0;
    won = lost = nev = 0;
    rst = sent = false;
    rlast = 0;
  }

  // Lane::store with the Progress of every slot < n written from the reset form
  __device__ __forceinline__ void store() {
    const uint32_t sf = self(), nn = n();
    const bool tl = tlast == last;
    // reset form: the self slot's Match = lastIndex, Next = lastIndex + 1 (the
    // noop's maybeUpdate keeps both so); as loaded, nothing touched it
    const bool sm = rst ? sf < nn : (meta0 & M_SM) != 0;
    // after a reset the n Progress entries are the reset form: M_RS instead of n x 20 bytes, when
    // rs_progress derives this reset's lastIndex (a leader's noop opened its term: tfirst = rlast + 1)
    // and its pauses (a leader with peers sent to them); otherwise they are written out
    const bool leader = state() == HB_STATE_LEADER;
    const bool rs = rst && (leader ? (tfirst == rlast + 1 && (sent || nn <= 1)) : (rlast == last && !sent));
    const uint64_t m2 = (meta & ~(M_TL | M_SM | M_RS)) | (tl ? M_TL : 0ull) | (sm ? M_SM : 0ull) |
                        (rs ? M_RS : (rst ? 0ull : (meta & M_RS)));
    if (m2 != meta) {
      meta = m2;
      dirty |= D_META;
    }
    if (!tl && (meta0 & M_TL)) dirty |= D_TRUN;
    if (dirty & D_META) S.meta[g] = meta;
    if (dirty & D_TERM) S.term[g] = term;
    if (dirty & D_COMMIT) S.commit[g] = committed;
    if (dirty & D_LAST) S.last[g] = last;
    if (dirty & D_TRUN) {
      S.tfirst[g] = tfirst;
      S.tlast[g] = tlast;
    }
    if (dirty & D_ELAPSED) S.elapsed[g] = 0;
    if (rst && !rs) {
      const uint32_t peer_pm = pm_make(HB_PR_PROBE, sent ? 1u : 0u, 0, 0);
#pragma unroll
      for (int s = 0; s < NMAX; ++s) {
        if ((uint32_t)s < nn) {
          const bool me = (uint32_t)s == sf;
          S.match[(size_t)s * S.G + g] = me ? last : 0ull;
          S.next[(size_t)s * S.G + g] = me ? last + 1 : rlast + 1;
          S.pm[(size_t)s * S.G + g] = me ? pm_make(HB_PR_PROBE, 0, 0, 0) : peer_pm;
        }
      }
    }
  }

  // Lane::reset / transition / poll (raft/raft.go:334-404, :445-460)
  __device__ __forceinline__ void reset(uint64_t t) {
    if (term != t) {
      if (tfirst != HB_NO_INDEX) tr_push(S, g, tfirst, term);
      term = t;
      set_vote(HB_REF_NONE);
      tfirst = HB_NO_INDEX;
      tlast = 0;
      dirty |= D_TERM | D_TRUN;
      ev(HB_EV_TERM, 0, 0, t);
    }
    set_lead(HB_REF_NONE);
    dirty |= D_ELAPSED;
    set_votes(0, 0);
    rst = true;
    sent = false;
    rlast = last;
  }
  __device__ __forceinline__ void transition(uint32_t kind, uint64_t t, uint32_t ld) {
    const uint64_t before = soft();
    reset(kind == HB_STATE_CANDIDATE ? term + 1 : (kind == HB_STATE_FOLLOWER ? t : term));
    set_lead(kind == HB_STATE_LEADER ? self() : (kind == HB_STATE_FOLLOWER ? ld : (uint32_t)HB_REF_NONE));
    if (kind == HB_STATE_CANDIDATE) set_vote(self());
    set_state(kind);
    if (soft() != before) ev(HB_EV_STATE, 0, 0, soft());
  }
  __device__ __forceinline__ uint32_t poll(uint32_t bit, bool v) {
    uint32_t resp = m_resp(meta), grant = m_grant(meta);
    if (!((resp >> bit) & 1u)) {
      resp |= 1u << bit;
      if (v) grant |= 1u << bit;
      set_votes(resp, grant);
    }
    return (uint32_t)__popc(grant);
  }

  // Whether this lane steps the message (false: hand the group over here).
  // The caller has dropped non-member responses (raft/multinode.go:235).
  __device__ __forceinline__ bool takes(uint32_t type, uint32_t from, uint64_t mterm) const {
    if (type == HB_MSG_HUP) return state() != HB_STATE_LEADER;
    if (!(type == HB_MSG_VOTE_RESP || type == HB_MSG_APP_RESP || type == HB_MSG_HEARTBEAT_RESP ||
          type == HB_MSG_UNREACHABLE || type == HB_MSG_SNAP_STATUS))
      return false;
    if (from >= n()) return false;  // (MsgSnapStatus: a non-member's would be a nil Progress)
    // a leader that keeps its term reads its Progress, except for the vote
    // tally it ignores after winning in this batch (Progress in reset form)
    const bool keeps = mterm == 0 || mterm == term;
    if (state() == HB_STATE_LEADER && keeps) return rst && type == HB_MSG_VOTE_RESP;
    return true;
  }

  // Lane::step for the messages takes() accepts
  __device__ __forceinline__ void step(uint32_t type, uint32_t from, uint64_t mterm, bool reject) {
    // ---- gate (raft/raft.go:462-486)
    if (type == HB_MSG_HUP) {
      transition(HB_STATE_CANDIDATE, 0, HB_REF_NONE);  // campaign -> becomeCandidate
    } else if (mterm != 0) {
      if (mterm < term) return;
      if (mterm > term) transition(HB_STATE_FOLLOWER, mterm, from);
    }
    const uint32_t nn = n(), sf = self();
    const uint32_t q = nn / 2 + 1;
    bool win = false, bcast = false;
    if (type == HB_MSG_HUP) {  // campaign :429-443: an immediate win sends nothing
      if (q == poll(sf, true)) {
        won++;
        win = true;
      } else {  // the MsgVotes (slot order) as one EVC_VBCAST word when there are two or more
        const uint32_t mask = ((1u << nn) - 1) & ~(1u << sf);
        if (mask & (mask - 1)) {
          emit_ev(E, g & (PART - 1), EVC_VBCAST, mask, 0, last);
          nev += __popc(mask);
        } else {
#pragma nounroll
          for (uint32_t s = 0; s < nn; ++s)
            if (s != sf) ev(HB_EV_VOTE, s, 0, last);
        }
      }
    } else if (state() == HB_STATE_CANDIDATE && type == HB_MSG_VOTE_RESP) {  // :603-612
      const uint32_t gr = poll(from, !reject);
      if (q == gr) {
        won++;
        win = true;
        bcast = true;
      } else if (q == (uint32_t)__popc(m_resp(meta)) - gr) {
        lost++;
        transition(HB_STATE_FOLLOWER, term, HB_REF_NONE);
      }
    }
    if (!win) return;
    // ---- becomeLeader (:406-427) + appendEntry of the noop (:351-360)
    transition(HB_STATE_LEADER, term, HB_REF_NONE);
    const uint64_t old = last;
    last += 1;
    if (tfirst == HB_NO_INDEX) tfirst = old + 1;
    tlast = last;
    dirty |= D_LAST | D_TRUN;
    ev(HB_EV_LAST, 0, 1, last);
    // maybeCommit: the only non-zero Match is self's (= last): the q-th largest
    // is last for n = 1 and 0 otherwise; term(last) == Term (the noop)
    if (nn == 1 && last > committed) {
      committed = last;
      dirty |= D_COMMIT;
      ev(HB_EV_COMMIT, 0, 0, last);
    }
    // bcastAppend (slot order): every peer is in Probe, not paused, Next =
    // rlast + 1 <= last: MsgApp{Index = rlast} and pause
    if (bcast) {  // one EVC_BCAST word for two or more sends (the same records once expanded)
      const uint32_t mask = ((1u << nn) - 1) & ~(1u << sf);
      const uint32_t lt = (tfirst <= rlast && rlast <= tlast) ? 1u : 0u;  // aux: term(Index) == Term
      if (mask & (mask - 1)) {
        emit_ev(E, g & (PART - 1), EVC_BCAST, mask, lt, rlast);
        nev += __popc(mask);
      } else if (mask) {
        ev(HB_EV_APP, __ffs(mask) - 1, lt, rlast);
      }
      sent = true;
    }
  }
};

}  // namespace hb
