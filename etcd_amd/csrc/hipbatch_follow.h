// hipbatch_follow.h — the follower side's steady state on the fast path.
//
// A node leads about 1/n of its groups and follows the rest, so most of the
// messages a MultiNode steps are the follower side of replication: the
// leader's MsgApp and MsgHeartbeat for a group this node follows
// (raft/raft.go:616-669 stepFollower, handleAppendEntries, handleHeartbeat;
// raft/log.go:72-88 maybeAppend).  k_follow (Lane<NMAX, true>) steps every
// follower-side case; FollowLane is its specialization for the common one, run
// by k_apply_fast (n = 3) and k_apply_lead (n >= 5) in the same pass as the
// leader lane:
//
//   * a follower (not M_RS, not M_NC) receiving, at its own Term, from a member:
//   * MsgHeartbeat with m.Commit <= lastIndex
//       r.elapsed = 0, r.lead = m.From, commitTo(m.Commit), MsgHeartbeatResp
//   * MsgApp whose Index is below committed (MsgAppResp{Index: committed}),
//     whose (Index, LogTerm) does not match the log (a reject, RejectHint
//     read by the host from its log), or that appends at the log's end
//     (Index == lastIndex, matching) entries that all carry m.Term (REC_UNI,
//     counted by the partition's first pass) with no size ring to extend, and
//     whose commitTo(min(m.Commit, lastnewi)) stays within the log:
//       maybeAppend without a conflict scan, commitTo(min(m.Commit, lastnewi)),
//       MsgAppResp{Index: lastnewi}
//   * any message below its Term (dropped by the Step gate, raft/raft.go:480)
//
// Everything else — a higher Term, a candidate, an Index inside the log
// (findConflict), older-term entries, a snapshot, a vote, a term(i) below the
// current-term run — hands the group to the general kernels at that message,
// exactly as the leader lane does.  The events are Lane<NMAX, true>'s, in its
// order: the step marker, a lead change, the append marker, the commit, the
// response.  m.LogTerm and m.Commit come with the route slot (the partition's
// X-mode extension, hipbatch.hip), not by arrival index.
#pragma once

#include "hipbatch_fast.h"

namespace hb {

// Base: FastLane (k_apply_fast, n = 3) or LeadLane (k_apply_lead, n >= 5),
// whose lanes step a partition's leaders and followers side by side.
template <int NMAX, class Base = FastLane<NMAX>>
struct FollowLane : Base {
  using B = Base;
  using B::S;
  using B::g;
  using B::arrival;
  using B::term;
  using B::committed;
  using B::first;
  using B::last;
  using B::tfirst;
  using B::tlast;
  using B::mlo;
  using B::dirty;
  using B::nev;
  static constexpr uint32_t F_ELAPSED = 1u << 26;  // dirty: r.elapsed = 0
  static constexpr uint32_t F_SELF = 1u << 27;     // dirty: the self slot's match / next were derived (M_SM)
  uint64_t self_last;                              // lastIndex when M_SM was dropped (the self Match)

  __device__ __forceinline__ uint32_t lead() const { return (mlo >> 9) & 0xF; }
  __device__ __forceinline__ uint32_t soft() const { return (mlo & 3) | (((mlo >> 9) & 0xF) << 8) | (((mlo >> 13) & 0xF) << 16); }
  // the remaining state a follower needs (term, committed, first, last, tfirst
  // and pm came with meta: FastLane::load_head)
  __device__ __forceinline__ void load_follow() {
    tlast = (mlo & (uint32_t)M_TL) ? last : at32(S.tlast, g);
    dirty = 0;
    nev = 0;
  }
  // raftLog.term(i) from the current-term run (raft/log.go:198-217); *known =
  // false when i lies in an older run (the general lane reads the run ring)
  __device__ __forceinline__ uint64_t term_at(uint64_t i, bool* known) const {
    *known = true;
    if (i + 1 < first || i > last) return 0;
    if (tfirst != HB_NO_INDEX && i >= tfirst) return term;
    *known = false;
    return 0;
  }
  // whether the message is one FollowLane steps (see the header comment)
  __device__ __forceinline__ bool takes_follow(uint32_t info, uint32_t from, uint64_t mterm, uint64_t index, uint64_t lterm,
                                        uint64_t mcommit) const {
    const uint32_t type = info & 0xF;
    if ((mlo & 3) != HB_STATE_FOLLOWER || (mlo & (uint32_t)M_RS) || from >= B::n()) return false;
    if (type != HB_MSG_APP && type != HB_MSG_HEARTBEAT) return false;
    if (mterm == 0 || mterm > term) return false;
    if (mterm < term) return true;  // the gate drops it
    if (type == HB_MSG_HEARTBEAT) return mcommit <= last || mcommit <= committed;
    if (index < committed) return true;
    bool known;
    const uint64_t t = term_at(index, &known);
    if (!known) return false;
    if (t != lterm) return true;  // the reject
    // no entries: nothing to scan or append; entries: appended at the log's end
    const uint64_t ne = rec_ne(info);
    if (!(info & REC_UNI) || !(ne == 0 || (index == last && !sz_on(S.max_msg_size)))) return false;
    // commitTo(min(m.Commit, lastnewi)) within the log: an empty MsgApp past the
    // log's end matches LogTerm 0 (raftLog.term is 0 there) and can commit past
    // lastIndex, the reference's panic (raft/log.go:175-176) — the general lane's
    return ne != 0 || umin64(mcommit, index) <= last;
  }
  __device__ __forceinline__ void set_lead(uint32_t from) {
    if (lead() == from) return;
    mlo = (mlo & ~(0xFu << 9)) | (from << 9);
    dirty |= D_META;
    B::ev(HB_EV_STATE, 0, 0, soft());
  }
  // commitTo raft/log.go:172-180 (takes() keeps `to` within the log; a
  // screening gap still faults as the general lane does, not silently)
  __device__ __forceinline__ void commit_to(uint64_t to) {
    if (committed < to) {
      if (last < to) {
        B::fault(HB_FAULT_COMMIT_RANGE);
        return;
      }
      committed = to;
      dirty |= D_COMMIT;
      B::ev(HB_EV_COMMIT, 0, 0, to);
    }
  }
  __device__ __forceinline__ void resp(uint32_t to, uint32_t kind, uint64_t x) { B::ev(HB_EV_RESP, to, kind, x); }
  // Step (raft/raft.go:462-490) -> stepFollower (:616-649) for a message takes() accepted
  __device__ __forceinline__ void step_follow(uint32_t info, uint32_t from, uint64_t mterm, uint64_t index, uint64_t lterm,
                                       uint64_t mcommit) {
    if (mterm < term) return;  // lower term: ignored
    const uint32_t type = info & 0xF;
    B::ev(HB_EV_FOLLOW, 0, HB_FOLLOW_STEP, B::arrival_x());
    dirty |= F_ELAPSED;  // r.elapsed = 0
    set_lead(from);      // r.lead = m.From
    if (type == HB_MSG_HEARTBEAT) {  // handleHeartbeat :666-669
      commit_to(mcommit);
      if (B::faulted()) B::ev(HB_EV_FAULT, 0, B::faulted(), B::arrival_x());
      else resp(from, HB_RESP_HEARTBEAT, 0);
      return;
    }
    // handleAppendEntries :651-665
    if (index < committed) {
      resp(from, HB_RESP_APP, committed);
      return;
    }
    bool known;
    if (term_at(index, &known) != lterm) {  // reject; RejectHint = lastIndex (the host reads its log)
      resp(from, HB_RESP_APP | HB_RESP_REJECT, index);
      return;
    }
    const uint64_t ne = rec_ne(info), lastnewi = index + ne;
    if (ne) {  // maybeAppend: every entry is past the log's end (no conflict scan), all at Term
      if (mlo & (uint32_t)M_SM) {  // the self Match / Next were derived from lastIndex: pin them
        self_last = last;
        mlo &= ~(uint32_t)M_SM;
        dirty |= D_META | F_SELF;
      }
      if (tfirst == HB_NO_INDEX) tfirst = index + 1;
      last = lastnewi;
      tlast = last;
      dirty |= D_LAST | D_TRUN | B::D_TFIRST;
      B::ev(HB_EV_FOLLOW, 0, HB_FOLLOW_APPEND, B::arrival_x());
    }
    commit_to(mcommit < lastnewi ? mcommit : lastnewi);
    if (B::faulted()) B::ev(HB_EV_FAULT, 0, B::faulted(), B::arrival_x());
    else resp(from, HB_RESP_APP, lastnewi);
  }
  __device__ __forceinline__ void store_follow() {
    // M_TL: the tlast array is kept only while tlast != last
    const bool tl = tlast == last;
    if (tl != ((mlo & (uint32_t)M_TL) != 0)) {
      mlo = tl ? (mlo | (uint32_t)M_TL) : (mlo & ~(uint32_t)M_TL);
      dirty |= D_META;
    }
    if (dirty & D_META) at32(reinterpret_cast<uint32_t*>(S.meta), 2 * g) = mlo;  // little-endian low word
    if (dirty & D_COMMIT) at32(S.commit, g) = committed;
    if (dirty & D_LAST) at32(S.last, g) = last;
    if (dirty & B::D_TFIRST) at32(S.tfirst, g) = tfirst;
    if ((dirty & D_TRUN) && !tl) at32(S.tlast, g) = tlast;
    if (dirty & F_ELAPSED) at32(S.elapsed, g) = 0u;
    if (dirty & F_SELF) {
      const uint32_t sf = B::self();
      at32(S.match, sf * S.G + g) = self_last;
      at32(S.next, sf * S.G + g) = self_last + 1;
    }
  }
};

}  // namespace hb
