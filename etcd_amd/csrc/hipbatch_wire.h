// hipbatch_wire.h — device decoder of raftpb.Message records (wire ingestion).
//
// Restates, per record and lane, the gogo-generated decoders the reference
// runs on every received message: Message.Unmarshal
// (raft/raftpb/raft.pb.go:549-799) with Entry (:256-364), Snapshot
// (:461-548), SnapshotMetadata (:365-460) and ConfState (:862-930), and
// gogo proto.Skip (Godeps/.../gogo/protobuf/proto/skip_gogo.go:34-105) for
// unknown fields.  Go semantics kept bit-exactly: varint fields OR into the
// field (a repeated field accumulates), Reject is assigned, shifts past the
// operand width contribute nothing (uint64 / int / int32 operands), the field
// number is int32(key >> 3), unknown fields restart at index -
// minimal_len(key), Entry errors are ignored, Snapshot errors propagate, int
// arithmetic wraps.  Outcomes Go cannot express as a value — a panic on a
// negative slice bound, a group loop that never returns — are reported as
// W_PANIC; groups nested past W_MAX_DEPTH go to the host (W_DEEP).
#pragma once
#include <cstdint>

namespace hb {

enum : int { W_OK = 0, W_ERR = 1, W_PANIC = 2, W_DEEP = 3 };
constexpr int W_MAX_DEPTH = 16;

struct WireMsg {
  int32_t type;
  uint64_t from, term, index, hint;
  bool reject;
};

__device__ __forceinline__ int64_t w_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

// varint into uint64 at d[*i] (the shared inner loop of every decoder)
__device__ __forceinline__ int w_varint(const uint8_t* d, int64_t l, int64_t* i, uint64_t* out) {
  uint64_t v = 0;
  for (uint32_t shift = 0;; shift += 7) {
    if (*i >= l) return W_ERR;  // io.ErrUnexpectedEOF
    const uint32_t b = d[*i];
    ++*i;
    if (shift < 64) v |= (uint64_t)(b & 0x7F) << shift;
    if (b < 0x80) break;
  }
  *out = v;
  return W_OK;
}

__device__ __forceinline__ int64_t w_size_of_wire(uint64_t w) {
  int64_t n = 0;
  do {
    ++n;
    w >>= 7;
  } while (w);
  return n;
}

// proto.Skip(d[0:l]) without recursion: frame k of the stack is the k-th
// nested Skip call (a wire-type-3 group walks its fields by calling Skip on
// each of them, skip_gogo.go:73-92).
__device__ int w_skip(const uint8_t* d0, int64_t l0, int64_t* n_out) {
  struct Frame {
    int64_t base, l, i, start, it;
  };
  enum { ENTER, RETURNED, GROUP };
  Frame st[W_MAX_DEPTH + 1];
  int top = 0;
  st[0].base = 0;
  st[0].l = l0;
  int state = ENTER;
  int64_t ret = 0;  // what the frame that just finished returned
  for (;;) {
    if (state == ENTER) {  // Skip(d[base : base + l]): one field
      Frame& f = st[top];
      if (f.l <= 0) return W_PANIC;  // panic("unreachable")
      const uint8_t* d = d0 + f.base;
      f.i = 0;
      uint64_t key;
      if (w_varint(d, f.l, &f.i, &key)) return W_ERR;
      const int wt = (int)(key & 7);
      state = RETURNED;
      if (wt == 0) {
        for (;;) {
          if (f.i >= f.l) return W_ERR;
          ++f.i;
          if (d[f.i - 1] < 0x80) break;
        }
        ret = f.i;
      } else if (wt == 1) {
        ret = w_add(f.i, 8);
      } else if (wt == 2) {
        uint64_t len;
        if (w_varint(d, f.l, &f.i, &len)) return W_ERR;
        ret = w_add(f.i, (int64_t)len);
      } else if (wt == 4) {
        ret = f.i;
      } else if (wt == 5) {
        ret = w_add(f.i, 4);
      } else if (wt == 3) {
        if (top >= W_MAX_DEPTH) return W_DEEP;
        f.it = 0;
        state = GROUP;
      } else {
        return W_ERR;  // illegal wireType
      }
    } else if (state == RETURNED) {
      if (top == 0) {
        *n_out = ret;
        return W_OK;
      }
      --top;
      st[top].i = w_add(st[top].start, ret);  // index = start + next
      state = GROUP;
    } else {  // GROUP: the next field of a start-group
      Frame& f = st[top];
      if (f.it++ > f.l + 1) return W_PANIC;  // `index` revisits a position: Go never returns
      f.start = f.i;
      if (f.i < 0) return W_PANIC;
      uint64_t k2;
      if (w_varint(d0 + f.base, f.l, &f.i, &k2)) return W_ERR;
      if ((k2 & 7) == 4) {
        ret = f.i;
        state = RETURNED;
      } else {  // next, err := Skip(data[start:])
        Frame& c = st[top + 1];
        c.base = f.base + f.start;
        c.l = f.l - f.start;
        ++top;
        state = ENTER;
      }
    }
  }
}

// the default: branch of every generated Unmarshal
__device__ __forceinline__ int w_skip_unknown(const uint8_t* d, int64_t l, int64_t* i, uint64_t key) {
  *i -= w_size_of_wire(key);
  int64_t skippy;
  const int rc = w_skip(d + *i, l - *i, &skippy);
  if (rc) return rc;
  const int64_t w = w_add(*i, skippy);
  if (w > l) return W_ERR;
  if (w < *i) return W_PANIC;  // data[index:index+skippy]
  *i = w;
  return W_OK;
}

__device__ __forceinline__ int w_span(const uint8_t* d, int64_t l, int64_t* i, int64_t* post) {
  uint64_t len;
  if (w_varint(d, l, i, &len)) return W_ERR;
  const int64_t p = w_add(*i, (int64_t)len);
  if (p > l) return W_ERR;
  if (p < *i) return W_PANIC;  // data[index:postIndex]
  *post = p;
  return W_OK;
}

// Entry / SnapshotMetadata / Snapshot / ConfState Unmarshal: validation only
// (their values are off the engine's path).  K: 0 Entry, 1 SnapshotMetadata,
// 2 Snapshot, 3 ConfState; the nesting (Snapshot -> Metadata -> ConfState) is
// fixed, so the calls are template instances, not recursion.
template <int K>
__device__ __forceinline__ int w_parse_sub(const uint8_t* d, int64_t l) {
  int64_t i = 0;
  for (int64_t it = 0; i < l; ++it) {
    // control flow depends on the index alone: more than l rounds repeat a
    // position (a field skipping zero bytes or back into its key) and Go
    // never returns
    if (it > l) return W_PANIC;
    uint64_t key;
    if (w_varint(d, l, &i, &key)) return W_ERR;
    const int32_t field = (int32_t)(uint32_t)(key >> 3);
    const int wt = (int)(key & 7);
    int want;
    if (K == 0) want = (field >= 1 && field <= 3) ? 0 : (field == 4 ? 2 : -1);
    else if (K == 1) want = field == 1 ? 2 : ((field == 2 || field == 3) ? 0 : -1);
    else if (K == 2) want = (field == 1 || field == 2) ? 2 : -1;
    else want = field == 1 ? 0 : -1;
    if (want < 0) {
      const int rc = w_skip_unknown(d, l, &i, key);
      if (rc) return rc;
      continue;
    }
    if (wt != want) return W_ERR;  // wrong wireType
    if (want == 0) {
      uint64_t v;
      if (w_varint(d, l, &i, &v)) return W_ERR;
      continue;
    }
    int64_t post;
    const int rc = w_span(d, l, &i, &post);
    if (rc) return rc;
    if constexpr (K == 1) {
      if (field == 1) {  // ConfState
        const int r2 = w_parse_sub<3>(d + i, post - i);
        if (r2) return r2;
      }
    } else if constexpr (K == 2) {
      if (field == 2) {  // Metadata
        const int r2 = w_parse_sub<1>(d + i, post - i);
        if (r2) return r2;
      }
    }
    i = post;
  }
  return W_OK;
}

// Fast path for the record shape Message.MarshalTo writes for the messages
// the engine consumes (raft/raftpb/raft.pb.go:1271-1330): every scalar field
// once, in field order, no entries, the empty Snapshot (data absent, empty
// ConfState, index 0, term 0), each varint at most 10 bytes.  On that shape
// the general parser runs the same field assignments in the same order, so
// the result is identical; anything else returns false and the record goes
// to w_unmarshal_message.  Straight-line code with a handful of registers, so
// the common case does not pay for the general parser's occupancy.
__device__ __forceinline__ bool w_fast_varint(const uint8_t* d, int64_t l, int64_t& i, uint64_t& v) {
  v = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    if (i >= l) return false;
    const uint32_t b = d[i++];
    v |= (uint64_t)(b & 0x7F) << (7 * k);  // k = 9: bits past 63 drop, as Go's shift
    if (b < 0x80) return true;
  }
  return false;
}

__device__ __forceinline__ bool w_fast_message(const uint8_t* d, int64_t l, WireMsg* m) {
  int64_t i = 0;
  uint64_t v[9];
  // keys of fields 1..6, 8 (varint), then the empty snapshot, 10, 11
  const uint8_t keys[7] = {0x08, 0x10, 0x18, 0x20, 0x28, 0x30, 0x40};
#pragma unroll
  for (int f = 0; f < 7; ++f) {
    if (i >= l || d[i] != keys[f]) return false;
    ++i;
    if (!w_fast_varint(d, l, i, v[f])) return false;
  }
  // 4a 08 | 12 06 | 0a 00 | 10 00 | 18 00 : Snapshot{Metadata{ConfState{}, 0, 0}}
  if (i + 10 > l) return false;
  const uint8_t snap[10] = {0x4a, 0x08, 0x12, 0x06, 0x0a, 0x00, 0x10, 0x00, 0x18, 0x00};
  bool same = true;
#pragma unroll
  for (int j = 0; j < 10; ++j) same &= d[i + j] == snap[j];
  if (!same) return false;
  i += 10;
  if (i >= l || d[i] != 0x50) return false;
  ++i;
  if (!w_fast_varint(d, l, i, v[7])) return false;
  if (i >= l || d[i] != 0x58) return false;
  ++i;
  if (!w_fast_varint(d, l, i, v[8])) return false;
  if (i != l) return false;
  // MessageType is int32: the low 32 bits of the accumulated varint (shifts
  // of 28 and more wrap inside int32, exactly the general parser's `t`)
  m->type = (int32_t)(uint32_t)v[0];
  m->from = v[2];
  m->term = v[3];
  m->index = v[5];
  m->reject = v[7] != 0;
  m->hint = v[8];
  return true;
}

// Message.Unmarshal (raft/raftpb/raft.pb.go:549-799)
__device__ int w_unmarshal_message(const uint8_t* d, int64_t l, WireMsg* m) {
  m->type = 0;
  m->from = m->term = m->index = m->hint = 0;
  m->reject = false;
  int64_t i = 0;
  for (int64_t it = 0; i < l; ++it) {
    if (it > l) return W_PANIC;  // a position repeats: Go never returns
    uint64_t key;
    if (w_varint(d, l, &i, &key)) return W_ERR;
    const int32_t field = (int32_t)(uint32_t)(key >> 3);
    const int wt = (int)(key & 7);
    if (field < 1 || field > 11) {
      const int rc = w_skip_unknown(d, l, &i, key);
      if (rc) return rc;
      continue;
    }
    const int want = (field == 7 || field == 9) ? 2 : 0;
    if (wt != want) return W_ERR;
    if (want == 2) {
      int64_t post;
      int rc = w_span(d, l, &i, &post);
      if (rc) return rc;
      rc = field == 7 ? w_parse_sub<0>(d + i, post - i) : w_parse_sub<2>(d + i, post - i);
      if (field == 7) {
        if (rc == W_PANIC || rc == W_DEEP) return rc;  // an Entry's error is dropped (:678)
      } else if (rc) {
        return rc;
      }
      i = post;
      continue;
    }
    if (field == 1) {  // MessageType is int32
      uint32_t t = 0;
      for (uint32_t shift = 0;; shift += 7) {
        if (i >= l) return W_ERR;
        const uint32_t b = d[i++];
        if (shift < 32) t |= (b & 0x7F) << shift;
        if (b < 0x80) break;
      }
      m->type |= (int32_t)t;
      continue;
    }
    uint64_t v;
    if (w_varint(d, l, &i, &v)) return W_ERR;
    if (field == 3) m->from |= v;
    else if (field == 4) m->term |= v;
    else if (field == 6) m->index |= v;
    else if (field == 10) m->reject = v != 0;  // assigned
    else if (field == 11) m->hint |= v;
    // to (2), logTerm (5), commit (8): decoded, not needed by the batch
  }
  return W_OK;
}

}  // namespace hb
