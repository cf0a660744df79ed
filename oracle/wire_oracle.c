/*
 * wire_oracle.c — CPU restatement of the reference's raftpb wire decoder.
 * TEST INFRASTRUCTURE ONLY (see raft_oracle.h): the checker for the engine's
 * hb_decode.  Follows raft/raftpb/raft.pb.go (gogo-generated, reference
 * holandes22/etcd @ 2.1.0-alpha):
 *   Entry.Unmarshal            :256-364
 *   SnapshotMetadata.Unmarshal :365-460
 *   Snapshot.Unmarshal         :461-548
 *   Message.Unmarshal          :549-799
 *   ConfState.Unmarshal        :862-930
 * and gogo proto.Skip (Godeps/_workspace/src/github.com/gogo/protobuf/proto/
 * skip_gogo.go:34-105), then multiNode.Step's local-message filter
 * (raft/multinode.go:432-439, IsLocalMsg raft/util.go:49-51).
 *
 * Go semantics kept: every varint field ORs into the field (a repeated field
 * accumulates), Reject is assigned (last wins); shifts past the operand width
 * contribute nothing (uint64 / int / int32 operands); the field number is
 * int32(key >> 3); unknown fields are skipped from index - minimal_len(key);
 * errors inside an Entry are ignored (:678), inside Snapshot they propagate.
 * Where Go would panic (slice bounds from a negative length) or never return
 * (a group whose inner Skip goes backwards) the result is WIRE_PANIC.
 */
#include "raft_oracle.h"

#include <string.h>

enum { U_OK = 0, U_ERR = 1, U_PANIC = 2, U_DEEP = 3 };

/* Go int arithmetic wraps */
static inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
#define MAX_GROUP_DEPTH 16

/* varint into uint64 (Go: (uint64(b) & 0x7F) << shift, zero past 63) */
static int varint_u64(const uint8_t* d, int64_t l, int64_t* i, uint64_t* out) {
  uint64_t v = 0;
  for (unsigned shift = 0;; shift += 7) {
    if (*i >= l) return U_ERR;                            /* io.ErrUnexpectedEOF */
    uint8_t b = d[(*i)++];
    if (shift < 64) v |= ((uint64_t)b & 0x7F) << shift;
    if (b < 0x80) break;
  }
  *out = v;
  return U_OK;
}

/* minimal varint length of a key value (the sizeOfWire loop) */
static int64_t size_of_wire(uint64_t w) {
  int64_t n = 0;
  do {
    n++;
    w >>= 7;
  } while (w);
  return n;
}

/* proto.Skip(data[0:l]) (skip_gogo.go:34-105): U_OK with *n, or U_ERR/U_PANIC/U_DEEP */
static int skip(const uint8_t* d, int64_t l, int64_t* n, int depth) {
  int64_t i = 0;
  if (l <= 0) return U_PANIC;                             /* panic("unreachable") */
  uint64_t key;
  if (varint_u64(d, l, &i, &key)) return U_ERR;
  switch ((int)(key & 7)) {
    case 0:
      for (;;) {
        if (i >= l) return U_ERR;
        i++;
        if (d[i - 1] < 0x80) break;
      }
      *n = i;
      return U_OK;
    case 1:
      *n = wadd(i, 8);
      return U_OK;
    case 2: {
      uint64_t len;
      if (varint_u64(d, l, &i, &len)) return U_ERR;      /* int accumulation = same bits */
      *n = wadd(i, (int64_t)len);
      return U_OK;
    }
    case 3:
      if (depth >= MAX_GROUP_DEPTH) return U_DEEP;
      for (int64_t it = 0;; it++) {
        /* the loop's state is `index` alone: more than l + 1 rounds revisit
         * a position, i.e. Go never returns */
        if (it > l + 1) return U_PANIC;
        int64_t start = i;
        uint64_t k2;
        if (i < 0) return U_PANIC;                        /* data[index] with index < 0 */
        if (varint_u64(d, l, &i, &k2)) return U_ERR;
        if ((k2 & 7) == 4) break;
        int64_t next;
        int rc = skip(d + start, l - start, &next, depth + 1);
        if (rc) return rc;
        i = wadd(start, next);
      }
      *n = i;
      return U_OK;
    case 4:
      *n = i;
      return U_OK;
    case 5:
      *n = i + 4;
      return U_OK;
    default:
      return U_ERR;                                       /* "proto: illegal wireType" */
  }
}

/* the default: branch shared by every generated Unmarshal */
static int skip_unknown(const uint8_t* d, int64_t l, int64_t* i, uint64_t key) {
  *i -= size_of_wire(key);
  int64_t skippy;
  int rc = skip(d + *i, l - *i, &skippy, 0);
  if (rc) return rc;
  const int64_t w = wadd(*i, skippy);
  if (w > l) return U_ERR;
  if (w < *i) return U_PANIC;                             /* data[index:index+skippy] */
  *i = w;
  return U_OK;
}

/* a length-delimited field: returns the [*i, *post) span */
static int span(const uint8_t* d, int64_t l, int64_t* i, int64_t* post) {
  uint64_t len;
  if (varint_u64(d, l, i, &len)) return U_ERR;
  int64_t p = wadd(*i, (int64_t)len);
  if (p > l) return U_ERR;
  if (p < *i) return U_PANIC;                             /* data[index:postIndex] with postIndex < index */
  *post = p;
  return U_OK;
}

enum { K_ENTRY, K_META, K_SNAP, K_CONF };

/* Entry / SnapshotMetadata / Snapshot / ConfState Unmarshal: validation only
 * (their values are not on the engine's path). */
static int parse_sub(int kind, const uint8_t* d, int64_t l) {
  int64_t i = 0;
  for (int64_t it = 0; i < l; it++) {
    /* control flow depends on `index` alone: a field that skips zero bytes
     * (or backwards into its own key) repeats a position and Go never returns */
    if (it > l) return U_PANIC;
    uint64_t key;
    if (varint_u64(d, l, &i, &key)) return U_ERR;
    int32_t field = (int32_t)(uint32_t)(key >> 3);
    int wt = (int)(key & 7);
    int want = -1, sub = -1;
    switch (kind) {
      case K_ENTRY: want = field == 1 || field == 2 || field == 3 ? 0 : field == 4 ? 2 : -1; break;
      case K_META:
        want = field == 1 ? 2 : (field == 2 || field == 3) ? 0 : -1;
        sub = field == 1 ? K_CONF : -1;
        break;
      case K_SNAP:
        want = field == 1 || field == 2 ? 2 : -1;
        sub = field == 2 ? K_META : -1;
        break;
      case K_CONF: want = field == 1 ? 0 : -1; break;
    }
    if (want < 0) {
      int rc = skip_unknown(d, l, &i, key);
      if (rc) return rc;
      continue;
    }
    if (wt != want) return U_ERR;                         /* "proto: wrong wireType" */
    if (want == 0) {
      uint64_t v;
      if (varint_u64(d, l, &i, &v)) return U_ERR;
    } else {
      int64_t post;
      int rc = span(d, l, &i, &post);
      if (rc) return rc;
      if (sub >= 0) {
        rc = parse_sub(sub, d + i, post - i);
        if (rc) return rc;
      }
      i = post;
    }
  }
  return U_OK;
}

int orc_unmarshal_message(const uint8_t* d, int64_t l, orc_wire_msg* m) {
  memset(m, 0, sizeof(*m));
  int64_t i = 0;
  for (int64_t it = 0; i < l; it++) {
    if (it > l) return U_PANIC;                           /* a position repeats: Go never returns */
    uint64_t key;
    if (varint_u64(d, l, &i, &key)) return U_ERR;
    int32_t field = (int32_t)(uint32_t)(key >> 3);
    int wt = (int)(key & 7);
    if (field < 1 || field > 11) {
      int rc = skip_unknown(d, l, &i, key);
      if (rc) return rc;
      continue;
    }
    const int want = (field == 7 || field == 9) ? 2 : 0;
    if (wt != want) return U_ERR;
    if (want == 2) {
      int64_t post;
      int rc = span(d, l, &i, &post);
      if (rc) return rc;
      if (field == 7) {
        m->nentries++;
        rc = parse_sub(K_ENTRY, d + i, post - i);
        if (rc == U_PANIC || rc == U_DEEP) return rc;     /* Entry errors are dropped (:678) */
      } else {
        rc = parse_sub(K_SNAP, d + i, post - i);
        if (rc) return rc;
      }
      i = post;
      continue;
    }
    uint64_t v = 0;
    if (field == 1) {                                     /* MessageType is int32 */
      uint32_t t = 0;
      for (unsigned shift = 0;; shift += 7) {
        if (i >= l) return U_ERR;
        uint8_t b = d[i++];
        if (shift < 32) t |= ((uint32_t)b & 0x7F) << shift;
        if (b < 0x80) break;
      }
      m->type |= (int32_t)t;
      continue;
    }
    if (varint_u64(d, l, &i, &v)) return U_ERR;
    switch (field) {
      case 2: m->to |= v; break;
      case 3: m->from |= v; break;
      case 4: m->term |= v; break;
      case 5: m->log_term |= v; break;
      case 6: m->index |= v; break;
      case 8: m->commit |= v; break;
      case 10: m->reject = v != 0; break;                 /* assigned */
      case 11: m->reject_hint |= v; break;
    }
  }
  return U_OK;
}

static int is_local(int32_t t) {                          /* raft/util.go:49-51 */
  return t == HB_MSG_HUP || t == HB_MSG_BEAT || t == HB_MSG_UNREACHABLE || t == HB_MSG_SNAP_STATUS;
}

void orc_decode_batch(const uint8_t* bytes, const uint64_t* off, const uint32_t* len, const uint32_t* group,
                      uint64_t n, uint32_t capacity, const uint32_t* group_n, const uint64_t* peers,
                      uint32_t* o_group, uint32_t* o_info, uint64_t* o_term, uint64_t* o_index, uint64_t* o_hint,
                      uint8_t* status) {
  for (uint64_t k = 0; k < n; k++) {
    orc_wire_msg m;
    int rc = orc_unmarshal_message(bytes + off[k], len[k], &m);
    uint8_t st;
    if (rc == U_ERR) st = HB_WIRE_ERROR;
    else if (rc == U_PANIC) st = HB_WIRE_PANIC;
    else if (rc == U_DEEP) st = HB_WIRE_HOST;
    else if (is_local(m.type)) st = HB_WIRE_LOCAL;
    else if (m.type != HB_MSG_APP_RESP && m.type != HB_MSG_VOTE_RESP && m.type != HB_MSG_HEARTBEAT_RESP)
      st = HB_WIRE_HOST;
    else if (group[k] >= capacity) st = HB_WIRE_BADGROUP;
    else st = HB_WIRE_OK;
    status[k] = st;
    uint32_t slot = HB_SLOT_NONE;
    if (st == HB_WIRE_OK) {
      const uint32_t g = group[k];
      for (uint32_t s = 0; s < group_n[g] && s < HB_MAX_REPLICAS; s++)
        if (m.from != 0 && peers[(uint64_t)g * HB_MAX_REPLICAS + s] == m.from) { slot = s; break; }
    }
    o_group[k] = st == HB_WIRE_OK ? group[k] : 0xFFFFFFFFu;
    o_info[k] = st == HB_WIRE_OK ? ((uint32_t)m.type | slot << 4 | (uint32_t)(m.reject != 0) << 8) : 0u;
    o_term[k] = st == HB_WIRE_OK ? m.term : 0;
    o_index[k] = st == HB_WIRE_OK ? m.index : 0;
    o_hint[k] = st == HB_WIRE_OK ? m.reject_hint : 0;
  }
}
