// hbnode.cpp — host side of raft.MultiNode over the MI355X engine (include/hbnode.h).
//
// The device (libhipbatch) steps the leader bookkeeping of every group in one
// launch per Ready cycle and reports what changed as an ordered event stream
// per group.  This file is the rest of the reference's `multiNode.run` loop
// (raft/multinode.go:166-322) that stays on the host:
//
//   MemoryStorage        raft/storage.go:63-248
//   raftLog (host half)  raft/log.go:23-308, unstable raft/log_unstable.go:20-140
//   newReady / commitReady / containsUpdates
//                        raft/node.go:82-100, 447-463; raft/multinode.go:137-164
//   message materialisation from the device's send intents
//                        raft/raft.go:227-321 (send, sendAppend, sendHeartbeat),
//                        :429-443 (campaign's MsgVote), :614-624 (MsgProp forward)
//   pendingConf          raft/raft.go:406-427 (becomeLeader scan), :500-513
//   CreateGroup          raft/multinode.go:181-217 + newRaft raft/raft.go:157-209
//   ApplyConfChange      raft/multinode.go:239-262, raft/raft.go:729-750
//   Status               raft/status.go:34-49
//
// Nothing here steps raft: every Step/Campaign/Propose/Report goes into the
// device batch, and the host only replays the events the device returns.
#include "../../include/hbnode.h"
#include "hbpool.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <string>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <type_traits>
#include <unordered_set>
#include <vector>

namespace {

thread_local std::string g_err;

struct Panic {
  std::string msg;
};
[[noreturn]] void panicf(const std::string& m) { throw Panic{m}; }

struct Fail {
  int code;
};

// ---------------------------------------------------------------- entries
struct Ent {
  uint64_t term = 0, index = 0;
  uint32_t type = HBN_ENTRY_NORMAL;
  bool has_data = false;
  std::string data;
};

Ent ent_from(const hbn_entry& e) {
  Ent x;
  x.term = e.term;
  x.index = e.index;
  x.type = e.type;
  x.has_data = e.has_data != 0;
  if (x.has_data && e.data_len) x.data.assign(reinterpret_cast<const char*>(e.data), e.data_len);
  return x;
}

uint64_t sov(uint64_t x) {  // sovRaft: varint length
  uint64_t n = 0;
  do {
    ++n;
    x >>= 7;
  } while (x);
  return n;
}

// Entry.Size() (raft/raftpb/raft.pb.go, gogo): Type, Term, Index always, Data if non-nil.
uint64_t ent_size(uint64_t type, uint64_t term, uint64_t index, bool has_data, uint64_t len) {
  uint64_t n = 1 + sov(type) + 1 + sov(term) + 1 + sov(index);
  if (has_data) n += 1 + len + sov(len);
  return n;
}
uint64_t ent_size(const Ent& e) { return ent_size(e.type, e.term, e.index, e.has_data, e.data.size()); }
uint32_t ent_desc(const Ent& e) {  // HB_ENT_DESC: the engine computes Entry.Size() from it
  if (e.data.size() > HB_ENT_MAX_DATA) throw std::length_error("entry data longer than HB_ENT_MAX_DATA");
  return HB_ENT_DESC(e.data.size(), e.type, e.has_data);
}

// limitSize raft/util.go:97-110
template <class V>
size_t limit_count(const V& ents, uint64_t max_size) {
  if (ents.empty()) return 0;
  uint64_t size = ent_size(ents[0]);
  size_t limit = 1;
  for (; limit < ents.size(); ++limit) {
    size += ent_size(ents[limit]);
    if (size > max_size) break;
  }
  return limit;
}

std::string marshal_varint(uint64_t v) {
  std::string s;
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
  return s;
}

// ConfChange.MarshalTo (raft/raftpb/raft.pb.go:1402-1426)
std::string marshal_conf_change(uint64_t id, uint32_t type, uint64_t node, const uint8_t* ctx, uint64_t ctx_len,
                                bool has_ctx) {
  std::string s;
  s.push_back(0x08);
  s += marshal_varint(id);
  s.push_back(0x10);
  s += marshal_varint(type);
  s.push_back(0x18);
  s += marshal_varint(node);
  if (has_ctx) {
    s.push_back(0x22);
    s += marshal_varint(ctx_len);
    if (ctx_len) s.append(reinterpret_cast<const char*>(ctx), ctx_len);
  }
  return s;
}

// ---------------------------------------------------------------- snapshot
struct Snap {
  uint64_t index = 0, term = 0;
  std::vector<uint64_t> nodes;
  bool has_data = false;
  std::string data;
};

void snap_view(const Snap& s, hbn_snapshot* o) {
  o->index = s.index;
  o->term = s.term;
  o->nodes = s.nodes.empty() ? nullptr : s.nodes.data();
  o->n_nodes = (uint32_t)s.nodes.size();
  o->has_data = s.has_data;
  o->data = s.data.empty() ? nullptr : reinterpret_cast<const uint8_t*>(s.data.data());
  o->data_len = s.data.size();
}

Snap snap_from(const hbn_snapshot& s) {
  Snap x;
  x.index = s.index;
  x.term = s.term;
  if (s.n_nodes) x.nodes.assign(s.nodes, s.nodes + s.n_nodes);
  x.has_data = s.has_data != 0;
  if (x.has_data && s.data_len) x.data.assign(reinterpret_cast<const char*>(s.data), s.data_len);
  return x;
}

// ---------------------------------------------------------------- entry blocks
// The storages' logs grow by one fixed-size deque block every few entries, on
// every group in the same Ready cycle.  From glibc malloc that is a million
// small allocations whose per-thread heaps grow page by page (mprotect under
// the process's address-space lock): 330 ms for 1M blocks on 8 threads, no
// faster than one thread.  These blocks come instead from 2 MiB chunks carved
// by a thread-local bump pointer (45 ms for the same 1M), and freed blocks are
// recycled through a per-thread cache backed by a global list.  Memory is kept
// for reuse, never returned to the system.
template <size_t BLOCK_BYTES>
class BlockPool {
 public:
  static constexpr size_t BLOCK = BLOCK_BYTES;
  static constexpr size_t CHUNK = size_t(2) << 20;
  static void* get() {
    Local& l = local();
    if (!l.free.empty()) {
      void* p = l.free.back();
      l.free.pop_back();
      return p;
    }
    if (refill(l)) {
      void* p = l.free.back();
      l.free.pop_back();
      return p;
    }
    if (l.left < BLOCK) {
      l.cur = chunk();
      l.left = CHUNK;
    }
    void* p = l.cur;
    l.cur += BLOCK;
    l.left -= BLOCK;
    return p;
  }
  static void put(void* p) {
    Local& l = local();
    l.free.push_back(p);
    if (l.free.size() >= 2 * BATCH) spill(l, BATCH);
  }

 private:
  static constexpr size_t BATCH = 256;
  struct Local {
    std::vector<void*> free;
    char* cur = nullptr;
    size_t left = 0;
    ~Local() {  // a thread ends: its cached blocks and the rest of its chunk go to the global list
      for (; left >= BLOCK; cur += BLOCK, left -= BLOCK) free.push_back(cur);
      spill(*this, free.size());
    }
  };
  static Local& local() {
    thread_local Local l;
    return l;
  }
  // the next CHUNK of the current region: regions of 1 GiB address space
  // (reserved, transparent huge pages where the system allows), mapped as
  // needed (one call per 4096 blocks: a lock is cheap here)
  static char* chunk() {
    static constexpr size_t REGION = size_t(1) << 30;
    static char* base = nullptr;
    static size_t top = REGION;
    std::lock_guard<std::mutex> lk(mu());
    if (top + CHUNK > REGION) {
      void* r = mmap(nullptr, REGION, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
      if (r == MAP_FAILED) throw std::bad_alloc();
      (void)madvise(r, REGION, MADV_HUGEPAGE);
      base = static_cast<char*>(r);
      top = 0;
    }
    top += CHUNK;
    return base + top - CHUNK;
  }
  static std::mutex& mu() {
    static std::mutex m;
    return m;
  }
  static std::vector<void*>& global() {
    static std::vector<void*>* g = new std::vector<void*>();  // (outlives every thread's Local)
    return *g;
  }
  static void spill(Local& l, size_t k) {
    std::lock_guard<std::mutex> lk(mu());
    std::vector<void*>& g = global();
    g.insert(g.end(), l.free.end() - k, l.free.end());
    l.free.resize(l.free.size() - k);
    pooled_blocks().store(g.size(), std::memory_order_relaxed);
  }
  static std::atomic<size_t>& pooled_blocks() {  // the global list's size, read without the lock
    static std::atomic<size_t> k{0};
    return k;
  }
  static bool refill(Local& l) {
    if (pooled_blocks().load(std::memory_order_relaxed) == 0) return false;
    std::lock_guard<std::mutex> lk(mu());
    std::vector<void*>& g = global();
    if (g.empty()) return false;
    const size_t k = std::min(BATCH, g.size());
    l.free.insert(l.free.end(), g.end() - k, g.end());
    g.resize(g.size() - k);
    pooled_blocks().store(g.size(), std::memory_order_relaxed);
    return true;
  }
};

// std::allocator, except for entry storage: a storage deque's blocks (512 /
// sizeof(Ent) entries, libstdc++'s node) and one-entry vectors (a proposal's
// entries, the unstable tail between Readys) come from the block pools.  A
// million proposals per cycle are allocated by the ingesting workers and
// freed by the replaying ones: from malloc, every free returns a chunk to
// another thread's arena under its lock.
template <class T>
struct BlockAlloc {
  using value_type = T;
  using is_always_equal = std::true_type;
  BlockAlloc() = default;
  template <class U>
  BlockAlloc(const BlockAlloc<U>&) {}
  static constexpr bool ENT = std::is_same<T, Ent>::value;
  static bool node(size_t n) { return ENT && sizeof(T) < 512 && n == 512 / sizeof(T); }
  static bool one(size_t n) { return ENT && n == 1 && sizeof(T) <= 64; }
  T* allocate(size_t n) {
    if (node(n)) return static_cast<T*>(BlockPool<512>::get());
    if (one(n)) return static_cast<T*>(BlockPool<64>::get());
    return std::allocator<T>().allocate(n);
  }
  void deallocate(T* p, size_t n) {
    if (node(n)) BlockPool<512>::put(p);
    else if (one(n)) BlockPool<64>::put(p);
    else std::allocator<T>().deallocate(p, n);
  }
  template <class U>
  bool operator==(const BlockAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const BlockAlloc<U>&) const { return false; }
};
using EntLog = std::deque<Ent, BlockAlloc<Ent>>;

// std::allocator whose value-less construct() default-initializes: a vector of
// integers grows without being zeroed (the batch arrays, written in full by
// the bulk workers right after they are sized)
template <class T>
struct RawAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = RawAlloc<U>;
  };
  RawAlloc() = default;
  template <class U>
  RawAlloc(const RawAlloc<U>&) {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
template <class T>
using RawVec = std::vector<T, RawAlloc<T>>;
using EntVec = std::vector<Ent, BlockAlloc<Ent>>;

}  // namespace

// ---------------------------------------------------------------- MemoryStorage
// raft/storage.go:63-248.  ents[i] has raft log position i + ents[0].Index.
struct hbn_storage {
  hbn_hard_state hs{0, 0, 0};
  Snap snap;
  // a deque: appends never move the entries already stored (a vector's
  // doubling re-copied a million groups' logs in the same Ready cycle)
  EntLog ents{Ent{}};
  std::vector<hbn_entry> view;  // hbn_storage_entries result
  // (node, group id) of every group whose raftLog reads this storage: Compact /
  // CreateSnapshot / ApplySnapshot first step the node's pending batch (the
  // reference stepped those messages before the call) and copy the entries of
  // the group's pending MsgApps, then the device's firstIndex / snapshot index
  // of the group is refreshed before its next step.
  std::vector<std::pair<hbn_node*, uint64_t>> users;

  uint64_t offset() const { return ents[0].index; }
  uint64_t last_index() const { return ents[0].index + ents.size() - 1; }
  uint64_t first_index() const { return ents[0].index + 1; }

  // Term :117-125
  int term(uint64_t i, uint64_t* t) const {
    if (i < offset()) return HBN_ECOMPACTED;
    if (i - offset() >= ents.size())
      panicf("runtime error: index out of range");  // ms.ents[i-offset] in Go
    *t = ents[i - offset()].term;
    return HB_OK;
  }
  // Entries :98-114 (returns the limited range [lo, lo+k))
  int entries(uint64_t lo, uint64_t hi, uint64_t max_size, size_t* first, size_t* count) const {
    if (lo <= offset()) return HBN_ECOMPACTED;
    if (hi > last_index() + 1) panicf("entries's hi(" + std::to_string(hi) + ") is out of bound lastindex(" +
                                      std::to_string(last_index()) + ")");
    if (ents.size() == 1) return HBN_EUNAVAILABLE;
    if (lo > hi) panicf("runtime error: slice bounds out of range");
    const size_t a = lo - offset(), b = hi - offset();
    size_t k = 0;
    if (max_size == HB_NO_LIMIT) {  // limitSize keeps everything
      k = b - a;
    } else if (b > a) {
      uint64_t size = ent_size(ents[a]);
      for (k = 1; a + k < b; ++k) {
        size += ent_size(ents[a + k]);
        if (size > max_size) break;
      }
    }
    *first = a;
    *count = k;
    return HB_OK;
  }
  // Append :217-248, straight from the caller's entries
  void append(const hbn_entry* in, uint64_t n) {
    if (n == 0) return;
    const uint64_t first = ents[0].index + 1;
    const uint64_t last = in[0].index + n - 1;
    if (last < first) return;
    uint64_t skip = 0;
    if (first > in[0].index) skip = first - in[0].index;
    const uint64_t off = in[skip].index - ents[0].index;
    if (ents.size() > off) {
      ents.resize(off);
    } else if (ents.size() != off) {
      panicf("missing log entry [last: " + std::to_string(last_index()) + ", append at: " +
             std::to_string(in[skip].index) + "]");
    }
    for (uint64_t i = skip; i < n; ++i) ents.push_back(ent_from(in[i]));
  }
};

namespace {

// ---------------------------------------------------------------- raftLog (host half)
struct Log {
  hbn_storage* st = nullptr;
  EntVec unstable;  // unstable.entries, position i + offset
  uint64_t offset = 0;
  uint64_t committed = 0, applied = 0;
  bool has_usnap = false;     // unstable.snapshot (set by the follower side's restore)
  Snap usnap;

  // newLog raft/log.go:41-63
  void init(hbn_storage* s) {
    st = s;
    offset = s->last_index() + 1;
    committed = s->first_index() - 1;
    applied = s->first_index() - 1;
  }
  uint64_t first_index() const { return has_usnap ? usnap.index + 1 : st->first_index(); }
  uint64_t last_index() const {
    if (!unstable.empty()) return offset + unstable.size() - 1;
    if (has_usnap) return usnap.index;
    return st->last_index();
  }
  // unstable.maybeTerm raft/log_unstable.go:54-73
  bool u_term(uint64_t i, uint64_t* t) const {
    if (i < offset) {
      if (has_usnap && usnap.index == i) {
        *t = usnap.term;
        return true;
      }
      return false;
    }
    if (unstable.empty() && !has_usnap) return false;
    if (i > last_index()) return false;
    if (i - offset >= unstable.size()) return false;
    *t = unstable[i - offset].term;
    return true;
  }
  // term raft/log.go:198-217
  uint64_t term(uint64_t i) const {
    const uint64_t dummy = first_index() - 1;
    if (i < dummy || i > last_index()) return 0;
    uint64_t t;
    if (u_term(i, &t)) return t;
    const int rc = st->term(i, &t);
    if (rc == HB_OK) return t;
    if (rc == HBN_ECOMPACTED) return 0;
    panicf("storage term error");
  }
  // append :89-98 + truncateAndAppend raft/log_unstable.go:100-122 (entries
  // moved in: the leader's proposals and the follower's MsgApp copies are
  // not read again)
  void append(EntVec&& ents) {
    if (ents.empty()) return;
    const uint64_t after = ents[0].index - 1;
    if (after < committed)
      panicf("after(" + std::to_string(after) + ") is out of range [committed(" + std::to_string(committed) + ")]");
    if (after == offset + unstable.size() - 1) {
      if (unstable.empty()) {
        unstable.swap(ents);
        return;
      }
    } else if (after < offset) {
      offset = after + 1;
      unstable.swap(ents);
      return;
    } else {
      unstable.resize(after + 1 - offset);
    }
    unstable.insert(unstable.end(), std::make_move_iterator(ents.begin()), std::make_move_iterator(ents.end()));
  }
  // slice raft/log.go:253-289 (copies)
  std::vector<Ent> slice(uint64_t lo, uint64_t hi, uint64_t max_size) const {
    if (lo > hi) panicf("invalid slice " + std::to_string(lo) + " > " + std::to_string(hi));
    const uint64_t fi = first_index(), len = last_index() - fi + 1;
    if (lo < fi || hi > fi + len)
      panicf("slice[" + std::to_string(lo) + "," + std::to_string(hi) + ") out of bound [" + std::to_string(fi) +
             "," + std::to_string(last_index()) + "]");
    std::vector<Ent> out;
    if (lo == hi) return out;
    if (lo < offset) {
      const uint64_t h = std::min(hi, offset);
      size_t a, k;
      const int rc = st->entries(lo, h, max_size, &a, &k);
      if (rc == HBN_ECOMPACTED)
        panicf("entries[" + std::to_string(lo) + ":" + std::to_string(h) + ") from storage is out of bound");
      if (rc == HBN_EUNAVAILABLE)
        panicf("entries[" + std::to_string(lo) + ":" + std::to_string(h) + ") is unavailable from storage");
      out.assign(st->ents.begin() + a, st->ents.begin() + a + k);
      if ((uint64_t)k < h - lo) return out;
    }
    if (hi > offset) {
      const uint64_t a = std::max(lo, offset);
      if (hi > offset + unstable.size())
        panicf("unstable.slice[" + std::to_string(a) + "," + std::to_string(hi) + ") out of bound");
      out.insert(out.end(), unstable.begin() + (a - offset), unstable.begin() + (hi - offset));
    }
    out.resize(limit_count(out, max_size));
    return out;
  }
  // slice(lo, hi, noLimit) as a visit over the entries in place (no copies)
  template <class F>
  void visit(uint64_t lo, uint64_t hi, F&& f) const {
    if (lo > hi) panicf("invalid slice " + std::to_string(lo) + " > " + std::to_string(hi));
    const uint64_t fi = first_index(), li = last_index();
    if (lo < fi || hi > li + 1)
      panicf("slice[" + std::to_string(lo) + "," + std::to_string(hi) + ") out of bound [" + std::to_string(fi) +
             "," + std::to_string(li) + "]");
    if (lo == hi) return;
    if (lo < offset) {
      const uint64_t h = std::min(hi, offset);
      size_t a, k;
      const int rc = st->entries(lo, h, HB_NO_LIMIT, &a, &k);
      if (rc == HBN_ECOMPACTED)
        panicf("entries[" + std::to_string(lo) + ":" + std::to_string(h) + ") from storage is out of bound");
      if (rc == HBN_EUNAVAILABLE)
        panicf("entries[" + std::to_string(lo) + ":" + std::to_string(h) + ") is unavailable from storage");
      auto it = st->ents.cbegin() + a;
      for (size_t i = 0; i < k; ++i, ++it) f(*it);
    }
    if (hi > offset) {
      const uint64_t a = std::max(lo, offset);
      for (uint64_t i = a; i < hi; ++i) f(unstable[i - offset]);
    }
  }
  // How many entries limitSize (raft/util.go:97-110) keeps of (lo-1, last]:
  // the first always, then each while the running Entry.Size() sum <= max.
  uint64_t limit_count_from(uint64_t lo, uint64_t max_size) const {
    const uint64_t li = last_index();
    if (lo > li) return 0;
    uint64_t size = 0, k = 0;
    bool stop = false;
    auto take = [&](const Ent& x) {
      if (stop) return;
      size += ent_size(x);
      if (k == 0 || size <= max_size) ++k;
      else stop = true;
    };
    uint64_t i = lo;  // storage part then unstable part, stopping early
    while (!stop && i <= li) {
      const uint64_t h = std::min(li + 1, i + 256);
      visit(i, h, take);
      i = h;
    }
    return k;
  }
  // entries :219-224
  std::vector<Ent> entries(uint64_t i, uint64_t max_size) const {
    if (i > last_index()) return {};
    return slice(i, last_index() + 1, max_size);
  }
  // nextEnts :135-141
  std::vector<Ent> next_ents() const {
    const uint64_t off = std::max(applied + 1, first_index());
    if (committed + 1 > off) return slice(off, committed + 1, HB_NO_LIMIT);
    return {};
  }
  Snap snapshot() const { return has_usnap ? usnap : st->snap; }
  // appliedTo :182-190
  void applied_to(uint64_t i) {
    if (i == 0) return;
    if (committed < i || i < applied)
      panicf("applied(" + std::to_string(i) + ") is out of range [prevApplied(" + std::to_string(applied) +
             "), committed(" + std::to_string(committed) + ")]");
    applied = i;
  }
  // stableTo raft/log_unstable.go:75-88
  void stable_to(uint64_t i, uint64_t t) {
    uint64_t gt;
    if (!u_term(i, &gt)) return;
    if (gt == t && i >= offset) {
      unstable.erase(unstable.begin(), unstable.begin() + (i + 1 - offset));
      offset = i + 1;
    }
  }
  void stable_snap_to(uint64_t i) {
    if (has_usnap && usnap.index == i) has_usnap = false;
  }
  // restore raft/log.go:294-298 + unstable.restore raft/log_unstable.go:94-98
  void restore(const Snap& s) {
    committed = s.index;
    offset = s.index + 1;
    unstable.clear();
    has_usnap = true;
    usnap = s;
  }
  // findConflict raft/log.go:112-123 over the entries index+1, index+2, ...
  uint64_t find_conflict(uint64_t index, const uint64_t* terms, uint64_t n) const {
    for (uint64_t k = 0; k < n; ++k)
      if (term(index + 1 + k) != terms[k]) return index + 1 + k;
    return 0;
  }
};

// ---------------------------------------------------------------- messages
// Two cache lines: a million groups hold a few of these each between Readys.
struct Msg {
  uint32_t type = 0, reject = 0;
  uint64_t to = 0, from = 0, term = 0, log_term = 0, index = 0, commit = 0, reject_hint = 0;
  EntVec entries;  // owned entries (proposals), or
  uint64_t ent_lo = 0, ent_hi = 0;  // log range [lo, hi) still to be read (MsgApp), when !owned
  bool owned = true;
  std::shared_ptr<const Snap> snap;  // MsgSnap's snapshot
};

// A group's MsgProps in flight through the device batch, arrival order: a
// vector drained from its head (steady state: one in, one out per Ready cycle,
// no allocation once the capacity is there).
struct MsgQueue {
  std::vector<Msg> v;
  size_t head = 0;
  bool empty() const { return head == v.size(); }
  Msg& front() { return v[head]; }
  Msg& back() { return v.back(); }
  void push_back(Msg&& m) { v.push_back(std::move(m)); }
  void pop_front() {
    v[head].entries = EntVec();
    if (++head == v.size()) {
      clear();
    } else if (head >= 64 && 2 * head >= v.size()) {  // a long-lived backlog: reclaim the drained part
      v.erase(v.begin(), v.begin() + head);
      head = 0;
    }
  }
  void clear() {
    v.clear();
    head = 0;
  }
};

// The ids of a group's prs in device slot order (at most HB_MAX_REPLICAS, the
// engine's limit): inline, so the per-message slot lookup stays in the group.
struct Peers {
  uint64_t id[HB_MAX_REPLICAS] = {};
  uint32_t k = 0;
  Peers() = default;
  Peers(const std::vector<uint64_t>& v) { *this = v; }
  Peers& operator=(const std::vector<uint64_t>& v) {
    if (v.size() > HB_MAX_REPLICAS) throw Fail{HBN_EUNSUPPORTED};
    k = (uint32_t)v.size();
    std::copy(v.begin(), v.end(), id);
    return *this;
  }
  operator std::vector<uint64_t>() const { return std::vector<uint64_t>(id, id + k); }
  size_t size() const { return k; }
  bool empty() const { return k == 0; }
  uint64_t operator[](size_t s) const { return id[s]; }
  uint64_t at(size_t s) const {
    if (s >= k) throw std::out_of_range("peer slot");
    return id[s];
  }
  void push_back(uint64_t x) {
    if (k == HB_MAX_REPLICAS) throw Fail{HBN_EUNSUPPORTED};
    id[k++] = x;
  }
  const uint64_t* begin() const { return id; }
  const uint64_t* end() const { return id + k; }
};

struct Soft {
  uint64_t lead = 0;
  uint32_t state = HB_STATE_FOLLOWER;
  bool operator==(const Soft& o) const { return lead == o.lead && state == o.state; }
};

bool hs_equal(const hbn_hard_state& a, const hbn_hard_state& b) {
  return a.term == b.term && a.vote == b.vote && a.commit == b.commit;
}
bool hs_empty(const hbn_hard_state& a) { return a.term == 0 && a.vote == 0 && a.commit == 0; }

constexpr uint32_t NO_SLOT = 0xFFFFFFFFu;

struct Delivered {
  bool has_soft = false;
  Soft soft;
  hbn_hard_state hard{0, 0, 0};
  bool has_last = false;
  uint64_t last_index = 0, last_term = 0;
  uint64_t snap_index = 0;
};


// Field order: what every message and every Ready cycle touches first (the
// ingestion path reads slot, flags, peers and the batch counters; the replay
// and the Ready build the terms, the log head and the message queues), the
// rarely used parts last.
struct Group {
  uint64_t id = 0;
  uint32_t slot = NO_SLOT;  // device slot, NO_SLOT while prs is empty (host-only)
  uint32_t fault = 0;
  // Ready bookkeeping flags (membership of the node's lists)
  bool touched = false, stepped = false, content = false, delivered = false;
  bool in_bx = false;
  bool bounds = false;  // storage changed: device firstIndex / snapshot index to refresh (hbn_node::bounds)
  bool pending_conf = false;
  bool reload = false;
  uint64_t bx = 0, bx_top = 0;  // entries the batch can append (sizes)
  uint64_t bxr = 0;             // term runs it can start: a noop per VoteResp / MsgHup, a MsgApp entry, a restore
  Peers peers;                  // device slot -> node id (prs, in slot order)
  uint64_t term = 0, vote = 0, lead = 0, hs_commit = 0;
  uint32_t state = HB_STATE_FOLLOWER;
  uint32_t election = 10, heartbeat = 1;
  Soft prev_soft;
  hbn_hard_state prev_hard{0, 0, 0};
  MsgQueue props;         // MsgProp in flight through the device batch, arrival order
  std::vector<Msg> msgs;  // r.msgs since the last Ready
  Log log;
  Delivered dlv;  // what the last Ready delivered for this group (commitReady input)
  // the device log index (hb_reserve_log): ring capacities reserved so far, an
  // upper bound on the term runs the device must keep (every run of the log),
  // and what the pending batch can add: entries and messages (each may start a
  // run or append a noop), and the top of its MsgApps' entries
  uint64_t lx_sz = 0, lx_tr = 0, lx_runs = 0;
  uint64_t prev_snapi = 0;
  // follower side: m.From of the message the device is stepping (HB_EV_FOLLOW)
  uint64_t cur_from = 0;
  std::vector<uint64_t> reload_nodes;  // a restored snapshot's ConfState, when it differs from peers
  bool solo = false;  // on hbn_node::solo (one peer: its tick can win an election)

  hbn_hard_state hard() const { return hbn_hard_state{term, vote, hs_commit}; }
  Soft soft() const { return Soft{lead, state}; }
  int slot_of(uint64_t node) const {
    for (uint32_t s = 0; s < peers.k; ++s)
      if (peers.id[s] == node) return (int)s;
    return -1;
  }
};

// ---------------------------------------------------------------- host threads
// (Pool and its CPU placement: hbpool.h)
using hbpool::Pool;
using hbpool::SMALL_CYCLE_MSGS;
using hbpool::PREWAKE_MIN_MSGS;

// [lo, hi) of n items for worker t of k
inline void split(size_t n, unsigned k, unsigned t, size_t* lo, size_t* hi) {
  *lo = n * t / k;
  *hi = n * (t + 1) / k;
}
// set a membership flag; true for the one caller that set it
// (a plain load first: most calls find the flag set already, and a locked
// exchange per call costs more than the rest of a small phase's per-group work)
inline bool flag_set(bool& f, bool shared = true) {
  if (__atomic_load_n(&f, __ATOMIC_RELAXED)) return false;
  if (!shared) return f = true;  // one worker: no other thread touches the flag
  return !__atomic_exchange_n(&f, true, __ATOMIC_RELAXED);
}
// a counter that several workers may bump (k > 1) or only this one
inline void bump(uint64_t& x, bool shared) {
  if (shared) __atomic_fetch_add(&x, 1, __ATOMIC_RELAXED);
  else ++x;
}

// membership lists a parallel phase appends to, one per worker (a cache line
// of its own: the workers push to them on every group)
struct alignas(64) Lists {
  std::vector<Group*> touched, content, delivered, reload, stepped, bx;
  void clear() {
    touched.clear();
    content.clear();
    delivered.clear();
    reload.clear();
    stepped.clear();
    bx.clear();
  }
};

// one worker's part of the last Ready (valid until the next call on the node)
struct alignas(64) Arena {
  std::vector<hbn_group_ready> out;
  std::vector<hbn_entry> ents;
  std::vector<hbn_message> msgs;
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off;  // per out: entries, committed, messages offsets
  std::deque<Snap> snaps;
  void clear() {
    out.clear();
    ents.clear();
    msgs.clear();
    bytes.clear();
    off.clear();
    snaps.clear();
  }
};

// host phase timers (hbn_profile): seconds and calls per phase
enum : uint32_t {
  PH_SYNC_LOADS, PH_RESERVE, PH_HB_STEP, PH_FETCH, PH_REPLAY, PH_STEPPED, PH_BUILD, PH_MERGE, PH_ADVANCE,
  PH_BULK_LOOKUP, PH_BULK_RESP, PH_BULK_PROP, PH_CLEAR, PH_COUNT_
};
struct PhaseClock {
  double* acc;
  std::chrono::steady_clock::time_point t0;
  PhaseClock(double* a) : acc(a), t0(std::chrono::steady_clock::now()) {}
  ~PhaseClock() { *acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
};
#define HBN_PHASE(n, ph) PhaseClock phase_clock_##ph(&(n)->prof[ph])

// The node's groups by id (raft/multinode.go:163 `groups map[uint64]*group`):
// open addressing over one flat array (linear probing, load <= 1/2,
// backward-shift deletion), so a lookup is one probe into a 16-byte slot
// rather than a bucket chain; the map owns its groups.
class IdMap {
 public:
  ~IdMap() { clear(); }
  size_t size() const { return n_; }
  Group* find(uint64_t id) const {
    if (!n_) return nullptr;
    for (size_t i = home(id);; i = (i + 1) & mask_) {
      const Slot& s = t_[i];
      if (!s.g) return nullptr;
      if (s.id == id) return s.g;
    }
  }
  // the slot a lookup of id starts at, for a prefetch ahead of find()
  const void* probe(uint64_t id) const { return t_.empty() ? nullptr : &t_[home(id)]; }
  void insert(uint64_t id, std::unique_ptr<Group> g) {
    if (2 * (n_ + 1) > t_.size()) grow();
    size_t i = home(id);
    while (t_[i].g) i = (i + 1) & mask_;
    t_[i] = Slot{id, g.release()};
    ++n_;
  }
  // removes and deletes id's group
  void erase(uint64_t id) {
    if (!n_) return;
    size_t i = home(id);
    while (t_[i].g && t_[i].id != id) i = (i + 1) & mask_;
    if (!t_[i].g) return;
    delete t_[i].g;
    t_[i] = Slot{};
    --n_;
    for (size_t j = (i + 1) & mask_; t_[j].g; j = (j + 1) & mask_) {  // close the gap
      const size_t h = home(t_[j].id);
      const bool stays = i <= j ? (i < h && h <= j) : (i < h || h <= j);
      if (stays) continue;
      t_[i] = t_[j];
      t_[j] = Slot{};
      i = j;
    }
  }
  template <class F>
  void each(F&& f) const {
    for (const Slot& s : t_)
      if (s.g) f(s.id, *s.g);
  }
  void clear() {
    for (Slot& s : t_) delete s.g;
    t_.clear();
    n_ = 0;
    mask_ = 0;
  }

 private:
  struct Slot {
    uint64_t id = 0;
    Group* g = nullptr;
  };
  size_t home(uint64_t id) const {
    uint64_t x = id;  // splitmix64's finalizer: sequential ids spread over the table
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return (size_t)(x ^ (x >> 31)) & mask_;
  }
  void grow() {
    std::vector<Slot> old;
    old.swap(t_);
    t_.assign(old.empty() ? 1024 : 2 * old.size(), Slot{});
    mask_ = t_.size() - 1;
    for (const Slot& s : old)
      if (s.g) {
        size_t i = home(s.id);
        while (t_[i].g) i = (i + 1) & mask_;
        t_[i] = s;
      }
  }
  std::vector<Slot> t_;
  size_t n_ = 0, mask_ = 0;
};

}  // namespace

struct hbn_node {
  double prof[PH_COUNT_] = {};
  hb_handle* h = nullptr;
  uint64_t id = 0;
  uint32_t capacity = 0, nmax = 0, W = 0;
  uint64_t max_msg = HB_NO_LIMIT, max_batch = 0;
  IdMap groups;
  std::vector<Group*> by_slot;
  std::vector<uint32_t> free_slots;
  // pending device batch (host SoA, HB_STEP_HOST_PTRS; the bulk paths size the
  // arrays and their workers write every element, so growth does not zero them)
  RawVec<uint32_t> b_group, b_info;
  RawVec<uint64_t> b_term, b_index, b_hint;
  // entries of the batch (hb_batch eoff / eterm / edesc): a MsgProp's (descriptors,
  // finite MaxSizePerMsg) and a MsgApp's (terms; payloads kept here for the replay)
  bool sized = false;
  RawVec<uint32_t> b_edesc;
  RawVec<uint64_t> b_eoff, b_eterm;
  std::vector<Ent> b_ents;  // the MsgApp entries' payloads, in batch order
  RawVec<uint32_t> b_kept;  // per message: its first entry in b_ents (MsgApp only)
  uint64_t b_nent = 0;
  // follower side (hb_batch commit; the sender ids and snapshots stay here)
  RawVec<uint64_t> b_commit, b_from;
  RawVec<uint32_t> b_snapi;  // per message: index into b_snaps, or NO_SLOT
  std::vector<Snap> b_snaps;
  bool b_app = false, b_follow = false;
  bool b_prop = false;  // the batch carries MsgProp rows (hb_step HB_STEP_MSG_PROPS)
  std::vector<Group*> reload;        // groups whose restored ConfState differs from their peers
  std::vector<Group*> pend_sz;  // groups (re)loaded on the device whose entry sizes are still to push
  std::vector<Group*> pend_tr;  // ... and whose older log term runs are still to push
  std::vector<Group*> stepped;  // groups whose raft.Step runs in the pending batch
  std::vector<Group*> bx;       // groups with messages in the pending batch (Group::bx)
  std::vector<Group*> solo;     // groups that had one peer when listed (Group::solo; pruned by hbn_tick)
  // the step's compact event words (hb_events_to_host, pinned: the device writes them)
  uint64_t* w_words = nullptr;
  uint64_t w_cap = 0;
  uint32_t* w_counts = nullptr;
  uint64_t* w_total = nullptr;
  uint32_t n_chunks = 0, chunk_groups = 0;
  std::vector<uint64_t> w_off;  // first word of each chunk
  // host threads (hbn_set_threads) and their per-phase lists
  std::unique_ptr<Pool> pool;
  std::vector<Lists> lists;
  std::vector<Arena> arenas;
  // CreateGroup loads, coalesced into one hb_load_groups / hb_load_timers per slot run
  std::vector<std::pair<uint32_t, hb_group>> pend_rec;
  std::vector<std::pair<uint32_t, hb_timer>> pend_tm;
  std::vector<Group*> bounds;  // groups whose storage changed since the last device sync (Group::bounds)
  // Ready bookkeeping (raft/multinode.go:166-322)
  std::vector<Group*> touched;    // rds candidates since the last delivery (Group::touched)
  std::vector<Group*> content;    // groups whose state-derived Ready may be non-empty (lazy, Group::content)
  std::vector<Group*> delivered;  // groups of the last Ready (Group::delivered)
  bool awaiting_advance = false;
  // the last Ready: one record per group (contiguous), its entries / messages in
  // the arena of the worker that built it
  std::unique_ptr<hbn_group_ready[]> r_out;  // (not value-initialised: every record is written)
  size_t r_cap = 0, r_n = 0;
};

namespace {

// ---------------------------------------------------------------- device records
uint32_t ref_of(const Group& g, uint64_t self, uint64_t node) {
  if (node == 0) return HB_REF_NONE;
  const int s = g.slot_of(node);
  if (s >= 0) return (uint32_t)s;
  if (node == self) return HB_REF_SELF;
  return HB_REF_OTHER;
}
uint64_t id_of_ref(const Group& g, uint64_t self, uint32_t ref, uint64_t keep) {
  if (ref == HB_REF_NONE) return 0;
  if (ref == HB_REF_SELF) return self;
  if (ref == HB_REF_OTHER) return keep;  // an id outside prs: only the host knows it
  if (ref < g.peers.size()) return g.peers[ref];
  return keep;
}

// [term_first, term_last]: the run of i in [first-1, last] with term(i) == Term.
void term_run(const Group& g, uint64_t* tf, uint64_t* tl) {
  const uint64_t lo = g.log.first_index() - 1, last = g.log.last_index();
  uint64_t i = last + 1;
  while (i > lo && g.log.term(i - 1) == g.term) --i;
  if (i == last + 1) {
    *tf = HB_NO_INDEX;
    *tl = 0;
  } else {
    *tf = i;
    *tl = last;
  }
}

void check(int rc) {
  if (rc != HB_OK) throw Fail{rc};
}

// A fresh device record from the host state; prs Progress as given.
hb_group make_record(const hbn_node* n, const Group& g, const std::vector<hb_progress>& prs) {
  hb_group r;
  std::memset(&r, 0, sizeof(r));
  r.term = g.term;
  r.committed = g.log.committed;
  r.first_index = g.log.first_index();
  r.last_index = g.log.last_index();
  term_run(g, &r.term_first, &r.term_last);
  r.snap_index = g.log.snapshot().index;
  r.state = g.state;
  r.n = (uint32_t)g.peers.size();
  const int ss = g.slot_of(n->id);
  r.self_slot = ss >= 0 ? (uint32_t)ss : HB_SLOT_NONE;
  r.lead = ref_of(g, n->id, g.lead);
  r.vote = ref_of(g, n->id, g.vote);
  // r.Commit (HardState.Commit) is committed, or 0 until the first Step of a
  // group created with an empty HardState (raft/raft.go:466,488,759)
  r.commit_zero = (g.hs_commit == 0 && g.log.committed != 0) ? 1u : 0u;
  for (size_t s = 0; s < prs.size(); ++s) r.pr[s] = prs[s];
  return r;
}

// list a one-peer group for hbn_tick's noop reservation
void note_solo(hbn_node* n, Group& g) {
  if (g.peers.size() == 1 && !g.solo) {
    g.solo = true;
    n->solo.push_back(&g);
  }
}

uint32_t alloc_slot(hbn_node* n) {
  if (n->free_slots.empty()) throw Fail{HB_ENOMEM};
  const uint32_t s = n->free_slots.back();
  n->free_slots.pop_back();
  return s;
}

// ---------------------------------------------------------------- event replay
void touch_into(std::vector<Group*>& v, Group& g, bool shared = true) {
  if (flag_set(g.touched, shared)) v.push_back(&g);
}
void touch(hbn_node* n, Group& g) { touch_into(n->touched, g, false); }  // (the API thread alone)

void mark_stepped(std::vector<Group*>& touched, Group& g, bool shared = true) {
  g.hs_commit = g.log.committed;  // r.Commit = r.raftLog.committed after Step (raft/raft.go:488)
  touch_into(touched, g, shared);
}

// worker lists merged into the node's, in worker order
void merge(std::vector<Group*>& dst, std::vector<Lists>& ls, std::vector<Group*> Lists::*m) {
  for (Lists& l : ls) {
    dst.insert(dst.end(), (l.*m).begin(), (l.*m).end());
    (l.*m).clear();
  }
}

// r.msgs entries are read from the log when the Ready is built; before the log
// can lose them (Advance's stableTo, a Ready withheld until Advance) they are copied.
void materialize(Group& g) {
  for (Msg& m : g.msgs) {
    if (m.owned) continue;
    m.entries.clear();
    if (m.ent_hi > m.ent_lo) g.log.visit(m.ent_lo, m.ent_hi, [&](const Ent& x) { m.entries.push_back(x); });
    m.owned = true;
  }
}

// a new message at the end of g's r.msgs (raft.send, raft/raft.go:227-236)
Msg& base_msg(const hbn_node* n, Group& g, uint32_t type, uint64_t to) {
  Msg& m = g.msgs.emplace_back();
  m.type = type;
  m.to = to;
  m.from = n->id;
  m.term = g.term;
  return m;
}

// ---- follower side (raft/raft.go:616-707): the device decided, the host log follows
uint64_t batch_ent_end(const hbn_node* n, uint64_t x) {
  return x + 1 < n->b_eoff.size() ? n->b_eoff[x + 1] : n->b_nent;
}

// HB_FOLLOW_APPEND: raftLog.maybeAppend of batch message x appended its entries
// from the first conflict (raft/log.go:72-88 -> append :89-98).
void follower_append(hbn_node* n, Group& g, uint64_t x) {
  if (x >= n->b_eoff.size()) panicf("device appended for a message outside the batch");
  const uint64_t e0 = n->b_eoff[x], e1 = batch_ent_end(n, x), index = n->b_index[x];
  const uint64_t ci = g.log.find_conflict(index, n->b_eterm.data() + e0, e1 - e0);
  if (ci == 0) panicf("device appended entries the host log already holds");
  materialize(g);  // pending MsgApps of this group read entries the append may cut
  const uint64_t k0 = n->b_kept[x];  // (the message's entries, contiguous in b_ents)
  EntVec ents(n->b_ents.begin() + (k0 + (ci - index - 1)), n->b_ents.begin() + (k0 + (e1 - e0)));
  g.log.append(std::move(ents));
}

// HB_FOLLOW_RESTORE: restore of batch message x's snapshot (raft/raft.go:684-707)
void follower_restore(hbn_node* n, Group& g, uint64_t x, Lists& L) {
  if (x >= n->b_snapi.size() || n->b_snapi[x] == NO_SLOT) panicf("device restored a snapshot the host does not hold");
  const Snap& s = n->b_snaps[n->b_snapi[x]];
  materialize(g);
  g.log.restore(s);
  // r.prs from the ConfState (every Progress reset, the device did that for the
  // current slots); a different peer set is reloaded after the batch
  std::vector<uint64_t> a = s.nodes, b = g.peers;
  std::sort(a.begin(), a.end());
  std::sort(b.begin(), b.end());
  if (a != b) {
    g.reload_nodes = s.nodes;
    if (!g.reload) {
      g.reload = true;
      L.reload.push_back(&g);
    }
  }
}

// HB_EV_RESP: the follower side's r.send of a response (raft/raft.go:227-236)
void follower_resp(hbn_node* n, Group& g, const hb_event& e) {
  const uint32_t kind = e.aux & 7u;
  const uint64_t to = e.to < g.peers.size() ? g.peers[e.to] : g.cur_from;  // HB_REF_OTHER: the sender
  const uint32_t type = kind == HB_RESP_APP ? HB_MSG_APP_RESP
                                            : (kind == HB_RESP_HEARTBEAT ? HB_MSG_HEARTBEAT_RESP : HB_MSG_VOTE_RESP);
  const uint64_t li = g.log.last_index();
  Msg& m = base_msg(n, g, type, to);
  m.reject = (e.aux & HB_RESP_REJECT) ? 1 : 0;
  if (kind == HB_RESP_APP) {
    m.index = e.x;
    if (m.reject) m.reject_hint = li;  // handleAppendEntries :661-663
  }
}

void on_event(hbn_node* n, Group& g, const hb_event& e, Lists& L) {
  if (g.fault) return;
  switch (e.type) {
    case HB_EV_TERM:  // reset (raft/raft.go:334-349)
      // Vote, lead and state arrive with the transition's STATE event, which the
      // device emits only when they differ from before the transition (a
      // candidate re-campaigning keeps Vote = self, so no STATE follows).
      g.term = e.x;
      g.pending_conf = false;
      break;
    case HB_EV_STATE: {
      const uint32_t st = (uint32_t)(e.x & 0xFF), lref = (uint32_t)((e.x >> 8) & 0xFF),
                     vref = (uint32_t)((e.x >> 16) & 0xFF);
      g.state = st;
      g.lead = (e.aux & HB_STATE_OTH_LEAD) ? g.cur_from : id_of_ref(g, n->id, lref, g.lead);
      g.vote = (e.aux & HB_STATE_OTH_VOTE) ? g.cur_from : id_of_ref(g, n->id, vref, g.vote);
      g.pending_conf = false;  // every become* runs reset
      if (st == HB_STATE_LEADER) {
        // becomeLeader's scan of the uncommitted tail (raft/raft.go:415-424)
        for (const Ent& x : g.log.entries(g.log.committed + 1, HB_NO_LIMIT)) {
          if (x.type != HBN_ENTRY_CONF_CHANGE) continue;
          if (g.pending_conf) {
            g.fault = HBN_FAULT_DOUBLE_CONF;
            return;
          }
          g.pending_conf = true;
        }
      }
      break;
    }
    case HB_EV_COMMIT:
      g.log.committed = e.x;
      break;
    case HB_EV_LAST: {
      const uint64_t li = g.log.last_index();
      EntVec ents;
      if (e.aux == 1) {
        ents.resize(1);  // becomeLeader's pb.Entry{Data: nil}
      } else {
        if (g.props.empty()) panicf("device appended entries without a pending proposal");
        ents = std::move(g.props.front().entries);
        g.props.pop_front();
        for (Ent& x : ents) {  // stepLeader MsgProp (raft/raft.go:500-513)
          if (x.type == HBN_ENTRY_CONF_CHANGE) {
            if (g.pending_conf) x = Ent{};
            g.pending_conf = true;
          }
        }
      }
      if (li + ents.size() != e.x) panicf("device lastIndex disagrees with the host log");
      for (size_t i = 0; i < ents.size(); ++i) {  // appendEntry (raft/raft.go:351-360)
        ents[i].term = g.term;
        ents[i].index = li + 1 + i;
      }
      g.log.append(std::move(ents));
      break;
    }
    case HB_EV_APP: {  // sendAppend (raft/raft.go:261-281)
      const uint64_t to = g.peers.at(e.to);
      const uint64_t lt = (e.aux & 1u) ? g.term : g.log.term(e.x);  // aux 1: the device saw term(Index) == Term
      // entries(Index+1, maxMsgSize): (Index, last] under noLimit, one entry under 0
      const uint64_t li = g.log.last_index();
      uint64_t hi;
      if (e.x + 1 > li) hi = e.x + 1;
      else if (n->max_msg == 0) hi = e.x + 2;
      else if (n->max_msg == HB_NO_LIMIT) hi = li + 1;
      else hi = e.x + 1 + g.log.limit_count_from(e.x + 1, n->max_msg);  // limitSize, as the device cut it
      Msg& m = base_msg(n, g, HB_MSG_APP, to);
      m.index = e.x;
      m.log_term = lt;
      m.owned = false;
      m.ent_lo = e.x + 1;
      m.ent_hi = hi;
      m.commit = g.log.committed;
      break;
    }
    case HB_EV_SNAP: {  // sendAppend, snapshot branch (:246-260)
      const uint64_t to = g.peers.at(e.to);
      auto snap = std::make_shared<const Snap>(g.log.snapshot());
      base_msg(n, g, HB_MSG_SNAP, to).snap = std::move(snap);
      break;
    }
    case HB_EV_HEARTBEAT: {  // sendHeartbeat (:285-299)
      const uint64_t to = g.peers.at(e.to);
      base_msg(n, g, HB_MSG_HEARTBEAT, to).commit = e.x;
      break;
    }
    case HB_EV_VOTE: {  // campaign (:429-443)
      const uint64_t to = g.peers.at(e.to);
      const uint64_t lt = g.log.term(g.log.last_index());
      Msg& m = base_msg(n, g, HB_MSG_VOTE, to);
      m.index = e.x;
      m.log_term = lt;
      break;
    }
    case HB_EV_PROP_FWD: {  // stepFollower MsgProp (:617-624): m.To = r.lead; r.send(m)
      if (g.props.empty()) panicf("device forwarded a proposal the host does not hold");
      Msg m = std::move(g.props.front());
      g.props.pop_front();
      m.to = id_of_ref(g, n->id, e.to, g.lead);
      m.from = n->id;  // MsgProp keeps its own Term
      g.msgs.push_back(std::move(m));
      break;
    }
    case HB_EV_PROP_DROP:
      if (!g.props.empty()) g.props.pop_front();
      break;
    case HB_EV_FAULT:
      g.fault = e.aux;
      g.props.clear();
      break;
    case HB_EV_FOLLOW:
      if (e.aux == HB_FOLLOW_STEP) {
        if (e.x >= n->b_from.size()) panicf("device stepped a message outside the batch");
        g.cur_from = n->b_from[e.x];
      } else if (e.aux == HB_FOLLOW_APPEND) {
        follower_append(n, g, e.x);
      } else if (e.aux == HB_FOLLOW_RESTORE) {
        follower_restore(n, g, e.x, L);
      }
      break;
    case HB_EV_RESP:
      follower_resp(n, g, e);
      break;
    default:
      panicf("unknown device event type " + std::to_string(e.type));
  }
}

// The step's events: the device's compact words (hb_events_to_host; one word
// per bcastAppend), replayed per group in order.  Partition p's groups have
// their words in chunks 2p and 2p+1, so workers take contiguous partition
// ranges (balanced by words) and never share a group.
void consume_events(hbn_node* n) {
  if (!n->w_counts) {
    check(hb_event_words_chunks(n->h, &n->n_chunks, &n->chunk_groups));
    void* p = nullptr;
    check(hb_alloc_pinned(n->n_chunks * 4ull + 64, &p));
    n->w_counts = static_cast<uint32_t*>(p);
    check(hb_alloc_pinned(64, &p));
    n->w_total = static_cast<uint64_t*>(p);
  }
  auto fetch0 = std::chrono::steady_clock::now();
  for (int attempt = 0;; ++attempt) {
    check(hb_events_to_host(n->h, n->w_words, n->w_cap, n->w_counts, n->w_total));
    check(hb_sync(n->h));
    if (*n->w_total <= n->w_cap) break;
    if (attempt) panicf("device event words exceed their buffer");
    if (n->w_words) (void)hb_free_pinned(n->w_words);
    n->w_words = nullptr;
    n->w_cap = 0;
    const uint64_t cap = *n->w_total + *n->w_total / 4 + 4096;
    void* p = nullptr;
    check(hb_alloc_pinned(cap * 8, &p));
    n->w_words = static_cast<uint64_t*>(p);
    n->w_cap = cap;
  }
  n->prof[PH_FETCH] += std::chrono::duration<double>(std::chrono::steady_clock::now() - fetch0).count();
  const uint64_t total = *n->w_total;
  if (total == 0) return;
  HBN_PHASE(n, PH_REPLAY);
  const uint32_t nc = n->n_chunks, np = nc / 2;
  n->w_off.resize(nc + 1);
  uint64_t run = 0;
  for (uint32_t c = 0; c < nc; ++c) {
    n->w_off[c] = run;
    run += n->w_counts[c];
  }
  n->w_off[nc] = run;
  if (run != total) panicf("device event word counts disagree");
  const unsigned k = n->pool->ways_small(total, 16384, 2048);
  n->pool->run(
      [&](unsigned t) {
        // partitions [p0, p1) of worker t: an equal share of the words
        uint32_t p0 = 0, p1 = np;
        if (k > 1) {
          const uint64_t w0 = total * t / k, w1 = total * (t + 1) / k;
          auto at = [&](uint64_t w) {  // first partition whose words start at or after w
            return (uint32_t)(std::lower_bound(n->w_off.begin(), n->w_off.begin() + nc, w) - n->w_off.begin() + 1) / 2;
          };
          p0 = t == 0 ? 0 : at(w0);
          p1 = t + 1 == k ? np : at(w1);
        }
        Lists& L = n->lists[t];
        const uint64_t* W = n->w_words;
        const bool ahead = total >= 65536;  // (a small node's groups sit in cache already)
        for (uint32_t p = p0; p < p1; ++p) {
          for (uint64_t i = n->w_off[2 * p], end = n->w_off[2 * p + 2]; i < end; ++i) {
            if (ahead && i + 16 < end) {  // the group of a word ahead: its hot lines (flags .. log head)
              const uint32_t ps = p * n->chunk_groups + ((uint32_t)(W[i + 16] >> 16) & 0xFF);
              if (ps < n->by_slot.size())
                if (const char* q = reinterpret_cast<const char*>(n->by_slot[ps]))
                  for (int l = 0; l < 5; ++l) __builtin_prefetch(q + 64 * l);
            }
            if (ahead && i + 8 < end) {  // ... and, nearer, the buffers it points to
              const uint32_t ps = p * n->chunk_groups + ((uint32_t)(W[i + 8] >> 16) & 0xFF);
              if (ps < n->by_slot.size())
                if (const Group* q = n->by_slot[ps]) {
                  __builtin_prefetch(q->msgs.data() + q->msgs.size());
                  if (!q->props.empty()) __builtin_prefetch(q->props.v.data() + q->props.head);
                }
            }
            const uint64_t w = W[i];
            const uint32_t type = (uint32_t)w & 0xF;
            if (type == HB_EVW_CONT) continue;
            const uint32_t slot = p * n->chunk_groups + ((uint32_t)(w >> 16) & 0xFF);
            if (slot >= n->by_slot.size() || !n->by_slot[slot]) continue;
            Group& g = *n->by_slot[slot];
            hb_event e;
            e.group = slot;
            e.x = w >> 24;
            if (((w >> 11) & 1u) && i + 1 < end) e.x |= (W[i + 1] >> 4) << 40;
            const uint32_t to = (uint32_t)(w >> 4) & 0x7F;
            if (type == HB_EVW_BCAST || type == HB_EVW_VBCAST) {  // to every slot of the mask, in slot order
              e.type = type == HB_EVW_BCAST ? HB_EV_APP : HB_EV_VOTE;
              e.aux = (uint16_t)((w >> 12) & 0xF);
              for (uint32_t s = 0; s < 7; ++s)
                if ((to >> s) & 1u) {
                  e.to = (uint8_t)s;
                  on_event(n, g, e, L);
                }
            } else {
              e.type = (uint8_t)type;
              e.to = (uint8_t)to;
              e.aux = (uint16_t)((w >> 12) & 0xF);
              on_event(n, g, e, L);
            }
            mark_stepped(L.touched, g, k > 1);
          }
        }
      },
      k);
  merge(n->touched, n->lists, &Lists::touched);
  merge(n->reload, n->lists, &Lists::reload);
}

// Push the queued CreateGroup records and timers to the device, one call per
// run of consecutive slots (a million groups load in a few calls).
template <class T, class F>
void load_runs(std::vector<std::pair<uint32_t, T>>& v, F&& load) {
  if (v.empty()) return;
  std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<T> run;
  size_t i = 0;
  while (i < v.size()) {
    size_t j = i;
    run.clear();
    while (j < v.size() && v[j].first == v[i].first + (j - i)) run.push_back(v[j++].second);
    check(load(v[i].first, (uint32_t)run.size(), run.data()));
    i = j;
  }
  v.clear();
}

// ---- the device log index (include/hipbatch.h, hb_reserve_log) ----
// The term runs of [lo, hi] of g's log, newest first (binary search per run:
// log terms never decrease with the index).
template <class F>
void log_runs(const Group& g, uint64_t lo, uint64_t hi, F&& f) {
  while (hi + 1 > lo) {
    const uint64_t t = g.log.term(hi);
    uint64_t a = lo, b = hi;  // smallest i in [lo, hi] with term(i) == t
    while (a < b) {
      const uint64_t mid = a + (b - a) / 2;
      if (g.log.term(mid) == t) b = mid;
      else a = mid + 1;
    }
    f(a, t);
    if (a == lo) break;
    hi = a - 1;
  }
}
// every term run of [firstIndex - 1, lastIndex]: the device's runs plus its current-term run
uint64_t count_runs(const Group& g) {
  uint64_t k = 0;
  log_runs(g, g.log.first_index() - 1, g.log.last_index(), [&](uint64_t, uint64_t) { ++k; });
  return k;
}
uint64_t pow2_at_least(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Capacity for g's rings before a step that can append up to extra_sz entries
// (and MsgApp entries up to g.bx_top) and start up to extra_runs term runs:
// sizes cover [firstIndex - 1, the new lastIndex], runs every run of the log
// plus the new ones.  Requested with 2x headroom (amortised); the exact run
// count is taken only when the bound grows past the reserved capacity.
void want_log(const hbn_node* n, Group& g, uint64_t extra_sz, uint64_t extra_runs, std::vector<uint32_t>& slots,
              std::vector<uint64_t>& szc, std::vector<uint64_t>& trc) {
  uint64_t need_sz = 0;
  if (n->sized) {
    const uint64_t lo = g.log.first_index() - 1;
    need_sz = std::max(g.log.last_index(), g.bx_top) + extra_sz - lo + 1;
  }
  uint64_t need_tr = g.lx_runs + extra_runs + 1;
  if (need_tr > g.lx_tr) {
    g.lx_runs = count_runs(g);
    need_tr = g.lx_runs + extra_runs + 1;
  }
  const bool gs = need_sz > g.lx_sz, gt = need_tr > g.lx_tr;
  if (!gs && !gt) return;
  if (gs) g.lx_sz = pow2_at_least(2 * need_sz);
  if (gt) g.lx_tr = pow2_at_least(2 * need_tr);
  slots.push_back(g.slot);
  szc.push_back(gs ? g.lx_sz : 0);
  trc.push_back(gt ? g.lx_tr : 0);
}
void reserve(hbn_node* n, const std::vector<uint32_t>& slots, const std::vector<uint64_t>& szc,
             const std::vector<uint64_t>& trc) {
  if (!slots.empty())
    check(hb_reserve_log(n->h, (uint32_t)slots.size(), slots.data(), n->sized ? szc.data() : nullptr, trc.data()));
}

// Finite MaxSizePerMsg: the sizes of every entry of (re)loaded groups
// (hb_load_entry_sizes: (firstIndex - 1, lastIndex]), so the device's limitSize
// serves a follower at any Next in the log.
void push_sizes(hbn_node* n) {
  if (n->pend_sz.empty()) return;
  std::vector<uint32_t> slots, cnt, sizes;
  std::vector<uint32_t> rs;
  std::vector<uint64_t> rz, rt;
  for (Group* g : n->pend_sz) {
    if (g->slot == NO_SLOT) continue;
    const uint64_t li = g->log.last_index(), fi = g->log.first_index();
    const uint64_t k = li + 1 - fi;
    slots.push_back(g->slot);
    cnt.push_back((uint32_t)k);
    g->log.visit(fi, li + 1, [&](const Ent& x) { sizes.push_back((uint32_t)ent_size(x)); });
    g->lx_sz = 0;  // a reload: reserve afresh
    want_log(n, *g, 0, 0, rs, rz, rt);
  }
  n->pend_sz.clear();
  reserve(n, rs, rz, rt);
  if (!slots.empty())
    check(hb_load_entry_sizes(n->h, (uint32_t)slots.size(), slots.data(), cnt.data(), sizes.data()));
}

// The follower side's raftLog.term() lookups below a (re)loaded group's
// current-term run: every older run down to firstIndex - 1 (hb_load_term_runs).
void push_term_runs(hbn_node* n) {
  if (n->pend_tr.empty()) return;
  std::vector<uint32_t> slots, cnt;
  std::vector<uint64_t> runs;
  std::vector<uint32_t> rs;
  std::vector<uint64_t> rz, rt;
  for (Group* g : n->pend_tr) {
    if (g->slot == NO_SLOT) continue;
    uint64_t tf, tl;
    term_run(*g, &tf, &tl);
    const uint64_t lo = g->log.first_index() - 1;
    std::vector<std::pair<uint64_t, uint64_t>> rr;  // newest first
    if (tf != lo) log_runs(*g, lo, tf == HB_NO_INDEX ? g->log.last_index() : tf - 1,
                           [&](uint64_t a, uint64_t t) { rr.emplace_back(a, t); });
    slots.push_back(g->slot);
    cnt.push_back((uint32_t)rr.size());
    for (auto it = rr.rbegin(); it != rr.rend(); ++it) {
      runs.push_back(it->first);
      runs.push_back(it->second);
    }
    g->lx_tr = 0;  // a reload: reserve afresh, with the exact count
    g->lx_runs = rr.size() + (tf != HB_NO_INDEX ? 1 : 0);
    want_log(n, *g, 0, 0, rs, rz, rt);
  }
  n->pend_tr.clear();
  reserve(n, rs, rz, rt);
  if (!slots.empty())
    check(hb_load_term_runs(n->h, (uint32_t)slots.size(), slots.data(), cnt.data(), runs.data()));
}

// Before hb_step: room in every batch group's rings for what the batch can add
// (workers over disjoint ranges of the batch's groups).
void reserve_batch(hbn_node* n) {
  const size_t nb = n->bx.size();
  const unsigned k = n->pool->ways(nb, 4096);
  std::vector<std::vector<uint32_t>> rs(k);
  std::vector<std::vector<uint64_t>> rz(k), rt(k);
  n->pool->run(
      [&](unsigned t) {
        size_t lo, hi;
        split(nb, k, t, &lo, &hi);
        for (size_t i = lo; i < hi; ++i) {
          Group& g = *n->bx[i];
          if (g.slot != NO_SLOT) want_log(n, g, g.bx, g.bxr, rs[t], rz[t], rt[t]);
          g.lx_runs += g.bxr;  // after the step: the bound on the log's runs grows by what it could add
          g.bx = g.bx_top = g.bxr = 0;
          g.in_bx = false;
        }
      },
      k);
  for (unsigned t = 1; t < k; ++t) {
    rs[0].insert(rs[0].end(), rs[t].begin(), rs[t].end());
    rz[0].insert(rz[0].end(), rz[t].begin(), rz[t].end());
    rt[0].insert(rt[0].end(), rt[t].begin(), rt[t].end());
  }
  reserve(n, rs[0], rz[0], rt[0]);
  n->bx.clear();
}

void sync_loads(hbn_node* n) {
  load_runs(n->pend_rec, [&](uint32_t f, uint32_t c, const hb_group* r) { return hb_load_groups(n->h, f, c, r); });
  load_runs(n->pend_tm, [&](uint32_t f, uint32_t c, const hb_timer* t) { return hb_load_timers(n->h, f, c, t); });
  push_sizes(n);
  push_term_runs(n);
  if (!n->bounds.empty()) {  // storage compactions / snapshots since the last step, one call
    std::vector<uint32_t> slots;
    std::vector<uint64_t> first, snap;
    for (Group* g : n->bounds) {
      g->bounds = false;
      if (g->slot == NO_SLOT) continue;
      slots.push_back(g->slot);
      first.push_back(g->log.first_index());
      snap.push_back(g->log.snapshot().index);
    }
    n->bounds.clear();
    if (!slots.empty())
      check(hb_set_log_bounds(n->h, (uint32_t)slots.size(), slots.data(), first.data(), snap.data()));
  }
}

void reload_prs(hbn_node* n, Group& g, const std::vector<uint64_t>& new_peers,
                const std::vector<std::pair<uint64_t, uint64_t>>& fresh, bool restored);

void flush(hbn_node* n) {
  {
    HBN_PHASE(n, PH_SYNC_LOADS);
    sync_loads(n);
  }
  if (n->b_group.empty()) return;
  hb_batch b{};
  b.n = n->b_group.size();
  b.group = n->b_group.data();
  b.info = n->b_info.data();
  b.term = n->b_term.data();
  b.index = n->b_index.data();
  b.hint = n->b_hint.data();
  b.props = nullptr;
  if (n->sized || n->b_app) {
    b.n_edesc = n->b_nent;
    b.eoff = n->b_eoff.data();
    if (n->sized) b.edesc = n->b_edesc.data();
    if (n->b_app) b.eterm = n->b_eterm.data();
  }
  if (n->b_follow) b.commit = n->b_commit.data();
  {
    HBN_PHASE(n, PH_RESERVE);
    reserve_batch(n);
  }
  {
    HBN_PHASE(n, PH_HB_STEP);
    check(hb_step(n->h, &b, HB_STEP_HOST_PTRS | (n->b_prop ? HB_STEP_MSG_PROPS : 0u)));
  }
  // A small cycle's replay and Ready build split over the partners: they wake
  // while the device steps and spin between the cycle's phases.  A cycle of
  // many messages runs its phases on the whole pool for far longer than a
  // wake-up, and a tiny one stays on the caller: no spinning for either.
  n->pool->set_small_cycle(b.n < SMALL_CYCLE_MSGS);
  if (b.n >= PREWAKE_MIN_MSGS) n->pool->prewake(n->pool->small_ways());
  consume_events(n);
  {
    HBN_PHASE(n, PH_STEPPED);
    const size_t ns = n->stepped.size();
    const unsigned k = n->pool->ways(ns, 16384);
    n->pool->run(
        [&](unsigned t) {
          size_t lo, hi;
          split(ns, k, t, &lo, &hi);
          std::vector<Group*>& touched = k == 1 ? n->touched : n->lists[t].touched;
          for (size_t i = lo; i < hi; ++i) {
            if (i + 8 < hi) __builtin_prefetch(n->stepped[i + 8]);
            Group& g = *n->stepped[i];
            g.stepped = false;
            mark_stepped(touched, g, k > 1);
          }
        },
        k);
    if (k > 1) merge(n->touched, n->lists, &Lists::touched);
    n->stepped.clear();
  }
  HBN_PHASE(n, PH_CLEAR);
  n->b_group.clear();
  n->b_info.clear();
  n->b_term.clear();
  n->b_index.clear();
  n->b_hint.clear();
  n->b_edesc.clear();
  n->b_eoff.clear();
  n->b_eterm.clear();
  n->b_ents.clear();
  n->b_kept.clear();
  n->b_nent = 0;
  n->b_commit.clear();
  n->b_from.clear();
  n->b_snapi.clear();
  n->b_snaps.clear();
  n->b_app = n->b_follow = n->b_prop = false;
  // restored snapshots whose ConfState differs from the peers: r.prs = the
  // ConfState's nodes, every Progress as setProgress made it (raft/raft.go:700-705)
  for (Group* g : n->reload) {
    g->reload = false;
    if (g->fault) continue;
    std::vector<std::pair<uint64_t, uint64_t>> fresh;
    for (uint64_t id : g->reload_nodes) fresh.emplace_back(id, g->log.last_index() + 1);
    reload_prs(n, *g, g->reload_nodes, fresh, true);
    g->reload_nodes.clear();
  }
  n->reload.clear();
}

bool is_response(uint32_t t) {  // IsResponseMsg raft/util.go:53-55
  return t == HB_MSG_APP_RESP || t == HB_MSG_VOTE_RESP || t == HB_MSG_HEARTBEAT_RESP || t == HB_MSG_UNREACHABLE;
}

// One message of the Ready cycle into the device batch (raft/multinode.go:224-237).
void push(hbn_node* n, Group& g, uint32_t type, uint64_t from, bool reject, uint64_t term, uint64_t index,
          uint64_t hint, uint64_t commit = 0, bool voted = false) {
  const int s = g.slot_of(from);
  const uint32_t fs = s >= 0 ? (uint32_t)s : HB_SLOT_NONE;
  touch(n, g);
  if (g.slot == NO_SLOT) {
    // prs is empty: every response is filtered (raft/multinode.go:235); anything
    // else would step a raft with no progress at all.
    if (is_response(type)) return;
    throw Fail{HBN_EUNSUPPORTED};
  }
  if (n->b_group.size() >= n->max_batch) flush(n);
  if (type == HB_MSG_PROP) n->b_prop = true;
  n->b_group.push_back(g.slot);
  n->b_info.push_back(HB_INFO(type, fs, reject) | (voted ? HB_INFO_VOTED : 0u));
  n->b_term.push_back(term);
  n->b_index.push_back(index);
  n->b_hint.push_back(hint);
  n->b_eoff.push_back(n->b_nent);  // a MsgProp's / MsgApp's entries follow (push_entry)
  n->b_commit.push_back(commit);
  n->b_from.push_back(from);
  n->b_snapi.push_back(NO_SLOT);
  n->b_kept.push_back((uint32_t)n->b_ents.size());
  g.bx++;  // a noop (becomeLeader) at most
  if (type == HB_MSG_HUP || type == HB_MSG_VOTE_RESP || type == HB_MSG_SNAP) g.bxr++;  // a noop's / restore's run
  if (!g.in_bx) {
    g.in_bx = true;
    n->bx.push_back(&g);
  }
  if ((s >= 0 || !is_response(type)) && !g.stepped) {
    g.stepped = true;
    n->stepped.push_back(&g);
  }
}

Group& group_of(hbn_node* n, uint64_t id) {
  Group* g = n->groups.find(id);
  if (!g) throw Fail{HBN_ENOGROUP};
  return *g;
}

// ---- bulk ingestion (hbn_step_many / hbn_propose_many) ----
// Pass 1 (parallel): each message's group, and whether it takes the bulk path
// (an existing, unfaulted group; for steps a response type).  The rest go one
// by one through the single-message path, which raises the reference's errors
// at the right position.
struct BulkRun {
  RawVec<Group*> gp;      // (every element written by the lookup's workers)
  RawVec<uint8_t> fast;
};
template <class Ok>
void bulk_lookup(hbn_node* n, uint64_t count, const uint64_t* gids, BulkRun& br, Ok&& ok) {
  HBN_PHASE(n, PH_BULK_LOOKUP);
  br.gp.resize(count);
  br.fast.resize(count);
  const unsigned k = n->pool->ways_small(count, 4096, n->pool->small_bulk());
  n->pool->run(
      [&](unsigned t) {
        size_t lo, hi;
        split(count, k, t, &lo, &hi);
        for (size_t i = lo; i < hi; ++i) {
          if (i + 16 < hi) __builtin_prefetch(n->groups.probe(gids[i + 16]));
          Group* g = n->groups.find(gids[i]);
          br.gp[i] = g;
          br.fast[i] = 0;
          if (!g) continue;
          br.fast[i] = !g->fault && ok(i, *g);
        }
      },
      k);
}

// Whether bad(i) holds for some i in [0, count) (argument checks of a bulk call,
// before anything is queued), workers over disjoint ranges.
template <class Bad>
bool bulk_any(hbn_node* n, uint64_t count, Bad&& bad) {
  const unsigned k = n->pool->ways(count, 65536);
  std::vector<uint8_t> hit(k, 0);
  n->pool->run(
      [&](unsigned t) {
        size_t lo, hi;
        split(count, k, t, &lo, &hi);
        for (size_t i = lo; i < hi; ++i)
          if (bad(i)) {
            hit[t] = 1;
            return;
          }
      },
      k);
  return std::find(hit.begin(), hit.end(), 1) != hit.end();
}

// Bulk push() of response messages [a, b) (all fast): rows at fixed batch
// positions, group flags by atomic exchange, lists per worker.  The batch has
// room for b - a rows.
void push_responses(hbn_node* n, const BulkRun& br, const hbn_message* m, size_t a, size_t b) {
  HBN_PHASE(n, PH_BULK_RESP);
  const size_t cnt = b - a;
  const unsigned k = n->pool->ways_small(cnt, 4096, n->pool->small_bulk());
  std::vector<size_t> rows(k + 1, 0);  // rows of each worker's range (groups with a device slot)
  n->pool->run(
      [&](unsigned t) {
        size_t lo, hi, c = 0;
        split(cnt, k, t, &lo, &hi);
        for (size_t i = a + lo; i < a + hi; ++i) {
          if (i + 16 < a + hi) __builtin_prefetch(br.gp[i + 16]);
          c += br.gp[i]->slot != NO_SLOT;
        }
        rows[t + 1] = c;
      },
      k);
  for (unsigned t = 0; t < k; ++t) rows[t + 1] += rows[t];
  const size_t base = n->b_group.size(), add = rows[k];
  for (auto* v : {&n->b_term, &n->b_index, &n->b_hint, &n->b_eoff, &n->b_commit, &n->b_from}) v->resize(base + add);
  n->b_group.resize(base + add);
  n->b_info.resize(base + add);
  n->b_snapi.resize(base + add);
  n->b_kept.resize(base + add);  // (read only for MsgApp)
  n->pool->run(
      [&](unsigned t) {
        size_t lo, hi;
        split(cnt, k, t, &lo, &hi);
        Lists& L = n->lists[t];
        size_t r = base + rows[t];
        for (size_t i = a + lo; i < a + hi; ++i) {
          if (i + 8 < a + hi) {  // the messages' groups are in network order: fetch ahead
            const char* q = reinterpret_cast<const char*>(br.gp[i + 8]);
            __builtin_prefetch(q);
            __builtin_prefetch(q + 64);
          }
          Group& g = *br.gp[i];
          const hbn_message& x = m[i];
          touch_into(L.touched, g, k > 1);
          if (g.slot == NO_SLOT) continue;  // prs is empty: responses are filtered (raft/multinode.go:235)
          const int s = g.slot_of(x.from);
          n->b_group[r] = g.slot;
          n->b_info[r] = HB_INFO(x.type, s >= 0 ? (uint32_t)s : HB_SLOT_NONE, x.reject != 0);
          n->b_term[r] = x.term;
          n->b_index[r] = x.index;
          n->b_hint[r] = x.reject_hint;
          n->b_eoff[r] = n->b_nent;
          n->b_commit[r] = 0;
          n->b_from[r] = x.from;
          n->b_snapi[r] = NO_SLOT;
          ++r;
          bump(g.bx, k > 1);
          if (x.type == HB_MSG_VOTE_RESP) bump(g.bxr, k > 1);
          if (flag_set(g.in_bx, k > 1)) L.bx.push_back(&g);
          if (s >= 0 && flag_set(g.stepped, k > 1)) L.stepped.push_back(&g);
        }
      },
      k);
  merge(n->touched, n->lists, &Lists::touched);
  merge(n->bx, n->lists, &Lists::bx);
  merge(n->stepped, n->lists, &Lists::stepped);
}

// Bulk propose() of one-entry proposals [a, b) (all fast: groups with a device
// slot).  A group's proposals keep their order in g.props, so each group
// belongs to one worker (slot % k); rows and entry positions are fixed.
void push_proposals(hbn_node* n, const BulkRun& br, const uint8_t* const* data, const uint64_t* len, size_t a,
                    size_t b) {
  HBN_PHASE(n, PH_BULK_PROP);
  const size_t cnt = b - a, base = n->b_group.size(), e0 = n->b_nent;
  const unsigned k = n->pool->ways_small(cnt, 4096, n->pool->small_bulk());
  for (auto* v : {&n->b_term, &n->b_index, &n->b_hint, &n->b_eoff, &n->b_commit, &n->b_from}) v->resize(base + cnt);
  n->b_group.resize(base + cnt);
  n->b_info.resize(base + cnt);
  n->b_snapi.resize(base + cnt);
  n->b_kept.resize(base + cnt);  // (read only for MsgApp)
  n->b_eterm.resize(e0 + cnt);
  if (n->sized) n->b_edesc.resize(e0 + cnt);
  RawVec<uint32_t> sl(cnt);  // each group's owner is slot % k
  n->pool->run(
      [&](unsigned t) {
        size_t lo, hi;
        split(cnt, k, t, &lo, &hi);
        for (size_t i = lo; i < hi; ++i) sl[i] = br.gp[a + i]->slot;
      },
      k);
  n->pool->run(
      [&](unsigned t) {
        Lists& L = n->lists[t];
        for (size_t j = 0; j < cnt; ++j) {
          if (k > 1 && sl[j] % k != t) continue;
          const size_t i = a + j, r = base + j;
          Group& g = *br.gp[i];
          Msg msg;
          msg.type = HB_MSG_PROP;
          msg.from = n->id;  // raft/multinode.go:228
          Ent e;
          e.has_data = data[i] != nullptr;
          if (len[i]) e.data.assign(reinterpret_cast<const char*>(data[i]), len[i]);
          if (n->sized) n->b_edesc[e0 + j] = ent_desc(e);
          msg.entries.push_back(std::move(e));
          g.props.push_back(std::move(msg));
          const int s = g.slot_of(n->id);
          n->b_group[r] = g.slot;
          n->b_info[r] = HB_INFO(HB_MSG_PROP, s >= 0 ? (uint32_t)s : HB_SLOT_NONE, false);
          n->b_term[r] = 0;
          n->b_index[r] = 1;
          n->b_hint[r] = 0;
          n->b_eoff[r] = e0 + j;
          n->b_commit[r] = 0;
          n->b_from[r] = n->id;
          n->b_snapi[r] = NO_SLOT;
          n->b_eterm[e0 + j] = 0;
          g.bx += 2;  // the message and its entry
          if (flag_set(g.touched, k > 1)) L.touched.push_back(&g);
          if (flag_set(g.in_bx, k > 1)) L.bx.push_back(&g);
          if (flag_set(g.stepped, k > 1)) L.stepped.push_back(&g);
        }
      },
      k);
  n->b_nent = e0 + cnt;
  n->b_prop = true;
  merge(n->touched, n->lists, &Lists::touched);
  merge(n->bx, n->lists, &Lists::bx);
  merge(n->stepped, n->lists, &Lists::stepped);
}

// Runs of bulk messages in [0, count), each cut to the batch's free rows (the
// batch is stepped when full, as push() does); the others one at a time.  A
// flush replays device events, which can fault a group or move its slot (a
// restore reload).  The message whose push triggers the flush was checked
// before it, as in push(); from the next one on, the run is re-checked with
// `still`, and a message that no longer qualifies goes through one(i), which
// raises the reference's error at its position, as hbn_step / hbn_propose do.
template <class Bulk, class One, class Still>
void bulk_runs(hbn_node* n, uint64_t count, BulkRun& br, uint64_t* done, Bulk&& bulk, One&& one, Still&& still) {
  size_t i = 0;
  while (i < count) {
    if (!br.fast[i]) {
      one(i);
      *done = ++i;
      continue;
    }
    size_t j = i;
    while (j < count && br.fast[j]) ++j;
    while (i < j) {
      if (n->b_group.size() >= n->max_batch) {
        flush(n);
        for (size_t k = i + 1; k < j; ++k)
          if (!still(k)) {
            br.fast[k] = 0;
            j = k;
            break;
          }
      }
      const size_t room = n->max_batch - n->b_group.size();
      const size_t e = std::min(j, i + room);
      bulk(i, e);
      *done = i = e;
    }
  }
}

// One entry of the last pushed message (its descriptor for the device's
// limitSize, its term for the follower side; `keep`: the payload for the replay).
void push_entry(hbn_node* n, const Ent& x, bool keep) {
  Group* g = n->by_slot[n->b_group.back()];
  g->bx++;  // one more entry the step can append
  if (keep) g->bxr++;  // a MsgApp entry can start a term run (a MsgProp entry continues the leader's)
  if (n->sized) n->b_edesc.push_back(ent_desc(x));
  n->b_eterm.push_back(x.term);
  if (keep) n->b_ents.push_back(x);
  n->b_nent++;
}

void propose(hbn_node* n, Group& g, Msg m) {
  if (g.fault) throw Fail{HBN_EPANIC};
  m.from = n->id;  // raft/multinode.go:228
  const uint64_t k = m.entries.size(), term = m.term;
  if (g.slot != NO_SLOT) g.props.push_back(std::move(m));
  push(n, g, HB_MSG_PROP, n->id, false, term, k, 0);
  if (g.slot != NO_SLOT)
    for (const Ent& x : g.props.back().entries) push_entry(n, x, false);
}

// The follower side of Step (MsgApp / MsgHeartbeat / MsgSnap / MsgVote,
// raft/raft.go:585-707): the device steps it; the payloads stay here.
void step_follower(hbn_node* n, Group& g, const hbn_message* m) {
  const uint32_t t = m->type;
  if (g.fault) throw Fail{HBN_EPANIC};
  if (g.slot == NO_SLOT) throw Fail{HBN_EUNSUPPORTED};  // a raft with no prs at all
  for (uint64_t k = 0; k < m->n_entries; ++k)  // the device numbers a MsgApp's entries Index+1, +2, ...
    if (m->entries[k].index != m->index + 1 + k) throw Fail{HB_EINVAL};
  bool voted = false;
  if (t == HB_MSG_VOTE && g.slot_of(m->from) < 0) {
    // r.Vote == m.From for a sender outside prs: only the host knows ids outside
    // prs, so the group's earlier messages of this batch are stepped first
    if (g.stepped) flush(n);
    voted = g.vote != 0 && g.vote == m->from;
  }
  uint64_t index = m->index, hint = m->log_term;
  if (t == HB_MSG_SNAP) {
    index = m->snapshot.index;
    hint = m->snapshot.term;
  }
  push(n, g, t, m->from, m->reject != 0, m->term, index, hint,
       (t == HB_MSG_APP || t == HB_MSG_HEARTBEAT) ? m->commit : 0, voted);
  n->b_follow = true;
  if (t == HB_MSG_APP && m->n_entries) {
    n->b_app = true;
    for (uint64_t k = 0; k < m->n_entries; ++k) push_entry(n, ent_from(m->entries[k]), true);
    g.bx_top = std::max(g.bx_top, m->index + m->n_entries);  // a MsgApp can cut the log and append up to here
  }
  if (t == HB_MSG_SNAP) {
    n->b_snapi.back() = (uint32_t)n->b_snaps.size();
    n->b_snaps.push_back(snap_from(m->snapshot));
    // a restore to another peer set reloads the group's prs after its batch: the
    // group's later messages must see the new prs, so the batch ends here
    std::vector<uint64_t> a = n->b_snaps.back().nodes, b = g.peers;
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    if (a != b) flush(n);
  }
}

// ---------------------------------------------------------------- Ready
void refresh_content(std::vector<Group*>& content, Group& g);
// (e.data holds the payload's offset in A.bytes until patch_arena)
void arena_entry(Arena& A, const Ent& x) {
  hbn_entry& e = A.ents.emplace_back();
  e.term = x.term;
  e.index = x.index;
  e.type = x.type;
  e.has_data = x.has_data;
  e.data_len = x.data.size();
  e.data = reinterpret_cast<const uint8_t*>(A.bytes.size());
  if (!x.data.empty()) A.bytes.insert(A.bytes.end(), x.data.begin(), x.data.end());
}

void clear_arena(hbn_node* n) {
  n->r_n = 0;
  for (Arena& A : n->arenas) A.clear();
}

// newReady (raft/node.go:447-463) of g into arena A when it containsUpdates
// (raft/node.go:96-100); the delivered part is remembered for commitReady.
void build_ready(Group& g, Arena& A, Lists& L) {
  g.touched = false;
  refresh_content(L.content, g);
  if (!g.content && g.msgs.empty() && !g.fault) return;
  hbn_group_ready& r = A.out.emplace_back();  // (zeroed)
  r.group = g.id;
  Delivered& d = g.dlv;
  d = Delivered{};
  if (!(g.soft() == g.prev_soft)) {
    r.has_soft_state = 1;
    r.raft_state = g.state;
    r.lead = g.lead;
    d.has_soft = true;
    d.soft = g.soft();
  }
  if (!hs_equal(g.hard(), g.prev_hard)) r.hard_state = d.hard = g.hard();
  if (g.log.has_usnap) {
    A.snaps.push_back(g.log.usnap);
    snap_view(A.snaps.back(), &r.snapshot);
    d.snap_index = g.log.usnap.index;
  }
  A.off.push_back(A.ents.size());  // Entries = unstableEntries
  for (const Ent& x : g.log.unstable) arena_entry(A, x);
  r.n_entries = g.log.unstable.size();
  if (r.n_entries) {
    d.has_last = true;
    d.last_index = g.log.unstable.back().index;
    d.last_term = g.log.unstable.back().term;
  }
  A.off.push_back(A.ents.size());  // CommittedEntries = nextEnts (raft/log.go:135-141)
  const uint64_t lo = std::max(g.log.applied + 1, g.log.first_index());
  if (g.log.committed + 1 > lo) g.log.visit(lo, g.log.committed + 1, [&](const Ent& x) { arena_entry(A, x); });
  r.n_committed = A.ents.size() - A.off.back();
  A.off.push_back(A.msgs.size());  // Messages = r.msgs, then cleared (raft/multinode.go:277-281)
  for (Msg& m : g.msgs) {
    hbn_message& x = A.msgs.emplace_back();  // (zeroed)
    x.type = m.type;
    x.reject = m.reject;
    x.to = m.to;
    x.from = m.from;
    x.term = m.term;
    x.log_term = m.log_term;
    x.index = m.index;
    x.commit = m.commit;
    x.reject_hint = m.reject_hint;
    const size_t e0 = A.ents.size();
    if (m.owned)
      for (const Ent& e : m.entries) arena_entry(A, e);
    else if (m.ent_hi > m.ent_lo)
      g.log.visit(m.ent_lo, m.ent_hi, [&](const Ent& e) { arena_entry(A, e); });
    x.n_entries = A.ents.size() - e0;
    x.entries = reinterpret_cast<const hbn_entry*>(e0);  // offset, patched below
    if (m.snap) {
      A.snaps.push_back(*m.snap);
      snap_view(A.snaps.back(), &x.snapshot);
    }
  }
  r.n_messages = g.msgs.size();
  g.msgs.clear();
  r.fault = g.fault;
  g.delivered = true;
  L.delivered.push_back(&g);
}

// A large touched list (the network input's order: random over the groups)
// is rebuilt in device slot order, i.e. the groups' allocation order, so the
// Ready build, the application's persisting and Advance walk memory forward
// instead of missing cache and TLB on every group (the Ready's group order is
// unspecified: the reference iterates a map).  Groups without a slot keep
// their place after the others.
void slot_order_touched(hbn_node* n) {
  const size_t nt = n->touched.size(), ns = n->by_slot.size();
  if (nt < 65536 || 8 * nt < ns) return;
  const unsigned k = n->pool->size();
  n->pool->run(
      [&](unsigned t) {
        size_t lo, hi;
        split(ns, k, t, &lo, &hi);
        std::vector<Group*>& v = n->lists[t].touched;
        for (size_t s = lo; s < hi; ++s) {
          Group* g = n->by_slot[s];
          if (g && g->touched) v.push_back(g);
        }
      },
      k);
  std::vector<Group*> host;
  for (Group* g : n->touched)
    if (g->slot == NO_SLOT) host.push_back(g);
  n->touched.clear();
  merge(n->touched, n->lists, &Lists::touched);
  n->touched.insert(n->touched.end(), host.begin(), host.end());
  if (n->touched.size() != nt) panicf("touched groups disagree with their flags");
}

// once no vector of A grows any more: offsets become pointers
void patch_arena(Arena& A) {
  for (hbn_entry& e : A.ents)
    e.data = e.data_len ? A.bytes.data() + reinterpret_cast<uintptr_t>(e.data) : nullptr;
  for (hbn_message& x : A.msgs)
    x.entries = x.n_entries ? A.ents.data() + reinterpret_cast<uintptr_t>(x.entries) : nullptr;
  for (size_t i = 0; i < A.out.size(); ++i) {
    hbn_group_ready& r = A.out[i];
    r.entries = r.n_entries ? A.ents.data() + A.off[3 * i] : nullptr;
    r.committed_entries = r.n_committed ? A.ents.data() + A.off[3 * i + 1] : nullptr;
    r.messages = r.n_messages ? A.msgs.data() + A.off[3 * i + 2] : nullptr;
  }
}

// commitReady raft/multinode.go:137-164
void commit_ready(Group& g, const Delivered& d) {
  if (d.has_soft) g.prev_soft = d.soft;
  if (!hs_empty(d.hard)) g.prev_hard = d.hard;
  if (g.prev_hard.commit != 0) g.log.applied_to(g.prev_hard.commit);
  if (d.has_last) g.log.stable_to(d.last_index, d.last_term);
  if (d.snap_index != 0) {
    g.prev_snapi = d.snap_index;
    g.log.stable_snap_to(d.snap_index);
  }
}

// containsUpdates of newReady(g) without building it
bool has_updates(const Group& g) {
  if (!(g.soft() == g.prev_soft) || !hs_equal(g.hard(), g.prev_hard)) {
    if (!(g.soft() == g.prev_soft) || !hs_empty(g.hard())) return true;
  }
  if (!g.log.unstable.empty() || (g.log.has_usnap && g.log.usnap.index != 0)) return true;
  return g.log.committed + 1 > std::max(g.log.applied + 1, g.log.first_index());
}

void refresh_content(std::vector<Group*>& content, Group& g) {
  const bool c = has_updates(g);
  if (c && !g.content) content.push_back(&g);
  g.content = c;
}

// Rebuild the device record of g after prs changed (ApplyConfChange; with
// `restored`, a snapshot restore's setProgress of every ConfState node).
void reload_prs(hbn_node* n, Group& g, const std::vector<uint64_t>& new_peers,
                const std::vector<std::pair<uint64_t, uint64_t>>& fresh /* id -> (match 0, next) */,
                bool restored) {
  if (new_peers.size() > n->nmax) throw Fail{HBN_EUNSUPPORTED};  // the engine's limit (hbn_start max_replicas <= 7)
  hb_group old;
  std::memset(&old, 0, sizeof(old));
  hb_timer tm;
  std::memset(&tm, 0, sizeof(tm));
  std::vector<std::vector<uint64_t>> ins;
  std::vector<uint32_t> ins_start;
  const std::vector<uint64_t> old_peers = g.peers;
  if (g.slot != NO_SLOT) {
    sync_loads(n);
    check(hb_get_groups(n->h, g.slot, 1, &old));
    check(hb_get_timers(n->h, g.slot, 1, &tm));
    ins.resize(old_peers.size());
    ins_start.resize(old_peers.size());
    std::vector<uint64_t> vals(n->W);
    for (size_t s = 0; s < old_peers.size(); ++s) {
      uint32_t st = 0, c = 0;
      check(hb_get_inflights(n->h, g.slot, (uint32_t)s, &st, &c, vals.data()));
      ins[s].assign(vals.begin(), vals.begin() + c);
      ins_start[s] = st;
    }
  }
  g.peers = new_peers;
  note_solo(n, g);
  if (new_peers.empty()) {
    if (g.slot != NO_SLOT) {
      check(hb_remove_groups(n->h, g.slot, 1));
      n->by_slot[g.slot] = nullptr;
      n->free_slots.push_back(g.slot);
      g.slot = NO_SLOT;
    }
    return;
  }
  std::vector<hb_progress> prs(new_peers.size());
  std::vector<int> from_old(new_peers.size(), -1);
  for (size_t s = 0; s < new_peers.size(); ++s) {
    std::memset(&prs[s], 0, sizeof(hb_progress));
    for (size_t o = 0; o < old_peers.size(); ++o)
      if (old_peers[o] == new_peers[s] && g.slot != NO_SLOT && !restored) from_old[s] = (int)o;
    if (restored) {  // raft/raft.go:700-705
      prs[s].next = g.log.last_index() + 1;
      prs[s].match = new_peers[s] == n->id ? g.log.last_index() : 0;
      prs[s].state = HB_PR_PROBE;
    } else if (from_old[s] >= 0) {
      prs[s] = old.pr[from_old[s]];
    } else {
      for (const auto& f : fresh)
        if (f.first == new_peers[s]) prs[s].next = f.second;
      prs[s].state = HB_PR_PROBE;
    }
  }
  const bool was_loaded = g.slot != NO_SLOT;
  hb_group r = make_record(n, g, prs);
  if (was_loaded) {
    r.term_first = old.term_first;
    r.term_last = old.term_last;
    r.fault = old.fault;
    // r.votes as slot bitmasks: move each responded peer's bit to its new slot
    uint32_t resp = 0, grant = 0;
    for (size_t o = 0; o < old_peers.size() + 1; ++o) {
      const uint32_t bit = o < old_peers.size() ? (uint32_t)o : 7u;
      if (!((old.votes_resp >> bit) & 1u)) continue;
      const uint64_t who = o < old_peers.size() ? old_peers[o] : n->id;
      const int ns = g.slot_of(who);
      const uint32_t nb = ns >= 0 ? (uint32_t)ns : (who == n->id ? 7u : 0xFFu);
      if (nb == 0xFFu) continue;  // a voter that left prs: its vote is still in r.votes, kept by no slot
      resp |= 1u << nb;
      if ((old.votes_grant >> bit) & 1u) grant |= 1u << nb;
    }
    r.votes_resp = resp;
    r.votes_grant = grant;
  } else {
    g.slot = alloc_slot(n);
    n->by_slot[g.slot] = &g;
    tm.elapsed = 0;
    tm.rand_pos = 0;
  }
  check(hb_load_groups(n->h, g.slot, 1, &r));
  if (n->sized) {
    n->pend_sz.push_back(&g);
    push_sizes(n);
  }
  n->pend_tr.push_back(&g);
  push_term_runs(n);
  hb_timer t2 = tm;
  t2.election_tick = (uint16_t)g.election;
  t2.heartbeat_tick = (uint16_t)g.heartbeat;
  check(hb_load_timers(n->h, g.slot, 1, &t2));
  for (size_t s = 0; s < new_peers.size(); ++s)
    if (from_old[s] >= 0 && !ins[from_old[s]].empty())
      check(hb_set_inflights(n->h, g.slot, (uint32_t)s, ins_start[from_old[s]], (uint32_t)ins[from_old[s]].size(),
                             ins[from_old[s]].data()));
}

// Before the application mutates storage `s` (Compact / CreateSnapshot /
// ApplySnapshot): the messages already handed to MultiNode.Step were stepped
// by the reference before this call, so a node with a pending batch steps it
// now; every MsgApp a group sent copied its entries at send time
// (raft/raft.go:265), so pending lazy messages are materialized.
void before_storage_change(hbn_storage* s) {
  for (auto& u : s->users) {
    if (!u.first->b_group.empty()) flush(u.first);
    Group* g = u.first->groups.find(u.second);
    if (g && g->log.st == s) materialize(*g);
  }
}
// After it: the group's device firstIndex / snapshot index are refreshed
// before its next step (sync_loads).
void after_storage_change(hbn_storage* s) {
  for (auto& u : s->users) {
    Group* gp = u.first->groups.find(u.second);
    if (!gp || gp->log.st != s) continue;
    Group& g = *gp;
    if (!g.bounds) {
      g.bounds = true;
      u.first->bounds.push_back(&g);
    }
  }
}

void drop_user(hbn_storage* s, hbn_node* n, uint64_t group) {
  auto& v = s->users;
  v.erase(std::remove(v.begin(), v.end(), std::make_pair(n, group)), v.end());
}

template <class F>
int guarded(F&& f) {
  try {
    f();
    return HB_OK;
  } catch (const Panic& p) {
    g_err = p.msg;
    return HBN_EPANIC;
  } catch (const Fail& e) {
    g_err = "failed with code " + std::to_string(e.code);
    return e.code;
  } catch (const std::bad_alloc&) {
    g_err = "out of host memory";
    return HB_ENOMEM;
  } catch (const std::exception& e) {
    g_err = e.what();
    return HBN_EPANIC;
  }
}

// Step (raft/multinode.go:431-439) of one message; throws the reference's errors.
void step_one(hbn_node* n, uint64_t group, const hbn_message* m) {
  const uint32_t t = m->type;
  // IsLocalMsg (raft/util.go:49-51): ignored when received over the network
  if (t == HB_MSG_HUP || t == HB_MSG_BEAT || t == HB_MSG_UNREACHABLE || t == HB_MSG_SNAP_STATUS) return;
  Group& g = group_of(n, group);
  if (t == HB_MSG_PROP) {
    Msg p;
    p.type = t;
    p.to = m->to;
    p.term = m->term;
    p.log_term = m->log_term;
    p.index = m->index;
    p.commit = m->commit;
    p.reject = m->reject;
    p.reject_hint = m->reject_hint;
    for (uint64_t i = 0; i < m->n_entries; ++i) p.entries.push_back(ent_from(m->entries[i]));
    propose(n, g, std::move(p));
    return;
  }
  if (t == HB_MSG_APP || t == HB_MSG_HEARTBEAT || t == HB_MSG_SNAP || t == HB_MSG_VOTE) {
    step_follower(n, g, m);
    return;
  }
  if (t != HB_MSG_APP_RESP && t != HB_MSG_VOTE_RESP && t != HB_MSG_HEARTBEAT_RESP) throw Fail{HBN_EUNSUPPORTED};
  if (g.fault) throw Fail{HBN_EPANIC};
  push(n, g, t, m->from, m->reject != 0, m->term, m->index, m->reject_hint);
}

// Propose (raft/multinode.go:377-385) of one entry.
void propose_one(hbn_node* n, uint64_t group, const uint8_t* data, uint64_t len) {
  Group& g = group_of(n, group);
  Msg m;
  m.type = HB_MSG_PROP;
  Ent e;
  e.has_data = data != nullptr;
  if (len) e.data.assign(reinterpret_cast<const char*>(data), len);
  m.entries.push_back(std::move(e));
  propose(n, g, std::move(m));
}

}  // namespace

// ======================================================================= C ABI
extern "C" {

const char* hbn_last_error(void) { return g_err.c_str(); }

uint64_t hbn_entry_size(const hbn_entry* e) {
  return e ? ent_size(e->type, e->term, e->index, e->has_data != 0, e->data_len) : 0;
}

// ---- MemoryStorage ----------------------------------------------------------
int hbn_storage_new(hbn_storage** out) {
  if (!out) return HB_EINVAL;
  return guarded([&] { *out = new hbn_storage(); });
}

int hbn_storage_new_with_entries(const hbn_entry* ents, uint64_t n, hbn_storage** out) {
  if (!out || (n && !ents)) return HB_EINVAL;
  return guarded([&] {
    auto* s = new hbn_storage();
    s->ents.clear();
    for (uint64_t i = 0; i < n; ++i) s->ents.push_back(ent_from(ents[i]));
    if (s->ents.empty()) s->ents.emplace_back();  // Go would index an empty slice; keep the dummy
    *out = s;
  });
}

int hbn_storage_free(hbn_storage* s) {
  if (s)  // groups still reading it keep no dangling back-reference
    for (auto& u : s->users) {
      Group* g = u.first->groups.find(u.second);
      if (g && g->log.st == s) g->log.st = nullptr;
    }
  delete s;
  return HB_OK;
}

int hbn_storage_initial_state(hbn_storage* s, hbn_hard_state* hs, uint64_t* nodes, uint32_t cap, uint32_t* n_nodes) {
  if (!s || !hs || !n_nodes) return HB_EINVAL;
  *hs = s->hs;
  *n_nodes = (uint32_t)s->snap.nodes.size();
  if (s->snap.nodes.size() > cap || (cap && !nodes && !s->snap.nodes.empty())) return HB_EINVAL;
  for (size_t i = 0; i < s->snap.nodes.size(); ++i) nodes[i] = s->snap.nodes[i];
  return HB_OK;
}

int hbn_storage_set_hard_state(hbn_storage* s, const hbn_hard_state* hs) {
  if (!s || !hs) return HB_EINVAL;
  s->hs = *hs;
  return HB_OK;
}

int hbn_storage_entries(hbn_storage* s, uint64_t lo, uint64_t hi, uint64_t max_size, const hbn_entry** out,
                        uint64_t* n) {
  if (!s || !out || !n) return HB_EINVAL;
  int rc = HB_OK;
  const int g = guarded([&] {
    size_t a = 0, k = 0;
    rc = s->entries(lo, hi, max_size, &a, &k);
    s->view.clear();
    if (rc != HB_OK) return;
    for (size_t i = 0; i < k; ++i) {
      const Ent& x = s->ents[a + i];
      s->view.push_back(hbn_entry{x.term, x.index, x.type, x.has_data,
                                  x.data.empty() ? nullptr : reinterpret_cast<const uint8_t*>(x.data.data()),
                                  x.data.size()});
    }
  });
  if (g != HB_OK) return g;
  *out = s->view.empty() ? nullptr : s->view.data();
  *n = s->view.size();
  return rc;
}

int hbn_storage_term(hbn_storage* s, uint64_t i, uint64_t* term) {
  if (!s || !term) return HB_EINVAL;
  int rc = HB_OK;
  *term = 0;
  const int g = guarded([&] { rc = s->term(i, term); });
  return g != HB_OK ? g : rc;
}

int hbn_storage_last_index(hbn_storage* s, uint64_t* out) {
  if (!s || !out) return HB_EINVAL;
  *out = s->last_index();
  return HB_OK;
}

int hbn_storage_first_index(hbn_storage* s, uint64_t* out) {
  if (!s || !out) return HB_EINVAL;
  *out = s->first_index();
  return HB_OK;
}

int hbn_storage_snapshot(hbn_storage* s, hbn_snapshot* out) {
  if (!s || !out) return HB_EINVAL;
  snap_view(s->snap, out);
  return HB_OK;
}

// ApplySnapshot raft/storage.go:150-159
int hbn_storage_apply_snapshot(hbn_storage* s, const hbn_snapshot* snap) {
  if (!s || !snap) return HB_EINVAL;
  return guarded([&] {
    before_storage_change(s);
    s->snap = snap_from(*snap);
    Ent d;
    d.term = snap->term;
    d.index = snap->index;
    s->ents.assign(1, d);
    after_storage_change(s);
  });
}

// CreateSnapshot :161-186
int hbn_storage_create_snapshot(hbn_storage* s, uint64_t i, const uint64_t* nodes, uint32_t n_nodes,
                                const uint8_t* data, uint64_t data_len, hbn_snapshot* out) {
  if (!s) return HB_EINVAL;
  int rc = HB_OK;
  const int g = guarded([&] {
    if (i <= s->snap.index) {
      rc = HBN_ESNAPOUTOFDATE;
      return;
    }
    if (i > s->last_index())
      panicf("snapshot " + std::to_string(i) + " is out of bound lastindex(" + std::to_string(s->last_index()) + ")");
    before_storage_change(s);
    s->snap.index = i;
    s->snap.term = s->ents[i - s->offset()].term;
    if (nodes || n_nodes == 0) {
      if (nodes) s->snap.nodes.assign(nodes, nodes + n_nodes);
    }
    s->snap.has_data = data != nullptr;
    s->snap.data.assign(data ? reinterpret_cast<const char*>(data) : "", data ? data_len : 0);
    after_storage_change(s);
  });
  if (g != HB_OK) return g;
  if (out) {
    if (rc == HB_OK)
      snap_view(s->snap, out);
    else
      std::memset(out, 0, sizeof(*out));
  }
  return rc;
}

// Compact :188-214
int hbn_storage_compact(hbn_storage* s, uint64_t i) {
  if (!s) return HB_EINVAL;
  int rc = HB_OK;
  const int g = guarded([&] {
    const uint64_t off = s->offset();
    if (i <= off) {
      rc = HBN_ECOMPACTED;
      return;
    }
    if (i > s->last_index())
      panicf("compact " + std::to_string(i) + " is out of bound lastindex(" + std::to_string(s->last_index()) + ")");
    before_storage_change(s);
    const size_t k = i - off;
    EntLog ents(1);
    ents[0].index = s->ents[k].index;
    ents[0].term = s->ents[k].term;
    ents.insert(ents.end(), s->ents.begin() + k + 1, s->ents.end());
    s->ents.swap(ents);
    after_storage_change(s);
  });
  return g != HB_OK ? g : rc;
}

int hbn_storage_append(hbn_storage* s, const hbn_entry* ents, uint64_t n) {
  if (!s || (n && !ents)) return HB_EINVAL;
  return guarded([&] { s->append(ents, n); });
}

// ---- MultiNode ----------------------------------------------------------------
int hbn_start(int device, uint64_t id, uint32_t capacity, uint32_t max_replicas, uint32_t max_inflight,
              uint64_t max_msg_size, uint64_t max_batch, hbn_node** out) {
  if (!out || id == 0 || capacity == 0 || max_batch == 0) return HB_EINVAL;
  hb_handle* h = nullptr;
  const int rc = hb_create(device, capacity, max_replicas, max_inflight, max_msg_size, max_batch, &h);
  if (rc != HB_OK) return rc;
  return guarded([&] {
    auto* n = new hbn_node();
    n->h = h;
    n->id = id;
    n->capacity = capacity;
    n->nmax = max_replicas;
    n->W = max_inflight;
    n->max_msg = max_msg_size;
    n->sized = max_msg_size != 0 && max_msg_size != HB_NO_LIMIT;
    n->max_batch = max_batch;
    unsigned th = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("HBN_THREADS")) th = (unsigned)std::min(256, std::max(1, std::atoi(e)));  // as hbn_set_threads
    n->pool.reset(new Pool(th));
    n->lists.resize(th);
    n->arenas.resize(th);
    n->by_slot.assign(capacity, nullptr);
    n->free_slots.reserve(capacity);
    for (uint32_t s = capacity; s > 0; --s) n->free_slots.push_back(s - 1);
    *out = n;
  });
}

int hbn_stop(hbn_node* n) {
  if (!n) return HB_EINVAL;
  n->groups.each([&](uint64_t id, Group& g) {
    if (g.log.st) drop_user(g.log.st, n, id);
  });
  if (n->w_words) (void)hb_free_pinned(n->w_words);
  if (n->w_counts) (void)hb_free_pinned(n->w_counts);
  if (n->w_total) (void)hb_free_pinned(n->w_total);
  const int rc = hb_destroy(n->h);
  delete n;
  return rc;
}

hb_handle* hbn_engine(hbn_node* n) { return n ? n->h : nullptr; }

int hbn_create_group(hbn_node* n, uint64_t group, const hbn_config* cfg, hbn_storage* storage,
                     const uint64_t* peer_ids, uint32_t n_peers) {
  if (!n || !cfg || !storage || (n_peers && !peer_ids) || cfg->election_tick == 0 || cfg->heartbeat_tick == 0 ||
      cfg->election_tick > 0xFFFF || cfg->heartbeat_tick > 0xFFFF)
    return HB_EINVAL;
  if (n->groups.find(group)) return HBN_EEXIST;
  return guarded([&] {
    auto gp = std::make_unique<Group>();
    Group& g = *gp;
    g.id = group;
    g.election = cfg->election_tick;
    g.heartbeat = cfg->heartbeat_tick;
    // newRaft raft/raft.go:157-209
    g.log.init(storage);
    g.peers = storage->snap.nodes;  // ConfState.Nodes (Config.peers is test-only and not taken here)
    if (!hs_empty(storage->hs)) {  // loadState :755-763
      const hbn_hard_state& hs = storage->hs;
      if (hs.commit < g.log.committed || hs.commit > g.log.last_index())
        panicf("state.commit " + std::to_string(hs.commit) + " is out of range [" + std::to_string(g.log.committed) +
               ", " + std::to_string(g.log.last_index()) + "]");
      g.log.committed = hs.commit;
      g.term = hs.term;
      g.vote = hs.vote;
      g.hs_commit = hs.commit;
    }
    if (cfg->applied > 0) g.log.applied_to(cfg->applied);
    // becomeFollower(r.Term, None)
    g.state = HB_STATE_FOLLOWER;
    g.lead = 0;
    std::vector<std::pair<uint64_t, uint64_t>> fresh;
    if (storage->last_index() == 0) {
      // new group (raft/multinode.go:194-211): becomeFollower(1, None), one
      // ConfChangeAddNode entry per peer, committed = len(peers), addNode each.
      if (g.term != 1) g.vote = 0;
      g.term = 1;
      EntVec ents(n_peers);
      for (uint32_t i = 0; i < n_peers; ++i) {
        ents[i].type = HBN_ENTRY_CONF_CHANGE;
        ents[i].term = 1;
        ents[i].index = i + 1;
        ents[i].has_data = true;
        ents[i].data = marshal_conf_change(0, HBN_CC_ADD_NODE, peer_ids[i], nullptr, 0, false);
      }
      g.log.append(std::move(ents));
      g.log.committed = n_peers;
      for (uint32_t i = 0; i < n_peers; ++i) {
        if (g.slot_of(peer_ids[i]) >= 0) continue;  // addNode ignores a known id
        g.peers.push_back(peer_ids[i]);
      }
    }
    if (g.peers.size() > n->nmax) throw Fail{HBN_EUNSUPPORTED};  // the engine's limit (hbn_start max_replicas <= 7)
    // Progress after reset / addNode: Next = lastIndex+1; Match = lastIndex for self
    // after reset, 0 after addNode (the bootstrap path).
    std::vector<hb_progress> prs(g.peers.size());
    const bool boot = storage->last_index() == 0;
    for (size_t s = 0; s < g.peers.size(); ++s) {
      std::memset(&prs[s], 0, sizeof(hb_progress));
      prs[s].next = g.log.last_index() + 1;
      prs[s].match = (!boot && g.peers[s] == n->id) ? g.log.last_index() : 0;
      prs[s].state = HB_PR_PROBE;
    }
    if (!g.peers.empty()) {
      g.slot = alloc_slot(n);
      n->pend_rec.emplace_back(g.slot, make_record(n, g, prs));
      hb_timer t;
      std::memset(&t, 0, sizeof(t));
      t.election_tick = (uint16_t)g.election;
      t.heartbeat_tick = (uint16_t)g.heartbeat;
      n->pend_tm.emplace_back(g.slot, t);
      n->by_slot[g.slot] = &g;
      if (n->sized) n->pend_sz.push_back(&g);
      n->pend_tr.push_back(&g);
    }
    note_solo(n, g);
    // the initial hard and soft states (:213-215)
    g.prev_soft = g.soft();
    g.prev_hard = g.hard();
    touch(n, g);
    storage->users.emplace_back(n, group);
    n->groups.insert(group, std::move(gp));
  });
}

int hbn_remove_group(hbn_node* n, uint64_t group) {
  if (!n) return HB_EINVAL;
  return guarded([&] {
    flush(n);
    Group* gp = n->groups.find(group);
    if (!gp) return;  // delete of a missing key is a no-op in Go
    Group& g = *gp;
    if (g.slot != NO_SLOT) {
      check(hb_remove_groups(n->h, g.slot, 1));
      n->by_slot[g.slot] = nullptr;
      n->free_slots.push_back(g.slot);
    }
    if (g.log.st) drop_user(g.log.st, n, group);
    for (auto* v : {&n->touched, &n->content, &n->delivered, &n->stepped, &n->bounds, &n->pend_sz, &n->pend_tr,
                    &n->reload, &n->bx, &n->solo})
      v->erase(std::remove(v->begin(), v->end(), &g), v->end());
    n->groups.erase(group);
  });
}

int hbn_set_rand(hbn_node* n, uint64_t first, uint64_t count, const uint64_t* draws) {
  if (!n) return HB_EINVAL;
  return hb_set_rand(n->h, first, count, draws);
}

// Tick (raft/multinode.go:264-275): every group ticks; every group is then a
// Ready candidate (those whose Ready was left un-advanced come back).
int hbn_tick(hbn_node* n) {
  if (!n) return HB_EINVAL;
  return guarded([&] {
    flush(n);  // (also pushes queued loads)
    if (!n->solo.empty()) {  // a one-peer group's tick can win an election at once and append its noop
      std::vector<uint32_t> rs;
      std::vector<uint64_t> rz, rt;
      size_t k = 0;
      for (Group* g : n->solo) {
        if (g->peers.size() != 1) {  // no longer one peer: off the list
          g->solo = false;
          continue;
        }
        n->solo[k++] = g;
        if (g->slot == NO_SLOT || g->state == HB_STATE_LEADER) continue;  // a leader's tick only beats
        want_log(n, *g, 1, 1, rs, rz, rt);
        g->lx_runs += 1;
      }
      n->solo.resize(k);
      reserve(n, rs, rz, rt);
    }
    check(hb_tick(n->h, 0));
    consume_events(n);
    size_t k = 0;  // every group with pending content is a Ready candidate again; drop stale entries
    for (Group* g : n->content)
      if (g->content) {
        touch(n, *g);
        n->content[k++] = g;
      }
    n->content.resize(k);
  });
}

int hbn_campaign(hbn_node* n, uint64_t group) {
  if (!n) return HB_EINVAL;
  return guarded([&] {
    Group& g = group_of(n, group);
    if (g.fault) throw Fail{HBN_EPANIC};
    push(n, g, HB_MSG_HUP, 0, false, 0, 0, 0);  // Step(MsgHup) (:369-375)
  });
}

int hbn_propose(hbn_node* n, uint64_t group, const uint8_t* data, uint64_t len) {
  if (!n || (len && !data)) return HB_EINVAL;
  return guarded([&] { propose_one(n, group, data, len); });
}

int hbn_propose_many(hbn_node* n, uint64_t count, const uint64_t* groups, const uint8_t* const* data,
                     const uint64_t* len, uint64_t* done) {
  if (!n || (count && (!groups || !data || !len))) return HB_EINVAL;
  if (bulk_any(n, count, [&](size_t i) { return len[i] && !data[i]; })) return HB_EINVAL;
  uint64_t d = 0;
  const int rc = guarded([&] {
    BulkRun br;
    bulk_lookup(n, count, groups, br, [](size_t, const Group& g) { return g.slot != NO_SLOT; });
    bulk_runs(n, count, br, &d, [&](size_t a, size_t b) { push_proposals(n, br, data, len, a, b); },
              [&](size_t i) { propose_one(n, groups[i], data[i], len[i]); },
              [&](size_t i) { return !br.gp[i]->fault && br.gp[i]->slot != NO_SLOT; });
  });
  if (done) *done = d;
  return rc;
}

int hbn_propose_conf_change(hbn_node* n, uint64_t group, uint64_t cc_id, uint32_t cc_type, uint64_t node_id,
                            const uint8_t* cc_context, uint64_t context_len) {
  if (!n) return HB_EINVAL;
  return guarded([&] {
    Group& g = group_of(n, group);
    Msg m;
    m.type = HB_MSG_PROP;
    Ent e;
    e.type = HBN_ENTRY_CONF_CHANGE;
    e.has_data = true;
    e.data = marshal_conf_change(cc_id, cc_type, node_id, cc_context, context_len, cc_context != nullptr);
    m.entries.push_back(std::move(e));
    propose(n, g, std::move(m));
  });
}

int hbn_step(hbn_node* n, uint64_t group, const hbn_message* m) {
  if (!n || !m || (m->n_entries && !m->entries)) return HB_EINVAL;
  return guarded([&] { step_one(n, group, m); });
}

int hbn_step_many(hbn_node* n, uint64_t count, const uint64_t* groups, const hbn_message* msgs, uint64_t* done) {
  if (!n || (count && (!groups || !msgs))) return HB_EINVAL;
  if (bulk_any(n, count, [&](size_t i) { return msgs[i].n_entries && !msgs[i].entries; })) return HB_EINVAL;
  uint64_t d = 0;
  const int rc = guarded([&] {
    BulkRun br;
    bulk_lookup(n, count, groups, br, [&](size_t i, const Group&) {
      const uint32_t t = msgs[i].type;
      return t == HB_MSG_APP_RESP || t == HB_MSG_VOTE_RESP || t == HB_MSG_HEARTBEAT_RESP;
    });
    bulk_runs(n, count, br, &d, [&](size_t a, size_t b) { push_responses(n, br, msgs, a, b); },
              [&](size_t i) { step_one(n, groups[i], &msgs[i]); }, [&](size_t i) { return !br.gp[i]->fault; });
  });
  if (done) *done = d;
  return rc;
}

int hbn_profile(hbn_node* n, double* out, uint32_t cap, uint32_t* count) {
  if (!n) return HB_EINVAL;
  if (count) *count = PH_COUNT_;
  for (uint32_t i = 0; i < cap && i < PH_COUNT_ && out; ++i) out[i] = n->prof[i];
  return HB_OK;
}

int hbn_set_threads(hbn_node* n, uint32_t threads) {
  if (!n || threads == 0 || threads > 256) return HB_EINVAL;
  return guarded([&] {
    n->pool.reset(new Pool(threads));
    n->lists.resize(threads);
    if (n->arenas.size() < threads) n->arenas.resize(threads);  // (the last Ready stays valid)
  });
}

int hbn_report_unreachable(hbn_node* n, uint64_t id, uint64_t group) {
  if (!n) return HB_EINVAL;
  return guarded([&] {
    Group& g = group_of(n, group);
    if (g.fault) throw Fail{HBN_EPANIC};
    push(n, g, HB_MSG_UNREACHABLE, id, false, 0, 0, 0);
  });
}

int hbn_report_snapshot(hbn_node* n, uint64_t id, uint64_t group, int failure) {
  if (!n) return HB_EINVAL;
  return guarded([&] {
    Group& g = group_of(n, group);
    if (g.fault) throw Fail{HBN_EPANIC};
    push(n, g, HB_MSG_SNAP_STATUS, id, failure != 0, 0, 0, 0);
  });
}

int hbn_apply_conf_change(hbn_node* n, uint64_t group, uint32_t cc_type, uint64_t node_id, uint64_t* nodes_out,
                          uint32_t* n_nodes) {
  if (!n) return HB_EINVAL;
  return guarded([&] {
    flush(n);
    Group& g = group_of(n, group);
    if (g.fault) throw Fail{HBN_EPANIC};
    touch(n, g);
    if (node_id != 0) {
      std::vector<uint64_t> np = g.peers;
      switch (cc_type) {
        case HBN_CC_ADD_NODE:  // addNode raft/raft.go:729-738
          if (g.slot_of(node_id) < 0) {
            np.push_back(node_id);
            reload_prs(n, g, np, {{node_id, g.log.last_index() + 1}}, false);
            g.pending_conf = false;
          }
          break;
        case HBN_CC_REMOVE_NODE:  // removeNode :740-743
          np.erase(std::remove(np.begin(), np.end(), node_id), np.end());
          if (np.size() != g.peers.size()) reload_prs(n, g, np, {}, false);
          g.pending_conf = false;
          break;
        case HBN_CC_UPDATE_NODE:
          g.pending_conf = false;
          break;
        default:
          panicf("unexpected conf type");
      }
    } else {
      g.pending_conf = false;  // resetPendingConf
    }
    std::vector<uint64_t> nodes = g.peers;
    std::sort(nodes.begin(), nodes.end());
    if (n_nodes) *n_nodes = (uint32_t)nodes.size();
    if (nodes_out)
      for (size_t i = 0; i < nodes.size(); ++i) nodes_out[i] = nodes[i];
  });
}

int hbn_ready(hbn_node* n, const hbn_group_ready** out, uint64_t* count) {
  if (!n || !out || !count) return HB_EINVAL;
  *out = nullptr;
  *count = 0;
  int rc = HB_OK;
  const int g0 = guarded([&] {
    flush(n);
    clear_arena(n);
    if (n->awaiting_advance) {
      // readyc is not selectable; r.msgs keep accumulating, so pin their entries
      for (Group* g : n->touched) materialize(*g);
      rc = HBN_EAGAIN;
      return;
    }
    for (Group* g : n->delivered) g->delivered = false;
    n->delivered.clear();
    // newReady for every touched group, workers over disjoint ranges of them
    auto build0 = std::chrono::steady_clock::now();
    slot_order_touched(n);
    const size_t nt = n->touched.size();
    const unsigned k = n->pool->ways_small(nt, 2048, 512);
    n->pool->run(
        [&](unsigned t) {
          size_t lo, hi;
          split(nt, k, t, &lo, &hi);
          Arena& A = n->arenas[t];
          const bool ahead = nt >= 65536;  // (a small node's groups sit in cache already)
          for (size_t i = lo; i < hi; ++i) {
            if (ahead && i + 4 < hi) {  // the group 4 ahead, then what the group 2 ahead points to
              const char* q = reinterpret_cast<const char*>(n->touched[i + 4]);
              for (int l = 0; l < 9; ++l) __builtin_prefetch(q + 64 * l);
            }
            if (ahead && i + 2 < hi) {
              const Group& q = *n->touched[i + 2];
              __builtin_prefetch(q.msgs.data());
              __builtin_prefetch(q.log.unstable.data());
              __builtin_prefetch(q.log.st);
            }
            build_ready(*n->touched[i], A, n->lists[t]);
          }
          patch_arena(A);
        },
        k);
    n->touched.clear();
    n->prof[PH_BUILD] += std::chrono::duration<double>(std::chrono::steady_clock::now() - build0).count();
    HBN_PHASE(n, PH_MERGE);
    merge(n->content, n->lists, &Lists::content);
    merge(n->delivered, n->lists, &Lists::delivered);
    size_t tot = 0;
    for (const Arena& A : n->arenas) tot += A.out.size();
    if (tot == 0) {
      rc = HBN_EAGAIN;
      return;
    }
    if (tot > n->r_cap) {
      n->r_out.reset(new hbn_group_ready[tot + tot / 4]);
      n->r_cap = tot + tot / 4;
    }
    // the workers' records, contiguous in worker order (each worker copies its own)
    std::vector<size_t> at(n->arenas.size() + 1, 0);
    for (size_t t = 0; t < n->arenas.size(); ++t) at[t + 1] = at[t] + n->arenas[t].out.size();
    const unsigned kc = tot < 4096 ? 1u : (unsigned)std::min<size_t>(n->pool->size(), n->arenas.size());
    n->pool->run(
        [&](unsigned t) {
          for (size_t a = t; a < n->arenas.size(); a += kc) {
            const std::vector<hbn_group_ready>& v = n->arenas[a].out;
            if (!v.empty()) std::memcpy(n->r_out.get() + at[a], v.data(), v.size() * sizeof(hbn_group_ready));
          }
        },
        kc);
    n->r_n = tot;
    n->awaiting_advance = true;
  });
  if (g0 != HB_OK) return g0;
  if (rc != HB_OK) return rc;
  *out = n->r_out.get();
  *count = n->r_n;
  return HB_OK;
}

int hbn_advance(hbn_node* n, const uint64_t* groups, uint64_t count) {
  if (!n || (count && !groups)) return HB_EINVAL;
  return guarded([&] {
    flush(n);
    HBN_PHASE(n, PH_ADVANCE);
    const unsigned k = n->pool->ways_small(count, 2048, n->pool->small_adv());
    n->pool->run(
        [&](unsigned t) {
          size_t lo, hi;
          split(count, k, t, &lo, &hi);
          Lists& L = n->lists[t];
          for (size_t i = lo; i < hi; ++i) {
            if (i + 16 < hi) __builtin_prefetch(n->groups.probe(groups[i + 16]));
            if (i + 8 < hi)
              if (const Group* q = n->groups.find(groups[i + 8])) {
                __builtin_prefetch(q);
                __builtin_prefetch(reinterpret_cast<const char*>(q) + 64);
                __builtin_prefetch(reinterpret_cast<const char*>(q) + 128);
              }
            Group* gp = n->groups.find(groups[i]);
            if (!gp) continue;
            Group& g = *gp;
            if (!__atomic_load_n(&g.delivered, __ATOMIC_RELAXED) ||
                !__atomic_exchange_n(&g.delivered, false, __ATOMIC_RELAXED))
              continue;  // (a group listed twice)
            materialize(g);  // messages stepped since the Ready still read the log
            commit_ready(g, g.dlv);
            // the recomputed Ready (raft/multinode.go:290-295) is a candidate again
            refresh_content(L.content, g);
            touch_into(L.touched, g, k > 1);
          }
        },
        k);
    merge(n->content, n->lists, &Lists::content);
    merge(n->touched, n->lists, &Lists::touched);
    n->awaiting_advance = false;
  });
}

int hbn_status(hbn_node* n, uint64_t group, hbn_group_status* out) {
  if (!n || !out) return HB_EINVAL;
  return guarded([&] {
    flush(n);
    Group& g = group_of(n, group);
    std::memset(out, 0, sizeof(*out));
    out->id = n->id;
    out->hard_state = g.hard();
    out->lead = g.lead;
    out->raft_state = g.state;
    out->applied = g.log.applied;
    if (g.state == HB_STATE_LEADER && g.slot != NO_SLOT) {
      hb_group r;
      check(hb_get_groups(n->h, g.slot, 1, &r));
      out->n_progress = (uint32_t)g.peers.size();
      for (size_t s = 0; s < g.peers.size(); ++s) {
        out->progress_id[s] = g.peers[s];
        out->progress[s] = r.pr[s];
      }
    }
  });
}

}  // extern "C"
