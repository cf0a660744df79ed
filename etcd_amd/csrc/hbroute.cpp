// hbroute.cpp — host owner routing across a node's GPUs (include/hbroute.h).
//
// One pass over an arrival-ordered stream, split into contiguous chunks over
// host threads: pass 1 counts each chunk's messages per rank, a prefix over
// (rank, chunk) gives every chunk its output offsets, pass 2 writes each
// message's stream position and local slot to its rank's arrays.  Chunks are
// contiguous and written at increasing offsets, so every rank's messages keep
// arrival order (raft/multinode.go:233-237 steps a group's messages in the
// order the run goroutine receives them).  The owner hash and slot of a group
// id come from one lookup: a flat table for a dense id space, else an
// open-addressing table (16-byte slots, load <= 1/2).
#include <algorithm>
#include <cstring>
#include <memory>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/hbroute.h"
#include "../../include/hipbatch.h"

namespace {

inline uint64_t splitmix64(uint64_t x) {  // etcd_amd/synth.py splitmix64
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr uint32_t NONE = 0xFFFFFFFFu;

// The exports' bodies run under this: nothing thrown crosses the C boundary
// (a Go / Python host would std::terminate).  A failed allocation is
// HB_ENOMEM, as in the rest of libhbnode (hbnode.cpp guarded()).
template <class F>
int route_guarded(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return HB_ENOMEM;
  } catch (const std::system_error&) {  // (thread resources: parallel() runs such a chunk inline)
    return HB_ENOMEM;
  } catch (...) {
    return HB_EINVARIANT;
  }
}

}  // namespace

constexpr uint32_t SLOT_BITS = 24;  // an engine holds at most 2^24 groups (hb_create)
constexpr uint32_t SLOT_MASK = (1u << SLOT_BITS) - 1;

struct hbn_router {
  uint32_t world = 1, threads = 1;
  uint64_t n = 0;
  // a group's place, rank << 24 | local slot (NONE: unknown): a flat table over
  // a dense id space, else open addressing (key UINT64_MAX = empty; that id
  // itself is kept aside)
  bool dense = false;
  std::vector<uint32_t> loc;
  std::vector<uint64_t> hkey;
  std::vector<uint32_t> hval;
  uint64_t hmask = 0;
  bool has_max = false;
  uint32_t max_val = NONE;
  std::vector<std::vector<uint64_t>> ids;  // per rank: slot -> id
  // the last hbn_route: each message's place, and per (chunk, rank) output offsets
  std::vector<uint32_t> place;
  std::vector<uint64_t> off;
  uint64_t n_last = 0, T_last = 0, per_last = 0;

  inline void prefetch(uint64_t id) const {
    if (dense) {
      if (id < loc.size()) __builtin_prefetch(&loc[id]);
    } else {
      __builtin_prefetch(&hkey[splitmix64(id ^ 0x5bd1e995ull) & hmask]);
    }
  }
  inline uint32_t find(uint64_t id) const {
    if (dense) return id < loc.size() ? loc[id] : NONE;
    if (id == ~0ull) return has_max ? max_val : NONE;
    uint64_t h = splitmix64(id ^ 0x5bd1e995ull) & hmask;
    while (true) {
      const uint64_t k = hkey[h];
      if (k == id) return hval[h];
      if (k == ~0ull) return NONE;
      h = (h + 1) & hmask;
    }
  }
  // body(t) for t in [0, T): chunk 0 on the calling thread; a chunk whose
  // thread cannot be started runs inline (the threads started are always joined)
  template <class F>
  void parallel(uint64_t T, F&& body) {
    std::vector<std::thread> th;
    th.reserve(T);
    std::vector<uint64_t> inl;
    for (uint64_t t = 1; t < T; ++t) {
      try {
        th.emplace_back(body, t);
      } catch (const std::system_error&) {
        inl.push_back(t);
      }
    }
    body(0);
    for (uint64_t t : inl) body(t);
    for (auto& x : th) x.join();
  }
};

namespace {

int router_create(const uint64_t* ids, uint64_t n, uint32_t world, uint32_t threads, hbn_router** out) {
  std::unique_ptr<hbn_router> r(new hbn_router);
  r->world = world;
  r->n = n;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  r->threads = threads ? threads : std::min(16u, hw);
  r->ids.assign(world, {});
  uint64_t mx = 0;
  for (uint64_t i = 0; i < n; ++i) mx = std::max(mx, ids[i]);
  r->dense = n > 0 && mx < 2 * n + 1024;
  if (r->dense) {
    r->loc.assign(mx + 1, NONE);
  } else {
    uint64_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    r->hkey.assign(cap, ~0ull);
    r->hval.assign(cap, NONE);
    r->hmask = cap - 1;
  }
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t id = ids[i];
    const uint32_t k = hbn_owner(id, world);
    if (r->ids[k].size() > SLOT_MASK) return HB_EINVAL;  // more than an engine holds
    const uint32_t v = (k << SLOT_BITS) | (uint32_t)r->ids[k].size();
    if (r->dense) {
      if (r->loc[id] != NONE) return HB_EINVAL;  // a duplicate id
      r->loc[id] = v;
    } else if (id == ~0ull) {
      if (r->has_max) return HB_EINVAL;
      r->has_max = true;
      r->max_val = v;
    } else {
      uint64_t h = splitmix64(id ^ 0x5bd1e995ull) & r->hmask;
      while (r->hkey[h] != ~0ull && r->hkey[h] != id) h = (h + 1) & r->hmask;
      if (r->hkey[h] == id) return HB_EINVAL;
      r->hkey[h] = id;
      r->hval[h] = v;
    }
    r->ids[k].push_back(id);
  }
  *out = r.release();
  return HB_OK;
}

int route(hbn_router* r, const uint64_t* gids, uint64_t n, uint64_t* counts, uint64_t* unknown) {
  const uint32_t W = r->world;
  // contiguous chunks of at least 64K messages, one per thread at most
  const uint64_t T = std::max<uint64_t>(1, std::min<uint64_t>(r->threads, (n + 65535) / 65536));
  const uint64_t per = (n + T - 1) / T;
  if (r->place.size() < n) r->place.resize(n);
  std::vector<uint64_t> cnt(T * (W + 1), 0);  // [chunk][rank], last column: unknown ids
  // the one pass over the stream: each message's place (the only random
  // accesses, prefetched ahead), counted per chunk and rank
  r->parallel(T, [&](uint64_t t) {
    const uint64_t lo = t * per, hi = std::min(n, lo + per);
    uint64_t* c = cnt.data() + t * (W + 1);
    uint32_t* pl = r->place.data();
    for (uint64_t i = lo; i < hi; ++i) {
      if (i + 24 < hi) r->prefetch(gids[i + 24]);
      const uint32_t v = r->find(gids[i]);
      pl[i] = v;
      c[v == NONE ? W : (v >> SLOT_BITS)]++;
    }
  });
  r->off.assign(T * W, 0);
  for (uint32_t k = 0; k < W; ++k) {
    uint64_t s = 0;
    for (uint64_t t = 0; t < T; ++t) {
      r->off[t * W + k] = s;
      s += cnt[t * (W + 1) + k];
    }
    counts[k] = s;
  }
  uint64_t unk = 0;
  for (uint64_t t = 0; t < T; ++t) unk += cnt[t * (W + 1) + W];
  if (unknown) *unknown = unk;
  r->n_last = n;
  r->T_last = T;
  r->per_last = per;
  return HB_OK;
}

int route_take(hbn_router* r, uint64_t* const* pos, uint32_t* const* slot) {
  const uint32_t W = r->world;
  const uint64_t n = r->n_last, T = r->T_last, per = r->per_last;
  // each chunk writes its messages at its offsets: sequential reads of the
  // places, sequential writes per rank
  r->parallel(T, [&](uint64_t t) {
    const uint64_t lo = t * per, hi = std::min(n, lo + per);
    uint64_t o[256];  // (world <= 255; nothing in a chunk's thread allocates, so nothing throws there)
    std::copy(r->off.begin() + t * W, r->off.begin() + (t + 1) * W, o);
    const uint32_t* pl = r->place.data();
    for (uint64_t i = lo; i < hi; ++i) {
      const uint32_t v = pl[i];
      if (v == NONE) continue;
      const uint32_t k = v >> SLOT_BITS;
      const uint64_t j = o[k]++;
      if (pos && pos[k]) pos[k][j] = i;
      if (slot && slot[k]) slot[k][j] = v & SLOT_MASK;
    }
  });
  return HB_OK;
}

}  // namespace

extern "C" {

uint32_t hbn_owner(uint64_t group_id, uint32_t world) {
  return world <= 1 ? 0u : (uint32_t)(splitmix64(group_id) % world);
}

int hbn_router_destroy(hbn_router* r) {
  delete r;
  return HB_OK;
}

uint64_t hbn_router_local_count(const hbn_router* r, uint32_t rank) {
  return (r && rank < r->world) ? r->ids[rank].size() : 0;
}

int hbn_router_local_ids(const hbn_router* r, uint32_t rank, uint64_t* ids) {
  if (!r || rank >= r->world || (!ids && !r->ids[rank].empty())) return HB_EINVAL;
  if (!r->ids[rank].empty()) std::memcpy(ids, r->ids[rank].data(), r->ids[rank].size() * 8);
  return HB_OK;
}

int hbn_router_create(const uint64_t* ids, uint64_t n, uint32_t world, uint32_t threads, hbn_router** out) {
  if (!out || world == 0 || world > 255 || (n && !ids)) return HB_EINVAL;
  *out = nullptr;
  return route_guarded([&] { return router_create(ids, n, world, threads, out); });
}

int hbn_route(hbn_router* r, const uint64_t* gids, uint64_t n, uint64_t* counts, uint64_t* unknown) {
  if (!r || !counts || (n && !gids)) return HB_EINVAL;
  return route_guarded([&] { return route(r, gids, n, counts, unknown); });
}

int hbn_route_take(hbn_router* r, uint64_t* const* pos, uint32_t* const* slot) {
  if (!r || (!pos && !slot)) return HB_EINVAL;
  return route_guarded([&] { return route_take(r, pos, slot); });
}

}  // extern "C"
