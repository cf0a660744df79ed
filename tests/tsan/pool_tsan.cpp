// ThreadSanitizer harness for libhbnode's host threading (no GPU needed):
// the Pool of etcd_amd/csrc/hbpool.h — run / prewake / post / STOP, the
// small-phase partners' spin on and off, small and large cycles, pools of 1-16
// workers, two nodes' pools side by side (the process-wide partner-core
// claims) — and the router's threaded passes (hbroute.cpp: hbn_route /
// hbn_route_take over multi-chunk streams, checked against a sequential
// restatement).  Built with -fsanitize=thread by tests/test_sanitizers.py;
// exits non-zero on a wrong result, and TSan reports any race it sees.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../etcd_amd/csrc/hbpool.h"
#include "../../include/hbroute.h"

using hbpool::Pool;

static int g_fail = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail = 1;                                                 \
    }                                                             \
  } while (0)

// One node's cycles: each phase splits an array over k workers (disjoint
// slices, as the replay and the Ready build do), the caller then reads it all.
static void drive_pool(unsigned workers, unsigned rounds, unsigned seed) {
  Pool pool(workers);
  std::vector<uint64_t> data(4096, 0);
  uint64_t expect = 0;
  for (unsigned r = 0; r < rounds; ++r) {
    const bool small = ((r + seed) % 3) != 0;
    pool.set_small_cycle(small);
    if ((r + seed) % 2) pool.prewake(pool.small_ways());
    const unsigned k = 1 + (r * 7 + seed) % pool.size();
    pool.run(
        [&](unsigned t) {
          const size_t lo = data.size() * t / k, hi = data.size() * (t + 1) / k;
          for (size_t i = lo; i < hi; ++i) data[i] += i + r;
        },
        k);
    for (size_t i = 0; i < data.size(); ++i) expect += i + r;
    uint64_t sum = 0;
    for (uint64_t v : data) sum += v;
    CHECK(sum == expect);
    if (r % 17 == 5 && k > 1) {  // a worker's exception reaches the caller, the pool stays usable
      bool caught = false;
      try {
        pool.run([&](unsigned t) {
          if (t == k - 1) throw std::runtime_error("boom");
        }, k);
      } catch (const std::runtime_error&) {
        caught = true;
      }
      CHECK(caught);
    }
    if (r % 11 == 3) std::this_thread::sleep_for(std::chrono::microseconds(200));  // partners go to sleep
  }
}

static void route_check(unsigned threads) {
  const uint64_t G = 50000, N = 600000;
  const uint32_t W = 3;
  std::vector<uint64_t> ids(G);
  for (uint64_t i = 0; i < G; ++i) ids[i] = i * 0x9E3779B97F4A7C15ull;  // sparse: the hash table
  hbn_router* r = nullptr;
  CHECK(hbn_router_create(ids.data(), G, W, threads, &r) == 0);
  if (!r) return;
  std::vector<uint64_t> gids(N), gidx(N);
  uint64_t x = 12345;
  for (uint64_t i = 0; i < N; ++i) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    gidx[i] = (x >> 33) % G;
    gids[i] = (i % 97 == 0) ? 7 : ids[gidx[i]];  // 7: an unknown id
  }
  uint64_t counts[W], unk = 0;
  CHECK(hbn_route(r, gids.data(), N, counts, &unk) == 0);
  std::vector<std::vector<uint64_t>> pos(W);
  std::vector<std::vector<uint32_t>> slot(W);
  uint64_t* pp[W];
  uint32_t* sp[W];
  for (uint32_t k = 0; k < W; ++k) {
    pos[k].resize(counts[k]);
    slot[k].resize(counts[k]);
    pp[k] = pos[k].data();
    sp[k] = slot[k].data();
  }
  CHECK(hbn_route_take(r, pp, sp) == 0);
  // sequential restatement: owner, slot = position among the rank's ids, arrival order
  std::vector<uint32_t> rank_of(G), slot_of(G);
  std::vector<uint32_t> fill(W, 0);
  for (uint64_t i = 0; i < G; ++i) {
    rank_of[i] = hbn_owner(ids[i], W);
    slot_of[i] = fill[rank_of[i]]++;
  }
  std::vector<size_t> at(W, 0);
  uint64_t n_unk = 0;
  for (uint64_t i = 0; i < N; ++i) {
    if (gids[i] == 7) {
      n_unk++;
      continue;
    }
    const uint64_t gi = gidx[i];
    const uint32_t k = rank_of[gi];
    CHECK(at[k] < counts[k] && pos[k][at[k]] == i && slot[k][at[k]] == slot_of[gi]);
    at[k]++;
  }
  CHECK(n_unk == unk);
  hbn_router_destroy(r);
}

int main() {
  for (const char* spin : {"0", "150"}) {
    setenv("HBN_SPIN_US", spin, 1);
    for (unsigned w : {1u, 2u, 4u, 8u, 16u}) drive_pool(w, 120, w);
    // two nodes in one process, started from two threads (one handle per GPU)
    std::thread a([] { drive_pool(8, 80, 1); });
    std::thread b([] { drive_pool(8, 80, 2); });
    a.join();
    b.join();
  }
  for (unsigned t : {1u, 4u, 16u}) route_check(t);
  std::puts(g_fail ? "pool_tsan FAILED" : "pool_tsan ok");
  return g_fail;
}
