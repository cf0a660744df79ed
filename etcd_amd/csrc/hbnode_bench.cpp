// hbnode_bench.cpp — an application driving raft.MultiNode through the public C
// ABI (include/hbnode.h) the way the reference's node_bench_test.go drives a
// node (raft/node_bench_test.go:24-52, without its 1 ms sleep), scaled to many
// groups: every round steps each leader's MsgAppResp
// from its followers (shuffled), proposes one entry per group, then takes the
// Ready, appends its entries to the group's MemoryStorage and advances.
// Bench infrastructure only (bench.py --workload multinode); it uses nothing
// but the exported API.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <sched.h>
#include <thread>
#include <vector>

#include "../../include/hbnode.h"

namespace {
using clk = std::chrono::steady_clock;
double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }
}  // namespace

extern "C" {

// out[0] timed seconds, [1] MsgAppResp stepped, [2] commit advances (groups x rounds),
// [3] seconds in hbn_ready, [4] seconds in hbn_step/hbn_propose, [5] seconds in
// storage append + hbn_advance, [6] entries committed seen in Ready, [7] faults,
// [8 .. 8 + 16) the node's host phase seconds over the timed rounds (hbn_profile),
// [24] seconds the application spent persisting (hbn_storage_append); out has 32 slots.
// flags: HBNB_BULK = the round's acks and proposals through hbn_step_many /
// hbn_propose_many (one call each) instead of one call per message;
// HBNB_PAR_APP = the application persists a Ready's entries to the groups'
// storages from `threads` threads (storages are independent).  threads: the
// node's host threads too (hbn_set_threads; 0 = the library default).
#define HBNB_BULK 1u
#define HBNB_PAR_APP 2u
// HBNB_PIN: the application pins its Ready-loop thread to the CPU it starts on,
// after hbn_start (whose small-phase partners share that CPU's L3; the
// threads the library starts inherit the unpinned mask)
#define HBNB_PIN 4u
int hbnb_run2(int device, uint32_t G, uint32_t n, uint32_t warmup, uint32_t rounds, uint32_t flags,
              uint32_t threads, double* out);
int hbnb_run(int device, uint32_t G, uint32_t n, uint32_t warmup, uint32_t rounds, double* out) {
  return hbnb_run2(device, G, n, warmup, rounds, 0, 0, out);
}

int hbnb_run2(int device, uint32_t G, uint32_t n, uint32_t warmup, uint32_t rounds, uint32_t flags,
              uint32_t threads, double* out) {
  if (G == 0 || n < 2 || n > HB_MAX_REPLICAS || !out) return HB_EINVAL;
  cpu_set_t old_mask;
  const bool pinned = (flags & HBNB_PIN) && sched_getaffinity(0, sizeof(old_mask), &old_mask) == 0;
  const int cpu0 = sched_getcpu();  // the CPU the loop starts on (the node's partners share its L3)
  struct Unpin {
    bool on;
    cpu_set_t* m;
    ~Unpin() {
      if (on) (void)sched_setaffinity(0, sizeof(*m), m);
    }
  } unpin{pinned, &old_mask};
  hbn_node* mn = nullptr;
  const uint64_t max_batch = (uint64_t)G * n + 16;
  int rc = hbn_start(device, 1, G, n, 256, HB_NO_LIMIT, max_batch, &mn);
  if (rc) return rc;
  if (threads) rc = hbn_set_threads(mn, threads);
  // pinned only once the node (and its threads) exist: a thread the library
  // starts inherits the creating thread's mask, which must not be one CPU
  if (pinned && cpu0 >= 0) {
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(cpu0, &one);
    (void)sched_setaffinity(0, sizeof(one), &one);
  }
  const uint32_t app_threads =
      (flags & HBNB_PAR_APP) ? (threads ? threads : std::min(16u, std::max(1u, std::thread::hardware_concurrency()))) : 1;
  std::vector<hbn_storage*> st(G, nullptr);
  std::vector<uint64_t> peers(n), last(G, 0), commit(G, 0), ids(G);
  for (uint32_t i = 0; i < n; ++i) peers[i] = i + 1;
  hbn_config cfg{10, 1, 0};
  for (uint32_t g = 0; g < G && !rc; ++g) {
    ids[g] = g + 1;
    rc = hbn_storage_new(&st[g]);
    if (!rc) rc = hbn_create_group(mn, ids[g], &cfg, st[g], peers.data(), n);
    if (!rc) rc = hbn_campaign(mn, ids[g]);
  }
  hbn_message m;
  std::memset(&m, 0, sizeof(m));
  m.type = HB_MSG_VOTE_RESP;
  m.term = 2;
  for (uint32_t g = 0; g < G && !rc; ++g)
    for (uint32_t p = 2; p <= n && !rc; ++p) {
      m.from = p;
      rc = hbn_step(mn, ids[g], &m);
    }
  uint64_t faults = 0, committed_entries = 0, advances = 0;
  double t_ready = 0, t_step = 0, t_adv = 0, t_persist = 0;
  std::vector<uint64_t> adv;  // the groups to advance (kept across cycles)
  // one Ready cycle: take the Ready, persist its entries, advance
  auto cycle = [&]() -> int {
    const hbn_group_ready* rds = nullptr;
    uint64_t cnt = 0;
    auto a = clk::now();
    int r = hbn_ready(mn, &rds, &cnt);
    auto b = clk::now();
    t_ready += secs(a, b);
    if (r == HBN_EAGAIN) return 0;
    if (r) return r;
    if (adv.size() < cnt) adv.resize(cnt);
    // the application's part: persist each group's entries (MemoryStorage.Append)
    // (counts kept in locals: the threads' result slots share a cache line)
    auto persist = [&](uint64_t lo, uint64_t hi, uint64_t* f, uint64_t* ce, uint64_t* av) -> int {
      uint64_t nf = 0, nce = 0, nav = 0;
      int rc2 = 0;
      for (uint64_t i = lo; i < hi && !rc2; ++i) {
        const hbn_group_ready& rd = rds[i];
        const uint64_t g = rd.group - 1;
        nf += rd.fault != 0;
        if (rd.n_entries) {
          rc2 = hbn_storage_append(st[g], rd.entries, rd.n_entries);
          last[g] = rd.entries[rd.n_entries - 1].index;
        }
        nce += rd.n_committed;
        if (rd.hard_state.commit > commit[g]) {
          commit[g] = rd.hard_state.commit;
          ++nav;
        }
        adv[i] = rd.group;
      }
      *f += nf;
      *ce += nce;
      *av += nav;
      return rc2;
    };
    auto p0 = clk::now();
    if (app_threads > 1 && cnt >= 4096) {
      std::vector<uint64_t> f(app_threads), ce(app_threads), av(app_threads);
      std::vector<int> er(app_threads);
      std::vector<std::thread> th;
      for (uint32_t t = 0; t < app_threads; ++t)
        th.emplace_back([&, t] {
          if (pinned) (void)sched_setaffinity(0, sizeof(old_mask), &old_mask);  // (not the loop thread's CPU)
          er[t] = persist(cnt * t / app_threads, cnt * (t + 1) / app_threads, &f[t], &ce[t], &av[t]);
        });
      for (auto& x : th) x.join();
      for (uint32_t t = 0; t < app_threads; ++t) {
        if (er[t]) return er[t];
        faults += f[t];
        committed_entries += ce[t];
        advances += av[t];
      }
    } else {
      r = persist(0, cnt, &faults, &committed_entries, &advances);
      if (r) return r;
    }
    t_persist += secs(p0, clk::now());
    r = hbn_advance(mn, adv.data(), cnt);
    t_adv += secs(b, clk::now());
    return r;
  };
  if (G >= 100000) std::fprintf(stderr, "hbnb: %u groups created, electing\n", G);
  for (int k = 0; k < 4 && !rc; ++k) rc = cycle();  // leaders elected, bootstrap + noop entries persisted
  std::vector<uint64_t> order((size_t)G * (n - 1));
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::mt19937_64 rng(1);
  std::shuffle(order.begin(), order.end(), rng);
  m.type = HB_MSG_APP_RESP;
  static const uint8_t foo[3] = {'f', 'o', 'o'};
  std::vector<uint64_t> bg(order.size());
  std::vector<hbn_message> bm(order.size());
  std::vector<const uint8_t*> pdata(G, foo);
  std::vector<uint64_t> plen(G, 3);
  auto t0 = clk::now();
  uint64_t acks = 0;
  double prof0[16] = {}, prof1[16] = {};
  for (uint32_t r = 0; r < warmup + rounds && !rc; ++r) {
    if (r == warmup) {
      t0 = clk::now();
      acks = 0;
      advances = 0;
      committed_entries = 0;
      t_ready = t_step = t_adv = t_persist = 0;
      hbn_profile(mn, prof0, 16, nullptr);
    }
    auto a = clk::now();
    if (flags & HBNB_BULK) {  // the round's network input and proposals, one call each
      auto fill = [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
          const uint64_t g = order[i] / (n - 1);
          bg[i] = ids[g];
          bm[i] = m;
          bm[i].from = 2 + order[i] % (n - 1);
          bm[i].index = last[g];
        }
      };
      const size_t no = order.size();
      if (app_threads > 1 && no >= 65536) {  // (the application builds a large round's messages on its threads)
        std::vector<std::thread> th;
        for (uint32_t t = 0; t < app_threads; ++t)
          th.emplace_back([&, t] {
            if (pinned) (void)sched_setaffinity(0, sizeof(old_mask), &old_mask);
            fill(no * t / app_threads, no * (t + 1) / app_threads);
          });
        for (auto& x : th) x.join();
      } else {
        fill(0, no);
      }
      uint64_t done = 0;
      rc = hbn_step_many(mn, order.size(), bg.data(), bm.data(), &done);
      acks += done;
      if (!rc) rc = hbn_propose_many(mn, G, ids.data(), pdata.data(), plen.data(), &done);
    } else {
      for (size_t i = 0; i < order.size() && !rc; ++i) {  // followers ack the last round's entries
        const uint64_t g = order[i] / (n - 1);
        m.from = 2 + order[i] % (n - 1);
        m.index = last[g];
        rc = hbn_step(mn, ids[g], &m);
        ++acks;
      }
      for (uint32_t g = 0; g < G && !rc; ++g) rc = hbn_propose(mn, ids[g], foo, 3);
    }
    t_step += secs(a, clk::now());
    if (!rc) rc = cycle();
    if (G >= 100000) {  // progress for long runs
      std::fprintf(stderr, "hbnb: round %u of %u (%.2f s)\n", r + 1, warmup + rounds, secs(t0, clk::now()));
      std::fflush(stderr);
    }
  }
  const double total = secs(t0, clk::now());
  hbn_profile(mn, prof1, 16, nullptr);
  for (int i = 0; i < 16; ++i) out[8 + i] = prof1[i] - prof0[i];
  out[0] = total;
  out[1] = (double)acks;
  out[2] = (double)advances;
  out[3] = t_ready;
  out[4] = t_step;
  out[5] = t_adv;
  out[6] = (double)committed_entries;
  out[7] = (double)faults;
  out[24] = t_persist;
  hbn_stop(mn);
  for (auto* s : st) hbn_storage_free(s);
  return rc;
}

}  // extern "C"
