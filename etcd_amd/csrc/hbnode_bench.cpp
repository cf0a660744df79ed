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
#include <vector>

#include "../../include/hbnode.h"

namespace {
using clk = std::chrono::steady_clock;
double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }
}  // namespace

extern "C" {

// out[0] timed seconds, [1] MsgAppResp stepped, [2] commit advances (groups x rounds),
// [3] seconds in hbn_ready, [4] seconds in hbn_step/hbn_propose, [5] seconds in
// storage append + hbn_advance, [6] entries committed seen in Ready, [7] faults.
int hbnb_run(int device, uint32_t G, uint32_t n, uint32_t warmup, uint32_t rounds, double* out) {
  if (G == 0 || n < 2 || n > HB_MAX_REPLICAS || !out) return HB_EINVAL;
  hbn_node* mn = nullptr;
  const uint64_t max_batch = (uint64_t)G * n + 16;
  int rc = hbn_start(device, 1, G, n, 256, HB_NO_LIMIT, max_batch, &mn);
  if (rc) return rc;
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
  double t_ready = 0, t_step = 0, t_adv = 0;
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
    std::vector<uint64_t> adv(cnt);
    for (uint64_t i = 0; i < cnt; ++i) {
      const hbn_group_ready& rd = rds[i];
      const uint64_t g = rd.group - 1;
      faults += rd.fault != 0;
      if (rd.n_entries) {
        r = hbn_storage_append(st[g], rd.entries, rd.n_entries);
        if (r) return r;
        last[g] = rd.entries[rd.n_entries - 1].index;
      }
      committed_entries += rd.n_committed;
      if (rd.hard_state.commit > commit[g]) {
        commit[g] = rd.hard_state.commit;
        ++advances;
      }
      adv[i] = rd.group;
    }
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
  auto t0 = clk::now();
  uint64_t acks = 0;
  for (uint32_t r = 0; r < warmup + rounds && !rc; ++r) {
    if (r == warmup) {
      t0 = clk::now();
      acks = 0;
      advances = 0;
      committed_entries = 0;
      t_ready = t_step = t_adv = 0;
    }
    auto a = clk::now();
    for (size_t i = 0; i < order.size() && !rc; ++i) {  // followers ack the last round's entries
      const uint64_t g = order[i] / (n - 1);
      m.from = 2 + order[i] % (n - 1);
      m.index = last[g];
      rc = hbn_step(mn, ids[g], &m);
      ++acks;
    }
    for (uint32_t g = 0; g < G && !rc; ++g) rc = hbn_propose(mn, ids[g], foo, 3);
    t_step += secs(a, clk::now());
    if (!rc) rc = cycle();
    if (G >= 100000) {  // progress for long runs
      std::fprintf(stderr, "hbnb: round %u of %u (%.2f s)\n", r + 1, warmup + rounds, secs(t0, clk::now()));
      std::fflush(stderr);
    }
  }
  const double total = secs(t0, clk::now());
  out[0] = total;
  out[1] = (double)acks;
  out[2] = (double)advances;
  out[3] = t_ready;
  out[4] = t_step;
  out[5] = t_adv;
  out[6] = (double)committed_entries;
  out[7] = (double)faults;
  hbn_stop(mn);
  for (auto* s : st) hbn_storage_free(s);
  return rc;
}

}  // extern "C"
