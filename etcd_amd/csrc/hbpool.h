// hbpool.h — the host thread pool of libhbnode (hbnode.cpp) and its CPU
// placement, in a header of its own so that the ThreadSanitizer harness
// (tests/tsan/pool_tsan.cpp) builds the same code without the engine.
#pragma once

#include <sched.h>
#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace hbpool {

// ---------------------------------------------------------------- host threads
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#endif
}
// CPUs of a sysfs cpu list ("0-7,128-135")
inline void parse_cpu_list(const char* path, cpu_set_t* set) {
  CPU_ZERO(set);
  FILE* f = std::fopen(path, "r");
  if (!f) return;
  char buf[1024];
  const size_t len = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[len] = 0;
  for (char* p = buf; *p;) {
    char* e = nullptr;
    const long a = std::strtol(p, &e, 10);
    if (e == p) break;
    long b = a;
    p = e;
    if (*p == '-') b = std::strtol(p + 1, &p, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET((int)c, set);
    while (*p == ',' || *p == '\n' || *p == ' ') ++p;
  }
}
// The CPUs a worker may run on: the creating thread's affinity mask (what a
// process-level taskset / numactl binding set, and what the workers inherit),
// else every online CPU.
inline void allowed_cpus(cpu_set_t* out) {
  CPU_ZERO(out);
  if (sched_getaffinity(0, sizeof(*out), out) != 0 || CPU_COUNT(out) == 0)
    parse_cpu_list("/sys/devices/system/cpu/online", out);
}
// Partner cores are handed out process-wide: two nodes (one per GPU, one
// process) started from threads on one CCD would otherwise pin their partners
// to the same cores and spin against each other.  A core already claimed is
// skipped; a node that finds none free pins nothing.
inline std::mutex g_core_mu;
inline std::vector<int> g_core_claims(CPU_SETSIZE, 0);
// One CPU per physical core sharing the calling thread's L3 (its CCD on
// EPYC), its own core excluded and only CPUs of its affinity mask, in core
// order; empty when the topology is unknown.
inline std::vector<int> l3_partner_cores() {
  std::vector<int> out;
  const int c = sched_getcpu();
  if (c < 0) return out;
  cpu_set_t l3, allowed, seen;
  char path[128];
  std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", c);
  parse_cpu_list(path, &l3);
  allowed_cpus(&allowed);
  CPU_ZERO(&seen);
  for (int i = 0; i < CPU_SETSIZE; ++i) {
    if (!CPU_ISSET(i, &l3) || CPU_ISSET(i, &seen)) continue;
    cpu_set_t sib;
    std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", i);
    parse_cpu_list(path, &sib);
    CPU_SET(i, &sib);
    CPU_OR(&seen, &seen, &sib);
    if (!CPU_ISSET(c, &sib) && CPU_ISSET(i, &allowed)) out.push_back(i);
  }
  return out;
}

// Groups are independent (raft/multinode.go:125-131), so the per-group host
// work of a Ready cycle — replaying the device's events, assembling Ready,
// Advance, bulk ingestion — runs on a pool of host threads, each owning a
// disjoint set of groups; the node's membership lists are appended per thread
// and merged in thread order.  The calling thread is worker 0.
class Pool {
 public:
  explicit Pool(unsigned n) : n_(n ? n : 1), w_(n_) {
    if (const char* e = std::getenv("HBN_SMALL_WAYS")) set_small_ways((unsigned)std::max(1, std::atoi(e)));
    if (const char* e = std::getenv("HBN_SMALL_ADV")) adv_min_ = (size_t)std::max(1, std::atoi(e));  // (A/B knob)
    if (const char* e = std::getenv("HBN_SPIN_US")) spin_us_ = (unsigned)std::max(0, std::atoi(e));
    if (const char* e = std::getenv("HBN_SMALL_BULK")) bulk_min_ = (size_t)std::max(1, std::atoi(e));
    for (unsigned t = 1; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
    // The small phases' partners (workers 1 .. small_ways-1) run on the creating
    // thread's L3 (CCD), one physical core each: the groups they replay and
    // assemble move between the threads' caches every phase, and across CCDs
    // each such line costs a remote fetch (measured: 1k-group cycles 2.5-3x
    // slower whenever the scheduler placed a partner on another CCD).
    // HBN_PIN_L3=0: no pinning.  Cores come from the creating thread's
    // affinity mask and are claimed process-wide (g_core_claims); a partner
    // without a free core of its own stays unpinned.
    // Every other worker keeps the mask it inherits from the creating thread
    // (measured at 1M groups: pinning them to the creating thread's NUMA node
    // changed nothing).
    const char* pin = std::getenv("HBN_PIN_L3");
    const std::vector<int> cores =
        (!pin || pin[0] != '0') && n_ > 1 ? l3_partner_cores() : std::vector<int>();
    std::lock_guard<std::mutex> lk(g_core_mu);
    size_t ci = 0;
    for (unsigned t = 1; t < n_ && t < small_; ++t) {
      while (ci < cores.size() && g_core_claims[cores[ci]] != 0) ++ci;
      if (ci == cores.size()) break;
      const int core = cores[ci++];
      cpu_set_t one;
      CPU_ZERO(&one);
      CPU_SET(core, &one);
      if (pthread_setaffinity_np(th_[t - 1].native_handle(), sizeof(one), &one) == 0) {
        g_core_claims[core]++;
        claimed_.push_back(core);
      }
    }
  }
  ~Pool() {
    for (unsigned t = 1; t < n_; ++t) post(t, STOP);
    for (auto& t : th_) t.join();
    std::lock_guard<std::mutex> lk(g_core_mu);
    for (int c : claimed_) g_core_claims[c]--;
  }
  // The partners spin (after a job, after a prewake) only while the node's
  // cycles are small (hbn_ready decides per cycle from its batch): a large
  // node's phases run for milliseconds, and spinning there only burns cores.
  void set_small_cycle(bool on) { small_cycle_.store(on, std::memory_order_relaxed); }
  bool small_cycle() const { return small_cycle_.load(std::memory_order_relaxed); }
  unsigned size() const { return n_; }
  // workers for `items` units of work of which one worker should take at least `grain`
  unsigned ways(size_t items, size_t grain) const {
    const size_t k = items / (grain ? grain : 1);
    return (unsigned)std::max<size_t>(1, std::min<size_t>(n_, k));
  }
  // ... and for the two long phases of a small node's Ready cycle (event replay,
  // Ready build: ~100 us each at 1k groups), up to small_ways() workers once
  // `items` reaches `small_min` — one futex wake per extra worker, which the
  // caller's own share hides
  unsigned ways_small(size_t items, size_t grain, size_t small_min) const {
    const unsigned k = ways(items, grain);
    if (k > 1 || items < small_min) return k;
    return std::min<unsigned>(n_, small_);
  }
  void set_small_ways(unsigned k) { small_ = k ? k : 1; }
  size_t small_adv() const { return adv_min_; }
  size_t small_bulk() const { return bulk_min_; }
  // Wake workers 1..k-1 ahead of a phase (hbn_ready: while the device steps),
  // so that, spinning for up to spin_us, they take the phase's job at once.
  void prewake(unsigned k) {
    if (!spin_us_ || !small_cycle()) return;
    for (unsigned t = 1; t < k && t < n_; ++t) {
      Worker& w = w_[t];
      w.poke.store(true);
      if (w.sleeping.load()) {
        std::lock_guard<std::mutex> lk(w.mu);
        w.cv.notify_one();
      }
    }
  }
  unsigned small_ways() const { return std::min(n_, small_); }
  // f(tid) for tid in [0, k) (k = use, at most size()); returns once every
  // worker finished; the first exception (lowest tid) is rethrown on the
  // calling thread
  template <class F>
  void run(F&& f, unsigned use = 0) {
    const unsigned k = use && use < n_ ? use : n_;
    if (k == 1) {  // the calling thread alone
      f(0u);
      return;
    }
    std::vector<std::exception_ptr> err(k);
    auto body = [&](unsigned t) {
      try {
        f(t);
      } catch (...) {
        err[t] = std::current_exception();
      }
    };
    if (k > 1) {
      job_ = body;
      left_.store(k - 1);
      for (unsigned t = 1; t < k; ++t) post(t, ++w_[t].seq);
      body(0);
      if (left_.load() != 0) {
        std::unique_lock<std::mutex> lk(mu_);
        waiting_.store(true);
        done_.wait(lk, [&] { return left_.load() == 0; });
        waiting_.store(false);
      }
      job_ = nullptr;
    } else {
      body(0);
    }
    for (auto& e : err)
      if (e) std::rethrow_exception(e);
  }

 private:
  static constexpr uint64_t STOP = ~0ull;
  // Only the workers a phase uses are woken (one futex each); nobody polls.
  // Polling for ~20-50 us between phases (r03, and again r04 with per-worker
  // wake-ups) made the 1k-group MultiNode 3-5x slower on the GPU box — every
  // phase, single-threaded ones included, slowed down next to the polling
  // threads under the box's 16-CPU quota — so small phases run on the calling
  // thread alone (ways()) and workers block between phases.  (Blocking
  // workers on 1k-group phases — grains 256-1024 — measured 0.37 and 1.22 ms
  // per cycle in two runs on one box against 0.43-0.44 ms single-threaded:
  // not kept.)
  struct alignas(64) Worker {
    std::atomic<uint64_t> post{0};  // the job sequence number posted to this worker (STOP: exit)
    std::atomic<bool> sleeping{false};
    std::atomic<bool> poke{false};  // prewake(): spin for the next job
    std::mutex mu;
    std::condition_variable cv;
    uint64_t seq = 0;  // (caller side) the last number posted
  };
  void post(unsigned t, uint64_t v) {
    Worker& w = w_[t];
    w.post.store(v);  // (seq_cst, against the worker's sleeping flag)
    if (w.sleeping.load()) {
      std::lock_guard<std::mutex> lk(w.mu);
      w.cv.notify_one();
    }
  }
  void loop(unsigned t) {
    Worker& w = w_[t];
    uint64_t seen = 0;
    bool spin = false;
    for (;;) {
      if (spin && spin_us_ && t < small_ && small_cycle()) {  // (a small-phase partner, after a job or a prewake) spin briefly
        const auto t0 = std::chrono::steady_clock::now();
        const auto lim = std::chrono::microseconds(spin_us_);
        while (w.post.load(std::memory_order_acquire) == seen && std::chrono::steady_clock::now() - t0 < lim)
          cpu_relax();
      }
      if (w.post.load() == seen) {
        std::unique_lock<std::mutex> lk(w.mu);
        w.sleeping.store(true);
        w.cv.wait(lk, [&] { return w.post.load() != seen || w.poke.load(); });
        w.sleeping.store(false);
        if (w.post.load() == seen) {  // poked: spin for the job
          w.poke.store(false);
          spin = true;
          continue;
        }
      }
      w.poke.store(false);
      spin = true;
      seen = w.post.load();
      if (seen == STOP) return;
      job_(t);
      if (left_.fetch_sub(1) == 1 && waiting_.load()) {
        std::lock_guard<std::mutex> lk(mu_);
        done_.notify_one();
      }
    }
  }
  unsigned n_;
  unsigned small_ = 4;
  unsigned spin_us_ = 150;  // HBN_SPIN_US: the small-phase partners spin this long after a job / prewake
  size_t adv_min_ = 512;  // Advance: split over the partners from this many groups on
  size_t bulk_min_ = 512;  // bulk ingestion (HBN_SMALL_BULK): the same, from this many messages
  std::vector<Worker> w_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable done_;
  std::function<void(unsigned)> job_;
  std::atomic<unsigned> left_{0};
  std::atomic<bool> waiting_{false};
  std::atomic<bool> small_cycle_{true};
  std::vector<int> claimed_;  // partner cores this pool holds in g_core_claims
};
// hbn_ready: a cycle below SMALL_CYCLE_MSGS messages lets the partners spin
// between its phases; from PREWAKE_MIN_MSGS on they are woken while the
// device steps (the replay of fewer messages' events stays on the caller).
constexpr uint64_t SMALL_CYCLE_MSGS = 65536;
constexpr uint64_t PREWAKE_MIN_MSGS = 256;

}  // namespace hbpool
