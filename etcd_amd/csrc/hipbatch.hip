// hipbatch.hip — MI355X (gfx950) batched Raft leader-bookkeeping engine.
//
// One hb_step() = three phases on the handle's stream:
//   1. partition  (k_radix_hist, k_scan_rows, k_radix_scatter x passes,
//      k_part_bounds): a stable LSD radix sort of the arrival-ordered batch by
//      partition = group >> PART_LOG, so every partition's segment keeps
//      arrival order.
//   2. apply      (k_apply<NMAX>): one 1024-lane workgroup per partition, one
//      lane per raft group.  The lane loads its group's SoA state into
//      registers once, steps the group's messages in arrival order (LDS
//      counting sort of the staged segment), emits events through a
//      wave-cooperative chunk allocator, and writes back only dirty fields.
//   3. finish     (k_finish): per-workgroup statistics are reduced to one
//      HB_STAT_COUNT vector (RCCL-reducible) and the event count is closed.
//
// The work is integer and HBM-bound; there is no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hipbatch_kernels.h"
#include "hipbatch_fast.h"

using namespace hb;

#define HB_CHECK(expr)                                                       \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) {                                                  \
      if (getenv("HB_DEBUG"))                                                \
        fprintf(stderr, "hipbatch: %s failed: %s (%s:%d)\n", #expr,          \
                hipGetErrorString(_e), __FILE__, __LINE__);                  \
      return HB_EDEVICE;                                                     \
    }                                                                        \
  } while (0)

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

// Block-wide exclusive scan (blockDim.x = 1024); returns exclusive prefix, *total = block sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh16, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan(v);
  if (lane == 63) sh16[wave] = incl;
  __syncthreads();
  if (wave == 0) {
    const uint32_t nw = blockDim.x >> 6;
    uint32_t x = lane < nw ? sh16[lane] : 0;
    x = wave_incl_scan(x);
    if (lane < nw) sh16[lane] = x;
  }
  __syncthreads();
  const uint32_t before = wave == 0 ? 0 : sh16[wave - 1];
  *total = sh16[(blockDim.x >> 6) - 1];
  __syncthreads();
  return before + incl - v;
}

// ============================================================================
// Phase 1: stable partition of the batch
//
// LSD radix sort of the messages by partition id (group >> PART_LOG), 6 bits
// (64 bins) per pass, 2 passes up to 4096 partitions (4M groups).  A 512-lane
// workgroup owns a tile of 2048 messages: it ranks them stably per digit
// (ballot matching inside a wave, per-wave counters across waves), stages the
// tile in LDS in digit order, and writes each digit's run contiguously, so the
// global stores are coalesced runs (~32 records per digit per tile) instead of
// scattered single records.  Messages of groups >= capacity are dropped in
// the first pass.  Arrival order is preserved within every partition.
// ============================================================================
struct BatchDev {
  const uint32_t* group;
  const uint32_t* info;
  const uint64_t* term;
  const uint64_t* index;
  const uint64_t* hint;
  const uint32_t* props;
  uint64_t n;
};

constexpr uint32_t RDX_BITS = 6;
constexpr uint32_t RDX_BINS = 1u << RDX_BITS;
constexpr uint32_t RDX_THREADS = 512;
constexpr uint32_t RDX_WAVES = RDX_THREADS / 64;
constexpr uint32_t RDX_ROUNDS = 4;
constexpr uint32_t RDX_TILE = RDX_THREADS * RDX_ROUNDS;  // 2048

struct RadixSrc {
  const uint32_t* group;
  const uint32_t* info;
  const uint32_t* orig;   // null: arrival index = position
  const uint64_t* term;
  const uint64_t* index;
  const uint32_t* n_dev;  // null: n
  uint32_t n;
};

struct RadixDst {
  uint32_t* group;
  uint32_t* info;
  uint32_t* orig;
  uint64_t* term;
  uint64_t* index;
};

__device__ __forceinline__ uint32_t src_n(const RadixSrc& s) { return s.n_dev ? *s.n_dev : s.n; }

__global__ void __launch_bounds__(RDX_THREADS) k_radix_hist(RadixSrc s, uint32_t G, uint32_t shift, uint32_t ntiles,
                                                           uint32_t* hist) {
  __shared__ uint32_t cnt[RDX_BINS];
  const uint32_t tid = threadIdx.x;
  if (tid < RDX_BINS) cnt[tid] = 0;
  __syncthreads();
  const uint32_t n = src_n(s);
  const uint32_t base = blockIdx.x * RDX_TILE;
#pragma unroll
  for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
    const uint32_t i = base + r * RDX_THREADS + tid;
    if (i < n) {
      const uint32_t g = s.group[i];
      if (g < G) atomicAdd(&cnt[((g >> PART_LOG) >> shift) & (RDX_BINS - 1)], 1u);
    }
  }
  __syncthreads();
  if (tid < RDX_BINS) hist[(size_t)tid * ntiles + blockIdx.x] = cnt[tid];
}

// Row scan: workgroup b turns row b of hist ([RDX_BINS][ntiles] tile counts)
// into exclusive per-tile prefixes and writes the row total to totals[b].
__global__ void __launch_bounds__(1024) k_scan_rows(uint32_t* hist, uint32_t ntiles, uint32_t* totals) {
  __shared__ uint32_t sh16[16];
  uint32_t* row = hist + (size_t)blockIdx.x * ntiles;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < ntiles; base += 4096) {
    const uint32_t i0 = base + threadIdx.x * 4;
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i0 + k < ntiles ? row[i0 + k] : 0u;
    uint32_t tot;
    uint32_t run = carry + block_excl_scan(v[0] + v[1] + v[2] + v[3], sh16, &tot);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i0 + k < ntiles) row[i0 + k] = run;
      run += v[k];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

__global__ void __launch_bounds__(RDX_THREADS) k_radix_scatter(RadixSrc s, RadixDst d, uint32_t G, uint32_t shift,
                                                              uint32_t ntiles, const uint32_t* off,
                                                              const uint32_t* totals, uint32_t* n_valid,
                                                              uint32_t final_pass) {
  __shared__ uint32_t s_off[RDX_BINS];
  __shared__ uint32_t s_wcnt[RDX_WAVES][RDX_BINS];
  __shared__ uint32_t s_dstart[RDX_BINS + 1];
  __shared__ uint32_t st_group[RDX_TILE];
  __shared__ uint32_t st_info[RDX_TILE];
  __shared__ uint32_t st_orig[RDX_TILE];
  __shared__ uint64_t st_term[RDX_TILE];
  __shared__ uint64_t st_index[RDX_TILE];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint32_t tile = blockIdx.x;
  if (tid < RDX_BINS) {
    // digit base = exclusive scan of the digit totals; + this tile's row prefix
    const uint32_t t = totals[tid];
    const uint32_t incl = wave_incl_scan(t);
    s_off[tid] = incl - t + off[(size_t)tid * ntiles + tile];
    if (tile == 0 && tid == RDX_BINS - 1) *n_valid = incl;
  }
  (&s_wcnt[0][0])[tid] = 0;  // RDX_WAVES * RDX_BINS == RDX_THREADS
  __syncthreads();
  const uint32_t n = src_n(s);
  const uint32_t base = tile * RDX_TILE;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t vg[RDX_ROUNDS], vi[RDX_ROUNDS], vo[RDX_ROUNDS], vd[RDX_ROUNDS], vr[RDX_ROUNDS];
  uint64_t vt[RDX_ROUNDS], vx[RDX_ROUNDS];
  bool vv[RDX_ROUNDS];
  // load (coalesced: round r, lane l -> element wave*256 + r*64 + l)
#pragma unroll
  for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
    const uint32_t e = wave * (64 * RDX_ROUNDS) + r * 64 + lane;
    const uint32_t i = base + e;
    vv[r] = i < n;
    vg[r] = vv[r] ? s.group[i] : 0u;
    vv[r] = vv[r] && vg[r] < G;
    vi[r] = vv[r] ? s.info[i] : 0u;
    vo[r] = vv[r] ? (s.orig ? s.orig[i] : i) : 0u;
    vt[r] = vv[r] ? s.term[i] : 0ull;
    vx[r] = vv[r] ? s.index[i] : 0ull;
    vd[r] = ((vg[r] >> PART_LOG) >> shift) & (RDX_BINS - 1);
  }
  // stable rank inside the wave: rounds in order, lanes in order
#pragma unroll
  for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
    uint64_t peers = __ballot(vv[r]);
#pragma unroll
    for (uint32_t k = 0; k < RDX_BITS; ++k) {
      const bool bit = (vd[r] >> k) & 1u;
      const uint64_t bk = __ballot(bit);
      peers &= bit ? bk : ~bk;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    const uint32_t before = vv[r] ? s_wcnt[wave][vd[r]] : 0u;
    vr[r] = before + rank;
    if (vv[r] && rank == 0) s_wcnt[wave][vd[r]] = before + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  // per digit: prefix over waves, then digit starts inside the tile
  if (tid < RDX_BINS) {
    uint32_t run = 0;
#pragma unroll
    for (uint32_t w = 0; w < RDX_WAVES; ++w) {
      const uint32_t c = s_wcnt[w][tid];
      s_wcnt[w][tid] = run;
      run += c;
    }
    const uint32_t incl = wave_incl_scan(run);
    s_dstart[tid] = incl - run;
    if (tid == RDX_BINS - 1) s_dstart[RDX_BINS] = incl;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
    if (vv[r]) {
      const uint32_t p = s_dstart[vd[r]] + s_wcnt[wave][vd[r]] + vr[r];
      st_group[p] = vg[r];
      st_info[p] = vi[r];
      st_orig[p] = vo[r];
      st_term[p] = vt[r];
      st_index[p] = vx[r];
    }
  }
  __syncthreads();
  const uint32_t valid = s_dstart[RDX_BINS];
#pragma unroll
  for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
    const uint32_t p = r * RDX_THREADS + tid;
    if (p < valid) {
      const uint32_t g = st_group[p];
      const uint32_t dg = ((g >> PART_LOG) >> shift) & (RDX_BINS - 1);
      const uint32_t o = s_off[dg] + (p - s_dstart[dg]);
      d.group[o] = g;
      d.info[o] = final_pass ? ((st_info[p] & 0xFFFFu) | ((g & (PART - 1)) << 16)) : st_info[p];
      d.orig[o] = st_orig[p];
      d.term[o] = st_term[p];
      d.index[o] = st_index[p];
    }
  }
}

// part_off[b] = first position of partition b in the sorted batch (b <= NB).
__global__ void k_part_bounds(const uint32_t* sorted_group, const uint32_t* n_dev, uint32_t NB, uint32_t* part_off) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > NB) return;
  uint32_t lo = 0, hi = *n_dev;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((sorted_group[mid] >> PART_LOG) < b) lo = mid + 1;
    else hi = mid;
  }
  part_off[b] = lo;
}

// ============================================================================
// Phase 2: apply
// ============================================================================
struct ApplyArgs {
  DevState S;
  const uint32_t* p_info;
  const uint32_t* p_orig;
  const uint64_t* p_term;
  const uint64_t* p_index;
  const uint64_t* hint;     // original-order RejectHint
  const uint32_t* props;    // dense proposals or null
  const uint32_t* part_off; // [NB+1]
  hb_event* ev;             // event region base
  uint32_t ev_per_msg;      // bound on events per stepped message (EV_MAX)
  uint32_t props_on;        // 1 if props[] is present (one proposal slot per group)
  uint32_t* ev_counts;      // [NB] records in each chunk
  uint64_t* ev_off;         // [NB] chunk offsets (records)
  uint64_t* stats_part;     // [NB][HB_STAT_COUNT]
  uint32_t* pflag;          // [NB][PART/32] groups handed from k_apply_fast to k_apply
  uint32_t* resume;         // [G] messages consumed by k_apply_fast | prop pending << 31
  uint64_t* commit0;        // [G] committed at batch start (for HB_STAT_COMMITS)
};

// stats slots reduced per workgroup
enum { ST_MSGS, ST_APPRESP, ST_VOTERESP, ST_DROPPED, ST_COMMITS, ST_WON, ST_LOST, ST_FAULTS, ST_ENTRIES, ST_N };

#ifndef HB_FAST_WAVES
#define HB_FAST_WAVES 4
#endif
constexpr uint32_t FLAG_WORDS = PART / 32;  // per-partition bitmask of groups handed to k_apply

// LDS staging of one round (<= CHUNK messages) of a partition's segment.
struct Stage {
  uint32_t info[CHUNK];
  uint32_t orig[CHUNK];
  uint64_t term[CHUNK];
  uint64_t index[CHUNK];
  uint16_t perm[CHUNK];
  uint32_t cnt[PART];
  uint32_t sh16[16];
};

// Stage messages [c0, c0+len) of the sorted batch and counting-sort them by
// group lane: on return the lane's messages are perm[*start, *start+*cnt), in
// arrival order (the segment is arrival-ordered; the per-lane run is
// re-sorted by position after the atomic placement).
__device__ __forceinline__ void stage_round(Stage& sl, const ApplyArgs& a, uint32_t c0, uint32_t len, uint32_t* start,
                                            uint32_t* cnt) {
  constexpr uint32_t PER = CHUNK / PART;
  const uint32_t tid = threadIdx.x;
  sl.cnt[tid] = 0;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < PER; ++k) {
    const uint32_t i = tid + k * PART;
    if (i < len) {
      const uint32_t inf = a.p_info[c0 + i];
      sl.info[i] = inf;
      sl.orig[i] = a.p_orig[c0 + i];
      sl.term[i] = a.p_term[c0 + i];
      sl.index[i] = a.p_index[c0 + i];
      atomicAdd(&sl.cnt[inf >> 16], 1u);
    }
  }
  __syncthreads();
  const uint32_t my_cnt = sl.cnt[tid];
  uint32_t total;
  const uint32_t my_start = block_excl_scan(my_cnt, sl.sh16, &total);
  sl.cnt[tid] = my_start;  // becomes the fill cursor
  __syncthreads();
  for (uint32_t i = tid; i < len; i += PART) {
    const uint32_t pos = atomicAdd(&sl.cnt[sl.info[i] >> 16], 1u);
    sl.perm[pos] = (uint16_t)i;
  }
  __syncthreads();
  for (uint32_t x = 1; x < my_cnt; ++x) {  // tiny insertion sort of the lane's run
    const uint16_t v = sl.perm[my_start + x];
    uint32_t y = x;
    while (y > 0 && sl.perm[my_start + y - 1] > v) {
      sl.perm[my_start + y] = sl.perm[my_start + y - 1];
      --y;
    }
    sl.perm[my_start + y] = v;
  }
  *start = my_start;
  *cnt = my_cnt;
}

__device__ __forceinline__ bool is_response(uint32_t type) {  // raft/util.go:53-55
  return type == HB_MSG_APP_RESP || type == HB_MSG_VOTE_RESP || type == HB_MSG_HEARTBEAT_RESP ||
         type == HB_MSG_UNREACHABLE;
}

// Reduce the lane statistics into the partition's stats row (accumulate: the
// general kernel adds to what the fast kernel wrote).
__device__ __forceinline__ void reduce_stats(const ApplyArgs& a, uint64_t* l_stats, const uint64_t (&vals)[ST_N],
                                             uint32_t part, bool accumulate) {
  const uint32_t tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < ST_N; ++k) {
    uint64_t v = vals[k];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    if ((tid & 63) == 0 && v) atomicAdd((unsigned long long*)&l_stats[k], (unsigned long long)v);
  }
  __syncthreads();
  if (tid < ST_N) {
    uint64_t* dst = &a.stats_part[(size_t)part * ST_N + tid];
    *dst = (accumulate ? *dst : 0ull) + l_stats[tid];
  }
}

// ---------------------------------------------------------------------------
// k_apply_fast: one workgroup per partition, one lane per group, steady-state
// leader operations only (FastLane).  The first message a lane cannot take
// (and everything after it) is handed to k_apply: the lane's bit is set in
// pflag[part] and resume[g] = messages already consumed | prop-pending bit.
// ---------------------------------------------------------------------------
template <int NMAX>
__global__ void __launch_bounds__(PART, (NMAX <= 3 ? HB_FAST_WAVES : 2)) k_apply_fast(ApplyArgs a) {
  __shared__ Stage sl;
  __shared__ uint32_t l_fill;
  __shared__ uint32_t l_flag[FLAG_WORDS];
  __shared__ uint64_t l_stats[ST_N];

  const uint32_t tid = threadIdx.x;
  const uint32_t part = blockIdx.x;
  const uint32_t g = part * PART + tid;
  const bool gvalid = g < a.S.G;

  // Exact chunk: every event is emitted while stepping a message (or the
  // group's proposal), at most ev_per_msg per message, so the partition's
  // chunk is ev_per_msg x (its messages + its proposal slots).
  const uint64_t ev_off = (uint64_t)a.ev_per_msg * ((uint64_t)a.part_off[part] + (uint64_t)part * PART * a.props_on);
  if (tid == 0) {
    l_fill = 0;
    a.ev_off[part] = ev_off;
  }
  if (tid < ST_N) l_stats[tid] = 0;
  if (tid < FLAG_WORDS) l_flag[tid] = 0;

  FastLane<NMAX> L;
  L.S = a.S;
  L.E.chunk = a.ev + ev_off;
  L.E.fill = &l_fill;
  L.g = g;
  const uint32_t seg_lo = a.part_off[part], seg_hi = a.part_off[part + 1];
  const bool wg_work = a.props_on || seg_hi > seg_lo;  // uniform over the workgroup
  L.mlo = gvalid ? reinterpret_cast<const uint32_t*>(a.S.meta)[2 * (size_t)g] : 0u;
  const uint32_t prop_raw = (a.props && gvalid) ? a.props[g] : 0u;
  // A group takes part when its slot is live (n > 0) and not faulted.
  const bool live = gvalid && L.n() != 0 && L.faulted() == 0;
  L.dirty = 0;
  L.last = L.committed = 0;
  if (wg_work && live) L.load();
  const uint64_t last0 = L.last, commit0 = L.committed;

  bool flagged = false;
  uint32_t resume = 0;
  uint32_t st_msgs = 0, st_drop = 0;

  const uint32_t prop_k = live ? prop_raw : 0u;
  if (prop_k) {
    if (L.prop_ok(prop_k)) {
      L.arrival = 0xFFFFFFFFu;
      L.prop(prop_k);
    } else {
      flagged = true;
      resume = 1u << 31;  // the proposal itself is pending
    }
  }

  uint32_t j = 0;  // messages of this lane consumed so far (all rounds)
  for (uint32_t c0 = seg_lo; c0 < seg_hi; c0 += CHUNK) {
    const uint32_t len = (seg_hi - c0) < CHUNK ? (seg_hi - c0) : CHUNK;
    uint32_t my_start, my_cnt;
    stage_round(sl, a, c0, len, &my_start, &my_cnt);
    if (live) {
      for (uint32_t x = 0; x < my_cnt; ++x) {
        if (flagged || L.faulted()) break;
        const uint32_t i = sl.perm[my_start + x];
        const uint32_t inf = sl.info[i];
        const uint32_t type = inf & 0xF, from = (inf >> 4) & 0xF;
        const bool reject = (inf >> 8) & 1u;
        if (from >= L.n() && is_response(type)) {  // raft/multinode.go:235
          st_drop++;
          j++;
          continue;
        }
        const uint64_t mterm = sl.term[i];
        if (!L.accept_ok(type, from, mterm, reject)) {
          flagged = true;
          resume = j;
          break;
        }
        L.arrival = sl.orig[i];
        L.accept(from, sl.index[i]);
        st_msgs++;
        j++;
      }
    }
    __syncthreads();
  }

  L.store();
  if (flagged) {
    atomicOr(&l_flag[tid >> 5], 1u << (tid & 31));
    a.resume[g] = resume;
    a.commit0[g] = commit0;
  }
  const uint64_t vals[ST_N] = {st_msgs,
                               st_msgs,  // every fast message is a MsgAppResp
                               0,
                               st_drop,
                               (uint64_t)(!flagged && L.committed != commit0),  // commitTo only raises
                               0,
                               0,
                               (uint64_t)(L.faulted() != 0 && live),
                               L.last - last0};
  reduce_stats(a, l_stats, vals, part, false);
  if (tid < FLAG_WORDS) a.pflag[(size_t)part * FLAG_WORDS + tid] = l_flag[tid];
  if (tid == 0) a.ev_counts[part] = l_fill;
  if (tid == 1) a.stats_part[(size_t)gridDim.x * ST_N + part] = l_fill;  // events reserved
}

// ---------------------------------------------------------------------------
// k_apply: the general state machine (Lane::step) for the groups k_apply_fast
// handed over, from their resume point.  Partitions without such groups exit
// after reading their flag words.
// ---------------------------------------------------------------------------
template <int NMAX>
__global__ void __launch_bounds__(PART, 2) k_apply(ApplyArgs a) {
  __shared__ Stage sl;
  __shared__ uint32_t l_fill;
  __shared__ uint32_t l_flag[FLAG_WORDS];
  __shared__ uint64_t l_stats[ST_N];

  const uint32_t tid = threadIdx.x;
  const uint32_t part = blockIdx.x;
  const uint32_t g = part * PART + tid;
  if (tid < FLAG_WORDS) l_flag[tid] = a.pflag[(size_t)part * FLAG_WORDS + tid];
  __syncthreads();
  uint32_t any = 0;
#pragma unroll
  for (uint32_t w = 0; w < FLAG_WORDS; ++w) any |= l_flag[w];
  if (!any) return;  // uniform
  const bool flagged = (l_flag[tid >> 5] >> (tid & 31)) & 1u;

  const uint64_t ev_off = a.ev_off[part];
  if (tid == 0) l_fill = a.ev_counts[part];  // append after the fast kernel's events
  if (tid < ST_N) l_stats[tid] = 0;

  Lane<NMAX> L;
  L.S = a.S;
  L.E.chunk = a.ev + ev_off;
  L.E.fill = &l_fill;
  L.g = g;
  L.won = 0;
  L.lost = 0;
  L.dirty = 0;
  L.meta = 0;
  L.last = 0;
  L.committed = 0;
  uint32_t resume = 0;
  uint64_t commit0 = 0;
  if (flagged) {  // live and not faulted when it was handed over
    L.meta = a.S.meta[g];
    L.load_all();
    resume = a.resume[g];
    commit0 = a.commit0[g];
  }
  const uint64_t last0 = L.last;
  uint32_t st_msgs = 0, st_app = 0, st_vote = 0, st_drop = 0;
  const uint32_t seg_lo = a.part_off[part], seg_hi = a.part_off[part + 1];

  if (flagged && (resume >> 31)) {
    L.arrival = 0xFFFFFFFFu;
    L.step(HB_MSG_PROP, L.self(), 0, a.props[g], false, 0);
  }
  const uint32_t skip = resume & 0x7FFFFFFFu;
  uint32_t j = 0;
  for (uint32_t c0 = seg_lo; c0 < seg_hi; c0 += CHUNK) {
    const uint32_t len = (seg_hi - c0) < CHUNK ? (seg_hi - c0) : CHUNK;
    uint32_t my_start, my_cnt;
    stage_round(sl, a, c0, len, &my_start, &my_cnt);
    if (flagged) {
      for (uint32_t x = 0; x < my_cnt; ++x, ++j) {
        if (j < skip) continue;
        const uint32_t i = sl.perm[my_start + x];
        const uint32_t inf = sl.info[i];
        const uint32_t type = inf & 0xF, from = (inf >> 4) & 0xF;
        const bool reject = (inf >> 8) & 1u;
        if (L.faulted()) break;
        if (from >= L.n() && is_response(type)) {  // raft/multinode.go:235
          st_drop++;
          continue;
        }
        L.arrival = sl.orig[i];
        L.step(type, from, sl.term[i], sl.index[i], reject, (reject && a.hint) ? a.hint[sl.orig[i]] : 0ull);
        st_msgs++;
        st_app += type == HB_MSG_APP_RESP;
        st_vote += type == HB_MSG_VOTE_RESP;
      }
    }
    __syncthreads();
  }

  if (flagged) L.store();
  const uint64_t vals[ST_N] = {st_msgs,
                               st_app,
                               st_vote,
                               st_drop,
                               (uint64_t)(flagged && L.committed != commit0),
                               L.won,
                               L.lost,
                               (uint64_t)(flagged && L.faulted() != 0),
                               L.last - last0};
  reduce_stats(a, l_stats, vals, part, true);
  if (tid == 0) a.ev_counts[part] = l_fill;
  if (tid == 1) a.stats_part[(size_t)gridDim.x * ST_N + part] = l_fill;  // events reserved
}

// ============================================================================
// Phase 3: finish
// ============================================================================
__global__ void __launch_bounds__(1024) k_finish(const uint64_t* stats_part, uint32_t NB, uint64_t* stats) {
  __shared__ uint64_t acc[HB_STAT_COUNT];
  if (threadIdx.x < HB_STAT_COUNT) acc[threadIdx.x] = 0;
  __syncthreads();
  uint64_t v[ST_N + 1] = {};
  for (uint32_t p = threadIdx.x; p < NB; p += blockDim.x) {
#pragma unroll
    for (int k = 0; k < ST_N; ++k) v[k] += stats_part[(size_t)p * ST_N + k];
    v[ST_N] += stats_part[(size_t)NB * ST_N + p];
  }
  const int map[ST_N + 1] = {HB_STAT_MSGS,  HB_STAT_APPRESP, HB_STAT_VOTERESP, HB_STAT_DROPPED, HB_STAT_COMMITS,
                             HB_STAT_WON,   HB_STAT_LOST,    HB_STAT_FAULTS,   HB_STAT_ENTRIES, HB_STAT_EVENTS};
#pragma unroll
  for (int k = 0; k <= ST_N; ++k) {
    uint64_t x = v[k];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
    if ((threadIdx.x & 63) == 0 && x) atomicAdd((unsigned long long*)&acc[map[k]], (unsigned long long)x);
  }
  __syncthreads();
  if (threadIdx.x < HB_STAT_COUNT) stats[threadIdx.x] = acc[threadIdx.x];
}

// ============================================================================
// group load / gather / inflights
// ============================================================================
__global__ void k_load(DevState S, uint32_t first, uint32_t count, const hb_group* src) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t g = first + i;
  const hb_group& r = src[i];
  S.term[g] = r.term;
  S.commit[g] = r.committed;
  S.first[g] = r.first_index;
  S.last[g] = r.last_index;
  S.tfirst[g] = r.term_first;
  S.tlast[g] = r.term_last;
  S.snap[g] = r.snap_index;
  S.meta[g] = meta_make(r.state, r.n, r.self_slot, r.lead, r.vote, r.fault, r.votes_resp, r.votes_grant);
  for (uint32_t s = 0; s < S.nmax; ++s) {
    const bool on = s < r.n;
    const size_t o = (size_t)s * S.G + g;
    S.match[o] = on ? r.pr[s].match : 0;
    S.next[o] = on ? r.pr[s].next : 0;
    S.pending[o] = on ? r.pr[s].pending_snapshot : 0;
    S.pm[o] = on ? pm_make(r.pr[s].state, r.pr[s].paused, r.pr[s].ins_start, r.pr[s].ins_count) : 0;
  }
}

__global__ void k_gather(DevState S, uint32_t first, uint32_t count, hb_group* dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t g = first + i;
  hb_group r;
  memset(&r, 0, sizeof(r));
  const uint64_t m = S.meta[g];
  r.term = S.term[g];
  r.committed = S.commit[g];
  r.first_index = S.first[g];
  r.last_index = S.last[g];
  r.term_first = S.tfirst[g];
  r.term_last = S.tlast[g];
  r.snap_index = S.snap[g];
  r.state = m_state(m);
  r.n = m_n(m);
  r.self_slot = m_self(m);
  r.lead = m_lead(m);
  r.vote = m_vote(m);
  r.fault = m_fault(m);
  r.votes_resp = m_resp(m);
  r.votes_grant = m_grant(m);
  for (uint32_t s = 0; s < S.nmax && s < r.n; ++s) {
    const size_t o = (size_t)s * S.G + g;
    const uint32_t p = S.pm[o];
    r.pr[s].match = S.match[o];
    r.pr[s].next = S.next[o];
    r.pr[s].state = pm_state(p);
    r.pr[s].paused = pm_paused(p);
    r.pr[s].ins_start = pm_start(p);
    r.pr[s].ins_count = pm_count(p);
    r.pr[s].pending_snapshot = pm_state(p) == HB_PR_SNAPSHOT ? S.pending[o] : 0;
  }
  dst[i] = r;
}

__global__ void k_remove(DevState S, uint32_t first, uint32_t count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) S.meta[first + i] = 0;
}

__global__ void k_set_ins(DevState S, uint32_t g, uint32_t s, uint32_t start, uint32_t count, const uint64_t* vals) {
  for (uint32_t i = threadIdx.x; i < count; i += blockDim.x) {
    uint32_t idx = start + i;
    if (idx >= S.W) idx -= S.W;
    S.ring[((size_t)s * S.W + idx) * S.G + g] = vals[i];
  }
  if (threadIdx.x == 0) {
    const size_t o = (size_t)s * S.G + g;
    const uint32_t p = S.pm[o];
    S.pm[o] = pm_make(pm_state(p), pm_paused(p), start, count);
  }
}

__global__ void k_get_ins(DevState S, uint32_t g, uint32_t s, uint64_t* vals, uint32_t* sc) {
  const size_t o = (size_t)s * S.G + g;
  const uint32_t p = S.pm[o];
  const uint32_t start = pm_start(p), count = pm_count(p);
  for (uint32_t i = threadIdx.x; i < count; i += blockDim.x) {
    uint32_t idx = start + i;
    if (idx >= S.W) idx -= S.W;
    vals[i] = S.ring[((size_t)s * S.W + idx) * S.G + g];
  }
  if (threadIdx.x == 0) {
    sc[0] = start;
    sc[1] = count;
  }
}

// Dense gather of the chunked events (chunk c at base + c*cap, counts[c]).
__global__ void __launch_bounds__(256) k_gather_events(const hb_event* base, const uint32_t* counts,
                                                       const uint64_t* offs, hb_event* out) {
  __shared__ uint64_t s_off;
  const uint32_t c = blockIdx.x;
  if (threadIdx.x == 0) {
    uint64_t off = 0;
    for (uint32_t k = 0; k < c; ++k) off += counts[k];
    s_off = off;
  }
  __syncthreads();
  const uint32_t cnt = counts[c];
  const hb_event* src = base + offs[c];
  for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) out[s_off + i] = src[i];
}

// ============================================================================
// host side
// ============================================================================
struct hb_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t G = 0, nmax = 0, W = 0, NB = 0;
  uint64_t max_msg_size = 0, max_batch = 0;
  DevState st{};
  std::vector<void*> allocs;
  // partition scratch
  uint32_t* hist = nullptr;       // [RDX_BINS][tiles]
  uint32_t* n_valid = nullptr;    // messages kept after pass 1 (device)
  uint32_t* totals = nullptr;     // [RDX_BINS] digit totals of the current pass
  uint32_t* part_off = nullptr;   // [NB + 1]
  RadixDst tmp[2] = {};           // intermediate passes (ping-pong)
  RadixDst fin = {};              // final pass = apply input
  uint32_t passes = 1;
  // host-pointer staging
  uint32_t* s_group = nullptr;
  uint32_t* s_info = nullptr;
  uint32_t* s_props = nullptr;
  uint64_t* s_term = nullptr;
  uint64_t* s_index = nullptr;
  uint64_t* s_hint = nullptr;
  // events
  hb_event* ev = nullptr;
  uint64_t ev_region = 0;  // records
  uint32_t ev_per_msg = 0;
  uint32_t* ev_counts = nullptr;  // [NB]
  uint64_t* ev_off = nullptr;     // [NB]
  uint64_t* stats_part = nullptr;
  uint64_t* stats = nullptr;
  // fast -> general hand-over
  uint32_t* pflag = nullptr;      // [NB][PART/32]
  uint32_t* resume = nullptr;     // [G]
  uint64_t* commit0 = nullptr;    // [G]
  static constexpr uint32_t PROF_RING = 256;
  hipEvent_t ph[PROF_RING][HB_PHASE_COUNT + 1] = {};
  uint32_t prof_n = 0;  // profiled steps since hb_phase_reset
  bool stepped = false;
};

namespace {

int dalloc(hb_handle* h, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (hipMalloc(p, bytes) != hipSuccess) return HB_ENOMEM;
  h->allocs.push_back(*p);
  return HB_OK;
}

template <class T>
int dalloc_t(hb_handle* h, T** p, size_t count) {
  return dalloc(h, reinterpret_cast<void**>(p), count * sizeof(T));
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

uint32_t ceil_log2(uint32_t x) {
  uint32_t b = 0;
  while ((1u << b) < x) ++b;
  return b;
}

template <int NMAX>
void launch_apply(hb_handle* h, const ApplyArgs& a) {
  hipLaunchKernelGGL(k_apply_fast<NMAX>, dim3(h->NB), dim3(PART), 0, h->stream, a);
  hipLaunchKernelGGL(k_apply<NMAX>, dim3(h->NB), dim3(PART), 0, h->stream, a);
}

}  // namespace

extern "C" {

int hb_abi_version(void) { return HB_ABI_VERSION; }

const char* hb_strerror(int code) {
  switch (code) {
    case HB_OK: return "ok";
    case HB_EINVAL: return "invalid argument";
    case HB_ENOMEM: return "out of memory";
    case HB_EDEVICE: return "device error";
    case HB_EINVARIANT: return "device invariant violated";
    default: return "unknown error";
  }
}

int hb_create(int device, uint32_t capacity, uint32_t max_replicas, uint32_t max_inflight,
              uint64_t max_msg_size, uint64_t max_batch, hb_handle** out) {
  if (!out || capacity == 0 || max_replicas < 1 || max_replicas > HB_MAX_REPLICAS || max_inflight < 1 ||
      max_inflight > HB_MAX_INFLIGHT || (max_msg_size != 0 && max_msg_size != HB_NO_LIMIT) ||
      max_batch >= (1ull << 31) || capacity > (1u << 24))
    return HB_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return HB_EDEVICE;
  DeviceGuard guard(device);
  hb_handle* h = new hb_handle();
  h->device = device;
  h->G = capacity;
  h->nmax = max_replicas <= 3 ? 3 : (max_replicas <= 5 ? 5 : 7);
  h->W = max_inflight;
  h->max_msg_size = max_msg_size;
  h->max_batch = max_batch;
  h->NB = (capacity + PART - 1) / PART;
  const size_t G = capacity, R = h->nmax;
  DevState& s = h->st;
  s.G = capacity;
  s.W = max_inflight;
  s.nmax = h->nmax;
  s.max_msg_size = max_msg_size;
  int rc = HB_OK;
#define ALLOC(ptr, count) \
  if (rc == HB_OK) rc = dalloc_t(h, &(ptr), (count))
  ALLOC(s.term, G);
  ALLOC(s.commit, G);
  ALLOC(s.first, G);
  ALLOC(s.last, G);
  ALLOC(s.tfirst, G);
  ALLOC(s.tlast, G);
  ALLOC(s.snap, G);
  ALLOC(s.meta, G);
  ALLOC(s.match, R * G);
  ALLOC(s.next, R * G);
  ALLOC(s.pending, R * G);
  ALLOC(s.pm, R * G);
  ALLOC(s.ring, R * (size_t)max_inflight * G);
  // partition scratch
  const size_t mb = max_batch ? max_batch : 1;
  const uint32_t pbits = std::max<uint32_t>(ceil_log2(h->NB), 1);
  h->passes = (pbits + RDX_BITS - 1) / RDX_BITS;
  const size_t tiles_max = (mb + RDX_TILE - 1) / RDX_TILE;
  ALLOC(h->hist, (size_t)RDX_BINS * tiles_max);
  ALLOC(h->n_valid, 4);
  ALLOC(h->totals, RDX_BINS);
  ALLOC(h->part_off, h->NB + 1);
  for (uint32_t k = 0; k < 3; ++k) {
    RadixDst& d = k < 2 ? h->tmp[k] : h->fin;
    if (k < 2 && h->passes < 2 + k) continue;  // ping-pong buffers only when needed
    ALLOC(d.group, mb);
    ALLOC(d.info, mb);
    ALLOC(d.orig, mb);
    ALLOC(d.term, mb);
    ALLOC(d.index, mb);
  }
  ALLOC(h->s_group, mb);
  ALLOC(h->s_info, mb);
  ALLOC(h->s_term, mb);
  ALLOC(h->s_index, mb);
  ALLOC(h->s_hint, mb);
  ALLOC(h->s_props, G);
  // events: (batch + one proposal slot per group) x EV_MAX (exact bound)
  h->ev_per_msg = h->nmax + 4;
  h->ev_region = (mb + (uint64_t)h->NB * PART) * h->ev_per_msg;
  ALLOC(h->ev, h->ev_region);
  ALLOC(h->ev_counts, h->NB);
  ALLOC(h->ev_off, h->NB);
  ALLOC(h->stats_part, (size_t)h->NB * (ST_N + 1) + 16);
  ALLOC(h->pflag, (size_t)h->NB * FLAG_WORDS);
  ALLOC(h->resume, G);
  ALLOC(h->commit0, G);
  ALLOC(h->stats, HB_STAT_COUNT);
#undef ALLOC
  if (rc != HB_OK) {
    hb_destroy(h);
    return rc;
  }
  for (auto& row : h->ph)
    for (auto& e : row)
      if (hipEventCreate(&e) != hipSuccess) {
        hb_destroy(h);
        return HB_EDEVICE;
      }
  // empty slots (n = 0), zeroed progress
  if (hipMemset(s.meta, 0, G * 8) != hipSuccess || hipMemset(s.pm, 0, R * G * 4) != hipSuccess ||
      hipMemset(h->stats, 0, HB_STAT_COUNT * 8) != hipSuccess ||
      hipMemset(h->ev_counts, 0, h->NB * 4ull) != hipSuccess || hipMemset(h->ev_off, 0, h->NB * 8ull) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    hb_destroy(h);
    return HB_EDEVICE;
  }
  *out = h;
  return HB_OK;
}

int hb_destroy(hb_handle* h) {
  if (!h) return HB_EINVAL;
  DeviceGuard guard(h->device);
  (void)hipDeviceSynchronize();
  for (void* p : h->allocs) (void)hipFree(p);
  for (auto& row : h->ph)
    for (auto& e : row)
      if (e) (void)hipEventDestroy(e);
  delete h;
  return HB_OK;
}

int hb_set_stream(hb_handle* h, void* stream) {
  if (!h) return HB_EINVAL;
  h->stream = reinterpret_cast<hipStream_t>(stream);
  return HB_OK;
}

int hb_sync(hb_handle* h) {
  if (!h) return HB_EINVAL;
  DeviceGuard guard(h->device);
  HB_CHECK(hipStreamSynchronize(h->stream));
  return HB_OK;
}

static bool valid_ref(uint32_t r, uint32_t n) {
  return r < n || r == HB_REF_OTHER || r == HB_REF_SELF || r == HB_REF_NONE;
}

int hb_load_groups(hb_handle* h, uint32_t first, uint32_t count, const hb_group* groups) {
  if (!h || !groups || (uint64_t)first + count > h->G) return HB_EINVAL;
  if (count == 0) return HB_OK;
  for (uint32_t i = 0; i < count; ++i) {
    const hb_group& r = groups[i];
    if (r.n < 1 || r.n > h->nmax || r.state > 2 || r.fault > 15) return HB_EINVAL;
    if (!(r.self_slot < r.n || r.self_slot == HB_SLOT_NONE)) return HB_EINVAL;
    if (!valid_ref(r.lead, r.n) || !valid_ref(r.vote, r.n)) return HB_EINVAL;
    if (r.first_index == 0 || r.last_index + 1 < r.first_index) return HB_EINVAL;
    if (r.term_first != HB_NO_INDEX &&
        (r.term_first > r.term_last || r.term_first + 1 < r.first_index || r.term_last > r.last_index))
      return HB_EINVAL;
    if ((r.votes_resp | r.votes_grant) > 0xFF || (r.votes_grant & ~r.votes_resp)) return HB_EINVAL;
    for (uint32_t s = 0; s < r.n; ++s) {
      const hb_progress& p = r.pr[s];
      if (p.state > 2 || p.paused > 1 || p.ins_start >= h->W || p.ins_count > h->W) return HB_EINVAL;
    }
  }
  DeviceGuard guard(h->device);
  hb_group* d = nullptr;
  HB_CHECK(hipMalloc(&d, sizeof(hb_group) * count));
  hipError_t e = hipMemcpyAsync(d, groups, sizeof(hb_group) * count, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_load, dim3((count + 255) / 256), dim3(256), 0, h->stream, h->st, first, count, d);
    e = hipStreamSynchronize(h->stream);
  }
  (void)hipFree(d);
  return e == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_get_groups(hb_handle* h, uint32_t first, uint32_t count, hb_group* out) {
  if (!h || !out || (uint64_t)first + count > h->G) return HB_EINVAL;
  if (count == 0) return HB_OK;
  DeviceGuard guard(h->device);
  hb_group* d = nullptr;
  HB_CHECK(hipMalloc(&d, sizeof(hb_group) * count));
  hipLaunchKernelGGL(k_gather, dim3((count + 255) / 256), dim3(256), 0, h->stream, h->st, first, count, d);
  hipError_t e = hipMemcpyAsync(out, d, sizeof(hb_group) * count, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  return e == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_remove_groups(hb_handle* h, uint32_t first, uint32_t count) {
  if (!h || (uint64_t)first + count > h->G) return HB_EINVAL;
  if (count == 0) return HB_OK;
  DeviceGuard guard(h->device);
  hipLaunchKernelGGL(k_remove, dim3((count + 255) / 256), dim3(256), 0, h->stream, h->st, first, count);
  HB_CHECK(hipStreamSynchronize(h->stream));
  return HB_OK;
}

int hb_set_inflights(hb_handle* h, uint32_t group, uint32_t slot, uint32_t start, uint32_t count,
                     const uint64_t* vals) {
  if (!h || group >= h->G || slot >= h->nmax || start >= h->W || count > h->W || (count && !vals))
    return HB_EINVAL;
  DeviceGuard guard(h->device);
  uint64_t* d = nullptr;
  HB_CHECK(hipMalloc(&d, 8ull * (count ? count : 1)));
  hipError_t e = hipSuccess;
  if (count) e = hipMemcpyAsync(d, vals, 8ull * count, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_set_ins, dim3(1), dim3(256), 0, h->stream, h->st, group, slot, start, count, d);
    e = hipStreamSynchronize(h->stream);
  }
  (void)hipFree(d);
  return e == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_get_inflights(hb_handle* h, uint32_t group, uint32_t slot, uint32_t* start, uint32_t* count,
                     uint64_t* vals) {
  if (!h || group >= h->G || slot >= h->nmax || !start || !count || !vals) return HB_EINVAL;
  DeviceGuard guard(h->device);
  uint64_t* d = nullptr;
  uint32_t* sc = nullptr;
  HB_CHECK(hipMalloc(&d, 8ull * h->W));
  if (hipMalloc(&sc, 8) != hipSuccess) {
    (void)hipFree(d);
    return HB_EDEVICE;
  }
  hipLaunchKernelGGL(k_get_ins, dim3(1), dim3(256), 0, h->stream, h->st, group, slot, d, sc);
  uint32_t hsc[2] = {0, 0};
  hipError_t e = hipMemcpyAsync(hsc, sc, 8, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e == hipSuccess && hsc[1]) e = hipMemcpy(vals, d, 8ull * hsc[1], hipMemcpyDeviceToHost);
  *start = hsc[0];
  *count = hsc[1];
  (void)hipFree(d);
  (void)hipFree(sc);
  return e == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_step(hb_handle* h, const hb_batch* b, uint32_t flags) {
  if (!h || !b || b->n > h->max_batch) return HB_EINVAL;
  if (b->n && (!b->group || !b->info || !b->term || !b->index)) return HB_EINVAL;
  DeviceGuard guard(h->device);
  hipStream_t st = h->stream;
  const bool prof = (flags & HB_STEP_PROFILE) != 0;
  BatchDev bd{b->group, b->info, b->term, b->index, b->hint, b->props, b->n};
  if (flags & HB_STEP_HOST_PTRS) {
    const size_t n = b->n;
    if (n) {
      HB_CHECK(hipMemcpyAsync(h->s_group, b->group, n * 4, hipMemcpyHostToDevice, st));
      HB_CHECK(hipMemcpyAsync(h->s_info, b->info, n * 4, hipMemcpyHostToDevice, st));
      HB_CHECK(hipMemcpyAsync(h->s_term, b->term, n * 8, hipMemcpyHostToDevice, st));
      HB_CHECK(hipMemcpyAsync(h->s_index, b->index, n * 8, hipMemcpyHostToDevice, st));
      if (b->hint) HB_CHECK(hipMemcpyAsync(h->s_hint, b->hint, n * 8, hipMemcpyHostToDevice, st));
    }
    if (b->props) HB_CHECK(hipMemcpyAsync(h->s_props, b->props, (size_t)h->G * 4, hipMemcpyHostToDevice, st));
    bd.group = h->s_group;
    bd.info = h->s_info;
    bd.term = h->s_term;
    bd.index = h->s_index;
    bd.hint = b->hint ? h->s_hint : nullptr;
    bd.props = b->props ? h->s_props : nullptr;
  }
  hipEvent_t* ev = h->ph[h->prof_n % hb_handle::PROF_RING];
  if (prof) HB_CHECK(hipEventRecord(ev[0], st));

  // ---- phase 1: partition ----------------------------------------------------
  const uint32_t NB = h->NB;
  if (b->n == 0) {
    HB_CHECK(hipMemsetAsync(h->part_off, 0, (NB + 1) * 4ull, st));
  } else {
    const uint32_t ntiles = (uint32_t)((b->n + RDX_TILE - 1) / RDX_TILE);
    RadixSrc src{bd.group, bd.info, nullptr, bd.term, bd.index, nullptr, (uint32_t)b->n};
    for (uint32_t p = 0; p < h->passes; ++p) {
      const bool last_pass = p + 1 == h->passes;
      const RadixDst& dst = last_pass ? h->fin : h->tmp[p & 1];
      const uint32_t shift = p * RDX_BITS;
      hipLaunchKernelGGL(k_radix_hist, dim3(ntiles), dim3(RDX_THREADS), 0, st, src, h->G, shift, ntiles, h->hist);
      hipLaunchKernelGGL(k_scan_rows, dim3(RDX_BINS), dim3(1024), 0, st, h->hist, ntiles, h->totals);
      hipLaunchKernelGGL(k_radix_scatter, dim3(ntiles), dim3(RDX_THREADS), 0, st, src, dst, h->G, shift, ntiles,
                         (const uint32_t*)h->hist, (const uint32_t*)h->totals, h->n_valid, last_pass ? 1u : 0u);
      src = RadixSrc{dst.group, dst.info, dst.orig, dst.term, dst.index, h->n_valid, (uint32_t)b->n};
    }
    hipLaunchKernelGGL(k_part_bounds, dim3((NB + 1 + 255) / 256), dim3(256), 0, st, (const uint32_t*)h->fin.group,
                       (const uint32_t*)h->n_valid, NB, h->part_off);
  }
  if (prof) HB_CHECK(hipEventRecord(ev[1], st));

  // ---- phase 2: apply ----------------------------------------------------------
  ApplyArgs aa;
  aa.S = h->st;
  aa.p_info = h->fin.info;
  aa.p_orig = h->fin.orig;
  aa.p_term = h->fin.term;
  aa.p_index = h->fin.index;
  aa.hint = bd.hint;
  aa.props = bd.props;
  aa.part_off = h->part_off;
  aa.ev = h->ev;
  aa.ev_per_msg = h->ev_per_msg;
  aa.props_on = bd.props ? 1u : 0u;
  aa.ev_counts = h->ev_counts;
  aa.ev_off = h->ev_off;
  aa.stats_part = h->stats_part;
  aa.pflag = h->pflag;
  aa.resume = h->resume;
  aa.commit0 = h->commit0;
  switch (h->nmax) {
    case 3: launch_apply<3>(h, aa); break;
    case 5: launch_apply<5>(h, aa); break;
    default: launch_apply<7>(h, aa); break;
  }
  if (prof) HB_CHECK(hipEventRecord(ev[2], st));
  // ---- phase 3: finish -----------------------------------------------------------
  hipLaunchKernelGGL(k_finish, dim3(1), dim3(1024), 0, st, h->stats_part, NB, h->stats);
  if (prof) HB_CHECK(hipEventRecord(ev[3], st));
  HB_CHECK(hipGetLastError());
  if (prof) h->prof_n++;
  h->stepped = true;
  return HB_OK;
}

int hb_events_device(hb_handle* h, const hb_event** base, const uint64_t** chunk_off, const uint32_t** counts,
                     uint32_t* n_chunks) {
  if (!h || !base || !chunk_off || !counts || !n_chunks) return HB_EINVAL;
  *base = h->ev;
  *chunk_off = h->ev_off;
  *counts = h->ev_counts;
  *n_chunks = h->NB;
  return HB_OK;
}

int hb_copy_events(hb_handle* h, hb_event* out, uint64_t cap, uint64_t* n) {
  if (!h || !n) return HB_EINVAL;
  DeviceGuard guard(h->device);
  uint64_t stats[HB_STAT_COUNT];
  HB_CHECK(hipMemcpyAsync(stats, h->stats, sizeof(stats), hipMemcpyDeviceToHost, h->stream));
  HB_CHECK(hipStreamSynchronize(h->stream));
  const uint64_t total = h->stepped ? stats[HB_STAT_EVENTS] : 0;
  *n = total;
  if (total == 0) return HB_OK;
  if (!out || cap < total) return HB_EINVAL;
  hb_event* d = nullptr;
  HB_CHECK(hipMalloc(&d, total * sizeof(hb_event)));
  hipLaunchKernelGGL(k_gather_events, dim3(h->NB), dim3(256), 0, h->stream, h->ev, h->ev_counts, h->ev_off, d);
  hipError_t e = hipMemcpyAsync(out, d, total * sizeof(hb_event), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  return e == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_stats_device(hb_handle* h, uint64_t** dev_stats) {
  if (!h || !dev_stats) return HB_EINVAL;
  *dev_stats = h->stats;
  return HB_OK;
}

int hb_stats(hb_handle* h, uint64_t* out) {
  if (!h || !out) return HB_EINVAL;
  DeviceGuard guard(h->device);
  HB_CHECK(hipMemcpyAsync(out, h->stats, HB_STAT_COUNT * 8, hipMemcpyDeviceToHost, h->stream));
  HB_CHECK(hipStreamSynchronize(h->stream));
  return HB_OK;
}

int hb_phase_ms(hb_handle* h, float* out, uint32_t* steps) {
  if (!h || !out) return HB_EINVAL;
  DeviceGuard guard(h->device);
  const uint32_t n = std::min<uint32_t>(h->prof_n, hb_handle::PROF_RING);
  if (steps) *steps = n;
  for (int i = 0; i < HB_PHASE_COUNT; ++i) out[i] = 0.f;
  if (n == 0) return HB_EINVAL;
  HB_CHECK(hipStreamSynchronize(h->stream));
  for (uint32_t k = 0; k < n; ++k) {
    for (int i = 0; i < HB_PHASE_COUNT; ++i) {
      float ms = 0.f;
      HB_CHECK(hipEventElapsedTime(&ms, h->ph[k][i], h->ph[k][i + 1]));
      out[i] += ms / (float)n;
    }
  }
  return HB_OK;
}

int hb_phase_reset(hb_handle* h) {
  if (!h) return HB_EINVAL;
  h->prof_n = 0;
  return HB_OK;
}

int hb_stats_to(hb_handle* h, uint64_t* dev_dst) {
  if (!h || !dev_dst) return HB_EINVAL;
  DeviceGuard guard(h->device);
  HB_CHECK(hipMemcpyAsync(dev_dst, h->stats, HB_STAT_COUNT * 8, hipMemcpyDeviceToDevice, h->stream));
  return HB_OK;
}

int hb_alloc_pinned(size_t bytes, void** out) {
  if (!out) return HB_EINVAL;
  return hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? HB_OK : HB_ENOMEM;
}

int hb_free_pinned(void* p) { return hipHostFree(p) == hipSuccess ? HB_OK : HB_EDEVICE; }

}  // extern "C"
