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
#include <type_traits>
#include <vector>

#include "hipbatch_kernels.h"
#include "hipbatch_fast.h"
#include "hipbatch_elect.h"
#include "hipbatch_lead.h"
#include "hipbatch_wire.h"

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
// Phase 1: partition the batch into buckets
//
// A bucket is 2^sis_log consecutive apply partitions (sis_log <= 4: up to
// 4096 groups, 7 at n = 3; hb_create picks the smallest that needs no extra pass, down to
// one k_route workgroup per bucket).  The batch is sorted by bucket id with a
// stable LSD radix sort, 8-bit digits: one pass up to 256 buckets, two up to
// 64K.  A 512-lane workgroup ranks a 2048-message tile stably (ballot
// matching inside a wave, per-wave counters across waves), stages it in LDS
// in digit order and writes each digit's run contiguously, so the global
// stores are coalesced runs (~8 records per digit per tile) instead of
// scattered single records.  Messages of groups >= capacity are dropped in
// the first pass.  Arrival order is preserved within every bucket.
//
// The final pass writes the apply input: one 16-byte MsgRec per message
// (info with the group's lane in bits 16-23 and its partition in the bucket
// in bits 24-27 (30-31 and 14 above 16 partitions: rec_sub), arrival index, Term and Index packed into one word, below).
// k_route reads the records and writes the partition once more as a key byte
// per message, contiguous, for the general kernel's bucket walk (a separate
// key array written here took 8-byte runs per digit per tile: partial lines).
//
// The 16-byte record: every pass over the messages (scatter write, route read
// and write, apply read) moves 16 instead of 24 bytes.  Term and Index share
// one u64 (Index in bits 0-39, Term in 40-63) when they fit, which is every
// message a raft cluster sends below 2^24 terms and 2^40 entries; otherwise
// the record is marked REC_LONG and the first pass keeps the full pair in
// the prep set's side table at the message's arrival index, where every
// reader takes it from (rec_unpack).  Bit-exact for every u64 value.
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

// A bucket is 2^sis_log apply partitions (hb_handle::sis_log, chosen at
// hb_create: at most SIS_MAX, fewer when that costs no extra radix pass, so
// that one k_route workgroup owns a whole bucket and reads it once).
constexpr uint32_t SIS_LOG_MAX = 4;
// HB_SIS_LOG_MAX3 > 4: n = 3 handles take buckets of up to 2^7 partitions
// (32K groups) when that saves a radix pass (8M groups: 256 buckets, one pass
// instead of two); k_route_fast's 16 sisters then read their bucket from L2,
// 16 times over.  Measured (cfg5, same box): partition 433 -> 241 us but
// k_route_fast 485 -> 1032 us (0.92 -> 1.27 ms/step): off.
#ifndef HB_SIS_LOG_MAX3
#define HB_SIS_LOG_MAX3 4
#endif
constexpr uint32_t SIS_LOG_MAX3 = HB_SIS_LOG_MAX3;
static_assert(SIS_LOG_MAX3 <= 7, "a record carries its partition in the bucket in 7 bits (rec_sub)");
// a prep set's counters: k_apply's 8 work-list lengths, k_elect's 8, k_follow's, the finish ticket —
// each on a 128-byte line of its own (CTR_STRIDE words): the returning atomics of every partition
// on one line serialise at the memory side (~7 ns each; 16K partitions put 16K on a list)
enum : uint32_t { CTR_STRIDE = 32, CTR_AP = 0, CTR_EL = 8 * CTR_STRIDE, CTR_FL = 16 * CTR_STRIDE,
                  CTR_DONE = 17 * CTR_STRIDE, CTR_WORDS = 18 * CTR_STRIDE };
// step statistics: NSH shards per value, each (value, shard) on a 128-byte line of its own
constexpr uint32_t NSH = 8;
constexpr uint64_t STAGE_MAX = 8ull << 20;  // host-pointer batches packed into one pinned copy up to this size  // (a shard per XCD slot; a finish lane per (value, shard))
__host__ __device__ constexpr uint32_t shard_at(uint32_t k, uint32_t sh) { return (k * NSH + sh) * 16; }
constexpr uint32_t RDX_BITS = 8;
constexpr uint32_t RDX_BINS = 1u << RDX_BITS;
#ifndef HB_RDX_THREADS  // measured (cfg2 / cfg5 A/B): 1024 x 2 beat 512 x 4 (-3 us / -46 us per step),
#define HB_RDX_THREADS 1024  // 256 x 4, 512 x 2, 512 x 8 and 1024 x 4
#endif
#ifndef HB_RDX_ROUNDS
#define HB_RDX_ROUNDS 2
#endif
constexpr uint32_t RDX_THREADS = HB_RDX_THREADS;
constexpr uint32_t RDX_WAVES = RDX_THREADS / 64;
constexpr uint32_t RDX_ROUNDS = HB_RDX_ROUNDS;
constexpr uint32_t RDX_TILE = RDX_THREADS * RDX_ROUNDS;  // 2048

struct MsgRec {      // apply input record (16 B)
  uint32_t info;     // type | from << 4 | reject << 8 | voted << 9 | lane << 16 | sub (rec_sub_bits) | long << 28
  uint32_t orig;     // arrival index in the batch
  uint64_t ti;       // Index | Term << 40 (REC_LONG: side[2 orig], side[2 orig + 1])
};
static_assert(sizeof(MsgRec) == 16, "one dwordx4 per record");
constexpr uint32_t REC_LONG = 1u << 28;
// Follower-side batches (hb_batch.commit present, "X mode"): every record also
// carries a 16-byte extension {hint (m.LogTerm / RejectHint), m.Commit} through
// the partition and the route (recx / slotx), and a MsgApp's info says how
// many entries it carries (bits 10-15) and REC_UNI when there are at most
// REC_UNI_MAX and every one has the message's Term — what the follower fast
// lane needs, with no gather by arrival index.
constexpr uint32_t REC_UNI = 1u << 29;
constexpr uint32_t REC_UNI_MAX = 8;
constexpr uint32_t REC_NE_SHIFT = 10;
__device__ __forceinline__ uint32_t rec_ne(uint32_t info) { return (info >> REC_NE_SHIFT) & 0xFu; }
// A final record's partition in its bucket (sub < 2^sis_log, at most 7 bits):
// bits 0-3 at 24-27, bits 4-5 at 30-31, bit 6 at 14 (the entry count above
// uses bits 10-13 only: REC_UNI_MAX = 8)
__device__ __forceinline__ uint32_t rec_sub_bits(uint32_t sub) {
  return ((sub & 0xFu) << 24) | (((sub >> 4) & 3u) << 30) | (((sub >> 6) & 1u) << 14);
}
__device__ __forceinline__ uint32_t rec_sub(uint32_t info) {
  return ((info >> 24) & 0xFu) | (((info >> 30) & 3u) << 4) | (((info >> 14) & 1u) << 6);
}
// the bits of a batch info word a record keeps (lane / partition bits are added by the final pass)
constexpr uint32_t REC_KEEP = 0x3FFFu | REC_LONG | REC_UNI;
constexpr uint32_t REC_IDX_BITS = 40;
constexpr uint64_t REC_IDX_MASK = (1ull << REC_IDX_BITS) - 1;
// pack (term, index) into ti; false: does not fit (REC_LONG)
__device__ __forceinline__ bool rec_pack(uint64_t term, uint64_t index, uint64_t* ti) {
  *ti = index | (term << REC_IDX_BITS);
  return index <= REC_IDX_MASK && term < (1ull << (64 - REC_IDX_BITS));
}
// a record's Term and Index (a long record's from the side table)
__device__ __forceinline__ void rec_unpack(uint32_t info, uint32_t orig, uint64_t ti, const uint64_t* side,
                                           uint64_t* term, uint64_t* index) {
  if (info & REC_LONG) {
    *term = side[2 * (size_t)orig];
    *index = side[2 * (size_t)orig + 1];
  } else {
    *term = ti >> REC_IDX_BITS;
    *index = ti & REC_IDX_MASK;
  }
}
// a route slot (lane-major [k][G], one dwordx4): info, arrival index, ti
__device__ __forceinline__ void slot_unpack(const uint4 r, const uint64_t* side, uint32_t* info, uint32_t* orig,
                                            uint64_t* term, uint64_t* index) {
  *info = r.x;
  *orig = r.y;
  rec_unpack(r.x, r.y, (uint64_t)r.z | ((uint64_t)r.w << 32), side, term, index);
}

struct RadixSrc {
  const uint32_t* group;
  const uint32_t* info;   // the batch's fields (first pass) ...
  const uint64_t* term;
  const uint64_t* index;
  const MsgRec* rec;      // ... or an intermediate pass's records (info without lane bits, arrival index)
  const uint32_t* n_dev;  // null: n
  uint64_t* side;         // first pass: the long records' (term, index) by arrival index
  uint32_t n;
  // X mode (hb_batch.commit present): the batch's hint / commit / entry arrays
  // (first pass) or the intermediate pass's extensions
  const uint64_t* hint;
  const uint64_t* mcommit;
  const uint64_t* eoff;
  const uint64_t* eterm;
  uint64_t n_ent;
  const uint4* recx;
};

// Intermediate pass output: the group ids (what the next pass's histogram
// reads) plus one 16-byte record per message, so that a digit's run of a tile
// is one contiguous store instead of several runs of 32-64 bytes (the SoA
// layout wrote 1.6x its bytes as partial lines on cfg4).
struct RadixDst {
  uint32_t* group;
  MsgRec* rec;
  uint4* recx;  // X mode
};

struct FinalDst {  // final pass output = apply input
  MsgRec* rec;
  uint4* recx;       // X mode: {hint, commit} beside each record
  uint32_t* bucket;  // bucket id per message (multi-pass only, for k_bucket_bounds)
  uint32_t* bk_off;  // [NBK + 1] written by the one-pass scatter
  uint32_t NBK;
  uint32_t sis_log;  // partitions per bucket (log2)
};

__device__ __forceinline__ uint32_t src_n(const RadixSrc& s) { return s.n_dev ? *s.n_dev : s.n; }
// shift = the bucket's log2 size + the pass's digit offset
// dbits = the pass's digit width (<= RDX_BITS; the first of two passes takes half the bits)
__device__ __forceinline__ uint32_t rdx_digit(uint32_t g, uint32_t shift, uint32_t dbits) {
  return (g >> shift) & ((1u << dbits) - 1u);
}

// Exclusive scan over the first 256 threads of the block (all threads call it).
__device__ __forceinline__ uint32_t excl_scan256(uint32_t v, uint32_t* sh4, uint32_t* total) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t incl = wave_incl_scan(v);
  if (tid < 256 && lane == 63) sh4[wave] = incl;
  __syncthreads();
  uint32_t before = 0;
#pragma unroll
  for (uint32_t w = 0; w < 4; ++w) before += (w < wave) ? sh4[w] : 0u;
  *total = sh4[0] + sh4[1] + sh4[2] + sh4[3];
  __syncthreads();
  return before + incl - v;
}

// Per-tile digit counts, HIST_TPB tiles per workgroup: every group id of the
// workgroup's tiles is loaded at once (more loads in flight per lane than one
// 2048-message tile gives), then counted tile by tile in LDS.
#ifndef HB_HIST_TPB
#define HB_HIST_TPB 4
#endif
constexpr uint32_t HIST_TPB = HB_HIST_TPB;
// One-pass partitions take each tile's digit offsets without a scan launch
// (HB_RDX_DIRECT): k_radix_hist also writes each workgroup's digit sums
// (DirectSums::agg) and adds them into its superblock's (SB_HW workgroups,
// agent-scope atomics), and the scatter sums the superblocks, aggregates and
// tiles before its own (k_radix_scatter_d).  The superblock sums rotate over
// three buffers: a step's hist clears the one the next step adds into (read
// by the scatter two steps ago), as far as that one was dirtied.
#ifndef HB_RDX_DIRECT
#define HB_RDX_DIRECT 1
#endif
constexpr uint32_t SB_HW = 32;
constexpr uint32_t SUP_BUFS = 3;
struct DirectSums {
  uint32_t* agg = nullptr;    // [hist workgroups][RDX_BINS]; null: k_scan_rows scans the counts
  uint32_t* sup = nullptr;    // [superblocks][RDX_BINS] of this step (zero on entry)
  uint32_t* clear = nullptr;  // the next step's superblock buffer: n_clear words to zero
  uint32_t n_clear = 0;
  uint32_t* bk_fill = nullptr;  // (k_scan_rows' clears)
  uint32_t NBK = 0;
  uint32_t* ctr = nullptr;
};
__global__ void __launch_bounds__(RDX_THREADS) k_radix_hist(RadixSrc s, uint32_t G, uint32_t shift, uint32_t dbits,
                                                           uint32_t ntiles, uint32_t* hist, uint32_t dm,
                                                           DirectSums ds) {
  __shared__ uint32_t cnt[HIST_TPB][RDX_BINS];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < HIST_TPB * RDX_BINS; i += RDX_THREADS) (&cnt[0][0])[i] = 0;
  __syncthreads();
  const uint32_t n = src_n(s);
  const uint32_t t0 = blockIdx.x * HIST_TPB;
  uint32_t gv[HIST_TPB][RDX_ROUNDS];
#pragma unroll
  for (uint32_t t = 0; t < HIST_TPB; ++t)
#pragma unroll
    for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
      const uint32_t i = (t0 + t) * RDX_TILE + r * RDX_THREADS + tid;
      gv[t][r] = i < n ? s.group[i] : 0xFFFFFFFFu;
    }
#pragma unroll
  for (uint32_t t = 0; t < HIST_TPB; ++t)
#pragma unroll
    for (uint32_t r = 0; r < RDX_ROUNDS; ++r)
      if (gv[t][r] < G) atomicAdd(&cnt[t][rdx_digit(gv[t][r], shift, dbits)], 1u);
  __syncthreads();
  for (uint32_t i = tid; i < (HIST_TPB << dbits); i += RDX_THREADS) {  // the pass's digits only
    if (dm) {  // [digit][tile]
      const uint32_t t = i % HIST_TPB, dg = i / HIST_TPB;
      if (t0 + t < ntiles) hist[(size_t)dg * ntiles + (t0 + t)] = cnt[t][dg];
    } else {  // [tile][digit]
      const uint32_t t = i >> dbits, dg = i & ((1u << dbits) - 1);
      if (t0 + t < ntiles) hist[((size_t)(t0 + t) << dbits) + dg] = cnt[t][dg];
    }
  }
  if (ds.agg) {  // uniform (one pass: dbits = RDX_BITS)
    if (tid < RDX_BINS) {
      uint32_t sum = 0;
#pragma unroll
      for (uint32_t t = 0; t < HIST_TPB; ++t) sum += cnt[t][tid];
      ds.agg[(size_t)blockIdx.x * RDX_BINS + tid] = sum;
      if (sum)
        __hip_atomic_fetch_add(&ds.sup[(size_t)(blockIdx.x / SB_HW) * RDX_BINS + tid], sum, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint32_t gi = blockIdx.x * RDX_THREADS + tid, gs = gridDim.x * RDX_THREADS;
    for (uint32_t i = gi; i < ds.n_clear; i += gs) ds.clear[i] = 0;
    for (uint32_t i = gi; i < ds.NBK; i += gs) ds.bk_fill[i * CTR_STRIDE] = 0;
    if (blockIdx.x == 0)
      for (uint32_t i = tid; i < CTR_WORDS; i += RDX_THREADS) ds.ctr[i] = 0;
  }
}

// Digit scan: workgroup d turns digit d's counts of every tile into exclusive
// per-tile prefixes and writes their total to totals[d].  Two-pass handles keep
// the counts digit-major ([nb][ntiles], dm: a streaming read per workgroup;
// tile-major rows made each workgroup read one word per row: cfg4 1.793 ->
// 1.765 ms, cfg5 0.982 -> 0.968 ms); a one-pass handle keeps them tile-major
// ([ntiles][nb]: the scatter reads its tile's row in one line; digit-major
// measured cfg2 +2 us), with the digits of one 128-byte line of every row
// scanned by workgroups of one XCD.  It also clears the per-bucket event-chunk
// cursors for the coming apply.
#ifndef HB_SCAN_PER
#define HB_SCAN_PER 16
#endif
constexpr uint32_t SCAN_PER = HB_SCAN_PER;
__global__ void __launch_bounds__(1024) k_scan_rows(uint32_t* hist, uint32_t ntiles, uint32_t dbits, uint32_t* totals,
                                                    uint32_t* bk_fill, uint32_t NBK, uint32_t* ctr, uint32_t dm) {
  __shared__ uint32_t sh16[16];
  const uint32_t nb = 1u << dbits;
  const uint32_t d = dm ? blockIdx.x : (nb >= 8 ? (blockIdx.x & 7) * (nb / 8) + (blockIdx.x >> 3) : blockIdx.x);
  uint32_t* col = dm ? hist + (size_t)d * ntiles : hist + d;
  const uint32_t CS = dm ? 0u : dbits;  // element i of the digit's counts at col[i << CS]
  for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < NBK; i += gridDim.x * 1024) bk_fill[i * CTR_STRIDE] = 0;
  if (blockIdx.x == 0)
    for (uint32_t i = threadIdx.x; i < CTR_WORDS; i += blockDim.x) ctr[i] = 0;
  // SCAN_PER consecutive tiles per lane, all loads of a chunk in flight at once
  uint32_t carry = 0;
  for (uint32_t base = 0; base < ntiles; base += 1024 * SCAN_PER) {
    const uint32_t i0 = base + threadIdx.x * SCAN_PER;
    uint32_t v[SCAN_PER], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; ++k) {
      v[k] = i0 + k < ntiles ? col[(size_t)(i0 + k) << CS] : 0u;
      sum += v[k];
    }
    uint32_t tot;
    uint32_t run = carry + block_excl_scan(sum, sh16, &tot);
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; ++k) {
      if (i0 + k < ntiles) col[(size_t)(i0 + k) << CS] = run;
      run += v[k];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) totals[d] = carry;
}

// Tile loads of k_radix_scatter (coalesced: round r, lane l -> element wave*256 + r*64 + l).
template <bool X>
struct ScatTile {
  uint32_t g[RDX_ROUNDS], i[RDX_ROUNDS], o[RDX_ROUNDS];
  uint64_t t[RDX_ROUNDS];  // packed ti
  bool v[RDX_ROUNDS];
};
template <bool X>
__device__ __forceinline__ void scat_load(const RadixSrc& s, uint32_t n, uint32_t G, uint32_t base, uint32_t wave,
                                          uint32_t lane, ScatTile<X>& T) {
#pragma unroll
  for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
    const uint32_t i = base + wave * (64 * RDX_ROUNDS) + r * 64 + lane;
    bool v = i < n;
    T.g[r] = v ? s.group[i] : 0u;
    v = v && T.g[r] < G;
    T.v[r] = v;
    if (s.rec) {
      MsgRec m{};
      if (v) m = s.rec[i];
      T.i[r] = m.info;
      T.o[r] = m.orig;
      T.t[r] = m.ti;
    } else {  // the batch: pack Term and Index (a long pair goes to the side table)
      const uint32_t inf = v ? s.info[i] : 0u;
      const uint64_t tm = v ? s.term[i] : 0ull, ix = v ? s.index[i] : 0ull;
      uint64_t ti;
      const bool fits = rec_pack(tm, ix, &ti);
      if (v && !fits) {
        s.side[2 * (size_t)i] = tm;
        s.side[2 * (size_t)i + 1] = ix;
      }
      uint32_t ie = (inf & 0x3FFu) | (fits ? 0u : REC_LONG);
      if constexpr (X) {
        // a MsgApp's entries: how many, and whether all carry m.Term (the
        // batch's entry arrays are in arrival order: near-contiguous per wave)
        if (v && (inf & 0xFu) == HB_MSG_APP && s.eoff && s.eterm) {
          const uint64_t e0 = s.eoff[i], e1 = i + 1 < n ? s.eoff[i + 1] : s.n_ent;
          const uint64_t ne = e1 - e0;
          bool uni = ne <= REC_UNI_MAX;
#pragma unroll
          for (uint32_t k = 0; k < REC_UNI_MAX; ++k)  // (bounded: the round loop stays unrolled)
            if (uni && k < ne) uni = s.eterm[e0 + k] == tm;
          if (uni) ie |= REC_UNI | ((uint32_t)ne << REC_NE_SHIFT);
        }
      }
      T.i[r] = ie;
      T.o[r] = v ? i : 0u;
      T.t[r] = ti;
    }
  }
}

// One workgroup scatters SCAT_TPW consecutive tiles; the next tile's loads
// are issued before the current tile is ranked, staged and written, so they
// are in flight during its LDS phases and stores.
#ifndef HB_SCAT_TPW
#define HB_SCAT_TPW 2
#endif
constexpr uint32_t SCAT_TPW = HB_SCAT_TPW;
// The scatter of TPW consecutive tiles from tile0 (`first`: the workgroup that
// writes n_valid and the one-pass bucket bounds); `off` / `totals` may be LDS.
// off[dg * ds + tile * ts]: a tile's exclusive prefix of digit dg.
// `pre` runs right after the first tile's loads are issued (k_radix_scatter_d
// sums its offsets there); off's tile index counts from tbase.
struct NoPre {
  __device__ void operator()() const {}
};
template <bool FINAL, bool X, uint32_t TPW, class Pre = NoPre>
__device__ __forceinline__ void scatter_tiles(const RadixSrc& s, const RadixDst& d, const FinalDst& f, uint32_t G,
                                              uint32_t shift, uint32_t dbits, uint32_t ntiles, uint32_t tile0,
                                              const uint32_t* off, uint32_t ds, uint32_t ts, const uint32_t* totals,
                                              uint32_t* n_valid, bool first, const Pre& pre = Pre{},
                                              uint32_t tbase = 0) {
  __shared__ uint32_t s_base[RDX_BINS];  // digit base in the pass output (exclusive scan of the totals)
  __shared__ uint32_t s_off[RDX_BINS];
  __shared__ uint32_t s_wcnt[RDX_WAVES][RDX_BINS];
  __shared__ uint32_t s_dstart[RDX_BINS + 1];
  __shared__ uint32_t sh4[4];
  // the tile staged in digit order: group / info / arrival (3 x 4 B) and ti (8 B)
  // per message; X mode then stages the extensions {hint, commit} (16 B) in the
  // same 40 KB once the records are written (two workgroups still fit a CU)
  __shared__ uint64_t st_buf[RDX_TILE * 5 / 2];
  uint32_t* const st_group = reinterpret_cast<uint32_t*>(st_buf);
  uint32_t* const st_info = st_group + RDX_TILE;
  uint32_t* const st_orig = st_info + RDX_TILE;
  uint64_t* const st_ti = st_buf + 3 * RDX_TILE / 2;
  uint4* const st_x = reinterpret_cast<uint4*>(st_buf);
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint32_t nb = 1u << dbits;  // the pass's digits (totals / off rows hold nb)
  const uint32_t n = src_n(s);
  ScatTile<X> cur, nxt;
  scat_load(s, n, G, tile0 * RDX_TILE, wave, lane, cur);
  pre();
  {
    const uint32_t t = tid < nb ? totals[tid] : 0u;
    uint32_t all;
    const uint32_t excl = excl_scan256(t, sh4, &all);
    if (tid < RDX_BINS) s_base[tid] = excl;
    if (first) {
      if (FINAL && f.bk_off && tid <= f.NBK && tid < RDX_BINS) f.bk_off[tid] = excl;
      if (tid == 0) {
        *n_valid = all;
        if (FINAL && f.bk_off && f.NBK == RDX_BINS) f.bk_off[RDX_BINS] = all;
      }
    }
  }
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (uint32_t j = 0; j < TPW; ++j) {
    const uint32_t tile = tile0 + j;
    if (tile >= ntiles) break;  // uniform
    // this tile's digit starts in the output; per-wave digit counters cleared
    if (tid < nb) s_off[tid] = s_base[tid] + off[(size_t)tid * ds + (size_t)(tile - tbase) * ts];
#pragma unroll
    for (uint32_t k = 0; k < RDX_WAVES * RDX_BINS / RDX_THREADS; ++k) (&s_wcnt[0][0])[tid + k * RDX_THREADS] = 0;
    __syncthreads();
    uint32_t vd[RDX_ROUNDS], vr[RDX_ROUNDS];
#pragma unroll
    for (uint32_t r = 0; r < RDX_ROUNDS; ++r) vd[r] = rdx_digit(cur.g[r], shift, dbits);
    // the next tile's loads go out now
    if (j + 1 < TPW && tile + 1 < ntiles) scat_load(s, n, G, (tile + 1) * RDX_TILE, wave, lane, nxt);
    // stable rank inside the wave: rounds in order, lanes in order
#pragma unroll
    for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
      uint64_t peers = __ballot(cur.v[r]);
#pragma unroll
      for (uint32_t k = 0; k < RDX_BITS; ++k) {
        if (k >= dbits) break;
        const bool bit = (vd[r] >> k) & 1u;
        const uint64_t bk = __ballot(bit);
        peers &= bit ? bk : ~bk;
      }
      const uint32_t rank = (uint32_t)__popcll(peers & lt);
      const uint32_t before = cur.v[r] ? s_wcnt[wave][vd[r]] : 0u;
      vr[r] = before + rank;
      if (cur.v[r] && rank == 0) s_wcnt[wave][vd[r]] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // per digit: prefix over waves, then digit starts inside the tile
    uint32_t run = 0;
    if (tid < RDX_BINS) {
#pragma unroll
      for (uint32_t w = 0; w < RDX_WAVES; ++w) {
        const uint32_t c = s_wcnt[w][tid];
        s_wcnt[w][tid] = run;
        run += c;
      }
    }
    {
      uint32_t all;
      const uint32_t excl = excl_scan256(tid < RDX_BINS ? run : 0u, sh4, &all);
      if (tid < RDX_BINS) s_dstart[tid] = excl;
      if (tid == 0) s_dstart[RDX_BINS] = all;
    }
    __syncthreads();
    uint32_t sp[RDX_ROUNDS];  // staging position of this thread's messages
#pragma unroll
    for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
      sp[r] = s_dstart[vd[r]] + s_wcnt[wave][vd[r]] + vr[r];
      if (cur.v[r]) {
        const uint32_t p = sp[r];
        st_group[p] = cur.g[r];
        st_info[p] = cur.i[r];
        st_orig[p] = cur.o[r];
        st_ti[p] = cur.t[r];
      }
    }
    // X mode: the extensions {m.LogTerm / RejectHint, m.Commit} are read now,
    // not with the tile (16 more VGPRs per tile in flight left one workgroup
    // per CU), and cross the records' output phase in flight
    uint4 xv[X ? RDX_ROUNDS : 1];
    if constexpr (X) {
#pragma unroll
      for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
        const uint32_t i = tile * RDX_TILE + wave * (64 * RDX_ROUNDS) + r * 64 + lane;
        xv[r] = make_uint4(0, 0, 0, 0);
        if (cur.v[r]) {
          if (s.rec) {
            xv[r] = s.recx[i];
          } else {
            const uint64_t h = s.hint ? s.hint[i] : 0ull, c = s.mcommit[i];
            xv[r] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)c, (uint32_t)(c >> 32));
          }
        }
      }
    }
    __syncthreads();
    const uint32_t valid = s_dstart[RDX_BINS];
    uint32_t wo[RDX_ROUNDS];  // output position of staging position r * RDX_THREADS + tid
#pragma unroll
    for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
      const uint32_t p = r * RDX_THREADS + tid;
      if (p < valid) {
        const uint32_t g = st_group[p];
        const uint32_t dg = rdx_digit(g, shift, dbits);
        const uint32_t o = s_off[dg] + (p - s_dstart[dg]);
        wo[r] = o;
        if (FINAL) {
          MsgRec m;
          m.info = (st_info[p] & REC_KEEP) | ((g & (PART - 1)) << 16) |
                   rec_sub_bits((g >> PART_LOG) & ((1u << f.sis_log) - 1));
          m.orig = st_orig[p];
          m.ti = st_ti[p];
          f.rec[o] = m;
          if (f.bucket) f.bucket[o] = g >> (PART_LOG + f.sis_log);
        } else {
          d.group[o] = g;
          MsgRec m;
          m.info = st_info[p];
          m.orig = st_orig[p];
          m.ti = st_ti[p];
          d.rec[o] = m;
        }
      }
    }
    if constexpr (X) {  // the extensions, through the same staging
      __syncthreads();
#pragma unroll
      for (uint32_t r = 0; r < RDX_ROUNDS; ++r)
        if (cur.v[r]) st_x[sp[r]] = xv[r];
      __syncthreads();
#pragma unroll
      for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
        const uint32_t p = r * RDX_THREADS + tid;
        if (p < valid) (FINAL ? f.recx : d.recx)[wo[r]] = st_x[p];
      }
    }
    __syncthreads();  // the next tile reuses s_off / s_wcnt / s_dstart / the staging
    cur = nxt;
  }
}
template <bool FINAL, bool X>
__global__ void __launch_bounds__(RDX_THREADS) __attribute__((amdgpu_waves_per_eu(8))) k_radix_scatter(RadixSrc s, RadixDst d, FinalDst f, uint32_t G,
                                                              uint32_t shift, uint32_t dbits, uint32_t ntiles, const uint32_t* off,
                                                              uint32_t ds, uint32_t ts, const uint32_t* totals, uint32_t* n_valid) {
  scatter_tiles<FINAL, X, SCAT_TPW>(s, d, f, G, shift, dbits, ntiles, blockIdx.x * SCAT_TPW, off, ds, ts, totals, n_valid,
                                    blockIdx.x == 0);
}

// One pass with direct offsets (HB_RDX_DIRECT): each tile's exclusive digit
// prefix = the superblocks before its own + the hist workgroups before its own
// in the superblock + the tiles before it in its hist workgroup; the digit
// totals = every superblock.  Four lanes per digit split those loads, all
// issued at once, while the first tile's loads are in flight.
constexpr uint32_t DQ = RDX_THREADS / RDX_BINS;  // lanes per digit
#ifndef HB_DIRECT_PER
#define HB_DIRECT_PER 16  // items per lane in one round trip (more: further round trips)
#endif
constexpr uint32_t DIRECT_PER = HB_DIRECT_PER;
static_assert(DQ * RDX_BINS == RDX_THREADS && SCAT_TPW <= HIST_TPB && HIST_TPB % SCAT_TPW == 0,
              "a scatter workgroup's tiles sit in one hist workgroup");
struct DirectPre {
  const uint32_t* hist;  // raw tile counts [tile][RDX_BINS]
  const uint32_t* agg;
  const uint32_t* sup;
  uint32_t ntiles, tile0;
  uint32_t* l_pre;  // [DQ][RDX_BINS]
  uint32_t* l_tsum;  // [DQ][RDX_BINS]
  uint32_t* l_off;  // [SCAT_TPW][RDX_BINS]: exclusive prefixes of the workgroup's tiles
  uint32_t* l_tot;  // [RDX_BINS]
  __device__ __forceinline__ const uint32_t* item(uint32_t i, uint32_t nsb, uint32_t na, uint32_t sb,
                                                  uint32_t hb) const {
    return i < nsb ? sup + (size_t)i * RDX_BINS
                   : i < nsb + na ? agg + (size_t)(sb * SB_HW + (i - nsb)) * RDX_BINS
                                  : hist + (size_t)(hb * HIST_TPB + (i - nsb - na)) * RDX_BINS;
  }
  __device__ void operator()() const {
    const uint32_t tid = threadIdx.x, dg = tid % RDX_BINS, q = tid / RDX_BINS;
    const uint32_t hb = tile0 / HIST_TPB, sb = hb / SB_HW;
    const uint32_t nhw = (ntiles + HIST_TPB - 1) / HIST_TPB, nsb = (nhw + SB_HW - 1) / SB_HW;
    const uint32_t na = hb - sb * SB_HW, nt = tile0 - hb * HIST_TPB, ni = nsb + na + nt;
    // the workgroup's own tiles but its last: their counts (lanes of quarter 0)
    uint32_t own[SCAT_TPW > 1 ? SCAT_TPW - 1 : 1];
#pragma unroll
    for (uint32_t j = 0; j + 1 < SCAT_TPW; ++j)
      own[j] = (q == 0 && tile0 + j < ntiles) ? hist[(size_t)(tile0 + j) * RDX_BINS + dg] : 0u;
    uint32_t pre = 0, tot = 0;
    for (uint32_t i0 = 0; i0 < ni; i0 += DQ * DIRECT_PER) {  // (one turn up to 16 superblocks: 8M messages)
      uint32_t v[DIRECT_PER];
#pragma unroll
      for (uint32_t k = 0; k < DIRECT_PER; ++k) {
        const uint32_t i = i0 + k * DQ + q;
        v[k] = i < ni ? item(i, nsb, na, sb, hb)[dg] : 0u;
      }
#pragma unroll
      for (uint32_t k = 0; k < DIRECT_PER; ++k) {
        const uint32_t i = i0 + k * DQ + q;
        if (i < nsb) {
          tot += v[k];
          if (i < sb) pre += v[k];
        } else {
          pre += v[k];
        }
      }
    }
    l_pre[q * RDX_BINS + dg] = pre;
    l_tsum[q * RDX_BINS + dg] = tot;
    __syncthreads();
    if (q == 0) {
      uint32_t p = 0, t = 0;
#pragma unroll
      for (uint32_t k = 0; k < DQ; ++k) {
        p += l_pre[k * RDX_BINS + dg];
        t += l_tsum[k * RDX_BINS + dg];
      }
      l_tot[dg] = t;
#pragma unroll
      for (uint32_t j = 0; j < SCAT_TPW; ++j) {
        l_off[j * RDX_BINS + dg] = p;
        if (j + 1 < SCAT_TPW) p += own[j];
      }
    }
    __syncthreads();
  }
};
template <bool X>
__global__ void __launch_bounds__(RDX_THREADS) __attribute__((amdgpu_waves_per_eu(8))) k_radix_scatter_d(
    RadixSrc s, FinalDst f, uint32_t G, uint32_t shift, uint32_t ntiles, const uint32_t* hist, const uint32_t* agg,
    const uint32_t* sup, uint32_t* n_valid) {
  __shared__ uint32_t l_pre[DQ * RDX_BINS], l_tsum[DQ * RDX_BINS];
  __shared__ uint32_t l_off[SCAT_TPW * RDX_BINS], l_tot[RDX_BINS];
  const uint32_t tile0 = blockIdx.x * SCAT_TPW;
  const DirectPre pre{hist, agg, sup, ntiles, tile0, l_pre, l_tsum, l_off, l_tot};
  scatter_tiles<true, X, SCAT_TPW>(s, RadixDst{}, f, G, shift, RDX_BITS, ntiles, tile0, l_off, 1u, RDX_BINS, l_tot,
                                   n_valid, blockIdx.x == 0, pre, tile0);
}

// One bucket (a node of at most 4,096 groups): the partition is the identity
// on the kept messages, so the final records are the batch's in arrival order
// minus the messages beyond capacity — a stable compaction (ballot prefixes
// per wave, one block scan per tile), no ranking or staging.  Same output as
// k_radix_small / the tiled kernels.
template <bool X>
__global__ void __launch_bounds__(RDX_THREADS) k_pack_one(RadixSrc s, FinalDst f, uint32_t G, uint32_t ntiles,
                                                         uint32_t* bk_fill, uint32_t NBK, uint32_t* ctr,
                                                         uint32_t* n_valid) {
  __shared__ uint32_t s_w[RDX_WAVES];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (uint32_t i = tid; i < NBK; i += RDX_THREADS) bk_fill[i * CTR_STRIDE] = 0;  // (k_scan_rows' clears)
  for (uint32_t i = tid; i < CTR_WORDS; i += RDX_THREADS) ctr[i] = 0;
  const uint32_t n = src_n(s);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t base = 0;
  ScatTile<X> cur, nxt;
  scat_load(s, n, G, 0, wave, lane, cur);
  for (uint32_t tile = 0; tile < ntiles; ++tile) {
    if (tile + 1 < ntiles) scat_load(s, n, G, (tile + 1) * RDX_TILE, wave, lane, nxt);
    // element wave * 64 R + r * 64 + lane: prefixes in (wave, r, lane) order = arrival order
    uint32_t rank[RDX_ROUNDS], wc = 0;
#pragma unroll
    for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
      const uint64_t b = __ballot(cur.v[r]);
      rank[r] = wc + (uint32_t)__popcll(b & lt);
      wc += (uint32_t)__popcll(b);
    }
    if (lane == 0) s_w[wave] = wc;
    __syncthreads();
    uint32_t before = base, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < RDX_WAVES; ++w) {
      const uint32_t c = s_w[w];
      before += w < wave ? c : 0u;
      all += c;
    }
    __syncthreads();  // (s_w is rewritten by the next tile)
#pragma unroll
    for (uint32_t r = 0; r < RDX_ROUNDS; ++r) {
      if (!cur.v[r]) continue;
      const uint32_t o = before + rank[r], g = cur.g[r];
      MsgRec m;
      m.info = (cur.i[r] & REC_KEEP) | ((g & (PART - 1)) << 16) | rec_sub_bits((g >> PART_LOG) & ((1u << f.sis_log) - 1));
      m.orig = cur.o[r];
      m.ti = cur.t[r];
      f.rec[o] = m;
      if constexpr (X) {
        const uint32_t i = cur.o[r];
        const uint64_t h = s.hint ? s.hint[i] : 0ull, c = s.mcommit[i];
        f.recx[o] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)c, (uint32_t)(c >> 32));
      }
    }
    base += all;
    cur = nxt;
  }
  if (tid == 0) {
    *n_valid = base;
    if (f.bk_off) {
      f.bk_off[0] = 0;
      f.bk_off[1] = base;
    }
  }
}

// A small one-pass batch (at most SMALL_TILES tiles: a MultiNode node's Ready
// cycle over a few thousand groups) in ONE workgroup: the tile histograms and
// their column scan in LDS, then the same scatter — k_radix_hist +
// k_scan_rows + k_radix_scatter in one launch, the same output.
constexpr uint32_t SMALL_TILES = 8;
template <bool X>
__global__ void __launch_bounds__(RDX_THREADS) k_radix_small(RadixSrc s, FinalDst f, uint32_t G, uint32_t shift,
                                                            uint32_t ntiles, uint32_t* bk_fill, uint32_t NBK,
                                                            uint32_t* ctr, uint32_t* n_valid) {
  __shared__ uint32_t s_hist[SMALL_TILES * RDX_BINS];  // [tile][digit]: counts, then exclusive prefixes
  __shared__ uint32_t s_tot[RDX_BINS];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < SMALL_TILES * RDX_BINS; i += RDX_THREADS) s_hist[i] = 0;
  for (uint32_t i = tid; i < NBK; i += RDX_THREADS) bk_fill[i * CTR_STRIDE] = 0;  // (k_scan_rows' clears)
  for (uint32_t i = tid; i < CTR_WORDS; i += RDX_THREADS) ctr[i] = 0;
  __syncthreads();
  const uint32_t n = src_n(s);
  for (uint32_t i = tid; i < n; i += RDX_THREADS) {
    const uint32_t g = s.group[i];
    if (g < G) atomicAdd(&s_hist[(i / RDX_TILE) * RDX_BINS + rdx_digit(g, shift, RDX_BITS)], 1u);
  }
  __syncthreads();
  if (tid < RDX_BINS) {
    uint32_t run = 0;
    for (uint32_t t = 0; t < ntiles; ++t) {
      const uint32_t c = s_hist[t * RDX_BINS + tid];
      s_hist[t * RDX_BINS + tid] = run;
      run += c;
    }
    s_tot[tid] = run;
  }
  __syncthreads();
  scatter_tiles<true, X, SMALL_TILES>(s, RadixDst{}, f, G, shift, RDX_BITS, ntiles, 0, s_hist, 1u, RDX_BINS, s_tot,
                                      n_valid, true);
}

// bk_off[b] = first position of bucket b in the sorted batch (b <= NBK); the
// multi-pass case (the one-pass scatter writes bk_off itself).
__global__ void k_bucket_bounds(const uint32_t* bucket, const uint32_t* n_dev, uint32_t NBK, uint32_t* bk_off) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > NBK) return;
  uint32_t lo = 0, hi = *n_dev;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (bucket[mid] < b) lo = mid + 1;
    else hi = mid;
  }
  bk_off[b] = lo;
}

// ============================================================================
// Phase 2: apply
// ============================================================================
#include "hipbatch_follow.h"  // (reads the record layout above)
struct ApplyArgs {
  DevState S;
  const MsgRec* rec;        // sorted batch: bucket order, arrival order inside a bucket
  uint8_t* key;             // partition-in-bucket of each record (k_route writes it for the walk)
  const uint32_t* bk_off;   // [NBK+1] bucket bounds in rec
  uint32_t* bk_fill;        // [NBK x CTR_STRIDE] event records reserved by the bucket's partitions (a line each)
  const uint64_t* hint;     // original-order RejectHint
  const uint32_t* props;    // dense proposals or null
  uint64_t* ev;             // event region base (compact words, hipbatch_kernels.h)
  uint32_t ev_per_msg;      // bound on event words per stepped message
  uint32_t props_on;        // 1 if props[] is present (one proposal slot per group)
  uint32_t NB;              // partitions
  uint32_t NBK;             // buckets
  uint32_t* ev_counts;      // [NB] records in each chunk
  uint64_t* ev_off;         // [NB] chunk offsets (records)
  uint64_t* stats_shard;    // step statistics, NSH shards per value (shard_at; atomic adds)
  uint32_t* pflag;          // [NB][PART/32] groups handed from k_apply_fast to k_apply
  uint32_t* ap_cnt;         // [8] k_apply's work lists: partitions k_apply_fast flagged, one list per
  uint32_t* ap_list;        // [8][NB]  XCD slot (blockIdx % 8) of the flagging workgroup
  uint32_t* fl_cnt;         // k_follow's work list: partitions with groups k_apply handed on
  uint32_t* fl_list;        // [NB]
  uint32_t* eflag;          // [NB][PART/32] (n >= 5) handed-over groups k_elect should try: not a
  uint32_t* el_cnt;         // [8]   leader, or a leader with a higher-term message in its slots;
  uint32_t* el_list;        // [8][NB]  k_elect's work lists (per XCD slot, as ap_list)
  uint32_t grid;            // apply_grid: virtual workgroups of the partition mapping (part_of)
  uint32_t sis_log;         // partitions per bucket (log2)
  uint32_t* done;           // k_apply workgroups finished (the last one runs the finish)
  uint64_t* stats;          // [HB_STAT_COUNT] this step's statistics (finish)
  uint64_t* accum;          // caller accumulator or null (finish)
  uint32_t* resume;         // [G] messages consumed by k_apply_fast | not loaded << 30 | prop pending << 31
  uint64_t* commit0;        // [G] committed at batch start (for HB_STAT_COMMITS)
  // k_route -> k_apply_fast / k_apply: each group's first kmax messages, lane-major
  uint32_t kmax;            // slots per group (= route_kmax(nmax))
  uint8_t* cnt;             // [G] messages of the group in this batch (saturated at 255)
  uint4* slot;              // [kmax][G] MsgRec {info, arrival index, ti} (slot_unpack)
  const uint64_t* side;     // [2 n] (term, index) of the REC_LONG records, by arrival index
  // X mode (follower-side batches): the records' extensions {hint, commit}
  const uint4* recx;        // beside rec (k_route input)
  uint4* slotx;             // [kmax][G] beside slot (null: no X mode this step)
  // storm hand-over (n >= 5, HB_ROUTE_STORM): k_route closes a partition whose
  // groups with messages are all busy leaders with a higher-term message, as
  // k_apply_lead would (flags, lists, event chunks), and k_apply_lead skips it
  uint32_t nmax;            // the handle's replica bound (5 or 7)
  uint32_t storm;           // 1: this step's route may close partitions (lskip), 2: and run k_elect's lane there
  uint8_t* lskip;           // [NB] 1: the route closed the partition
};

// Message slots k_route keeps per group: n - 1 (one MsgAppResp per follower,
// what k_apply_fast consumes), plus HB_KS_EXTRA for n >= 5 so that k_apply
// reads a handed-over group's messages from its slots (an election: MsgHup +
// n - 1 MsgVoteResp + a step-down) instead of walking the bucket.
#ifndef HB_KS_EXTRA
#define HB_KS_EXTRA 2
#endif
// n = 5 keeps 8 slots (4 acks + up to 4 heartbeat responses of a cfg3 step fit,
// so the general kernel's bucket walk is almost never needed)
#ifndef HB_KS5
#define HB_KS5 8
#endif
// n = 3 keeps up to 3: a leader's two MsgAppResp plus the MsgProp a MultiNode
// application proposes in the same Ready cycle stay on the fast lane when the
// batch says it carries MsgProp messages (HB_STEP_MSG_PROPS); otherwise 2 —
// the third slot costs cfg2 4 % (route at one workgroup per CU, one more slot
// per lane: 118.4-120.0 vs 123.5-124.6 us in two same-box pairs)
constexpr uint32_t route_kmax(int nmax) {
  return nmax <= 3 ? 3u : (nmax <= 5 ? (uint32_t)HB_KS5 : (uint32_t)(nmax - 1 + HB_KS_EXTRA));
}
// the slots a step uses (route_kmax is the most any step uses: the allocation)
inline uint32_t step_kmax(uint32_t nmax, uint32_t flags) {
  return nmax <= 3 ? ((flags & HB_STEP_MSG_PROPS) ? 3u : 2u) : route_kmax((int)nmax);
}
static_assert(route_kmax(3) <= 8 && route_kmax(5) <= 8 && route_kmax(7) <= 8,
              "the slot sorts carry slot numbers as 4-bit nibbles of one uint32_t");

// stats slots reduced per workgroup
enum { ST_MSGS, ST_APPRESP, ST_VOTERESP, ST_DROPPED, ST_COMMITS, ST_WON, ST_LOST, ST_FAULTS, ST_ENTRIES, ST_N };

#ifndef HB_FAST_WAVES
#define HB_FAST_WAVES 4
#endif
constexpr uint32_t FLAG_WORDS = PART / 32;  // per-partition bitmask of groups handed to k_apply
// Set (or clear) lane `lane`'s bit of a partition flag mask.  `lane & 63` must
// be the hardware lane and `lane >> 6` the wave's slot in the partition, so a
// wave owns words 2w and 2w + 1.  With HB_FLAG_BALLOT the wave ballots the
// predicate and its lowest active lane issues at most two LDS atomics, instead
// of one per flagged lane all landing on the same word (32-way serialised).
#ifndef HB_FLAG_BALLOT
#define HB_FLAG_BALLOT 1
#endif
template <bool SET>
__device__ __forceinline__ void flag_put(uint32_t* words, uint32_t lane, bool on) {
#if HB_FLAG_BALLOT
  const uint64_t act = __ballot(1);
  const uint64_t b = __ballot(on);
  if (b && (lane & 63) == (uint32_t)__ffsll((long long)act) - 1) {
    const uint32_t w = (lane >> 6) * 2, lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    if (lo) SET ? atomicOr(&words[w], lo) : atomicAnd(&words[w], ~lo);
    if (hi) SET ? atomicOr(&words[w + 1], hi) : atomicAnd(&words[w + 1], ~hi);
  }
#else
  if (on) SET ? atomicOr(&words[lane >> 5], 1u << (lane & 31)) : atomicAnd(&words[lane >> 5], ~(1u << (lane & 31)));
#endif
}
constexpr uint32_t KPL = 64;                // bucket key bytes scanned per lane per segment
constexpr uint32_t SEG = PART * KPL;        // positions per key-scan segment

// blockIdx -> partition.  The sister partitions of a bucket get block ids
// with equal blockIdx % 8, i.e. one XCD under the round-robin placement, so
// the bucket's keys and records are fetched into one L2 (speed only).
__device__ __forceinline__ uint32_t part_of(uint32_t x, uint32_t sl) {
  const uint32_t r = x & 7, q = x >> 3;
  return ((((q >> sl) << 3) | r) << sl) | (q & ((1u << sl) - 1));
}
__device__ __forceinline__ uint32_t block_part(uint32_t sl) { return part_of(blockIdx.x, sl); }

// LDS staging of one round (<= CH messages) of a partition's messages.
// w[j][i] = word j of the round's i-th MsgRec (info, orig, term lo/hi, index lo/hi).
// (Gathering the records by LDS-DMA, global_load_lds_dword x6, measured slower
// than register staging: 6 requests per record instead of 2-3.)
template <uint32_t CH>
struct Stage {
  static constexpr uint32_t CHUNK = CH;
  uint32_t rbuf[CH];      // bucket-relative positions, increasing (= arrival order)
  uint32_t w[6][CH];
  uint16_t perm[CH];
  uint32_t cnt[PART];
  uint32_t sh16[16];
  uint64_t bcast;
  __device__ __forceinline__ uint32_t info(uint32_t i) const { return w[0][i]; }
  __device__ __forceinline__ uint32_t orig(uint32_t i) const { return w[1][i]; }
  __device__ __forceinline__ uint64_t term(uint32_t i) const { return (uint64_t)w[2][i] | ((uint64_t)w[3][i] << 32); }
  __device__ __forceinline__ uint64_t index(uint32_t i) const { return (uint64_t)w[4][i] | ((uint64_t)w[5][i] << 32); }
};

// This lane's KPL key bytes of segment `seg` (positions seg + tid*KPL + k).
// load_keys only issues the loads, so the caller can overlap them with other
// work; eval_keys returns bit k set where the key equals `sub` and the
// position is in [lo, hi).  Four keys per dword: a SWAR zero-byte test, then
// the four byte flags are gathered into a nibble by one multiply.
struct Keys {
  uint4 q[KPL / 16];
  uint32_t base;
};
__device__ __forceinline__ Keys load_keys(const uint8_t* key, uint32_t seg, uint32_t lo, uint32_t hi) {
  Keys k;
  k.base = seg + threadIdx.x * KPL;
  const uint4* p = reinterpret_cast<const uint4*>(key + k.base);
#pragma unroll
  for (int q = 0; q < (int)(KPL / 16); ++q) k.q[q] = (k.base < hi && k.base + KPL > lo) ? p[q] : make_uint4(0, 0, 0, 0);
  return k;
}
__device__ __forceinline__ uint64_t eval_keys(const Keys& k, uint32_t lo, uint32_t hi, uint32_t sub) {
  const uint32_t base = k.base;
  if (base >= hi || base + KPL <= lo) return 0;
  const uint32_t rep = sub * 0x01010101u;
  uint64_t eq = 0;
#pragma unroll
  for (int q = 0; q < (int)(KPL / 16); ++q) {
    const uint32_t w[4] = {k.q[q].x, k.q[q].y, k.q[q].z, k.q[q].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t x = w[j] ^ rep;
      const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // 0x80 where byte == sub
      const uint32_t c = (((z >> 7) * 0x01020408u) >> 24) & 0xFu;                 // bytes 0..3 -> bits 0..3
      eq |= (uint64_t)c << (16 * q + 4 * j);
    }
  }
  const uint32_t a = lo > base ? lo - base : 0u;                // < KPL
  const uint32_t b = hi - base < KPL ? hi - base : KPL;          // > a
  const uint64_t vm = (b >= 64 ? ~0ull : ((1ull << b) - 1)) & (~0ull << a);
  return eq & vm;
}
__device__ __forceinline__ uint64_t scan_keys(const uint8_t* key, uint32_t seg, uint32_t lo, uint32_t hi,
                                              uint32_t sub) {
  return eval_keys(load_keys(key, seg, lo, hi), lo, hi, sub);
}

// Walk the partition's messages of bucket [lo, hi) in arrival order, in
// rounds of at most CHUNK.  on_total(total) runs once (all threads) before
// the first round with the partition's message count; round(fill) runs per
// round with sl.rbuf[0, fill) = the round's bucket-relative positions.
// `first`: the keys of segment 0, already loaded by the caller (or null).
template <class St, class OnTotal, class Round>
__device__ __forceinline__ void walk_partition(St& sl, const ApplyArgs& a, uint32_t lo, uint32_t hi, uint32_t sub,
                                               const Keys* first, OnTotal&& on_total, Round&& round) {
  constexpr uint32_t CHUNK = St::CHUNK;
  const uint32_t tid = threadIdx.x;
  const uint32_t seg0 = lo & ~15u;
  const uint32_t nseg = hi > lo ? (hi - seg0 + SEG - 1) / SEG : 0u;  // uniform
  if (nseg != 1) {
    uint32_t total = 0;
    for (uint32_t s = 0; s < nseg; ++s) {
      uint32_t t;
      (void)block_excl_scan((uint32_t)__popcll(scan_keys(a.key, seg0 + s * SEG, lo, hi, sub)), sl.sh16, &t);
      total += t;
    }
    on_total(total);
  }
  uint32_t fill = 0;  // uniform
  for (uint32_t s = 0; s < nseg; ++s) {
    const uint32_t seg = seg0 + s * SEG;
    const uint64_t eq = (s == 0 && first) ? eval_keys(*first, lo, hi, sub) : scan_keys(a.key, seg, lo, hi, sub);
    uint32_t tot;
    const uint32_t pre = block_excl_scan((uint32_t)__popcll(eq), sl.sh16, &tot);
    if (nseg == 1) on_total(tot);
    const uint32_t base = seg + tid * KPL - lo;
    for (uint32_t done = 0; done < tot;) {
      const uint32_t take = (tot - done) < (CHUNK - fill) ? (tot - done) : (CHUNK - fill);
      uint64_t m = eq;
      uint32_t idx = pre;
      while (m) {
        const uint32_t k = (uint32_t)__ffsll((long long)m) - 1;
        m &= m - 1;
        if (idx >= done && idx < done + take) sl.rbuf[fill + idx - done] = base + k;
        ++idx;
      }
      fill += take;
      done += take;
      if (fill == CHUNK) {
        __syncthreads();
        round(fill);
        fill = 0;
      }
    }
  }
  if (fill) {
    __syncthreads();
    round(fill);
  }
}

// Gather the round's records into LDS and counting-sort them by lane: on
// return the lane's messages are perm[*start, *start + *cnt), in arrival order.
// `issued()` runs once the round's record loads are in flight.
template <class St, class Issued>
__device__ __forceinline__ void gather_round(St& sl, const ApplyArgs& a, uint32_t lo, uint32_t fill,
                                             uint32_t* start, uint32_t* cnt, Issued&& issued) {
  constexpr uint32_t PER = St::CHUNK / PART;
  const uint32_t tid = threadIdx.x;
  sl.cnt[tid] = 0;
  __syncthreads();
  MsgRec m[PER];
#pragma unroll
  for (uint32_t k = 0; k < PER; ++k) {
    const uint32_t i = tid + k * PART;
    if (i < fill) m[k] = a.rec[lo + sl.rbuf[i]];
  }
  issued();
#pragma unroll
  for (uint32_t k = 0; k < PER; ++k) {
    const uint32_t i = tid + k * PART;
    if (i < fill) {
      uint64_t tm, ix;
      rec_unpack(m[k].info, m[k].orig, m[k].ti, a.side, &tm, &ix);
      sl.w[0][i] = m[k].info;
      sl.w[1][i] = m[k].orig;
      sl.w[2][i] = (uint32_t)tm;
      sl.w[3][i] = (uint32_t)(tm >> 32);
      sl.w[4][i] = (uint32_t)ix;
      sl.w[5][i] = (uint32_t)(ix >> 32);
      atomicAdd(&sl.cnt[(m[k].info >> 16) & (PART - 1)], 1u);
    }
  }
  __syncthreads();
  const uint32_t my_cnt = sl.cnt[tid];
  uint32_t total;
  const uint32_t my_start = block_excl_scan(my_cnt, sl.sh16, &total);
  sl.cnt[tid] = my_start;  // becomes the fill cursor
  __syncthreads();
  for (uint32_t i = tid; i < fill; i += PART) {
    const uint32_t pos = atomicAdd(&sl.cnt[(sl.info(i) >> 16) & (PART - 1)], 1u);
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

// The arrival order of a lane's KS route slots as slot numbers in nibbles of
// one word (nibble x = the slot of the lane's x-th message): key[k] = slot k's
// arrival index (0xFFFFFFFF for an unused slot, which sorts last); an
// odd-even transposition network carries the nibbles through its exchanges.
// (Ranking each slot by counting — KS^2 compares, no exchanges — measured
// neutral on cfg3 / cfg4.)
template <uint32_t KS>
__device__ __forceinline__ uint32_t arrival_perm(uint32_t (&key)[KS]) {
  uint32_t perm = 0;
#pragma unroll
  for (uint32_t k = 0; k < KS; ++k) perm |= k << (4 * k);
#pragma unroll
  for (uint32_t r = 0; r < KS; ++r) {
#pragma unroll
    for (uint32_t k = (r & 1); k + 1 < KS; k += 2) {
      const uint32_t k0 = key[k], k1 = key[k + 1];
      const bool sw = k1 < k0;
      key[k] = sw ? k1 : k0;
      key[k + 1] = sw ? k0 : k1;
      const uint32_t p0 = (perm >> (4 * k)) & 0xF, p1 = (perm >> (4 * (k + 1))) & 0xF;
      const uint32_t swp = (perm & ~(0xFFu << (4 * k))) | (p1 << (4 * k)) | (p0 << (4 * (k + 1)));
      perm = sw ? swp : perm;
    }
  }
  return perm;
}

__device__ __forceinline__ bool is_response(uint32_t type) {  // raft/util.go:53-55
  return type == HB_MSG_APP_RESP || type == HB_MSG_VOTE_RESP || type == HB_MSG_HEARTBEAT_RESP ||
         type == HB_MSG_UNREACHABLE;
}

// Reduce the lane statistics of the workgroup and add them (plus the events
// it reserved) to this XCD slot's shard of the step statistics: one no-return
// atomic per value per workgroup, spread over 8 shards; k_finish sums them.
// vals[ST_N] = the lane's events (public count).
template <class T>
__device__ __forceinline__ void reduce_stats(const ApplyArgs& a, uint64_t* l_stats, const T (&vals)[ST_N + 1]) {
  const uint32_t tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k <= ST_N; ++k) {
    uint64_t v = vals[k];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    if ((tid & 63) == 0 && v) atomicAdd((unsigned long long*)&l_stats[k], (unsigned long long)v);
  }
  __syncthreads();
  const uint64_t v = tid <= ST_N ? l_stats[tid] : 0ull;
  if (tid <= ST_N && v)
    atomicAdd((unsigned long long*)&a.stats_shard[shard_at(tid, blockIdx.x & (NSH - 1))], (unsigned long long)v);
}

// The fast and leader kernels' lane statistics are small per-lane counts
// (messages, responses, drops: at most the route slots; commits, faults: 0 or
// 1): four 16-bit fields per word keep a wave's sums exact (< 2^16 while each
// lane's count is < 1024), so ten values take four wave reductions, not ten.
template <>
__device__ __forceinline__ void reduce_stats<uint32_t>(const ApplyArgs& a, uint64_t* l_stats,
                                                       const uint32_t (&vals)[ST_N + 1]) {
  const uint32_t tid = threadIdx.x;
  uint64_t w[4] = {(uint64_t)vals[ST_MSGS] | (uint64_t)vals[ST_APPRESP] << 16 | (uint64_t)vals[ST_DROPPED] << 32 |
                       (uint64_t)vals[ST_COMMITS] << 48,
                   (uint64_t)vals[ST_VOTERESP] | (uint64_t)vals[ST_WON] << 16 | (uint64_t)vals[ST_LOST] << 32 |
                       (uint64_t)vals[ST_FAULTS] << 48,
                   (uint64_t)vals[ST_ENTRIES], (uint64_t)vals[ST_N]};
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) w[k] += __shfl_xor(w[k], d);
  if ((tid & 63) == 0) {
    const uint64_t v[ST_N + 1] = {w[0] & 0xFFFF, (w[0] >> 16) & 0xFFFF, w[1] & 0xFFFF, (w[0] >> 32) & 0xFFFF,
                                  w[0] >> 48,    (w[1] >> 16) & 0xFFFF, (w[1] >> 32) & 0xFFFF, w[1] >> 48,
                                  w[2],          w[3]};
    static_assert(ST_MSGS == 0 && ST_APPRESP == 1 && ST_VOTERESP == 2 && ST_DROPPED == 3 && ST_COMMITS == 4 &&
                      ST_WON == 5 && ST_LOST == 6 && ST_FAULTS == 7 && ST_ENTRIES == 8 && ST_N == 9,
                  "the unpacking above follows the ST_ order");
#pragma unroll
    for (int k = 0; k <= ST_N; ++k)
      if (v[k]) atomicAdd((unsigned long long*)&l_stats[k], (unsigned long long)v[k]);
  }
  __syncthreads();
  const uint64_t v = tid <= ST_N ? l_stats[tid] : 0ull;
  if (tid <= ST_N && v)
    atomicAdd((unsigned long long*)&a.stats_shard[shard_at(tid, blockIdx.x & (NSH - 1))], (unsigned long long)v);
}

// ---------------------------------------------------------------------------
// k_route<KMAX>: W = BK / RG workgroups per bucket, each owning RG groups
// (RG x KMAX message slots fit in LDS: RG = 2048 / 1024 for KMAX = 2 / > 2,
// half that in X mode).  Each workgroup streams its bucket's records (coalesced; the W
// sisters of a bucket share one XCD's L2), ranks the messages of its groups
// with one LDS counter per group, stages each group's first KMAX messages in
// LDS and writes them out lane-major (slot k of group g at slots.*[k][g]) with
// coalesced stores, so k_apply_fast reads them in the same round trip as the
// group state.  Counter ranks follow LDS-atomic order, not arrival order:
// k_apply_fast sorts a group's slots by arrival index and hands a group with
// more than KMAX messages to k_apply whole.  cnt[g] = the group's message
// count (saturated at 255).  Each partition reserves its M event chunk in the
// bucket's region (one atomic per partition).  No raft logic runs here.
// ---------------------------------------------------------------------------
constexpr uint32_t ROUTE_THREADS = 1024;
// cnt[g]: the group's message count (saturated at 127) | CNT_HIGHER when some
// message of the group carries a Term above the group's (n >= 5 routes of
// leader-side batches without dense proposals: k_apply_lead then hands a busy leader — an
// election storm's — over without reading its slots or state; cfg4 1.914 ->
// 1.83 ms.  With dense proposals the check cost cfg3 1.3 % for nothing: a
// leader there proposes, and one without the flag is loaded and stepped up to
// the higher term, as before)
constexpr uint32_t CNT_MASK = 0x7F, CNT_HIGHER = 0x80;
// HB_ROUTE_SORTED=1: the route writes a group's slots in arrival order when
// they hold all its messages (a sort of the <= KMAX arrival indices per group
// in the write-out), so k_apply_lead reads slot x for message x straight from
// HBM instead of staging all slots in LDS to sort them (32 KB per workgroup at
// n = 5: 4 waves/SIMD instead of 3 with HB_LEAD_WAVES=4).  Measured (r05,
// same box): cfg3 0.457-0.460 vs 0.461-0.463 ms, follow n = 5 lane 66.4 vs
// 71.7 us but its step 0.193 vs 0.190 ms and cfg4 1.912 vs 1.871 ms (the
// route's sort): off.
#ifndef HB_ROUTE_SORTED
#define HB_ROUTE_SORTED 0
#endif
#ifndef HB_ROUTE_UNROLL
#define HB_ROUTE_UNROLL 4
#endif
#ifndef HB_ROUTE_STORM
#define HB_ROUTE_STORM 1
#endif
constexpr uint32_t ROUTE_UNROLL = HB_ROUTE_UNROLL;  // records in flight per lane
// Route groups per workgroup (log2), measured on MI355X with 16-byte records
// (same-box A/B, r04): KMAX = 2 at 2048 (2 sisters per 4096-group bucket, 72 KB
// LDS) vs 1024: cfg2 119.2 vs 120.5 us, cfg5 0.995 vs 1.004 ms; KMAX = 6 / 8 at
// 1024 vs 512 (buckets of at least 1024 groups): cfg4 1.949 vs 2.020 ms, cfg3
// neutral.  X mode stages twice the bytes per slot, so it keeps half as many.
constexpr uint32_t route_rg_log(uint32_t kmax, bool x = false) {
  return (kmax <= 3 ? 11u : 10u) - (x ? 1u : 0u);
}
template <int KMAX, bool X> struct RouteGeom {
  static constexpr uint32_t RG_LOG = route_rg_log(KMAX, X);
  static constexpr uint32_t RG = 1u << RG_LOG;     // groups per workgroup
  // workgroups per bucket: 2^(PART_LOG + sis_log - RG_LOG) (sis_log >= RG_LOG - PART_LOG)
};

// EN > 0 (n = EN, storm mode 2): the election lane runs in the route's
// workgroup over the partitions it closes, from the LDS slots (§3.2)
template <int KMAX, bool X, int EN = 0>
__global__ void __launch_bounds__(ROUTE_THREADS) k_route(ApplyArgs a) {
  using RGm = RouteGeom<KMAX, X>;
  constexpr uint32_t RG = RGm::RG, NP = RG / PART;
  const uint32_t sl = a.sis_log, W = 1u << (PART_LOG + sl - RGm::RG_LOG);
  __shared__ uint32_t l_cnt[RG];
  __shared__ uint4 l_slot[KMAX][RG];  // the group's first KMAX records as they will be stored
  __shared__ uint4 l_slotx[X ? KMAX : 1][X ? RG : 1];  // X mode: their extensions
  __shared__ uint32_t l_ptot[NP];
  constexpr bool HI = KMAX >= 5;  // (CNT_HIGHER)
  constexpr bool ST = HI && !X && HB_ROUTE_STORM;
  static_assert(!ST || RG % ROUTE_THREADS == 0, "the storm ballots run at loop level");
  __shared__ uint32_t l_pf[ST ? RG / 32 : 1];  // groups k_apply_lead would hand over unloaded (pflag words)
  __shared__ uint32_t l_ef[ST ? RG / 32 : 1];  // ... of them, k_elect's (eflag words)
  __shared__ uint32_t l_ok[ST ? NP : 1];       // 1: the partition needs no k_apply_lead
  constexpr bool EL = ST && EN > 0;
  static_assert(!EL || (RG == ROUTE_THREADS && !HB_ROUTE_SORTED), "EL: one group per lane, slots as routed");
  __shared__ uint64_t l_moff[EL ? NP : 1];      // EL: the partitions' M chunks
  __shared__ uint32_t l_efill[EL ? NP : 1];     // ... and their fill
  __shared__ uint64_t l_stats[EL ? ST_N + 1 : 1];
  // blockIdx -> (bucket, w): the W sisters of a bucket share blockIdx % 8 (one XCD)
  const uint32_t x = blockIdx.x, q = x >> 3;
  const uint32_t bk = ((q / W) << 3) | (x & 7), w = q % W;
  if (bk >= a.NBK) return;  // uniform: grid padding
  const uint32_t tid = threadIdx.x;
  const uint32_t G = a.S.G;
  const uint32_t lg0 = w * RG;  // first group (in the bucket) of this workgroup
  // (uniform; a follower-side batch's route measured +12 us with it)
  const bool hi_on = HI && !X && !a.props_on;
  const bool storm = ST && a.storm;  // (the host sets it only without props and X)
  for (uint32_t i = tid; i < RG; i += ROUTE_THREADS) l_cnt[i] = 0;
  if (tid < NP) l_ptot[tid] = 0;
  if (ST && tid < NP) l_ok[tid] = 1;
  if (EL && tid < NP) l_efill[tid] = 0;
  if (EL && tid <= ST_N) l_stats[tid] = 0;
  __syncthreads();
  const uint32_t lo = a.bk_off[bk], hi = a.bk_off[bk + 1];
  const uint32_t sub_lo = lg0 >> PART_LOG, sub_hi = (lg0 + RG) >> PART_LOG;
  for (uint32_t base = lo; base < hi; base += ROUTE_THREADS * ROUTE_UNROLL) {
    MsgRec m[ROUTE_UNROLL];
    uint4 mx[X ? ROUTE_UNROLL : 1];
    uint32_t sub[ROUTE_UNROLL];
#pragma unroll
    for (uint32_t u = 0; u < ROUTE_UNROLL; ++u) {
      const uint32_t p = base + u * ROUTE_THREADS + tid;
      if (p < hi) m[u] = a.rec[p];
      if constexpr (X) mx[u] = p < hi ? a.recx[p] : make_uint4(0, 0, 0, 0);
      sub[u] = p < hi ? rec_sub(m[u].info) : 0xFFu;  // the partition in the bucket
    }
    if (w == 0) {  // the key bytes the general kernel's bucket walk scans (one coalesced store per lane)
#pragma unroll
      for (uint32_t u = 0; u < ROUTE_UNROLL; ++u) {
        const uint32_t p = base + u * ROUTE_THREADS + tid;
        if (p < hi) a.key[p] = (uint8_t)sub[u];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < ROUTE_UNROLL; ++u) {
      const uint32_t p = base + u * ROUTE_THREADS + tid;
      const bool own = p < hi && sub[u] >= sub_lo && sub[u] < sub_hi;
      const uint32_t l = own ? (((sub[u] - sub_lo) << PART_LOG) | ((m[u].info >> 16) & (PART - 1))) : RG;
      if (l < RG) {
        const uint32_t r = atomicAdd(&l_cnt[l], 1u);
        if (r < (uint32_t)KMAX) {
          l_slot[r][l] = make_uint4(m[u].info, m[u].orig, (uint32_t)m[u].ti, (uint32_t)(m[u].ti >> 32));
          if constexpr (X) l_slotx[r][l] = mx[X ? u : 0];
        }
      }
    }
  }
  __syncthreads();
  const uint32_t gbase = (bk << (PART_LOG + sl)) + lg0;
  const bool el = EL && storm;            // slots written after the election lane (EL)
  uint32_t e_c = 0;                       // (EL: the lane's group, i = tid)
  bool e_hand = false, e_elect = false;
  uint64_t e_meta = 0;
  for (uint32_t i = tid; i < RG; i += ROUTE_THREADS) {
    const uint32_t c = l_cnt[i], g = gbase + i;
    bool hand = false, elect = false, ok = true;  // (storm)
    if (g < G) {
      // a group whose messages all sit in its slots: any Term above its own?
      bool hib = false;
      uint64_t meta = 0;
      if (storm && c > 0)
        meta = EL ? a.S.meta[g] : (uint64_t)at32(reinterpret_cast<const uint32_t*>(a.S.meta), 2 * g);
      const uint32_t mlo = (uint32_t)meta;
      if (hi_on && c <= (uint32_t)KMAX) {
        const uint64_t t = a.S.term[g];
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)KMAX; ++k) {
          if (k < c) {
            const uint4 r = l_slot[k][i];
            uint64_t tm, ix;
            rec_unpack(r.x, r.y, (uint64_t)r.z | ((uint64_t)r.w << 32), a.side, &tm, &ix);
            hib |= tm > t;
          }
        }
      }
      a.cnt[g] = (uint8_t)((c < CNT_MASK ? c : CNT_MASK) | (hib ? CNT_HIGHER : 0u));
      if (storm && c > 0) {
        // what k_apply_lead (no proposals, no X) hands over unloaded at message 0:
        // a live group that is no leader, a leader whose r.Commit is unknown
        // (M_NC), and a busy leader (more messages than n - 1, all in its slots)
        // with a higher-term message (busy_hi); k_elect tries all but M_NC leaders
        const bool live = m_n(mlo) != 0 && m_fault(mlo) == 0;
        const bool leader = m_state(mlo) == HB_STATE_LEADER, nc = (mlo & (uint32_t)M_NC) != 0;
        const bool busy_hi = leader && !nc && c > a.nmax - 1 && c <= (uint32_t)KMAX && hib;
        hand = live && (!leader || nc || busy_hi);
        elect = live && (!leader || busy_hi);
        ok = !live || hand;  // (a leader to step: k_apply_lead runs the partition)
        if (hand) a.resume[g] = 1u << 30;
      }
      if constexpr (EL) {
        e_c = c;
        e_hand = hand;
        e_elect = elect;
        e_meta = meta;
      }
      // arrival order of a group whose messages all fit (odd-even transposition
      // over the arrival indices, slot numbers riding along as nibbles)
      uint32_t perm = 0, key[KMAX];
#pragma unroll
      for (uint32_t k = 0; k < (uint32_t)KMAX; ++k) {
        perm |= k << (4 * k);
        key[k] = (HB_ROUTE_SORTED && k < c && c <= (uint32_t)KMAX) ? l_slot[k][i].y : 0xFFFFFFFFu;
      }
      if (HB_ROUTE_SORTED && c > 1 && c <= (uint32_t)KMAX) {
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)KMAX; ++r) {
#pragma unroll
          for (uint32_t k = (r & 1); k + 1 < (uint32_t)KMAX; k += 2) {
            const uint32_t k0 = key[k], k1 = key[k + 1];
            const bool sw = k1 < k0;
            key[k] = sw ? k1 : k0;
            key[k + 1] = sw ? k0 : k1;
            const uint32_t p0 = (perm >> (4 * k)) & 0xF, p1 = (perm >> (4 * (k + 1))) & 0xF;
            const uint32_t swp = (perm & ~(0xFFu << (4 * k))) | (p1 << (4 * k)) | (p0 << (4 * (k + 1)));
            perm = sw ? swp : perm;
          }
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < (uint32_t)KMAX; ++k) {
        if (k < c && !el) {
          const uint32_t src = (perm >> (4 * k)) & 0xF;
          at32(a.slot, k * G + g) = l_slot[src][i];
          if constexpr (X) at32(a.slotx, k * G + g) = l_slotx[src][i];
        }
      }
    }
    uint32_t s = c;  // the wave's 64 groups lie in one partition
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    if ((tid & 63) == 0 && s) atomicAdd(&l_ptot[i >> PART_LOG], s);
    if constexpr (ST) {
      if (storm) {
        const uint64_t b = __ballot(hand), e = __ballot(elect), bad = __ballot(!ok);
        if ((tid & 63) == 0) {
          l_pf[i >> 5] = (uint32_t)b;
          l_pf[(i >> 5) + 1] = (uint32_t)(b >> 32);
          l_ef[i >> 5] = (uint32_t)e;
          l_ef[(i >> 5) + 1] = (uint32_t)(e >> 32);
          if (bad) atomicAnd(&l_ok[i >> PART_LOG], 0u);
        }
      }
    }
  }
  __syncthreads();
  if (tid < NP) {
    const uint32_t part = (bk << sl) + w * NP + tid;
    if (part < a.NB) {
      const uint32_t r = atomicAdd(&a.bk_fill[bk * CTR_STRIDE], a.ev_per_msg * (l_ptot[tid] + PART * a.props_on));
      const uint64_t mo =
          (uint64_t)a.ev_per_msg * ((uint64_t)a.NB * PART + lo + ((uint64_t)bk * PART << sl) * a.props_on) + r;
      a.ev_off[2 * part + 1] = mo;
      if constexpr (EL) l_moff[tid] = mo;
    }
  }
  if constexpr (EL) {
    if (el) {  // ---- the election lane over the closed partitions (k_elect's work, slots from LDS)
      __syncthreads();  // l_moff
      const uint32_t p = __builtin_amdgcn_readfirstlane(tid >> PART_LOG);
      const uint32_t g = gbase + tid;
      const bool closed = l_ok[p] != 0;  // (uniform per wave)
      bool done = false;
      uint32_t st_msgs = 0, st_app = 0, st_vote = 0, st_drop = 0, st_commit = 0;
      ElectLane<EN> L;
      L.won = L.lost = L.nev = 0;
      L.committed = L.last = 0;
      uint64_t last0 = 0;
      if (closed) {
        L.S = a.S;
        L.E.chunk = a.ev + l_moff[p];
        L.E.fill = &l_efill[p];
        L.g = g;
        L.meta = e_meta;
        // k_elect's own groups: no leader, or a busy leader with a higher-term message (resume 0, not loaded)
        const bool mine = e_elect && e_c <= (uint32_t)KMAX && L.self() < L.n() && !(L.meta & M_NC);
        if (mine) {
          L.load();
          last0 = L.last;
          const uint64_t commit0 = L.committed;
          uint32_t key[KMAX];
#pragma unroll
          for (uint32_t k = 0; k < (uint32_t)KMAX; ++k) key[k] = k < e_c ? l_slot[k][tid].y : 0xFFFFFFFFu;
          const uint32_t perm = arrival_perm<(uint32_t)KMAX>(key);
          uint32_t x = 0;
#pragma nounroll
          for (; x < e_c; ++x) {
            uint32_t inf, org;
            uint64_t mterm, ix;
            slot_unpack(l_slot[(perm >> (4 * x)) & 0xF][tid], a.side, &inf, &org, &mterm, &ix);
            const uint32_t type = inf & 0xF, from = (inf >> 4) & 0xF;
            if (from >= L.n() && is_response(type)) {  // raft/multinode.go:235
              st_drop++;
              continue;
            }
            if (!L.takes(type, from, mterm)) break;
            L.step(type, from, mterm, (inf >> 8) & 1u);
            st_msgs++;
            st_app += type == HB_MSG_APP_RESP;
            st_vote += type == HB_MSG_VOTE_RESP;
          }
          if (x > 0) {
            L.store();
            if (x == e_c) {
              done = true;  // the group's batch ends here
            } else {        // k_apply resumes at message x, loading what was stored
              a.resume[g] = x;
              a.commit0[g] = commit0;
            }
          }
          st_commit = done && L.committed != commit0;
        }
        flag_put<false>(&l_pf[p * FLAG_WORDS], tid & (PART - 1), done);
      }
      // the slots k_apply (or k_apply_lead / k_elect of an open partition) reads
      if (g < G && e_c > 0 && (!closed || (e_hand && !done))) {
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)KMAX; ++k)
          if (k < e_c) at32(a.slot, k * G + g) = l_slot[k][tid];
      }
      const uint32_t vals[ST_N + 1] = {st_msgs, st_app, st_vote, st_drop, st_commit, L.won, L.lost, 0,
                                       (uint32_t)(L.last - last0), L.nev};
      reduce_stats(a, l_stats, vals);  // (ends with a barrier: l_pf and l_efill are final)
    }
  }
  if constexpr (ST) {
    if (storm) {  // close the partitions k_apply_lead would only hand over (its fast_close)
      if (tid < NP * FLAG_WORDS) {
        const uint32_t p = tid / FLAG_WORDS, j = tid % FLAG_WORDS, part = (bk << sl) + w * NP + p;
        if (part < a.NB && l_ok[p]) {
          a.pflag[(size_t)part * FLAG_WORDS + j] = l_pf[p * FLAG_WORDS + j];
          if (!el) a.eflag[(size_t)part * FLAG_WORDS + j] = l_ef[p * FLAG_WORDS + j];
        }
      }
      if (tid < NP) {
        const uint32_t part = (bk << sl) + w * NP + tid;
        if (part < a.NB) {
          a.lskip[part] = (uint8_t)l_ok[tid];
          if (l_ok[tid]) {
            a.ev_off[2 * part] = (uint64_t)part * PART * a.ev_per_msg;
            a.ev_counts[2 * part] = 0;
            a.ev_counts[2 * part + 1] = EL ? l_efill[EL ? tid : 0] : 0u;
            uint32_t any = 0, eany = 0;
#pragma unroll
            for (uint32_t j = 0; j < FLAG_WORDS; ++j) {
              any |= l_pf[tid * FLAG_WORDS + j];
              eany |= l_ef[tid * FLAG_WORDS + j];
            }
            const uint32_t xs = blockIdx.x & 7;  // (= the bucket's XCD slot, as k_apply_lead's)
            if (any) a.ap_list[(size_t)xs * a.NB + atomicAdd(&a.ap_cnt[xs * CTR_STRIDE], 1u)] = part;
            if (eany && !el) a.el_list[(size_t)xs * a.NB + atomicAdd(&a.el_cnt[xs * CTR_STRIDE], 1u)] = part;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_apply_fast: one workgroup per partition, one lane per group, steady-state
// leader operations only (FastLane).  Every load of the lane (state, its
// message count, its first KMAX messages) is issued at once; no LDS staging,
// no barrier until the statistics.  The first message a lane cannot take
// (and everything after it, and messages beyond KMAX) is handed to k_apply:
// the lane's bit is set in pflag[part] and resume[g] = messages already
// consumed | prop-pending bit.
// ---------------------------------------------------------------------------
// The fast lane's work on one group once its loads are in: the dense proposal into the
// partition's P chunk, then the slot messages in arrival order into its M
// chunk, as far as FastLane takes them.  Sets the group's hand-over bit in
// l_flag (and, n >= 5, its k_elect bit in l_eflag), resume / commit0, and
// returns the statistics of the lane.
// lead: a leader whose state is loaded (the fast path may step it); leader:
// the group is a leader (for k_elect's test) — a leader with more messages
// than slots and no proposal is handed over with its state unloaded.
// fol (X mode): a follower whose messages all sit in its slots, stepped by
// FollowLane as far as it takes them (s_h / s_c: m.LogTerm, m.Commit).
template <int NMAX, uint32_t KS>
__device__ __forceinline__ bool fast_step(const ApplyArgs& a, FollowLane<NMAX>& L, uint32_t part, uint32_t lane,
                                          bool live, bool lead, bool leader, bool fol, uint32_t prop_raw, uint32_t cnt,
                                          uint32_t (&s_info)[KS], uint32_t (&s_orig)[KS],
                                          uint64_t (&s_term)[KS], uint64_t (&s_index)[KS],
                                          uint64_t (&s_h)[KS], uint64_t (&s_c)[KS],
                                          uint64_t moff, uint32_t* l_pfill, uint32_t* l_fill, uint32_t* l_flag,
                                          uint32_t* l_eflag, uint32_t (&vals)[ST_N + 1]) {
  constexpr uint32_t KMAX = KS;
  const uint32_t g = part * PART + lane;
  const uint64_t last0 = L.last, commit0 = L.committed;

  bool flagged = false;
  uint32_t resume = 0;
  uint32_t st_msgs = 0, st_drop = 0, st_app = 0;

  // ---- the dense proposal: its events go to the partition's P chunk (fixed
  // slot of ev_per_msg x PART words), before any message event of the group.
  const uint64_t poff = (uint64_t)part * PART * a.ev_per_msg;
  if (lane == 0) a.ev_off[2 * part] = poff;
  L.E.chunk = a.ev + poff;
  L.E.fill = l_pfill;
  const uint32_t prop_k = live ? prop_raw : 0u;
  if (prop_k) {
    if (lead && L.prop_ok(prop_k)) {
      L.arrival = 0xFFFFFFFFu;
      L.prop(prop_k);
    } else {
      flagged = true;
      resume = 1u << 31;  // the proposal itself is pending (stepped by k_apply into the M chunk)
    }
  }

  // ---- the lane's messages, arrival order (M chunk reserved by k_route).  The
  // slots arrive in k_route's counter order: sort them by arrival index
  // (odd-even transposition over KMAX registers; unused slots sort last).
#pragma unroll
  for (uint32_t k = 0; k < KMAX; ++k) s_orig[k] = k < cnt ? s_orig[k] : 0xFFFFFFFFu;
#pragma unroll
  for (uint32_t r = 0; r < KMAX; ++r) {
#pragma unroll
    for (uint32_t k = (r & 1); k + 1 < KMAX; k += 2) {
      const bool sw = s_orig[k + 1] < s_orig[k];
      const uint32_t i0 = s_info[k], o0 = s_orig[k];
      const uint64_t t0 = s_term[k], x0 = s_index[k], h0 = s_h[k], c0 = s_c[k];
      s_info[k] = sw ? s_info[k + 1] : i0;
      s_orig[k] = sw ? s_orig[k + 1] : o0;
      s_term[k] = sw ? s_term[k + 1] : t0;
      s_index[k] = sw ? s_index[k + 1] : x0;
      s_h[k] = sw ? s_h[k + 1] : h0;
      s_c[k] = sw ? s_c[k + 1] : c0;
      s_info[k + 1] = sw ? i0 : s_info[k + 1];
      s_orig[k + 1] = sw ? o0 : s_orig[k + 1];
      s_term[k + 1] = sw ? t0 : s_term[k + 1];
      s_index[k + 1] = sw ? x0 : s_index[k + 1];
      s_h[k + 1] = sw ? h0 : s_h[k + 1];
      s_c[k + 1] = sw ? c0 : s_c[k + 1];
    }
  }
  L.E.chunk = a.ev + moff;
  L.E.fill = l_fill;
  uint32_t j = 0;  // messages consumed
  if (live && !lead && !fol && cnt > 0 && !flagged) {
    flagged = true;
    resume = 0;
  }
  if (live && cnt > KMAX && !flagged && !L.faulted()) {  // the slots hold an arbitrary KMAX: all to k_apply
    flagged = true;
    resume = 0;
  }
  if (lead) {
#pragma unroll
    for (uint32_t k = 0; k < KMAX; ++k) {
      if (k >= cnt || flagged || L.faulted()) break;
      const uint32_t inf = s_info[k];
      const uint32_t type = inf & 0xF, from = (inf >> 4) & 0xF;
      const bool reject = (inf >> 8) & 1u;
      if (from >= L.n() && is_response(type)) {  // raft/multinode.go:235
        st_drop++;
        j++;
        continue;
      }
      if (KMAX >= 3 && type == HB_MSG_PROP) {  // a local proposal (Term 0; Index = its entry count): stepLeader MsgProp
        if (s_term[k] != 0 || s_index[k] > 0xFFFFFFFFull || !L.prop_ok((uint32_t)s_index[k])) {
          flagged = true;
          resume = j;
          break;
        }
        L.arrival = s_orig[k];
        L.prop((uint32_t)s_index[k]);
        st_msgs++;
        j++;
        continue;
      }
      if (!L.accept_ok(type, from, s_term[k], reject)) {
        flagged = true;
        resume = j;
        break;
      }
      L.arrival = s_orig[k];
      L.accept(from, s_index[k]);
      st_msgs++;
      if (KMAX >= 3) st_app++;
      j++;
    }
  }
  bool fstepped = false;  // FollowLane stepped a message: its state is stored
  if (fol) {
#pragma unroll
    for (uint32_t k = 0; k < KMAX; ++k) {
      if (k >= cnt || flagged || L.faulted()) break;
      const uint32_t inf = s_info[k];
      const uint32_t from = (inf >> 4) & 0xF;
      if (!L.takes_follow(inf, from, s_term[k], s_index[k], s_h[k], s_c[k])) {
        flagged = true;
        resume = j;
        break;
      }
      L.arrival = s_orig[k];
      L.step_follow(inf, from, s_term[k], s_index[k], s_h[k], s_c[k]);
      fstepped = true;
      st_msgs++;
      j++;
    }
  }

  if (lead) L.store();
  if (fstepped) L.store_follow();
  const bool stored = lead || fstepped;
  if constexpr (NMAX >= 5) {  // k_elect's candidates: an election (or a step-down) is likely
    bool higher = false;
#pragma unroll
    for (uint32_t k = 0; k < KMAX; ++k) higher |= k < cnt && s_term[k] > L.term;
    flag_put<true>(l_eflag, lane, flagged && (!leader || higher));
  }
  flag_put<true>(l_flag, lane, flagged);
  if (flagged) {
    at32(a.resume, g) = resume | (stored ? 0u : 1u << 30);
    if (stored) at32(a.commit0, g) = commit0;
  }
  vals[ST_MSGS] = st_msgs;
  vals[ST_APPRESP] = KMAX >= 3 ? st_app : (lead ? st_msgs : 0u);  // (two slots: every leader message is a MsgAppResp)
  vals[ST_VOTERESP] = 0;
  vals[ST_DROPPED] = st_drop;
  vals[ST_COMMITS] = (uint32_t)(!flagged && L.committed != commit0);  // commitTo only raises
  vals[ST_WON] = 0;
  vals[ST_LOST] = 0;
  vals[ST_FAULTS] = (uint32_t)(L.faulted() != 0 && live);
  vals[ST_ENTRIES] = (uint32_t)(L.last - last0);  // (entries appended to one group in one step)
  vals[ST_N] = L.nev;
  return flagged;
}

// The partition's bookkeeping after its lanes (one lane: `lane == 0`'s thread):
// event fills, and the k_apply / k_elect work lists of this XCD slot.
__device__ __forceinline__ void fast_close(const ApplyArgs& a, uint32_t part, const uint32_t* l_flag,
                                           const uint32_t* l_eflag, uint32_t pfill, uint32_t fill) {
  a.ev_counts[2 * part] = pfill;
  a.ev_counts[2 * part + 1] = fill;
  uint32_t any = 0, eany = 0;
#pragma unroll
  for (uint32_t w = 0; w < FLAG_WORDS; ++w) {
    any |= l_flag[w];
    eany |= l_eflag ? l_eflag[w] : 0u;
  }
  const uint32_t xs = blockIdx.x & 7;
  if (any)  // the partition joins k_apply's list of its XCD slot
    a.ap_list[(size_t)xs * a.NB + atomicAdd(&a.ap_cnt[xs * CTR_STRIDE], 1u)] = part;
  if (eany)  // ... and k_elect's
    a.el_list[(size_t)xs * a.NB + atomicAdd(&a.el_cnt[xs * CTR_STRIDE], 1u)] = part;
}

// (n = 3 only: n >= 5 runs k_apply_lead)
template <int NMAX, bool X, uint32_t KMAX>  // KMAX: one MsgAppResp per follower per batch (+ a MsgProp)
__global__ void __launch_bounds__(PART, HB_FAST_WAVES) k_apply_fast(ApplyArgs a) {
  static_assert(NMAX <= 3, "n >= 5 leaders and followers step in k_apply_lead");
  __shared__ uint32_t l_fill, l_pfill;
  __shared__ uint32_t l_flag[FLAG_WORDS];
  __shared__ uint32_t l_eflag[FLAG_WORDS];
  __shared__ uint64_t l_stats[ST_N + 1];

  const uint32_t part = block_part(a.sis_log);
  if (part >= a.NB) return;  // uniform: grid padding
  const uint32_t tid = threadIdx.x;
  const uint32_t g = part * PART + tid;
  const bool gvalid = g < a.S.G;
  if (tid == 0) l_fill = l_pfill = 0;
  if (tid <= ST_N) l_stats[tid] = 0;
  if (tid < FLAG_WORDS) l_flag[tid] = l_eflag[tid] = 0;

  // ---- every load of the lane, one round trip
  FollowLane<NMAX> L;
  L.S = a.S;
  L.g = g;
  L.mlo = gvalid ? at32(reinterpret_cast<uint32_t*>(a.S.meta), 2 * g) : 0u;
  const uint32_t prop_raw = (a.props && gvalid) ? at32(a.props, g) : 0u;
  const uint32_t cnt = gvalid ? at32(a.cnt, g) & CNT_MASK : 0u;
  // The state that depends on nothing is loaded beside meta (one round trip
  // fewer for every leader; a group with no fast-path work wastes 52 bytes)
  if (gvalid) L.load_head();
  // A group takes part when its slot is live (n > 0) and not faulted.
  const bool live = gvalid && L.n() != 0 && L.faulted() == 0;
  // Only a leader has fast-path work: any other live group is handed to
  // k_apply whole, without loading its state here (resume bit 30: commit0 =
  // its committed as k_apply loads it).
  const bool leader = live && L.state() == HB_STATE_LEADER;
  // a group that has not stepped since an empty HardState (r.Commit = 0, M_NC)
  // is the general lane's: its first Step sets r.Commit
  const bool nc = (L.mlo & (uint32_t)M_NC) != 0;
  // a leader the fast path cannot finish (more messages than slots) and
  // without a dense proposal is handed over whole, its state unloaded (cfg4:
  // every group; k_elect / k_apply load it)
  const bool lead = leader && !nc && (cnt <= KMAX || prop_raw != 0);
  // X mode: a follower whose messages all sit in its slots and that has no
  // dense proposal (stepFollower MsgProp forwards it: the general lane)
  const bool fol = X && live && !nc && L.state() == HB_STATE_FOLLOWER && cnt > 0 && cnt <= KMAX && prop_raw == 0;
  L.dirty = 0;
  L.nev = 0;
  if (lead) {
    L.load_rest();
  } else if (fol) {
    L.load_follow();
  } else {
    L.last = L.committed = 0;
    if (!(NMAX >= 5 && leader)) L.term = 0;
  }
  uint32_t s_info[KMAX], s_orig[KMAX];
  uint64_t s_term[KMAX], s_index[KMAX], s_h[KMAX], s_c[KMAX];
  // a leader's (follower's) used slots, in the state loads' round trip (both
  // wait for meta and the count); a group the fast path cannot finish reads none
  const bool slots = (lead || fol) && cnt <= KMAX;
  uint4 raw[KMAX];
#pragma unroll
  for (uint32_t k = 0; k < KMAX; ++k) {
    // (n >= 5: a busier leader's terms too, for k_elect's step-down test below)
    const bool u = NMAX >= 5 ? leader && k < cnt : slots && k < cnt;
    raw[k] = u ? at32(a.slot, k * a.S.G + g) : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (uint32_t k = 0; k < KMAX; ++k) slot_unpack(raw[k], a.side, &s_info[k], &s_orig[k], &s_term[k], &s_index[k]);
#pragma unroll
  for (uint32_t k = 0; k < KMAX; ++k) {
    uint4 x = make_uint4(0, 0, 0, 0);
    if (X && fol && k < cnt) x = at32(a.slotx, k * a.S.G + g);
    s_h[k] = (uint64_t)x.x | ((uint64_t)x.y << 32);
    s_c[k] = (uint64_t)x.z | ((uint64_t)x.w << 32);
  }
  uint32_t vals[ST_N + 1];
  (void)fast_step<NMAX, KMAX>(a, L, part, tid, live, lead, leader, fol, prop_raw, cnt, s_info, s_orig, s_term, s_index, s_h,
                        s_c, a.ev_off[2 * part + 1], &l_pfill, &l_fill, l_flag, l_eflag, vals);
  reduce_stats(a, l_stats, vals);
  if (tid < FLAG_WORDS) a.pflag[(size_t)part * FLAG_WORDS + tid] = l_flag[tid];
  if constexpr (NMAX >= 5) {
    if (tid < FLAG_WORDS) a.eflag[(size_t)part * FLAG_WORDS + tid] = l_eflag[tid];
  }
  if (tid == 0) fast_close(a, part, l_flag, NMAX >= 5 ? l_eflag : nullptr, l_pfill, l_fill);
}

// ---------------------------------------------------------------------------
// k_route_fast<KMAX, X>: k_route<KMAX, X> and k_apply_fast<3, X, KMAX> in one
// workgroup (n = 3, prep and apply on one stream).  The route phase stages
// each of the workgroup's RG groups' first KMAX messages (and, X mode, their
// extensions) in LDS exactly as k_route does; the fast lane then reads them
// from there instead of from the slot arrays, so the slots are neither
// written nor read back (16 + 16 B per message in X mode, plus the count, each
// way).  Only a group the fast lane hands over gets its count and slots
// written to HBM, where k_apply reads them.  512 lanes per workgroup and at
// most ~73 KB of LDS (RG = 2048 groups for two leader-side slots, fewer when
// a group keeps more bytes): two workgroups per CU, each lane stepping
// RG / 512 groups in turn, with no barrier between them (the partitions'
// event cursors and hand-over masks stay in LDS until the end).  Measured on
// cfg2 (same-box A/Bs) and not kept: 1024-group workgroups of 256 or 512
// lanes (+6-9 %), 8 or 16 records in flight per lane in the route phase
// (0 / +1.5 %), the slots staged as four 4-byte planes (neutral), the group
// loop not unrolled (neutral), the next group's first-round loads issued
// before this group's second round (+8 %: 128 VGPRs already, it spills).
// ---------------------------------------------------------------------------
#ifndef HB_ROUTE_FAST
#define HB_ROUTE_FAST 1
#endif
#ifndef HB_RF_UNROLL
#define HB_RF_UNROLL 4  // records in flight per lane in the route phase
#endif
#ifndef HB_RF_THREADS
#define HB_RF_THREADS 512
#endif
#ifndef HB_RF_RG_LOG
#define HB_RF_RG_LOG 11  // (two leader-side slots; each doubling of a group's LDS bytes halves it)
#endif
#ifndef HB_RF_WAVES
#define HB_RF_WAVES 4
#endif
constexpr uint32_t RF_THREADS = HB_RF_THREADS;
constexpr uint32_t RF_UNROLL = HB_RF_UNROLL;
template <uint32_t KMAX, bool X> struct RouteFastGeom {
  // 16 B per slot, twice in X mode: 2 slots x 2048, 3 x 1024, X 2 x 1024, X 3 x 512 groups
  static constexpr uint32_t RG_LOG = HB_RF_RG_LOG - (KMAX > 2 ? 1u : 0u) - (X ? 1u : 0u);
  static constexpr uint32_t RG = 1u << RG_LOG;  // groups per workgroup
  static constexpr uint32_t NP = RG / PART;     // partitions per workgroup
};
template <uint32_t KMAX, bool X>
__global__ void __launch_bounds__(RF_THREADS, HB_RF_WAVES) k_route_fast(ApplyArgs a) {
  constexpr int NMAX = 3;
  using GM = RouteFastGeom<KMAX, X>;
  constexpr uint32_t RG = GM::RG, NP = GM::NP;
  const uint32_t sl = a.sis_log, W = 1u << (PART_LOG + sl - GM::RG_LOG);
  __shared__ uint32_t l_cnt[RG];
  __shared__ uint4 l_slot[KMAX][RG];
  __shared__ uint4 l_slotx[X ? KMAX : 1][X ? RG : 1];
  __shared__ uint32_t l_ptot[NP];
  __shared__ uint64_t l_moff[NP];
  __shared__ uint32_t l_fill[NP], l_pfill[NP];
  __shared__ uint32_t l_flag[NP][FLAG_WORDS];
  __shared__ uint64_t l_stats[ST_N + 1];
  const uint32_t x = blockIdx.x, q = x >> 3;
  const uint32_t bk = ((q / W) << 3) | (x & 7), w = q % W;
  if (bk >= a.NBK) return;  // uniform: grid padding
  const uint32_t tid = threadIdx.x;
  const uint32_t G = a.S.G;
  const uint32_t lg0 = w * RG;
  for (uint32_t i = tid; i < RG; i += RF_THREADS) l_cnt[i] = 0;
  if (tid < NP) {
    l_ptot[tid] = 0;
    l_fill[tid] = l_pfill[tid] = 0;
  }
  for (uint32_t i = tid; i < NP * FLAG_WORDS; i += RF_THREADS) (&l_flag[0][0])[i] = 0;
  if (tid <= ST_N) l_stats[tid] = 0;
  __syncthreads();
  // ---- route: the bucket's records, the workgroup's groups ranked into LDS (as k_route)
  const uint32_t lo = a.bk_off[bk], hi = a.bk_off[bk + 1];
  const uint32_t sub_lo = lg0 >> PART_LOG, sub_hi = (lg0 + RG) >> PART_LOG;
  for (uint32_t base = lo; base < hi; base += RF_THREADS * RF_UNROLL) {
    MsgRec m[RF_UNROLL];
    uint4 mx[X ? RF_UNROLL : 1];
    uint32_t sub[RF_UNROLL];
#pragma unroll
    for (uint32_t u = 0; u < RF_UNROLL; ++u) {
      const uint32_t p = base + u * RF_THREADS + tid;
      if (p < hi) m[u] = a.rec[p];
      if constexpr (X) mx[u] = p < hi ? a.recx[p] : make_uint4(0, 0, 0, 0);
      sub[u] = p < hi ? rec_sub(m[u].info) : 0xFFu;
    }
    if (w == 0) {  // the key bytes of the general kernel's bucket walk
#pragma unroll
      for (uint32_t u = 0; u < RF_UNROLL; ++u) {
        const uint32_t p = base + u * RF_THREADS + tid;
        if (p < hi) a.key[p] = (uint8_t)sub[u];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < RF_UNROLL; ++u) {
      const uint32_t p = base + u * RF_THREADS + tid;
      const bool own = p < hi && sub[u] >= sub_lo && sub[u] < sub_hi;
      const uint32_t l = own ? (((sub[u] - sub_lo) << PART_LOG) | ((m[u].info >> 16) & (PART - 1))) : RG;
      if (l < RG) {
        const uint32_t r = atomicAdd(&l_cnt[l], 1u);
        if (r < KMAX) {
          l_slot[r][l] = make_uint4(m[u].info, m[u].orig, (uint32_t)m[u].ti, (uint32_t)(m[u].ti >> 32));
          if constexpr (X) l_slotx[r][l] = mx[X ? u : 0];
        }
      }
    }
  }
  __syncthreads();
  // ---- each partition's M event chunk in its bucket's region (as k_route)
  for (uint32_t i = tid; i < RG; i += RF_THREADS) {
    uint32_t s = l_cnt[i];  // (a wave's 64 groups lie in one partition)
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    if ((tid & 63) == 0 && s) atomicAdd(&l_ptot[i >> PART_LOG], s);
  }
  __syncthreads();
  const uint32_t part0 = (bk << sl) + w * NP;
  if (tid < NP) {
    const uint32_t part = part0 + tid;
    uint64_t mo = 0;
    if (part < a.NB) {
      const uint32_t r = atomicAdd(&a.bk_fill[bk * CTR_STRIDE], a.ev_per_msg * (l_ptot[tid] + PART * a.props_on));
      mo = (uint64_t)a.ev_per_msg * ((uint64_t)a.NB * PART + lo + ((uint64_t)bk * PART << sl) * a.props_on) + r;
      a.ev_off[2 * part + 1] = mo;
    }
    l_moff[tid] = mo;
  }
  __syncthreads();
  // ---- the fast lane (as k_apply_fast) over the workgroup's groups, RG / RF_THREADS per lane
  uint32_t acc[ST_N + 1];
#pragma unroll
  for (int k = 0; k <= ST_N; ++k) acc[k] = 0;
  for (uint32_t i = tid; i < RG; i += RF_THREADS) {
    const uint32_t p = i >> PART_LOG, part = part0 + p, lane = i & (PART - 1);
    const uint32_t g = part * PART + lane;
    const bool gvalid = part < a.NB && g < G;
    FollowLane<NMAX> L;
    L.S = a.S;
    L.g = g;
    L.mlo = gvalid ? at32(reinterpret_cast<uint32_t*>(a.S.meta), 2 * g) : 0u;
    const uint32_t prop_raw = (a.props && gvalid) ? at32(a.props, g) : 0u;
    const uint32_t c = gvalid ? l_cnt[i] : 0u;
    const uint32_t cnt = c < CNT_MASK ? c : CNT_MASK;
    if (gvalid) L.load_head();
    const bool live = gvalid && L.n() != 0 && L.faulted() == 0;
    const bool leader = live && L.state() == HB_STATE_LEADER;
    const bool nc = (L.mlo & (uint32_t)M_NC) != 0;
    const bool lead = leader && !nc && (cnt <= KMAX || prop_raw != 0);
    const bool fol = X && live && !nc && L.state() == HB_STATE_FOLLOWER && cnt > 0 && cnt <= KMAX && prop_raw == 0;
    L.dirty = 0;
    L.nev = 0;
    if (lead) {
      L.load_rest();
    } else if (fol) {
      L.load_follow();
    } else {
      L.last = L.committed = 0;
      L.term = 0;
    }
    uint32_t s_info[KMAX], s_orig[KMAX];
    uint64_t s_term[KMAX], s_index[KMAX], s_h[KMAX], s_c[KMAX];
    const bool slots = (lead || fol) && cnt <= KMAX;
#pragma unroll
    for (uint32_t k = 0; k < KMAX; ++k) {
      const bool u = slots && k < cnt;
      slot_unpack(u ? l_slot[k][i] : make_uint4(0, 0, 0, 0), a.side, &s_info[k], &s_orig[k], &s_term[k], &s_index[k]);
      uint4 xe = make_uint4(0, 0, 0, 0);
      if constexpr (X) {
        if (fol && k < cnt) xe = l_slotx[k][i];
      }
      s_h[k] = (uint64_t)xe.x | ((uint64_t)xe.y << 32);
      s_c[k] = (uint64_t)xe.z | ((uint64_t)xe.w << 32);
    }
    uint32_t vals[ST_N + 1];
    const bool flagged = fast_step<NMAX, KMAX>(a, L, part, lane, live, lead, leader, fol, prop_raw, cnt, s_info, s_orig,
                                               s_term, s_index, s_h, s_c, l_moff[p], &l_pfill[p], &l_fill[p], l_flag[p],
                                               nullptr, vals);
#pragma unroll
    for (int k = 0; k <= ST_N; ++k) acc[k] += vals[k];
    if (flagged) {  // what k_apply reads of a group it takes over: its count and slots
      a.cnt[g] = (uint8_t)cnt;
#pragma unroll
      for (uint32_t k = 0; k < KMAX; ++k) {
        if (k < c) {
          at32(a.slot, k * G + g) = l_slot[k][i];
          if constexpr (X) at32(a.slotx, k * G + g) = l_slotx[k][i];
        }
      }
    }
  }
  reduce_stats(a, l_stats, acc);  // (ends with a barrier: the partitions' fills and flags are final)
  for (uint32_t j = tid; j < NP * FLAG_WORDS; j += RF_THREADS) {
    const uint32_t p = j / FLAG_WORDS, part = part0 + p;
    if (part < a.NB) a.pflag[(size_t)part * FLAG_WORDS + j % FLAG_WORDS] = l_flag[p][j % FLAG_WORDS];
  }
  if (tid < NP && part0 + tid < a.NB) fast_close(a, part0 + tid, l_flag[tid], nullptr, l_pfill[tid], l_fill[tid]);
}

// ---------------------------------------------------------------------------
// k_apply: the general state machine (Lane::step) for the groups
// k_apply_fast handed over, from their resume point: every leader / candidate
// message type; at a group's first follower-side message (MsgApp /
// MsgHeartbeat / MsgSnap / MsgVote) the group is handed on to a second pass
// over the same partition with the follower-capable lane (Lane<NMAX, true>).
// Only partitions k_apply_fast put on a work list are visited.  A group whose
// messages all sit in its k_route slots (count <= route_kmax) steps them from
// there, in arrival order; the bucket is walked (LDS rounds) only when some
// group of the partition has more messages than slots.
// ---------------------------------------------------------------------------
#ifndef HB_GEN_WAVES
#define HB_GEN_WAVES 2
#endif
struct GenShared {
  Stage<CHUNK> sl;
  uint32_t l_fill;
  uint32_t l_flag[FLAG_WORDS];
  uint32_t l_next[FLAG_WORDS];  // groups handed on to the follower-side pass
  uint64_t l_stats[ST_N + 1];
};

// One partition through the general lane.  FOLLOW = false: the groups
// k_apply_fast flagged (pflag); returns whether any was handed on at a
// follower-side message (sh.l_next).  FOLLOW = true, chained: those groups,
// right after, in the same workgroup (flags and the chunk fill from LDS).
template <int NMAX, bool FOLLOW>
__device__ __forceinline__ bool apply_part(const ApplyArgs& a, uint32_t part, GenShared& sh, bool chained) {
  const uint32_t tid = threadIdx.x;
  const uint32_t bk = part >> a.sis_log, sub = part & ((1u << a.sis_log) - 1);
  const uint32_t g = part * PART + tid;
  const uint32_t fill0 = chained ? sh.l_fill : a.ev_counts[2 * part + 1];
  if (tid < FLAG_WORDS) {
    sh.l_flag[tid] = chained ? sh.l_next[tid] : a.pflag[(size_t)part * FLAG_WORDS + tid];
    sh.l_next[tid] = 0;
  }
  __syncthreads();
  uint32_t any = 0;
#pragma unroll
  for (uint32_t w = 0; w < FLAG_WORDS; ++w) any |= sh.l_flag[w];
  if (!any) return false;  // uniform
  const bool flagged = (sh.l_flag[tid >> 5] >> (tid & 31)) & 1u;

  if (tid == 0) sh.l_fill = fill0;  // append to the M chunk after the previous kernels' events
  if (tid <= ST_N) sh.l_stats[tid] = 0;

  Lane<NMAX, FOLLOW> L;
  L.S = a.S;
  L.E.chunk = a.ev + a.ev_off[2 * part + 1];
  L.E.fill = &sh.l_fill;
  L.g = g;
  L.won = 0;
  L.lost = 0;
  L.nev = 0;
  L.dirty = 0;
  L.prog = false;
  L.voted = false;
  L.meta = 0;
  L.last = 0;
  L.committed = 0;
  uint32_t resume = 0;
  uint64_t commit0 = 0;
  if (flagged) {  // live and not faulted when it was handed over
    L.meta = a.S.meta[g];
    L.load_group();
    resume = a.resume[g];
    commit0 = ((resume >> 30) & 1u) ? L.committed : a.commit0[g];
  }
  const uint64_t last0 = L.last;
  uint32_t st_msgs = 0, st_app = 0, st_vote = 0, st_drop = 0;
  const uint32_t skip = resume & 0x3FFFFFFFu;
  uint32_t j = 0;
  bool handed = false;  // (!FOLLOW) a follower-side message: the group goes on to the follower pass
  uint32_t hand_at = 0;
  const uint32_t lo = a.bk_off[bk], hi = a.bk_off[bk + 1];

  constexpr uint32_t KS = route_kmax(NMAX);
  const uint32_t cnt = flagged ? a.cnt[g] & CNT_MASK : 0u;
  const bool by_slot = flagged && cnt <= a.kmax;  // (a.kmax <= KS: the step's slot count)
  const bool by_walk = flagged && !by_slot;
  __syncthreads();  // l_fill
  // one message through the lane; false: handed on (k_apply only)
  auto step_one = [&](uint32_t inf, uint32_t morig, uint64_t mterm, uint64_t mindex, uint32_t ordinal) -> bool {
    const uint32_t type = inf & 0xF, from = (inf >> 4) & 0xF;
    const bool reject = (inf >> 8) & 1u;
    if (!FOLLOW && is_follower_type(type)) {
      handed = true;
      hand_at = ordinal;
      return false;
    }
    if (from >= L.n() && is_response(type)) {  // raft/multinode.go:235
      st_drop++;
      return true;
    }
    L.arrival = morig;
    L.voted = (inf & HB_INFO_VOTED) != 0;
    // RejectHint of a rejected MsgAppResp; m.LogTerm / the snapshot term of the follower side
    const bool wants_hint = (reject && type == HB_MSG_APP_RESP) || (FOLLOW && is_follower_type(type));
    L.step(type, from, mterm, mindex, reject, (wants_hint && a.hint) ? a.hint[morig] : 0ull);
    st_msgs++;
    st_app += type == HB_MSG_APP_RESP;
    st_vote += type == HB_MSG_VOTE_RESP;
    return true;
  };
  if (by_slot) {
    if (resume >> 31) {
      L.arrival = 0xFFFFFFFFu;
      L.step(HB_MSG_PROP, L.self(), 0, a.props[g], false, 0);
    }
    // arrival order of the slots: odd-even transposition over the arrival
    // indices, the slot numbers riding along as nibbles of `perm`
    uint32_t key[KS];
    uint32_t perm = 0;
#pragma unroll
    for (uint32_t k = 0; k < KS; ++k) {
      key[k] = k < cnt ? at32(a.slot, k * a.S.G + g).y : 0xFFFFFFFFu;
      perm |= k << (4 * k);
    }
#pragma unroll
    for (uint32_t r = 0; r < KS; ++r) {
#pragma unroll
      for (uint32_t k = (r & 1); k + 1 < KS; k += 2) {
        const uint32_t k0 = key[k], k1 = key[k + 1];
        const bool sw = k1 < k0;
        key[k] = sw ? k1 : k0;
        key[k + 1] = sw ? k0 : k1;
        const uint32_t p0 = (perm >> (4 * k)) & 0xF, p1 = (perm >> (4 * (k + 1))) & 0xF;
        const uint32_t swp = (perm & ~(0xFFu << (4 * k))) | (p1 << (4 * k)) | (p0 << (4 * (k + 1)));
        perm = sw ? swp : perm;
      }
    }
    // the next message's loads are issued before this one is stepped (one
    // rolled loop: Lane::step is inlined once per call site)
    uint32_t inf_n = 0, orig_n = 0;
    uint64_t term_n = 0, index_n = 0;
    if (cnt > skip)
      slot_unpack(at32(a.slot, ((perm >> (4 * skip)) & 0xF) * a.S.G + g), a.side, &inf_n, &orig_n, &term_n, &index_n);
#pragma nounroll
    for (uint32_t x = skip; x < cnt; ++x) {
      if (L.faulted()) break;
      const uint32_t inf = inf_n, morig = orig_n;
      const uint64_t mterm = term_n, mindex = index_n;
      if (x + 1 < cnt)
        slot_unpack(at32(a.slot, ((perm >> (4 * (x + 1))) & 0xF) * a.S.G + g), a.side, &inf_n, &orig_n, &term_n,
                    &index_n);
      if (!step_one(inf, morig, mterm, mindex, x)) break;
    }
  }

  auto on_total = [&](uint32_t) {
    __syncthreads();  // l_fill
    if (by_walk && (resume >> 31)) {
      L.arrival = 0xFFFFFFFFu;
      L.step(HB_MSG_PROP, L.self(), 0, a.props[g], false, 0);
    }
  };
  auto round = [&](uint32_t fill) {
    uint32_t my_start, my_cnt;
    gather_round(sh.sl, a, lo, fill, &my_start, &my_cnt, []() {});
    if (by_walk) {
      for (uint32_t x = 0; x < my_cnt; ++x, ++j) {
        if (j < skip || handed) continue;
        if (L.faulted()) break;
        const uint32_t i = sh.sl.perm[my_start + x];
        (void)step_one(sh.sl.info(i), sh.sl.orig(i), sh.sl.term(i), sh.sl.index(i), j);
      }
    }
    __syncthreads();
  };
  if (__syncthreads_or(by_walk)) walk_partition(sh.sl, a, lo, hi, sub, nullptr, on_total, round);

  if (flagged) L.store();
  if (handed) {  // the follower-side pass resumes the group at its follower-side message
    atomicOr(&sh.l_next[tid >> 5], 1u << (tid & 31));
    a.resume[g] = hand_at;
    a.commit0[g] = commit0;
  }
  const bool done = flagged && !handed;  // the group's batch ends in this kernel
  const uint64_t vals[ST_N + 1] = {st_msgs,
                                   st_app,
                                   st_vote,
                                   st_drop,
                                   (uint64_t)(done && L.committed != commit0),
                                   L.won,
                                   L.lost,
                                   (uint64_t)(done && L.faulted() != 0),
                                   L.last - last0,
                                   L.nev};
  reduce_stats(a, sh.l_stats, vals);  // (ends with a barrier: l_next and l_fill are final)
  if (tid == 0) a.ev_counts[2 * part + 1] = sh.l_fill;
  uint32_t nx = 0;
  if constexpr (!FOLLOW) {
#pragma unroll
    for (uint32_t w = 0; w < FLAG_WORDS; ++w) nx |= sh.l_next[w];
  }
  return nx != 0;
}

// k_apply runs over k_apply_fast's work lists, on the apply grid: workgroup w
// takes entry w / 8 of the list of XCD slot w % 8 (the slot of the workgroup
// that flagged the partition, so a bucket's sisters stay on one XCD; a list
// holds at most grid / 8 entries).  Partitions it hands on at a follower-side
// message (MsgApp / MsgHeartbeat / MsgSnap / MsgVote) go to k_follow's list.
#ifndef HB_FOLLOW_GRID
#define HB_FOLLOW_GRID 128
#endif
constexpr uint32_t FOLLOW_GRID = HB_FOLLOW_GRID;
// k_apply's grid: 0 = one workgroup per partition (each takes at most one list
// entry); else a persistent grid of that many (a multiple of 8).  Measured on
// MI355X: 512 saves ~1.5 us on an empty cfg2 step but cost 5-7 % on cfg3 /
// cfg4 while every partition was on the lists.  Since the leader lane
// (k_apply_lead) the n >= 5 lists are short, and the per-partition grid of a
// 256-VGPR, 31 KB-LDS kernel is itself ~40 us of dispatch (cfg3).
#ifndef HB_GEN_GRID
#define HB_GEN_GRID 1024
#endif
constexpr uint32_t GEN_GRID = HB_GEN_GRID;
#ifndef HB_GEN_GRID3
#define HB_GEN_GRID3 512  // n = 3 (cfg2 / cfg5: few partitions handed over): persistent, 2 per CU
#endif
constexpr uint32_t GEN_GRID3 = HB_GEN_GRID3;
static_assert(GEN_GRID % 8 == 0, "k_apply strides its XCD-slot lists by gridDim.x / 8");

// The step's finish (as k_finish), run by the last k_follow workgroup: the
// statistics shards (agent-scope atomics of every apply kernel) summed into
// stats (+ accum), the shards and the work lists cleared for the next step.
static_assert((ST_N + 1) * NSH <= PART && (NSH & (NSH - 1)) == 0, "a finish lane per (value, shard)");
__device__ __forceinline__ void finish_step(const ApplyArgs& a) {
  const int map[ST_N + 1] = {HB_STAT_MSGS,  HB_STAT_APPRESP, HB_STAT_VOTERESP, HB_STAT_DROPPED, HB_STAT_COMMITS,
                             HB_STAT_WON,   HB_STAT_LOST,    HB_STAT_FAULTS,   HB_STAT_ENTRIES, HB_STAT_EVENTS};
  // one lane per (value, shard): one round trip; the NSH lanes of a value are adjacent in a wave
  const uint32_t t = threadIdx.x, k = t / NSH;
  uint64_t v = 0;
  if (k <= ST_N) {
    v = __hip_atomic_load(&a.stats_shard[shard_at(k, t % NSH)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.stats_shard[shard_at(k, t % NSH)], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (uint32_t d = 1; d < NSH; d <<= 1) v += __shfl_xor(v, d);
  if (k <= ST_N && t % NSH == 0) {
    a.stats[map[k]] = v;
    if (a.accum) a.accum[map[k]] += v;
  }
}

// The workgroups that finish the step take tickets; the step's finish runs
// in the last.  Only workgroups that had work take one (`working` of them, a
// count every workgroup derives from the work-list lengths): a ticket per
// workgroup of the grid serialises hundreds of atomics on one word (~11 ns
// each).  With no work anywhere, workgroup 0 finishes at once.  (The
// work-list counters and the ticket word belong to the prep set and are
// cleared by the next prep that reuses it, never by a workgroup still
// reading them.)
__device__ __forceinline__ void finish_by_ticket(const ApplyArgs& a, bool worked, uint32_t working,
                                                 uint32_t* l_last) {
  if (working == 0) {
    if (blockIdx.x == 0) finish_step(a);  // uniform
    return;
  }
  if (!worked) return;  // uniform
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's stats atomics are performed
  __syncthreads();
  if (threadIdx.x == 0)
    *l_last = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == working - 1;
  __syncthreads();
  if (*l_last) finish_step(a);  // uniform
}

// CHAIN (n = 3): the follower-side pass runs chained in the same workgroup
// and k_apply's last workgroup runs the step's finish — no k_follow launch
// (n = 3's general kernel does not spill either way; at n >= 5 the follower
// lane's registers stay out of the hot general kernel).
template <int NMAX>
__global__ void __launch_bounds__(PART, HB_GEN_WAVES) k_apply(ApplyArgs a) {
  constexpr bool CHAIN = NMAX <= 3;
  __shared__ GenShared sh;
  __shared__ uint32_t l_last;
  // persistent over the list of its XCD slot when the grid is smaller than
  // the partitions (HB_GEN_GRID)
  const uint32_t xs = blockIdx.x & 7, stride = gridDim.x >> 3;
  uint32_t nl = 0, working = 0;
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    const uint32_t c = __hip_atomic_load(&a.ap_cnt[k * CTR_STRIDE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    nl = k == xs ? c : nl;
    working += c < stride ? c : stride;  // workgroups of slot k with at least one entry
  }
  for (uint32_t i = blockIdx.x >> 3; i < nl; i += stride) {  // uniform
    const uint32_t part = a.ap_list[(size_t)xs * a.NB + i];
    if (apply_part<NMAX, false>(a, part, sh, false)) {  // uniform: the partition goes on to the follower pass
      if constexpr (CHAIN) {
        __syncthreads();
        (void)apply_part<NMAX, true>(a, part, sh, true);
      } else {
        if (threadIdx.x < FLAG_WORDS) a.pflag[(size_t)part * FLAG_WORDS + threadIdx.x] = sh.l_next[threadIdx.x];
        if (threadIdx.x == 0) a.fl_list[atomicAdd(a.fl_cnt, 1u)] = part;
      }
    }
    __syncthreads();  // sh is reused by the next partition
  }
  if constexpr (CHAIN) finish_by_ticket(a, (blockIdx.x >> 3) < nl, working, &l_last);
}

// k_elect: the election lane (hipbatch_elect.h) over k_apply_fast's work
// lists, before k_apply (n >= 5, unsized logs): a handed-over group whose
// messages all sit in its route slots is stepped by ElectLane as far as it
// takes them; a group it finishes leaves the partition's flags, a group it
// hands over resumes in k_apply at the first message it did not take.
#ifndef HB_ELECT_WAVES
#define HB_ELECT_WAVES 4
#endif
#ifndef HB_ELECT_GRID  // persistent over the XCD-slot lists (cfg4 -9 to -11 us, cfg3 -3 to -6 us vs one
#define HB_ELECT_GRID 1024  // workgroup per partition: an empty or short list launched 16K workgroups)
#endif
#ifndef HB_ELECT_EAGER
#define HB_ELECT_EAGER 1
#endif
#ifndef HB_ELECT_PF
#define HB_ELECT_PF 1
#endif
constexpr uint32_t ELECT_GRID = HB_ELECT_GRID;
static_assert(ELECT_GRID % 8 == 0, "k_elect strides its XCD-slot lists by gridDim.x / 8");

template <int NMAX>
__global__ void __launch_bounds__(PART, HB_ELECT_WAVES) k_elect(ApplyArgs a) {
  constexpr uint32_t KS = route_kmax(NMAX);
  __shared__ uint32_t l_fill;
  __shared__ uint32_t l_flag[FLAG_WORDS];
  __shared__ uint32_t l_eflag[FLAG_WORDS];
  __shared__ uint64_t l_stats[ST_N + 1];
  // each lane's route slots, read once: the arrival keys come from them and the
  // messages are then read back in arrival order (reading the keys from HBM and
  // the slots again fetched every slot line twice: 16-byte slots, 4-byte keys)
  __shared__ uint4 l_slot[KS][PART];
  const uint32_t tid = threadIdx.x;
  const uint32_t xs = blockIdx.x & 7, stride = gridDim.x >> 3;
  const uint32_t nl = __hip_atomic_load(&a.el_cnt[xs * CTR_STRIDE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if HB_ELECT_PF
  // the partition list two ahead and the next partition's flags and event fill
  // are fetched during this partition's work (two round trips off each turn)
  const uint32_t* list = a.el_list + (size_t)xs * a.NB;
  uint32_t i = blockIdx.x >> 3;
  uint32_t part = i < nl ? list[i] : 0u;
  uint32_t nxt = i + stride < nl ? list[i + stride] : 0u;
  uint32_t pf = 0, pe = 0, pfill = 0;
  if (i < nl) {
    if (tid < FLAG_WORDS) {
      pf = a.pflag[(size_t)part * FLAG_WORDS + tid];
      pe = a.eflag[(size_t)part * FLAG_WORDS + tid];
    }
    if (tid == 0) pfill = a.ev_counts[2 * part + 1];
  }
  for (; i < nl; i += stride) {  // uniform
    const uint32_t g = part * PART + tid;
    if (tid < FLAG_WORDS) {
      l_flag[tid] = pf;
      l_eflag[tid] = pe;
    }
    if (tid == 0) l_fill = pfill;  // after k_apply_fast's events
    if (tid <= ST_N) l_stats[tid] = 0;
    __syncthreads();
#else
  for (uint32_t i = blockIdx.x >> 3; i < nl; i += stride) {  // uniform
    const uint32_t part = a.el_list[(size_t)xs * a.NB + i];
    const uint32_t g = part * PART + tid;
    if (tid < FLAG_WORDS) {
      l_flag[tid] = a.pflag[(size_t)part * FLAG_WORDS + tid];
      l_eflag[tid] = a.eflag[(size_t)part * FLAG_WORDS + tid];
    }
    if (tid == 0) l_fill = a.ev_counts[2 * part + 1];  // after k_apply_fast's events
    if (tid <= ST_N) l_stats[tid] = 0;
    __syncthreads();
#endif
    const bool flagged = (l_eflag[tid >> 5] >> (tid & 31)) & 1u;  // (a subset of the k_apply flags)
    ElectLane<NMAX> L;
    L.S = a.S;
    L.E.chunk = a.ev + a.ev_off[2 * part + 1];
    L.E.fill = &l_fill;
    L.g = g;
    L.meta = flagged ? a.S.meta[g] : 0ull;
    const uint32_t cnt = flagged ? a.cnt[g] & CNT_MASK : 0u;
    const uint32_t resume = flagged ? a.resume[g] : 0u;
    // (flagged groups are live and not faulted; a pending dense proposal goes to k_apply)
    const bool mine = flagged && cnt <= KS && (resume >> 31) == 0 && L.self() < L.n() && !(L.meta & M_NC);
    uint32_t st_msgs = 0, st_app = 0, st_vote = 0, st_drop = 0;
    bool done = false;
    uint64_t last0 = 0, commit0 = 0;
    L.won = L.lost = L.nev = 0;
    L.committed = L.last = 0;
    uint32_t key[KS];  // the slots' arrival keys (0xFFFFFFFF past cnt)
#if HB_ELECT_EAGER
    // every load of a flagged lane in the round trip of meta / cnt / resume: the
    // state, commit0 and all KS slots (those past cnt are masked here)
    uint64_t c0 = 0;
    if (flagged) {
      L.load();
      c0 = a.commit0[g];
      uint4 sl[KS];
#pragma unroll
      for (uint32_t k = 0; k < KS; ++k) sl[k] = at32(a.slot, k * a.S.G + g);
#pragma unroll
      for (uint32_t k = 0; k < KS; ++k) {
        const uint4 r = k < cnt ? sl[k] : make_uint4(0, 0xFFFFFFFFu, 0, 0);
        l_slot[k][tid] = r;
        key[k] = r.y;
      }
    }
#endif
#if HB_ELECT_PF
    const uint32_t nn = i + 2 * stride < nl ? list[i + 2 * stride] : 0u;
    if (i + stride < nl) {
      if (tid < FLAG_WORDS) {
        pf = a.pflag[(size_t)nxt * FLAG_WORDS + tid];
        pe = a.eflag[(size_t)nxt * FLAG_WORDS + tid];
      }
      if (tid == 0) pfill = a.ev_counts[2 * nxt + 1];
    }
#endif
    if (mine) {
#if !HB_ELECT_EAGER
      L.load();
#endif
      last0 = L.last;
#if HB_ELECT_EAGER
      commit0 = ((resume >> 30) & 1u) ? L.committed : c0;
#else
      commit0 = ((resume >> 30) & 1u) ? L.committed : a.commit0[g];
#pragma unroll
      for (uint32_t k = 0; k < KS; ++k) {
        const uint4 r = k < cnt ? at32(a.slot, k * a.S.G + g) : make_uint4(0, 0xFFFFFFFFu, 0, 0);
        l_slot[k][tid] = r;
        key[k] = r.y;
      }
#endif
      // arrival order of the slots (odd-even transposition, slot numbers as nibbles)
      const uint32_t perm = arrival_perm<KS>(key);
      const uint32_t skip = resume & 0x3FFFFFFFu;
      uint32_t x = skip;
#pragma nounroll
      for (; x < cnt; ++x) {
        uint32_t inf, org;  // (from the lane's LDS copy)
        uint64_t mterm, ix;
        slot_unpack(l_slot[(perm >> (4 * x)) & 0xF][tid], a.side, &inf, &org, &mterm, &ix);
        const uint32_t type = inf & 0xF, from = (inf >> 4) & 0xF;
        if (from >= L.n() && is_response(type)) {  // raft/multinode.go:235
          st_drop++;
          continue;
        }
        if (!L.takes(type, from, mterm)) break;
        L.step(type, from, mterm, (inf >> 8) & 1u);
        st_msgs++;
        st_app += type == HB_MSG_APP_RESP;
        st_vote += type == HB_MSG_VOTE_RESP;
      }
      if (x > skip) {
        L.store();
        if (x == cnt) {
          done = true;  // the group's batch ends here
        } else {  // k_apply resumes at message x, loading what was stored
          a.resume[g] = x;
          a.commit0[g] = commit0;
        }
      }
    }
    flag_put<false>(l_flag, tid, done);
    const uint64_t vals[ST_N + 1] = {st_msgs,
                                     st_app,
                                     st_vote,
                                     st_drop,
                                     (uint64_t)(done && L.committed != commit0),
                                     L.won,
                                     L.lost,
                                     0,
                                     mine ? L.last - last0 : 0ull,
                                     L.nev};
    reduce_stats(a, l_stats, vals);  // (ends with a barrier: l_flag and l_fill are final)
    if (tid < FLAG_WORDS) a.pflag[(size_t)part * FLAG_WORDS + tid] = l_flag[tid];
    if (tid == 0) a.ev_counts[2 * part + 1] = l_fill;
    __syncthreads();  // the next partition reuses the LDS
#if HB_ELECT_PF
    part = nxt;
    nxt = nn;
#endif
  }
}

#ifndef HB_LEAD_XSTAGE
#define HB_LEAD_XSTAGE 1
#endif
#ifndef HB_LEAD_XWAVES  // k_apply_lead<5> in X mode (LDS: 4 staged slots + the lane rows = 36 KB)
#define HB_LEAD_XWAVES 4
#endif
#ifndef HB_LEAD_WAVES
#define HB_LEAD_WAVES 3  // (n = 5: 125 VGPRs, 53 KB of LDS: 3 workgroups per CU)
#endif

#ifndef HB_LEAD7_WAVES  // k_apply_lead<7> (measured on cfg4: 2 waves +3 %, 4 waves -0.6 % with 128 B/lane of scratch)
#define HB_LEAD7_WAVES 3
#endif
// ---------------------------------------------------------------------------
// k_apply_lead (n >= 5, replaces k_apply_fast there): one workgroup per
// partition, one lane per group, the leader lane (hipbatch_lead.h) for every
// leader whose messages all sit in its route slots: the dense proposal, then
// the slot messages in arrival order as far as LeadLane::takes allows — every
// response a leader steps at its own term.  One load and one store of the
// group's state for the whole batch.  What it cannot take is handed over as
// k_apply_fast does (resume word, pflag; eflag for k_elect: a group that is no
// leader, or a leader stopped by a higher-term message).  A leader without a
// proposal and with more messages than n - 1 (an election storm's leader)
// first reads only its Term and its slots' terms: with a higher term among
// them it is handed over unloaded.
// ---------------------------------------------------------------------------
// X mode (follower-side batches): a follower whose messages all sit in its
// first FOLLOW_SLOTS route slots is stepped by FollowLane in the same pass
// (the follower side of a node with n >= 5 replicas: about (n-1)/n of its
// groups), the slots' {m.LogTerm, m.Commit} extensions staged beside them.
constexpr uint32_t FOLLOW_SLOTS = 4;
// Leaders' Match / Next in LDS (LeadLaneL) or in registers (LeadLane), per n
#ifndef HB_LEAD_LDS5
#define HB_LEAD_LDS5 1
#endif
#ifndef HB_LEAD_LDS7
#define HB_LEAD_LDS7 0  // n = 7: 28 KB of {Match, Next} leave 2 workgroups per CU (cfg4 2.018 vs 1.918 ms)
#endif
template <int NMAX> struct LeadOf {
  static constexpr bool LDS = NMAX <= 5 ? HB_LEAD_LDS5 : HB_LEAD_LDS7;
  using T = typename std::conditional<LDS, LeadLaneL<NMAX>, LeadLane<NMAX>>::type;
};
template <int NMAX, bool X>
__global__ void __launch_bounds__(PART, NMAX <= 5 ? (X && HB_LEAD_XSTAGE ? HB_LEAD_XWAVES : HB_LEAD_WAVES)
                                                 : HB_LEAD7_WAVES) k_apply_lead(ApplyArgs a) {
  constexpr uint32_t KS = route_kmax(NMAX);
  constexpr uint32_t FS = X ? FOLLOW_SLOTS : 1u;
  constexpr bool LDS = LeadOf<NMAX>::LDS;
  __shared__ uint32_t l_fill, l_pfill;
  __shared__ uint32_t l_flag[FLAG_WORDS];
  __shared__ uint32_t l_eflag[FLAG_WORDS];
  __shared__ uint64_t l_stats[ST_N + 1];
  // the lane's route slots, read once (as in k_elect) — unless the route wrote
  // them in arrival order (HB_ROUTE_SORTED): then slot x is read for message x.
  // X mode stages only the first FS (a follower's; a leader reads the rest from
  // HBM), so that the kernel fits 4 workgroups per CU (HB_LEAD_XSTAGE)
  constexpr uint32_t SR = HB_ROUTE_SORTED ? 0u : ((X && HB_LEAD_XSTAGE) ? FS : KS);
  __shared__ uint4 l_slot[SR ? SR : 1][SR ? PART : 1];
  // per lane, one 16-byte word per slot: a leader's {Match, Next} (LeadLaneL) or,
  // X mode, a follower's slot extensions {m.LogTerm, m.Commit} — a lane is one or the other
  constexpr uint32_t LW = LDS ? (NMAX > FS ? NMAX : FS) : (X ? FS : 1u);
  __shared__ uint4 l_lane[LW][(LDS || X) ? PART : 1];
  const uint32_t part = block_part(a.sis_log);
  if (part >= a.NB) return;  // uniform: grid padding
  if (!X && a.storm && a.lskip[part]) return;  // uniform: the route closed it (storm hand-over)
  const uint32_t tid = threadIdx.x;
  const uint32_t g = part * PART + tid;
  const bool gvalid = g < a.S.G;
  auto slot_at = [&](uint32_t k) -> uint4 {
    if constexpr (SR == 0) return at32(a.slot, k * a.S.G + g);
    else if constexpr (SR < KS) return k < SR ? l_slot[k < SR ? k : 0][threadIdx.x] : at32(a.slot, k * a.S.G + g);
    else return l_slot[k][threadIdx.x];
  };
  if (tid == 0) l_fill = l_pfill = 0;
  if (tid <= ST_N) l_stats[tid] = 0;
  if (tid < FLAG_WORDS) l_flag[tid] = l_eflag[tid] = 0;

  FollowLane<NMAX, typename LeadOf<NMAX>::T> L;
  L.S = a.S;
  L.g = g;
  if constexpr (LDS) L.lp = &l_lane[0][tid];
  L.mlo = gvalid ? reinterpret_cast<const uint32_t*>(a.S.meta)[2 * (size_t)g] : 0u;
  const uint32_t prop_raw = (a.props && gvalid) ? a.props[g] : 0u;
  const uint32_t craw = gvalid ? a.cnt[g] : 0u, cnt = craw & CNT_MASK;
  // X mode (a MultiNode node's batch: it leads some groups and follows most):
  // the per-group fields every role steps with come in meta's round trip
  L.last = L.committed = 0;
  L.term = 0;
  if (X && gvalid) L.load_state_head();
  const bool live = gvalid && L.n() != 0 && L.faulted() == 0;
  const bool leader = live && L.state() == HB_STATE_LEADER;
  const bool fits = cnt <= KS;  // every message of the group is in its slots
  // r.Commit = 0 (M_NC): the general lane steps the group's first message
  const bool nc = (L.mlo & (uint32_t)M_NC) != 0;
  // a leader with a proposal or at most one message per follower loads at once
  const bool spec = leader && !nc && (prop_raw != 0 || (fits && cnt <= (uint32_t)NMAX - 1));
  // X mode: a follower whose messages all sit in its first FS slots, without a
  // dense proposal (stepFollower forwards it: the general lane)
  const bool fol = X && live && !nc && L.state() == HB_STATE_FOLLOWER && cnt > 0 && cnt <= FS && prop_raw == 0;
  L.dirty = 0;
  L.nev = 0;
  // (without X, loading the state beside meta, as k_apply_fast does, measured
  // neutral on cfg3 and +4.5 % on cfg4, whose lanes are mostly not leaders)
  // (a busy leader with a higher-term message — the route's CNT_HIGHER — is
  // handed over without reading its slots or its state)
  const bool busy_hi = leader && !nc && fits && !spec && (craw & CNT_HIGHER) != 0;
  const bool slots = (leader && !nc && fits && !busy_hi) || fol;
  if constexpr (SR > 0) {
#pragma unroll
    for (uint32_t k = 0; k < SR; ++k)
      if (slots && k < cnt) l_slot[k][tid] = at32(a.slot, k * a.S.G + g);
  }
  if constexpr (X) {
#pragma unroll
    for (uint32_t k = 0; k < FS; ++k)
      if (fol && k < cnt) l_lane[k][tid] = at32(a.slotx, k * a.S.G + g);
  }
  if (spec) L.load(X);
  if (fol) L.load_follow();  // (a follower reads no Progress)
  bool loaded = spec, higher = busy_hi;
  if (slots && !spec && !fol) {  // a busy leader without a proposal and no higher term: load it
    L.load(X);
    loaded = true;
  }
  // the slots' arrival indices, only for a group this kernel steps (an election
  // storm's leaders go to k_elect without them)
  uint32_t key[KS];
  const bool keys = (slots && loaded) || fol;
#pragma unroll
  for (uint32_t k = 0; k < KS; ++k) key[k] = (!HB_ROUTE_SORTED && keys && k < cnt) ? slot_at(k).y : 0xFFFFFFFFu;
  // arrival order of the slots (slot numbers as nibbles)
  uint32_t perm = 0;
  if (HB_ROUTE_SORTED) {
#pragma unroll
    for (uint32_t k = 0; k < KS; ++k) perm |= k << (4 * k);
  } else {
    perm = arrival_perm<KS>(key);
  }
  const uint64_t last0 = L.last, commit0 = L.committed;
  bool flagged = false;
  uint32_t resume = 0;
  uint32_t st_msgs = 0, st_app = 0, st_vote = 0, st_drop = 0;

  // ---- the dense proposal: the partition's P chunk (fixed slot), before any message event
  const uint64_t poff = (uint64_t)part * PART * a.ev_per_msg;
  if (tid == 0) a.ev_off[2 * part] = poff;
  L.E.chunk = a.ev + poff;
  L.E.fill = &l_pfill;
  const uint32_t prop_k = live ? prop_raw : 0u;
  if (prop_k) {
    if (loaded && L.prop_ok(prop_k)) {
      L.arrival = 0xFFFFFFFFu;
      L.prop(prop_k);
    } else {
      flagged = true;
      resume = 1u << 31;  // the proposal itself is pending (stepped by k_apply into the M chunk)
    }
  }
  // ---- the slot messages in arrival order (M chunk reserved by k_route)
  L.E.chunk = a.ev + a.ev_off[2 * part + 1];
  L.E.fill = &l_fill;
  bool fstepped = false;  // FollowLane stepped a message: its state is stored
  if (X && fol) {
#pragma nounroll
    for (uint32_t x = 0; x < cnt; ++x) {
      if (L.faulted()) break;
      const uint32_t ks = (perm >> (4 * x)) & 0xF;
      uint32_t inf, morig;
      uint64_t mterm, mindex;
      slot_unpack(slot_at(ks), a.side, &inf, &morig, &mterm, &mindex);
      const uint4 ext = l_lane[ks < FS ? ks : 0][(LDS || X) ? tid : 0];
      const uint64_t lt = (uint64_t)ext.x | ((uint64_t)ext.y << 32), mc = (uint64_t)ext.z | ((uint64_t)ext.w << 32);
      const uint32_t from = (inf >> 4) & 0xF;
      if (!L.takes_follow(inf, from, mterm, mindex, lt, mc)) {
        flagged = true;
        resume = x;
        break;
      }
      L.arrival = morig;
      L.step_follow(inf, from, mterm, mindex, lt, mc);
      fstepped = true;
      st_msgs++;
    }
  } else if (live && cnt > 0 && !flagged && !L.faulted()) {
    if (!loaded || !fits) {  // all to k_apply (or k_elect)
      flagged = true;
      resume = 0;
    } else {
      uint32_t x = 0;
      uint4 nx = slot_at(perm & 0xF);  // (sorted slots: the next one's load runs ahead of this step)
#pragma nounroll
      for (; x < cnt; ++x) {
        if (L.faulted()) break;
        uint32_t inf, morig;
        uint64_t mterm, mindex;
        const uint4 cur = nx;
        if (x + 1 < cnt) nx = slot_at((perm >> (4 * (x + 1))) & 0xF);
        slot_unpack(cur, a.side, &inf, &morig, &mterm, &mindex);
        const uint32_t type = inf & 0xF, from = (inf >> 4) & 0xF;
        const bool reject = (inf >> 8) & 1u;
        if (from >= L.n() && is_response(type)) {  // raft/multinode.go:235
          st_drop++;
          continue;
        }
        if (!L.takes(type, from, mterm)) {
          flagged = true;
          resume = x;
          higher = mterm > L.term;
          break;
        }
        L.arrival = morig;
        L.step(type, from, mterm, mindex, reject,
               (reject && type == HB_MSG_APP_RESP && a.hint) ? a.hint[morig] : 0ull);
        st_msgs++;
        st_app += type == HB_MSG_APP_RESP;
        st_vote += type == HB_MSG_VOTE_RESP;
      }
    }
  }
  if (loaded) L.store();
  if (fstepped) L.store_follow();
  const bool stored = loaded || fstepped;
  // k_elect's candidates (n >= 5): no leader, or a leader a higher term steps down
  if constexpr (NMAX >= 5) flag_put<true>(l_eflag, tid, flagged && (!leader || higher));
  flag_put<true>(l_flag, tid, flagged);
  if (flagged) {
    a.resume[g] = resume | (stored ? 0u : 1u << 30);
    if (stored) a.commit0[g] = commit0;
  }
  const uint32_t vals[ST_N + 1] = {st_msgs,
                                   st_app,
                                   st_vote,
                                   st_drop,
                                   (uint32_t)(!flagged && L.committed != commit0),
                                   0,
                                   0,
                                   (uint32_t)(L.faulted() != 0 && live),
                                   (uint32_t)(L.last - last0),
                                   L.nev};
  reduce_stats(a, l_stats, vals);
  if (tid < FLAG_WORDS) {
    a.pflag[(size_t)part * FLAG_WORDS + tid] = l_flag[tid];
    if (NMAX >= 5) a.eflag[(size_t)part * FLAG_WORDS + tid] = l_eflag[tid];
  }
  if (tid == 0) fast_close(a, part, l_flag, NMAX >= 5 ? l_eflag : nullptr, l_pfill, l_fill);
}

// k_follow: the follower-capable lane (Lane<NMAX, true>) for the groups
// k_apply handed on at a follower-side message, over k_apply's work list (its
// registers and code stay out of k_apply, the hot general kernel of cfg3 /
// cfg4).  Its last workgroup out runs the step's finish: the statistics are
// agent-scope atomics, performed at the memory side, so each workgroup waits
// for its own (vmcnt(0)) before taking a ticket, and the last reads the shards
// with agent-scope loads.
template <int NMAX>
__global__ void __launch_bounds__(PART, HB_GEN_WAVES) k_follow(ApplyArgs a) {
  __shared__ GenShared sh;
  __shared__ uint32_t l_last;
  const uint32_t nl = __hip_atomic_load(a.fl_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    (void)apply_part<NMAX, true>(a, a.fl_list[i], sh, false);
    __syncthreads();
  }
  finish_by_ticket(a, blockIdx.x < nl, nl < gridDim.x ? nl : gridDim.x, &l_last);
}

// ---------------------------------------------------------------------------
// k_tick: one MultiNode.Tick (raft/multinode.go:264-275) — every live group
// runs tickHeartbeat (leader) or tickElection (raft/raft.go:362-382), the
// draw of isElectionTimeout (:765-771) read from the node's r.rand stream at
// the group's own position; a leader's due MsgBeat sends its heartbeats from
// Match / pm alone, a due MsgHup is stepped at once by the general state
// machine.  Events go to the partition's P chunk (at most one
// step per group, so the chunk's ev_per_msg x PART words bound them).
// ---------------------------------------------------------------------------
#ifndef HB_TICK_ELECT
#define HB_TICK_ELECT 1  // a tick's campaigns through ElectLane (reset form, M_RS)
#endif
template <int NMAX>
__global__ void __launch_bounds__(PART, 2) k_tick(ApplyArgs a) {
  __shared__ uint32_t l_fill;
  __shared__ uint64_t l_stats[ST_N + 1];
  const uint32_t part = block_part(a.sis_log);
  if (part >= a.NB) return;  // uniform: grid padding
  const uint32_t tid = threadIdx.x;
  const uint32_t g = part * PART + tid;
  if (tid == 0) l_fill = 0;
  if (tid <= ST_N) l_stats[tid] = 0;
  __syncthreads();

  const uint64_t poff = (uint64_t)part * PART * a.ev_per_msg;
  Lane<NMAX> L;
  L.S = a.S;
  L.E.chunk = a.ev + poff;
  L.E.fill = &l_fill;
  L.g = g;
  L.won = 0;
  L.lost = 0;
  L.nev = 0;
  L.dirty = 0;
  L.meta = 0;
  L.last = 0;
  L.committed = 0;
  L.arrival = 0xFFFFFFFFu;
  uint32_t type = 0xFF;
  bool live = false;
  // meta's low word (state, n, self, flags) decides a tick; the high word (the
  // vote tally) is read only by a group that steps or faults (4 B per group)
  const uint32_t* meta32 = reinterpret_cast<const uint32_t*>(a.S.meta);
  auto meta_hi = [&]() { L.meta |= (uint64_t)at32(meta32, 2 * g + 1) << 32; };
  if (g < a.S.G) {
    L.meta = at32(meta32, 2 * g);
    live = L.n() != 0 && !L.faulted();
  }
  if (live) {
    const uint32_t cfg = a.S.tcfg[g];
    const uint32_t et = cfg & 0xFFFFu, ht = cfg >> 16;
    uint32_t el = a.S.elapsed[g];
    if (L.state() == HB_STATE_LEADER) {  // tickHeartbeat
      if (++el >= ht) {
        el = 0;
        type = HB_MSG_BEAT;
      }
    } else if (L.self() == HB_SLOT_NONE) {  // tickElection: !promotable()
      el = 0;
    } else if (++el >= et) {  // isElectionTimeout: d = elapsed - et >= 0 takes a draw
      const uint32_t pos = a.S.rpos[g];
      if (pos >= a.S.nrnd) {
        meta_hi();
        L.fault(HB_FAULT_RAND_EXHAUSTED);
        L.dirty |= D_META;
        L.ev(HB_EV_FAULT, 0, HB_FAULT_RAND_EXHAUSTED, HB_NO_INDEX);
      } else {
        a.S.rpos[g] = pos + 1;
        if ((uint64_t)(el - et) > a.S.rnd[pos] % et) {
          el = 0;
          type = HB_MSG_HUP;
        }
      }
    }
    a.S.elapsed[g] = el;
  }
  uint64_t last0 = 0, commit0 = 0;
  if (type == HB_MSG_BEAT && !(L.meta & (M_RS | M_NC))) {
    // stepLeader MsgBeat -> bcastHeartbeat (raft/raft.go:495-498, :290-300):
    // a MsgHeartbeat to every peer in slot order at min(Match, committed), each
    // Progress resumed.  Only those fields are read and only a cleared pause bit
    // is written (Lane::step would load the whole group, ring heads included,
    // and write every peer's Progress back unchanged).  The self slot, whose
    // arrays may be stale under M_SM, is skipped.
    const uint64_t committed = a.S.commit[g];
    const uint32_t nn = L.n(), sf = L.self();
    uint64_t mt[NMAX];
    uint32_t pmv[NMAX];
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      const bool on = (uint32_t)s < nn && (uint32_t)s != sf;
      mt[s] = on ? a.S.match[(size_t)s * a.S.G + g] : 0ull;
      pmv[s] = on ? a.S.pm[(size_t)s * a.S.G + g] : 0u;
    }
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      if ((uint32_t)s >= nn || (uint32_t)s == sf) continue;
      L.ev(HB_EV_HEARTBEAT, s, 0, umin64(mt[s], committed));
      if (pmv[s] & PM_PAUSED) a.S.pm[(size_t)s * a.S.G + g] = pmv[s] & ~PM_PAUSED;
    }
  } else if (type == HB_MSG_HUP && HB_TICK_ELECT && !sz_on(a.S.max_msg_size) && !(L.meta & M_NC) &&
             L.self() < L.n()) {
    // a non-leader's election timeout: campaign through the election lane
    // (hipbatch_elect.h, as k_elect steps it), which leaves the n Progress
    // entries in the reset form (M_RS) instead of writing them — ~4 % of the
    // groups campaign per tick, each writing n x 20 scattered bytes through
    // the general lane (the tick's 2.3 x traffic over its byte model, r05)
    meta_hi();
    ElectLane<NMAX> E;
    E.S = a.S;
    E.E = L.E;
    E.g = g;
    E.meta = L.meta;
    E.load();
    last0 = E.last;
    commit0 = E.committed;
    E.step(HB_MSG_HUP, L.self(), 0, false);
    E.store();
    L.meta = E.meta;
    L.last = E.last;
    L.committed = E.committed;
    L.won = E.won;
    L.lost = E.lost;
    L.nev = E.nev;
    L.dirty = 0;  // (stored)
  } else if (type != 0xFF) {  // MsgHup (or the MsgBeat of a reset-form / M_NC leader): the general state machine
    meta_hi();
    L.load_all();
    last0 = L.last;
    commit0 = L.committed;
    L.step(type, L.self(), 0, 0, false, 0);
  }
  if (live && L.dirty) {
    if (type == 0xFF) L.S.meta[g] = L.meta;  // the fault only
    else L.store();
  }
  const bool stepped = type != 0xFF;
  const uint64_t vals[ST_N + 1] = {(uint64_t)stepped,
                                   0,
                                   0,
                                   0,
                                   (uint64_t)(stepped && L.committed != commit0),
                                   L.won,
                                   L.lost,
                                   (uint64_t)(live && L.faulted() != 0),
                                   stepped ? L.last - last0 : 0ull,
                                   L.nev};
  reduce_stats(a, l_stats, vals);
  if (tid == 0) {
    a.ev_off[2 * part] = poff;
    a.ev_off[2 * part + 1] = poff;
    a.ev_counts[2 * part] = l_fill;
    a.ev_counts[2 * part + 1] = 0;
  }
}

// ---------------------------------------------------------------------------
// k_decode: wire ingestion (hb_decode).  One lane per record: Message.Unmarshal
// (hipbatch_wire.h), multiNode.Step's local-message filter (raft/multinode.go:
// 432-439), m.From -> slot through the group's peer ids, one batch record out.
// ---------------------------------------------------------------------------
struct DecodeArgs {
  const uint8_t* bytes;
  const uint64_t* off;
  const uint32_t* len;
  const uint32_t* group;
  uint64_t n;
  const uint64_t* meta;
  const uint4* peer;  // [G] rows of HB_PEER_ROW node ids (64 B), or null
  uint32_t G, nmax;
  uint32_t* o_group;
  uint32_t* o_info;
  uint64_t* o_term;
  uint64_t* o_index;
  uint64_t* o_hint;
  uint8_t* status;
};

constexpr uint32_t HB_PEER_ROW = 8;  // u64 per group peer row: node ids of slots 0..6, then n

// Outcome of one record -> batch record + status (shared by both passes).
__device__ __forceinline__ void dec_emit(const DecodeArgs& a, uint64_t k, int rc, const WireMsg& m, uint32_t g, bool gok,
                                         const uint64_t* ids) {
  uint32_t st;
  if (rc == W_ERR) st = HB_WIRE_ERROR;
  else if (rc == W_PANIC) st = HB_WIRE_PANIC;
  else if (rc == W_DEEP) st = HB_WIRE_HOST;
  else if (m.type == HB_MSG_HUP || m.type == HB_MSG_BEAT || m.type == HB_MSG_UNREACHABLE ||
           m.type == HB_MSG_SNAP_STATUS)
    st = HB_WIRE_LOCAL;  // IsLocalMsg raft/util.go:49-51
  else if (m.type != HB_MSG_APP_RESP && m.type != HB_MSG_VOTE_RESP && m.type != HB_MSG_HEARTBEAT_RESP)
    st = HB_WIRE_HOST;
  else if (!gok) st = HB_WIRE_BADGROUP;
  else st = HB_WIRE_OK;
  uint32_t slot = HB_SLOT_NONE;
  if (st == HB_WIRE_OK && a.peer && m.from != 0) {
    const uint32_t nn = (uint32_t)ids[HB_PEER_ROW - 1];
#pragma unroll
    for (uint32_t s = 0; s < HB_MAX_REPLICAS; ++s)
      if (s < nn && slot == HB_SLOT_NONE && ids[s] == m.from) slot = s;
  }
  const bool ok = st == HB_WIRE_OK;
  a.o_group[k] = ok ? g : 0xFFFFFFFFu;
  a.o_info[k] = ok ? ((uint32_t)m.type | (slot << 4) | ((uint32_t)m.reject << 8)) : 0u;
  a.o_term[k] = ok ? m.term : 0ull;
  a.o_index[k] = ok ? m.index : 0ull;
  a.o_hint[k] = ok ? m.hint : 0ull;
  a.status[k] = (uint8_t)st;
}

// Pass 1 (k_decode): a wave's 64 records are contiguous in the usual layout,
// so the wave copies their span into its own LDS window with coalesced
// 16-byte loads (bytes at the unaligned ends one by one, so nothing outside
// the span is read) and each lane runs the straight-line MarshalTo-shape
// parser (w_fast_message) from LDS.  A record of any other shape (or a wave
// whose span does not fit the window) is queued for pass 2, k_decode_general,
// which runs the full Message.Unmarshal restatement over the queue only: its
// register and scratch footprint never limits the occupancy of pass 1.
constexpr uint32_t DEC_THREADS = 256;
constexpr uint32_t DEC_WIN = 4096;  // bytes of records staged per wave
constexpr uint32_t DEC_GEN_BLOCKS = 128;  // pass 2 is the exception path; scratch-heavy waves are costly to launch
__global__ void __launch_bounds__(DEC_THREADS) k_decode(DecodeArgs a, uint32_t* q, uint32_t* qn) {
  __shared__ uint4 l_win[DEC_THREADS / 64][DEC_WIN / 16 + 2];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t k = (uint64_t)blockIdx.x * DEC_THREADS + threadIdx.x;
  const bool live = k < a.n;
  const uint64_t o = live ? a.off[k] : 0ull;
  const uint32_t len = live ? a.len[k] : 0u;
  uint64_t lo = live ? o : ~0ull, hi = live ? o + len : 0ull;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t l2 = __shfl_xor(lo, d), h2 = __shfl_xor(hi, d);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
  }
  const bool fits = hi > lo && hi - lo <= DEC_WIN;  // uniform in the wave
  uint8_t* win = reinterpret_cast<uint8_t*>(&l_win[wave][0]);
  const uintptr_t A = reinterpret_cast<uintptr_t>(a.bytes) + lo, B = reinterpret_cast<uintptr_t>(a.bytes) + hi;
  const uintptr_t base = A & ~(uintptr_t)15;
  if (fits) {
    const uintptr_t A16 = (A + 15) & ~(uintptr_t)15, B16 = B & ~(uintptr_t)15;
    if (A16 < B16) {
      const uint32_t nc = (uint32_t)((B16 - A16) >> 4), c0 = (uint32_t)((A16 - base) >> 4);
      for (uint32_t c = lane; c < nc; c += 64) l_win[wave][c0 + c] = reinterpret_cast<const uint4*>(A16)[c];
      for (uintptr_t x = A + lane; x < A16; x += 64) win[x - base] = *reinterpret_cast<const uint8_t*>(x);
      for (uintptr_t x = B16 + lane; x < B; x += 64) win[x - base] = *reinterpret_cast<const uint8_t*>(x);
    } else {
      for (uintptr_t x = A + lane; x < B; x += 64) win[x - base] = *reinterpret_cast<const uint8_t*>(x);
    }
  }
  __syncthreads();
  if (!live) return;
  // the group's peer row and meta are random gathers: issue them before the
  // parse so their latency hides behind it
  const uint32_t g = a.group[k];
  const bool gok = g < a.G;
  uint4 prow[4] = {};
  if (gok && a.peer) {
#pragma unroll
    for (int j = 0; j < 4; ++j) prow[j] = a.peer[(size_t)g * 4 + j];
  }
  WireMsg m;
  const bool fast = fits && w_fast_message(win + (reinterpret_cast<uintptr_t>(a.bytes) + o - base), (int64_t)len, &m);
  // wave-aggregated append of the other records to the pass-2 queue
  const uint64_t slow = __ballot(!fast);
  if (slow) {
    const uint32_t cnt = (uint32_t)__popcll(slow);
    const uint32_t leader = (uint32_t)__ffsll((long long)slow) - 1;
    uint32_t b0 = 0;
    if (lane == leader) b0 = atomicAdd(qn, cnt);
    b0 = __shfl(b0, (int)leader);
    if (!fast) q[b0 + (uint32_t)__popcll(slow & ((1ull << lane) - 1))] = (uint32_t)k;
  }
  if (!fast) return;
  dec_emit(a, k, W_OK, m, g, gok, reinterpret_cast<const uint64_t*>(prow));
}

// row[7] of a group's peer row = its replica count n (from meta), so the
// From -> slot lookup reads one 64-byte row and no meta.  Refreshed whenever
// either side (hb_load_groups / hb_load_peers) changes.
__global__ void k_peer_n(uint64_t* peer, const uint64_t* meta, uint32_t first, uint32_t count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) peer[(size_t)(first + i) * HB_PEER_ROW + HB_PEER_ROW - 1] = m_n(meta[first + i]);
}

// Pass 2: Message.Unmarshal (hipbatch_wire.h) for the queued records, read
// from global memory.  Grid-stride over the queue length written by pass 1;
// the last workgroup to finish clears the queue for the next hb_decode.
__global__ void __launch_bounds__(DEC_THREADS) k_decode_general(DecodeArgs a, const uint32_t* q, uint32_t* qn) {
  const uint32_t total = *(volatile uint32_t*)qn;
  for (uint32_t j = blockIdx.x * DEC_THREADS + threadIdx.x; j < total; j += gridDim.x * DEC_THREADS) {
    const uint64_t k = q[j];
    const uint32_t g = a.group[k];
    const bool gok = g < a.G;
    uint64_t ids[HB_PEER_ROW] = {};
    if (gok && a.peer) {
      const uint64_t* row = reinterpret_cast<const uint64_t*>(a.peer) + (size_t)g * HB_PEER_ROW;
#pragma unroll
      for (uint32_t s = 0; s < HB_PEER_ROW; ++s) ids[s] = row[s];
    }
    WireMsg m;
    const int rc = w_unmarshal_message(a.bytes + a.off[k], (int64_t)a.len[k], &m);
    dec_emit(a, k, rc, m, g, gok, ids);
  }
  // qn[1] counts finished workgroups; the last one resets both words
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(qn + 1, 1u) == gridDim.x - 1) {
      qn[0] = 0;
      qn[1] = 0;
      __threadfence();
    }
  }
}

// ============================================================================
// Phase 3: finish
// ============================================================================
__global__ void __launch_bounds__(128) k_finish(uint64_t* shard, uint64_t* stats, uint64_t* accum) {
  const int map[ST_N + 1] = {HB_STAT_MSGS,  HB_STAT_APPRESP, HB_STAT_VOTERESP, HB_STAT_DROPPED, HB_STAT_COMMITS,
                             HB_STAT_WON,   HB_STAT_LOST,    HB_STAT_FAULTS,   HB_STAT_ENTRIES, HB_STAT_EVENTS};
  const uint32_t t = threadIdx.x, k = t / NSH;
  uint64_t v = 0;
  if (k <= ST_N) {
    v = shard[shard_at(k, t % NSH)];
    shard[shard_at(k, t % NSH)] = 0;  // ready for the next step
  }
#pragma unroll
  for (uint32_t d = 1; d < NSH; d <<= 1) v += __shfl_xor(v, d);
  if (k <= ST_N && t % NSH == 0) {
    stats[map[k]] = v;
    if (accum) accum[map[k]] += v;
  }
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
  uint64_t m = meta_make(r.state, r.n, r.self_slot, r.lead, r.vote, r.fault, r.votes_resp, r.votes_grant);
  if (r.term_last == r.last_index) m |= M_TL;
  if (r.self_slot < r.n && r.pr[r.self_slot].match == r.last_index && r.pr[r.self_slot].next == r.last_index + 1)
    m |= M_SM;
  if (r.commit_zero && r.committed != 0) m |= M_NC;  // r.Commit = 0 until the group's first Step
  S.meta[g] = m;
  S.elapsed[g] = 0;  // newRaft: fresh r.rand, becomeFollower -> reset
  S.rpos[g] = 0;
  if (S.szx) {  // finite max_msg_size: no entry sizes yet (hb_load_entry_sizes)
    S.szlo[g] = r.last_index;
    *cum_at(S.szx[g], r.last_index) = 0;
  }
  S.trc[g] = 0;  // no older term runs yet (hb_load_term_runs)
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
  r.term_last = (m & M_TL) ? r.last_index : S.tlast[g];
  r.snap_index = S.snap[g];
  r.state = m_state(m);
  r.n = m_n(m);
  r.self_slot = m_self(m);
  r.lead = m_lead(m);
  r.vote = m_vote(m);
  r.fault = m_fault(m);
  r.votes_resp = m_resp(m);
  r.votes_grant = m_grant(m);
  r.commit_zero = (m & M_NC) ? 1u : 0u;
  for (uint32_t s = 0; s < S.nmax && s < r.n; ++s) {
    const size_t o = (size_t)s * S.G + g;
    uint32_t p = S.pm[o];
    const bool kept = !((m & M_SM) && s == r.self_slot);  // M_SM: materialized from last
    r.pr[s].match = kept ? S.match[o] : r.last_index;
    r.pr[s].next = kept ? S.next[o] : r.last_index + 1;
    if (m & M_RS) rs_progress(m, s, r.last_index, r.term_first, &r.pr[s].match, &r.pr[s].next, &p);
    r.pr[s].state = pm_state(p);
    r.pr[s].paused = pm_paused(p);
    r.pr[s].ins_start = pm_start(p);
    r.pr[s].ins_count = pm_count(p);
    r.pr[s].pending_snapshot = pm_state(p) == HB_PR_SNAPSHOT ? S.pending[o] : 0;
  }
  dst[i] = r;
}

__global__ void k_set_bounds(DevState S, uint32_t count, const uint32_t* groups, const uint64_t* first,
                             const uint64_t* snap) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t g = groups[i];
  S.first[g] = first[i];
  S.snap[g] = snap[i];
}

// hb_load_term_runs: group groups[i] takes runs (start, term) off[i] .. + n_i
__global__ void k_load_runs(DevState S, uint32_t count, const uint32_t* groups, const uint32_t* n_runs,
                            const uint64_t* off, const uint64_t* runs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t g = groups[i], k = n_runs[i];
  uint64_t* R = lx_base(S.trx[g]);  // the host reserved >= k runs
  for (uint32_t j = 0; j < k; ++j) {
    R[2 * j] = runs[2 * (off[i] + j)];
    R[2 * j + 1] = runs[2 * (off[i] + j) + 1];
  }
  S.trc[g] = k;  // count k, head 0
}

// hb_load_entry_sizes: group groups[i] takes the sizes of its entries
// (last - n_i, last], concatenated at sizes + off[i]
__global__ void k_load_sizes(DevState S, uint32_t count, const uint32_t* groups, const uint32_t* n_sizes,
                             const uint64_t* off, const uint32_t* sizes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t g = groups[i], k = n_sizes[i];
  const uint64_t last = S.last[g], lo = last - k, x = S.szx[g];  // the host reserved > k entries
  const uint32_t* z = sizes + off[i];
  uint64_t acc = 0;
  *cum_at(x, lo) = 0;
  for (uint32_t j = 1; j <= k; ++j) {
    acc += z[j - 1];
    *cum_at(x, lo + j) = acc;
  }
  S.szlo[g] = lo;
}

// hb_reserve_log: move job i's ring to a larger extent, keeping its content.
// A job is 4 words: group | kind << 32 (0 sizes, 1 runs), old extent word, new extent word, unused.
__global__ void k_regrow(DevState S, uint32_t count, const uint64_t* jobs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint64_t* j = jobs + 4 * (size_t)i;
  const uint32_t g = (uint32_t)j[0], kind = (uint32_t)(j[0] >> 32);
  const uint64_t ox = j[1], nx = j[2];
  if (kind == 0) {  // cum(i) for i in [szlo, last]: same index, new mask
    const uint64_t lo = S.szlo[g], last = S.last[g];
    for (uint64_t k = lo; k <= last; ++k) *cum_at(nx, k) = *cum_at(ox, k);
    S.szx[g] = nx;
  } else {  // runs in ring order, to the front of the new ring (head 0)
    const uint64_t c = S.trc[g];
    const uint32_t n = (uint32_t)c, h = (uint32_t)(c >> 32);
    const uint64_t om = lx_cap(ox) - 1;
    const uint64_t* O = lx_base(ox);
    uint64_t* N = lx_base(nx);
    for (uint32_t k = 0; k < n; ++k) {
      const uint64_t o = 2 * ((h + k) & om);
      N[2 * k] = O[o];
      N[2 * k + 1] = O[o + 1];
    }
    S.trx[g] = nx;
    S.trc[g] = n;
  }
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
    const uint64_t m = S.meta[g];
    if (m & M_RS) {  // the reset form written out first: this slot's window changes alone
      for (uint32_t k = 0; k < m_n(m); ++k) {
        const size_t ok = (size_t)k * S.G + g;
        uint64_t mt, nx;
        uint32_t pk;
        rs_progress(m, k, S.last[g], S.tfirst[g], &mt, &nx, &pk);
        if (!((m & M_SM) && k == m_self(m))) {
          S.match[ok] = mt;
          S.next[ok] = nx;
        }
        S.pm[ok] = pk;
      }
      S.meta[g] = m & ~M_RS;
    }
    const size_t o = (size_t)s * S.G + g;
    const uint32_t p = S.pm[o];
    S.pm[o] = pm_make(pm_state(p), pm_paused(p), start, count);
  }
}

__global__ void k_get_ins(DevState S, uint32_t g, uint32_t s, uint64_t* vals, uint32_t* sc) {
  const size_t o = (size_t)s * S.G + g;
  const uint32_t p = (S.meta[g] & M_RS) ? 0u : S.pm[o];  // the reset form: an empty window
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

// Dense gather of the chunked events: chunk c (counts[c] compact words at
// base + offs[c]; chunk 2p / 2p+1 = partition p's P / M chunk) is expanded
// into public hb_event records at out + dst[c], dst = exclusive scan of the
// per-chunk event counts.
__device__ __forceinline__ uint32_t evc_outputs(uint64_t w) {
  const uint32_t t = (uint32_t)w & 0xF;
  if (t == EVC_CONT) return 0;
  if (t == EVC_BCAST || t == EVC_VBCAST) return __popc((uint32_t)(w >> 4) & 0x7F);
  return 1;
}
__global__ void __launch_bounds__(256) k_chunk_events(const uint64_t* base, const uint32_t* counts,
                                                      const uint64_t* offs, uint32_t* out_counts) {
  __shared__ uint32_t sh16[16];
  const uint32_t c = blockIdx.x, n = counts[c];
  const uint64_t* src = base + offs[c];
  uint32_t k = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) k += evc_outputs(src[i]);
  uint32_t tot;
  (void)block_excl_scan(k, sh16, &tot);
  if (threadIdx.x == 0) out_counts[c] = tot;
}
__global__ void __launch_bounds__(1024) k_scan_counts(const uint32_t* counts, uint32_t n, uint64_t* dst) {
  __shared__ uint32_t sh16[16];
  const uint32_t per = (n + 1023) / 1024, b0 = threadIdx.x * per;
  uint64_t sum = 0;
  for (uint32_t i = b0; i < b0 + per && i < n; ++i) sum += counts[i];
  uint32_t tot;
  uint64_t run = block_excl_scan((uint32_t)sum, sh16, &tot);  // total events < 2^32
  for (uint32_t i = b0; i < b0 + per && i < n; ++i) {
    dst[i] = run;
    run += counts[i];
  }
}
__global__ void __launch_bounds__(256) k_expand_events(const uint64_t* base, const uint32_t* counts,
                                                       const uint64_t* offs, const uint64_t* dst, hb_event* out) {
  __shared__ uint32_t sh16[16];
  const uint32_t c = blockIdx.x, n = counts[c], part = c >> 1;
  const uint64_t* src = base + offs[c];
  uint64_t run = dst[c];
  for (uint32_t t0 = 0; t0 < n; t0 += blockDim.x) {
    const uint32_t i = t0 + threadIdx.x;
    const uint64_t w = i < n ? src[i] : (uint64_t)EVC_CONT;
    const uint32_t k = evc_outputs(w);
    uint32_t tot;
    const uint32_t ex = block_excl_scan(k, sh16, &tot);
    if (k) {
      const uint32_t type = (uint32_t)w & 0xF, to = (uint32_t)(w >> 4) & 0x7F, aux = (uint32_t)(w >> 12) & 0xF;
      const uint32_t group = part * PART + ((uint32_t)(w >> 16) & 0xFF);
      uint64_t x = w >> 24;
      if ((w >> 11) & 1u) x |= (src[i + 1] >> 4) << 40;
      hb_event* o = out + run + ex;
      if (type == EVC_BCAST || type == EVC_VBCAST) {
        const uint8_t et = type == EVC_BCAST ? (uint8_t)HB_EV_APP : (uint8_t)HB_EV_VOTE;
        uint32_t m = to, r = 0;
        while (m) {
          const uint32_t s = __ffs(m) - 1;
          m &= m - 1;
          o[r++] = hb_event{x, group, et, (uint8_t)s, (uint16_t)aux};
        }
      } else {
        o[0] = hb_event{x, group, (uint8_t)type, (uint8_t)to, (uint16_t)aux};
      }
    }
    run += tot;
  }
}

// The compact delta to the host (hb_events_to_host): the words themselves,
// densely in chunk order, plus the words per chunk and their total.  Host
// destinations are pinned memory the kernels write through (posted PCIe writes,
// one coalesced 512-byte run per wave), so the copy is sized on the device.
__global__ void __launch_bounds__(1024) k_scan_words(const uint32_t* counts, uint32_t n, uint64_t* dst,
                                                     uint32_t* h_counts, uint64_t* h_total) {
  __shared__ uint32_t sh16[16];
  const uint32_t per = (n + 1023) / 1024, b0 = threadIdx.x * per;
  uint64_t sum = 0;
  for (uint32_t i = b0; i < b0 + per && i < n; ++i) sum += counts[i];
  uint32_t tot;
  uint64_t run = block_excl_scan((uint32_t)sum, sh16, &tot);  // total words < 2^32
  for (uint32_t i = b0; i < b0 + per && i < n; ++i) {
    dst[i] = run;
    run += counts[i];
  }
  for (uint32_t i = threadIdx.x; i < n; i += 1024) h_counts[i] = counts[i];
  if (threadIdx.x == 0) {
    dst[n] = tot;
    *h_total = tot;
  }
}
__global__ void __launch_bounds__(256) k_gather_words(const uint64_t* base, const uint32_t* counts,
                                                      const uint64_t* offs, const uint64_t* dst, uint64_t* out,
                                                      uint64_t cap) {
  const uint32_t c = blockIdx.x, n = counts[c];
  if (dst[gridDim.x] > cap) return;  // the caller's buffer is too small: counts and total only
  const uint64_t* src = base + offs[c];
  uint64_t* o = out + dst[c];
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) o[i] = src[i];
}

// Both in one workgroup when the chunks are few (a small node: 2 chunks per
// 256 groups): chunk offsets scanned in LDS, then a wave per chunk copies.
constexpr uint32_t WORDS_SMALL = 1024;
__global__ void __launch_bounds__(1024) k_words_small(const uint32_t* counts, uint32_t n, const uint64_t* base,
                                                      const uint64_t* offs, uint64_t* out, uint64_t cap,
                                                      uint32_t* h_counts, uint64_t* h_total) {
  __shared__ uint32_t sh16[16];
  __shared__ uint64_t s_dst[WORDS_SMALL];
  const uint32_t tid = threadIdx.x;
  const uint32_t c = tid < n ? counts[tid] : 0u;
  uint32_t tot;
  const uint32_t run = block_excl_scan(c, sh16, &tot);  // total words < 2^32
  if (tid < n) {
    s_dst[tid] = run;
    h_counts[tid] = c;
  }
  if (tid == 0) *h_total = tot;
  __syncthreads();
  if (tot > cap) return;  // the caller's buffer is too small: counts and total only
  const uint32_t wave = tid >> 6, lane = tid & 63;
  for (uint32_t k = wave; k < n; k += 16) {
    const uint32_t m = counts[k];
    const uint64_t* src = base + offs[k];
    uint64_t* o = out + s_dst[k];
    for (uint32_t i = lane; i < m; i += 64) o[i] = src[i];
  }
}

// ============================================================================
// host side
// ============================================================================
// What one step's prep (partition + route) hands to its apply.  Two sets, so
// the prep of batch k+1 (on the prep stream) can run while batch k applies.
struct PrepSet {
  MsgRec* rec = nullptr;          // final pass = apply input
  uint8_t* key = nullptr;         // partition-in-bucket per record (+ SEG bytes of padding)
  uint32_t* bucket = nullptr;     // bucket id per record (multi-pass only)
  uint32_t* bk_off = nullptr;     // [NBK + 1]
  uint32_t* bk_fill = nullptr;    // [NBK] event words reserved in each bucket's region (k_route)
  uint32_t* ctr = nullptr;        // [CTR_WORDS] work-list counters + finish ticket (cleared by this set's prep)
  uint8_t* cnt = nullptr;         // [G]
  uint8_t* dstage = nullptr;      // device copy of the packed host batch (grown on demand)
  uint64_t dstage_cap = 0;
  uint4* slot = nullptr;          // [route_kmax][G]
  uint64_t* side = nullptr;       // [2 max_batch] long records' (term, index)
  uint4* recx = nullptr;          // X mode: [max_batch] beside rec
  uint4* slotx = nullptr;         // X mode: [route_kmax][G] beside slot
  uint64_t* ev_off = nullptr;     // [2 NB] event chunk offsets (route writes the M chunks)
  uint32_t* ev_counts = nullptr;  // [2 NB]
  hipEvent_t prepped = nullptr;   // prep stream: this set is ready
  hipEvent_t applied = nullptr;   // apply stream: the last apply reading this set is done
  bool used = false;
};

// The log pool: extents of the per-group log index rings (DevState szx / trx),
// power-of-two sizes carved from device slabs, recycled through per-size free
// lists.  Only the host allocates (hb_reserve_log, hb_load_*): the device never
// grows a ring, it relies on the capacity reserved before the step.
struct LogPool {
  std::vector<void*> slabs;
  char* cur = nullptr;
  size_t left = 0;
  std::vector<uint64_t> free_[48];  // by log2(bytes)
  uint64_t bytes_live = 0;
  // an extent of 2^lb bytes (lb >= 7: 128-byte aligned, the extent word's tag bits stay free)
  uint64_t get(uint32_t lb) {
    if (!free_[lb].empty()) {
      const uint64_t a = free_[lb].back();
      free_[lb].pop_back();
      bytes_live += 1ull << lb;
      return a;
    }
    const size_t bytes = 1ull << lb;
    const size_t align = bytes < 4096 ? bytes : 4096;
    size_t pad = (align - (reinterpret_cast<uintptr_t>(cur) & (align - 1))) & (align - 1);
    if (!cur || left < pad + bytes) {
      const size_t slab = std::max<size_t>(bytes, 256ull << 20);
      void* p = nullptr;
      if (hipMalloc(&p, slab) != hipSuccess) return 0;
      slabs.push_back(p);
      cur = static_cast<char*>(p);
      left = slab;
      pad = 0;
    }
    const uint64_t a = reinterpret_cast<uint64_t>(cur + pad);
    cur += pad + bytes;
    left -= pad + bytes;
    bytes_live += bytes;
    return a;
  }
  void put(uint64_t a, uint32_t lb) {
    free_[lb].push_back(a);
    bytes_live -= 1ull << lb;
  }
  void release() {
    for (void* p : slabs) (void)hipFree(p);
    slabs.clear();
  }
};
constexpr uint32_t SZ_LOG_MIN = 4;  // a size ring starts at 16 entries (128 B)
constexpr uint32_t TR_LOG_MIN = 3;  // a run ring at 8 runs (128 B)

struct hb_handle {
  int device = 0;
  hipStream_t stream = nullptr;   // apply stream (hb_set_stream)
  hipStream_t prep = nullptr;     // partition + route (library-owned)
  hipStream_t in_stream = nullptr;  // where the batch inputs are produced (hb_set_input_stream)
  bool in_stream_set = false;
  hipEvent_t in_ready = nullptr;
  uint32_t G = 0, nmax = 0, W = 0, NB = 0;
  uint64_t max_msg_size = 0, max_batch = 0;
  DevState st{};
  std::vector<void*> allocs;
  // the log index (host mirror of DevState szx / trx: extent address | log2 capacity)
  LogPool pool;
  std::vector<uint64_t> h_szx, h_trx;
  uint64_t* lx_jobs = nullptr;     // device scratch of hb_reserve_log's regrow jobs
  uint64_t lx_jobs_cap = 0;
  // partition scratch
  uint32_t* hist = nullptr;       // [tiles][RDX_BINS]
  uint32_t* n_valid = nullptr;    // messages kept after pass 1 (device)
  uint32_t* totals = nullptr;     // [RDX_BINS] digit totals of the current pass
  // one-pass direct offsets (HB_RDX_DIRECT): hist workgroup sums, rotating superblock sums
  uint32_t* hagg = nullptr;       // [hist workgroups][RDX_BINS]
  uint32_t* hsup = nullptr;       // [SUP_BUFS][sup_max][RDX_BINS]
  uint32_t sup_max = 0, sup_k = 0;
  uint32_t sup_used[SUP_BUFS] = {};  // superblocks each buffer holds non-zero (cleared by a later hist)
  RadixDst tmp[2] = {};           // intermediate passes (ping-pong)
  PrepSet set[2];
  uint32_t next_set = 0, cur = 0;  // set of the next / the last step
  uint32_t NBK = 0;               // buckets
  uint32_t sis_log = SIS_LOG_MAX;  // partitions per bucket (log2)
  uint32_t passes = 1;
  // small steps (a few thousand messages, hb_step / hb_events_to_host): one
  // launch for the partition and one for the event words; HB_SMALL_STEP=0
  // turns that off (same output: the A/B and the parity tests compare both)
  bool no_small = false;
  uint32_t kern = 0;  // hb_step_kernels of the last step
  uint32_t fuse = 2;  // k_route_fast: 0 never, 1 one-pass handles, 2 every geometry (HB_ROUTE_FUSE at hb_create)
  uint32_t storm = 2;  // n >= 5: the route's storm hand-over, 2: with the election lane (HB_STORM=0/1/2 at hb_create)
  uint32_t agrid = 0;  // the apply kernels' grid (apply_grid_for)
  uint32_t bk_bits = 1;            // bits of a bucket id
  // host-pointer staging
  uint32_t* s_group = nullptr;
  uint32_t* s_info = nullptr;
  uint32_t* s_props = nullptr;
  uint64_t* s_term = nullptr;
  uint64_t* s_index = nullptr;
  uint64_t* s_hint = nullptr;
  uint64_t* s_eoff = nullptr;     // [max_batch]
  uint64_t* s_commit = nullptr;   // [max_batch]
  uint64_t* s_peoff = nullptr;    // [G] (finite max_msg_size)
  uint32_t* s_edesc = nullptr;    // grown on demand
  uint64_t s_edesc_cap = 0;
  uint64_t* s_eterm = nullptr;    // grown on demand
  uint64_t s_eterm_cap = 0;
  // events
  uint64_t* ev = nullptr;   // compact event words
  uint64_t ev_region = 0;  // records
  uint32_t ev_per_msg = 0;
  uint64_t* stats_shard = nullptr;  // shard_at(value, shard)
  uint64_t* stats_accum = nullptr;  // optional caller buffer (hb_set_stats_accum)
  uint64_t* stats_pin = nullptr;    // [HB_STAT_COUNT] pinned readback (hb_copy_events' count)
  // host-pointer batches up to STAGE_MAX bytes: packed into one pinned block, one H2D copy
  uint8_t* hstage = nullptr;        // pinned host block
  uint64_t hstage_cap = 0;
  hipEvent_t hstage_done = nullptr; // the last copy out of hstage has completed
  uint64_t* stats = nullptr;
  // fast -> general hand-over
  uint32_t* pflag = nullptr;      // [NB][PART/32]
  uint32_t* ap_list = nullptr;    // [8][NB]
  uint32_t* fl_list = nullptr;    // [NB]
  uint32_t* eflag = nullptr;      // [NB][PART/32] k_elect's groups (n >= 5)
  uint8_t* lskip = nullptr;       // [NB] partitions the route closed (n >= 5 storm hand-over)
  uint32_t* el_list = nullptr;    // [8][NB]
  uint32_t* done = nullptr;       // k_apply workgroups finished this step
  uint32_t* resume = nullptr;     // [G]
  uint64_t* commit0 = nullptr;    // [G]
  uint64_t* peer = nullptr;       // [G][HB_PEER_ROW] node ids (hb_load_peers), allocated on first use
  uint32_t* dec_q = nullptr;      // hb_decode pass-2 queue (record indices)
  uint64_t dec_cap = 0;
  uint32_t* dec_qn = nullptr;     // [queue length, finished pass-2 workgroups]
  void* evx = nullptr;            // hb_copy_events expansion scratch, grown on demand
  uint64_t evx_cap = 0;
  uint64_t* evw = nullptr;        // hb_events_to_host: per-chunk word offsets + total
  uint64_t evw_cap = 0;
  uint64_t* rnd = nullptr;        // the r.rand stream (hb_set_rand), grown on demand
  uint64_t rnd_cap = 0;
  static constexpr uint32_t PROF_RING = 256;
  // per profiled step: prep start, prep end (prep stream), apply start, fast end,
  // general end, finish end (apply stream)
  static constexpr uint32_t PH_EVENTS = 6;
  hipEvent_t ph[PROF_RING][PH_EVENTS] = {};
  bool prof_full[PROF_RING] = {};  // all phases recorded (else only HB_PHASE_APPLY)
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
uint32_t ceil_log2_64(uint64_t x) {
  uint32_t b = 0;
  while (b < 63 && (1ull << b) < x) ++b;
  return b;
}

// Grow the log-index rings of groups[i] to hold at least szcap[i] entry sizes
// and trcap[i] term runs (null array or 0: unchanged); the content moves
// along (k_regrow).  Never shrinks.
int reserve_log(hb_handle* h, uint32_t count, const uint32_t* groups, const uint64_t* szcap, const uint64_t* trcap) {
  struct Need {
    uint32_t g;
    uint64_t sz, tr;
  };
  std::vector<Need> need;
  need.reserve(count);
  for (uint32_t i = 0; i < count; ++i) {
    if (groups[i] >= h->G) return HB_EINVAL;
    const uint64_t sz = (szcap && h->st.szx) ? szcap[i] : 0, tr = trcap ? trcap[i] : 0;
    const bool grow_sz = sz > (1ull << (h->h_szx.empty() ? 0 : (h->h_szx[groups[i]] & LX_TAG)));
    const bool grow_tr = tr > (1ull << (h->h_trx[groups[i]] & LX_TAG));
    if ((sz && grow_sz) || (tr && grow_tr)) need.push_back({groups[i], sz, tr});
  }
  if (need.empty()) return HB_OK;
  // one job per (group, ring): duplicates of a group merge to their largest need
  std::sort(need.begin(), need.end(), [](const Need& a, const Need& b) { return a.g < b.g; });
  std::vector<uint64_t> jobs;
  std::vector<std::pair<uint64_t, uint32_t>> old;  // extents to recycle once the copies ran
  for (size_t i = 0; i < need.size();) {
    Need m = need[i++];
    while (i < need.size() && need[i].g == m.g) {
      m.sz = std::max(m.sz, need[i].sz);
      m.tr = std::max(m.tr, need[i].tr);
      ++i;
    }
    for (uint32_t kind = 0; kind < 2; ++kind) {
      const uint64_t want = kind ? m.tr : m.sz;
      uint64_t& hx = kind ? h->h_trx[m.g] : h->h_szx[m.g];
      const uint32_t lc = (uint32_t)(hx & LX_TAG);
      if (!want || want <= (1ull << lc)) continue;
      const uint32_t l = ceil_log2_64(want), rec = kind ? 4 : 3;  // 16-byte runs, 8-byte sizes
      const uint64_t a = h->pool.get(l + rec);
      if (!a) return HB_ENOMEM;
      const uint64_t nx = lx_word(a, l);
      jobs.insert(jobs.end(), {(uint64_t)m.g | ((uint64_t)kind << 32), hx, nx, 0});
      old.emplace_back(hx & ~LX_TAG, lc + rec);
      hx = nx;
    }
  }
  const uint32_t nj = (uint32_t)(jobs.size() / 4);
  if (h->lx_jobs_cap < jobs.size()) {
    if (h->lx_jobs) (void)hipFree(h->lx_jobs);
    h->lx_jobs = nullptr;
    h->lx_jobs_cap = 0;
    if (hipMalloc(&h->lx_jobs, jobs.size() * 8) != hipSuccess) return HB_ENOMEM;
    h->lx_jobs_cap = jobs.size();
  }
  HB_CHECK(hipMemcpyAsync(h->lx_jobs, jobs.data(), jobs.size() * 8, hipMemcpyHostToDevice, h->stream));
  hipLaunchKernelGGL(k_regrow, dim3((nj + 255) / 256), dim3(256), 0, h->stream, h->st, nj, (const uint64_t*)h->lx_jobs);
  HB_CHECK(hipStreamSynchronize(h->stream));
  for (auto& o : old) h->pool.put(o.first, o.second);
  return HB_OK;
}

template <int KMAX>
uint32_t route_grid(const hb_handle* h, bool x) {
  return ((h->NBK + 7) & ~7u) << (PART_LOG + h->sis_log - (x ? RouteGeom<KMAX, true>::RG_LOG : RouteGeom<KMAX, false>::RG_LOG));
}
template <int KMAX>
void launch_route(hb_handle* h, const ApplyArgs& a, hipStream_t st) {
  if constexpr (KMAX >= 5) {
    if (!a.slotx && a.storm >= 2) {  // the storm hand-over with the election lane in the route
      if (h->nmax <= 5)
        hipLaunchKernelGGL((k_route<KMAX, false, 5>), dim3(route_grid<KMAX>(h, false)), dim3(ROUTE_THREADS), 0, st, a);
      else
        hipLaunchKernelGGL((k_route<KMAX, false, 7>), dim3(route_grid<KMAX>(h, false)), dim3(ROUTE_THREADS), 0, st, a);
      return;
    }
  }
  if (a.slotx) hipLaunchKernelGGL((k_route<KMAX, true>), dim3(route_grid<KMAX>(h, true)), dim3(ROUTE_THREADS), 0, st, a);
  else hipLaunchKernelGGL((k_route<KMAX, false>), dim3(route_grid<KMAX>(h, false)), dim3(ROUTE_THREADS), 0, st, a);
}

// XCD-aware grid (see block_part()): whole groups of 8 buckets x 2^sis_log
// partitions, cut after the last block that maps to a real partition (a small
// handle's 4 partitions sit at blocks 0, 8, 16, 24 of a 128-block grid).
uint32_t apply_grid_for(uint32_t NBK, uint32_t sl, uint32_t NB) {
  const uint32_t full = ((NBK + 7) & ~7u) << sl;
  uint32_t need = 0;
  for (uint32_t x = 0; x < full; ++x) {
    const uint32_t r = x & 7, q = x >> 3;  // part_of() on the host
    if ((((((q >> sl) << 3) | r) << sl) | (q & ((1u << sl) - 1))) < NB) need = x + 1;
  }
  return (need + 7) & ~7u;
}
uint32_t apply_grid(const hb_handle* h) { return h->agrid; }

// The apply kernels; ev = this step's phase events (HB_STEP_PROFILE) or null.
template <uint32_t KMAX, bool X>
void launch_route_fast_t(hb_handle* h, const ApplyArgs& a) {
  hipLaunchKernelGGL((k_route_fast<KMAX, X>),
                     dim3(((h->NBK + 7) & ~7u) << (PART_LOG + h->sis_log - RouteFastGeom<KMAX, X>::RG_LOG)),
                     dim3(RF_THREADS), 0, h->stream, a);
}
void launch_route_fast(hb_handle* h, const ApplyArgs& a) {
  if (a.kmax == 3) {
    if (a.slotx) launch_route_fast_t<3, true>(h, a);
    else launch_route_fast_t<3, false>(h, a);
  } else {
    if (a.slotx) launch_route_fast_t<2, true>(h, a);
    else launch_route_fast_t<2, false>(h, a);
  }
}
// the largest route-fast workgroup (groups, log2) of a step
inline uint32_t route_fast_rg_log(uint32_t kmax, bool x) {
  return kmax == 3 ? (x ? RouteFastGeom<3, true>::RG_LOG : RouteFastGeom<3, false>::RG_LOG)
                   : (x ? RouteFastGeom<2, true>::RG_LOG : RouteFastGeom<2, false>::RG_LOG);
}
// fused: k_route_fast stood in for k_route + k_apply_fast (launched by hb_step)
template <int NMAX>
void launch_apply(hb_handle* h, const ApplyArgs& a, hipEvent_t* ev, bool full, bool fused = false) {
  const uint32_t grid = apply_grid(h);
  if (ev) (void)hipEventRecord(ev[2], h->stream);
  if (fused) {
    if constexpr (NMAX <= 3) launch_route_fast(h, a);
  } else if constexpr (NMAX >= 5) {
    if (a.slotx) hipLaunchKernelGGL((k_apply_lead<NMAX, true>), dim3(grid), dim3(PART), 0, h->stream, a);
    else hipLaunchKernelGGL((k_apply_lead<NMAX, false>), dim3(grid), dim3(PART), 0, h->stream, a);
  }
  else if (a.kmax == 3) {
    if (a.slotx) hipLaunchKernelGGL((k_apply_fast<NMAX, true, 3>), dim3(grid), dim3(PART), 0, h->stream, a);
    else hipLaunchKernelGGL((k_apply_fast<NMAX, false, 3>), dim3(grid), dim3(PART), 0, h->stream, a);
  } else {
    if (a.slotx) hipLaunchKernelGGL((k_apply_fast<NMAX, true, 2>), dim3(grid), dim3(PART), 0, h->stream, a);
    else hipLaunchKernelGGL((k_apply_fast<NMAX, false, 2>), dim3(grid), dim3(PART), 0, h->stream, a);
  }
  if (ev) (void)hipEventRecord(ev[3], h->stream);
  // the list kernels loop over their XCD slot's list, so a small handle (a
  // MultiNode node of a few thousand groups: 4 partitions under a 128-entry
  // virtual grid) launches one workgroup per list entry it can have, at least 8
  const uint32_t lists = std::max(8u, (h->NB + 7) & ~7u);
  if constexpr (NMAX >= 5) {  // the general kernel spills at n >= 5: elections go first
    if (!sz_on(h->max_msg_size))
      hipLaunchKernelGGL(k_elect<NMAX>, dim3(std::min(lists, ELECT_GRID ? std::min(grid, ELECT_GRID) : grid)),
                         dim3(PART), 0, h->stream, a);
  }
  if constexpr (NMAX <= 3) {  // chained follower pass; the last workgroup runs the finish
    const uint32_t gg = std::min(lists, GEN_GRID3 ? std::min(grid, GEN_GRID3) : grid);
    hipLaunchKernelGGL(k_apply<NMAX>, dim3(gg), dim3(PART), 0, h->stream, a);
  } else {
    hipLaunchKernelGGL(k_apply<NMAX>, dim3(std::min(lists, GEN_GRID ? std::min(grid, GEN_GRID) : grid)), dim3(PART), 0,
                       h->stream, a);
    // k_follow's last workgroup also runs the step's finish (k_finish)
    hipLaunchKernelGGL(k_follow<NMAX>, dim3(FOLLOW_GRID), dim3(PART), 0, h->stream, a);
  }
  if (ev && full) (void)hipEventRecord(ev[4], h->stream);
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
      max_inflight > HB_MAX_INFLIGHT || max_batch >= (1ull << 31) || capacity > (1u << 24))
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
  if (const char* e = getenv("HB_SMALL_STEP")) h->no_small = e[0] == '0';
  if (const char* e = getenv("HB_ROUTE_FUSE")) h->fuse = (uint32_t)atoi(e);
  if (const char* e = getenv("HB_STORM")) h->storm = (uint32_t)atoi(e);
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
  ALLOC(s.elapsed, G);
  ALLOC(s.rpos, G);
  ALLOC(s.tcfg, G);
  ALLOC(s.trx, G);  // the log index (DevState): older term runs (follower side) ...
  ALLOC(s.trc, G);
  if (sz_on(max_msg_size)) {  // ... and, for limitSize, the entries' cumulative sizes
    ALLOC(s.szx, G);
    ALLOC(s.szlo, G);
  }
  // partition scratch
  const size_t mb = max_batch ? max_batch : 1;
  // buckets: SIS_MAX partitions each, or fewer — down to one k_route
  // workgroup per bucket — while that needs no extra radix pass
  auto nbk_for = [&](uint32_t sl) { return (capacity + (PART << sl) - 1) / (PART << sl); };
  auto passes_for = [&](uint32_t sl) {
    return (std::max<uint32_t>(ceil_log2(nbk_for(sl)), 1) + RDX_BITS - 1) / RDX_BITS;
  };
  const uint32_t sl_max = h->nmax <= 3 ? SIS_LOG_MAX3 : SIS_LOG_MAX;
  h->sis_log = sl_max;
  const uint32_t sl_min = route_rg_log(route_kmax(h->nmax)) - PART_LOG;
  while (h->sis_log > sl_min && passes_for(h->sis_log - 1) == passes_for(sl_max)) --h->sis_log;
  if (const char* e = getenv("HB_SIS_LOG")) {  // (A/B knob: a fixed bucket size, within the allowed range)
    const int v = atoi(e);
    if (v >= (int)sl_min && v <= (int)sl_max) h->sis_log = (uint32_t)v;
  }
  h->NBK = nbk_for(h->sis_log);
  h->passes = passes_for(h->sis_log);
  h->bk_bits = std::max<uint32_t>(ceil_log2(h->NBK), 1);
  h->agrid = apply_grid_for(h->NBK, h->sis_log, h->NB);
  const size_t tiles_max = (mb + RDX_TILE - 1) / RDX_TILE;
  ALLOC(h->hist, (size_t)RDX_BINS * tiles_max);
  ALLOC(h->n_valid, 4);
  ALLOC(h->totals, RDX_BINS);
  if (h->passes == 1) {
    const size_t nhw = (tiles_max + HIST_TPB - 1) / HIST_TPB;
    h->sup_max = (uint32_t)((nhw + SB_HW - 1) / SB_HW);
    ALLOC(h->hagg, nhw * RDX_BINS);
    ALLOC(h->hsup, (size_t)SUP_BUFS * h->sup_max * RDX_BINS);
    if (rc == HB_OK && hipMemset(h->hsup, 0, (size_t)SUP_BUFS * h->sup_max * RDX_BINS * 4) != hipSuccess)
      rc = HB_EDEVICE;
  }
  for (uint32_t k = 0; k + 1 < h->passes && k < 2; ++k) {  // ping-pong buffers of intermediate passes
    RadixDst& d = h->tmp[k];
    ALLOC(d.group, mb);
    ALLOC(d.rec, mb);
    ALLOC(d.recx, mb);
  }
  for (PrepSet& ps : h->set) {
    ALLOC(ps.rec, mb);
    ALLOC(ps.key, mb + SEG);
    if (h->passes > 1) ALLOC(ps.bucket, mb);
    ALLOC(ps.bk_off, h->NBK + 1);
    ALLOC(ps.bk_fill, (size_t)h->NBK * CTR_STRIDE);
    ALLOC(ps.ctr, CTR_WORDS);
    ALLOC(ps.cnt, G);
    ALLOC(ps.slot, route_kmax(R) * G);
    ALLOC(ps.side, 2 * mb);
    ALLOC(ps.recx, mb);
    ALLOC(ps.slotx, route_kmax(R) * G);
    ALLOC(ps.ev_counts, 2ull * h->NB);
    ALLOC(ps.ev_off, 2ull * h->NB);
  }
  ALLOC(h->s_group, mb);
  ALLOC(h->s_info, mb);
  ALLOC(h->s_term, mb);
  ALLOC(h->s_index, mb);
  ALLOC(h->s_hint, mb);
  ALLOC(h->s_props, G);
  ALLOC(h->s_eoff, mb);
  ALLOC(h->s_commit, mb);
  if (sz_on(max_msg_size)) ALLOC(h->s_peoff, G);
  // events: (batch + one proposal slot per group) x EV_MAX (exact bound)
  h->ev_per_msg = EVC_WORDS_MAX * (h->nmax + 4);  // events per message <= nmax + 4, <= 2 words each
  // P chunks (one per partition, dense proposals) then the bucket regions of M chunks
  h->ev_region = ((uint64_t)h->NB * PART + mb + ((uint64_t)h->NBK * PART << h->sis_log)) * h->ev_per_msg;
  ALLOC(h->ev, h->ev_region);
  ALLOC(h->stats_shard, shard_at(ST_N + 1, 0));
  ALLOC(h->pflag, (size_t)h->NB * FLAG_WORDS);
  ALLOC(h->ap_list, 8ull * h->NB);
  ALLOC(h->fl_list, h->NB);
  if (h->nmax >= 5) {
    ALLOC(h->eflag, (size_t)h->NB * FLAG_WORDS);
    ALLOC(h->lskip, (size_t)h->NB);
    ALLOC(h->el_list, 8ull * h->NB);
  }
  ALLOC(h->resume, G);
  ALLOC(h->commit0, G);
  ALLOC(h->stats, HB_STAT_COUNT);
#undef ALLOC
  if (rc != HB_OK) {
    hb_destroy(h);
    return rc;
  }
  // the prep stream runs at the lowest priority: its kernels fill what the
  // apply stage leaves idle instead of competing with it
  int prio_least = 0, prio_greatest = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
  bool ok = hipStreamCreateWithPriority(&h->prep, hipStreamNonBlocking, prio_least) == hipSuccess &&
            hipEventCreateWithFlags(&h->in_ready, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&h->hstage_done, hipEventDisableTiming) == hipSuccess &&
            hipHostMalloc(reinterpret_cast<void**>(&h->stats_pin), HB_STAT_COUNT * 8, hipHostMallocDefault) == hipSuccess;
  for (PrepSet& ps : h->set)
    ok = ok && hipEventCreateWithFlags(&ps.prepped, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&ps.applied, hipEventDisableTiming) == hipSuccess;
  for (auto& row : h->ph)
    for (auto& e : row) ok = ok && hipEventCreate(&e) == hipSuccess;
  if (!ok) {
    hb_destroy(h);
    return HB_EDEVICE;
  }
  // empty slots (n = 0), zeroed progress
  if (hipMemset(s.meta, 0, G * 8) != hipSuccess || hipMemset(s.pm, 0, R * G * 4) != hipSuccess ||
      hipMemset(s.elapsed, 0, G * 4) != hipSuccess || hipMemset(s.rpos, 0, G * 4) != hipSuccess ||
      hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(s.tcfg), 10u | (1u << 16), G) != hipSuccess ||
      hipMemset(h->stats, 0, HB_STAT_COUNT * 8) != hipSuccess || hipMemset(h->stats_shard, 0, shard_at(ST_N + 1, 0) * 8ull) != hipSuccess ||
      hipMemset(h->set[0].ctr, 0, CTR_WORDS * 4) != hipSuccess || hipMemset(h->set[1].ctr, 0, CTR_WORDS * 4) != hipSuccess ||
      hipMemset(h->set[0].ev_counts, 0, h->NB * 8ull) != hipSuccess ||
      hipMemset(h->set[0].ev_off, 0, h->NB * 16ull) != hipSuccess ||
      hipMemset(s.trc, 0, G * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    hb_destroy(h);
    return HB_EDEVICE;
  }
  // the log index: every group starts with a 128-byte extent per ring, carved
  // from one slab each (hb_reserve_log moves a group to a larger one)
  auto init_rings = [&](std::vector<uint64_t>& hx, uint64_t* dx, uint32_t log2cap) {
    void* slab = nullptr;
    if (hipMalloc(&slab, G * 128) != hipSuccess) return false;
    h->pool.slabs.push_back(slab);
    hx.resize(G);
    const uint64_t base = reinterpret_cast<uint64_t>(slab);
    for (size_t g = 0; g < G; ++g) hx[g] = lx_word(base + 128 * g, log2cap);
    return hipMemcpy(dx, hx.data(), G * 8, hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!init_rings(h->h_trx, s.trx, TR_LOG_MIN) || (s.szx && !init_rings(h->h_szx, s.szx, SZ_LOG_MIN))) {
    hb_destroy(h);
    return HB_ENOMEM;
  }
  *out = h;
  return HB_OK;
}

int hb_destroy(hb_handle* h) {
  if (!h) return HB_EINVAL;
  DeviceGuard guard(h->device);
  (void)hipDeviceSynchronize();
  for (void* p : h->allocs) (void)hipFree(p);
  h->pool.release();
  if (h->lx_jobs) (void)hipFree(h->lx_jobs);
  for (auto& row : h->ph)
    for (auto& e : row)
      if (e) (void)hipEventDestroy(e);
  for (PrepSet& ps : h->set) {
    if (ps.prepped) (void)hipEventDestroy(ps.prepped);
    if (ps.applied) (void)hipEventDestroy(ps.applied);
  }
  if (h->rnd) (void)hipFree(h->rnd);
  if (h->evx) (void)hipFree(h->evx);
  if (h->evw) (void)hipFree(h->evw);
  for (PrepSet& ps : h->set)
    if (ps.dstage) (void)hipFree(ps.dstage);
  if (h->hstage) (void)hipHostFree(h->hstage);
  if (h->stats_pin) (void)hipHostFree(h->stats_pin);
  if (h->hstage_done) (void)hipEventDestroy(h->hstage_done);
  if (h->s_edesc) (void)hipFree(h->s_edesc);
  if (h->s_eterm) (void)hipFree(h->s_eterm);
  if (h->peer) (void)hipFree(h->peer);
  if (h->dec_q) (void)hipFree(h->dec_q);
  if (h->dec_qn) (void)hipFree(h->dec_qn);
  if (h->in_ready) (void)hipEventDestroy(h->in_ready);
  if (h->prep) (void)hipStreamDestroy(h->prep);
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
  HB_CHECK(hipStreamSynchronize(h->prep));
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
    if (h->peer)
      hipLaunchKernelGGL(k_peer_n, dim3((count + 255) / 256), dim3(256), 0, h->stream, h->peer, h->st.meta, first,
                         count);
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

int hb_set_log_bounds(hb_handle* h, uint32_t count, const uint32_t* groups, const uint64_t* first_index,
                      const uint64_t* snap_index) {
  if (!h || (count && (!groups || !first_index || !snap_index))) return HB_EINVAL;
  if (count == 0) return HB_OK;
  for (uint32_t i = 0; i < count; ++i)
    if (groups[i] >= h->G || first_index[i] == 0) return HB_EINVAL;
  DeviceGuard guard(h->device);
  char* d = nullptr;
  const size_t bytes = (size_t)count * (4 + 8 + 8);
  HB_CHECK(hipMalloc(&d, bytes));
  uint64_t* dfirst = reinterpret_cast<uint64_t*>(d);
  uint64_t* dsnap = dfirst + count;
  uint32_t* dgroup = reinterpret_cast<uint32_t*>(dsnap + count);
  hipError_t e = hipMemcpyAsync(dfirst, first_index, count * 8ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dsnap, snap_index, count * 8ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dgroup, groups, count * 4ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_set_bounds, dim3((count + 255) / 256), dim3(256), 0, h->stream, h->st, count,
                       (const uint32_t*)dgroup, (const uint64_t*)dfirst, (const uint64_t*)dsnap);
    e = hipStreamSynchronize(h->stream);
  }
  (void)hipFree(d);
  return e == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_load_term_runs(hb_handle* h, uint32_t count, const uint32_t* groups, const uint32_t* n_runs,
                      const uint64_t* runs) {
  if (!h || (count && (!groups || !n_runs))) return HB_EINVAL;
  if (count == 0) return HB_OK;
  std::vector<uint64_t> off(count), cap(count);
  uint64_t tot = 0;
  for (uint32_t i = 0; i < count; ++i) {
    if (groups[i] >= h->G) return HB_EINVAL;
    off[i] = tot;
    tot += n_runs[i];
    cap[i] = (uint64_t)n_runs[i] + 1;  // room for the reset that pushes the current-term run
  }
  if (tot && !runs) return HB_EINVAL;
  DeviceGuard guard(h->device);
  const int rc = reserve_log(h, count, groups, nullptr, cap.data());
  if (rc != HB_OK) return rc;
  char* d = nullptr;
  const size_t bytes = count * (8ull + 4 + 4) + tot * 16 + 16;
  HB_CHECK(hipMalloc(&d, bytes));
  uint64_t* doff = reinterpret_cast<uint64_t*>(d);
  uint64_t* druns = doff + count;
  uint32_t* dgrp = reinterpret_cast<uint32_t*>(druns + 2 * tot);
  uint32_t* dn = dgrp + count;
  hipError_t e = hipMemcpyAsync(doff, off.data(), count * 8ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess && tot) e = hipMemcpyAsync(druns, runs, tot * 16ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dgrp, groups, count * 4ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dn, n_runs, count * 4ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_load_runs, dim3((count + 255) / 256), dim3(256), 0, h->stream, h->st, count,
                       (const uint32_t*)dgrp, (const uint32_t*)dn, (const uint64_t*)doff, (const uint64_t*)druns);
    e = hipStreamSynchronize(h->stream);
  }
  (void)hipFree(d);
  return e == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_load_entry_sizes(hb_handle* h, uint32_t count, const uint32_t* groups, const uint32_t* n_sizes,
                        const uint32_t* sizes) {
  if (!h || (count && (!groups || !n_sizes))) return HB_EINVAL;
  if (!sz_on(h->max_msg_size)) return HB_EINVAL;
  if (count == 0) return HB_OK;
  std::vector<uint64_t> off(count), cap(count);
  uint64_t tot = 0;
  for (uint32_t i = 0; i < count; ++i) {
    if (groups[i] >= h->G) return HB_EINVAL;
    off[i] = tot;
    tot += n_sizes[i];
    cap[i] = (uint64_t)n_sizes[i] + 1;  // the base entry plus n sizes
  }
  if (tot && !sizes) return HB_EINVAL;
  DeviceGuard guard(h->device);
  const int rc = reserve_log(h, count, groups, cap.data(), nullptr);
  if (rc != HB_OK) return rc;
  char* d = nullptr;
  const size_t bytes = count * (4ull + 4 + 8) + tot * 4 + 16;
  HB_CHECK(hipMalloc(&d, bytes));
  uint64_t* doff = reinterpret_cast<uint64_t*>(d);
  uint32_t* dgrp = reinterpret_cast<uint32_t*>(doff + count);
  uint32_t* dn = dgrp + count;
  uint32_t* dsz = dn + count;
  hipError_t e = hipMemcpyAsync(doff, off.data(), count * 8ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dgrp, groups, count * 4ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dn, n_sizes, count * 4ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess && tot) e = hipMemcpyAsync(dsz, sizes, tot * 4ull, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_load_sizes, dim3((count + 255) / 256), dim3(256), 0, h->stream, h->st, count,
                       (const uint32_t*)dgrp, (const uint32_t*)dn, (const uint64_t*)doff, (const uint32_t*)dsz);
    e = hipStreamSynchronize(h->stream);
  }
  (void)hipFree(d);
  return e == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_reserve_log(hb_handle* h, uint32_t count, const uint32_t* groups, const uint64_t* size_cap,
                   const uint64_t* run_cap) {
  if (!h || (count && !groups)) return HB_EINVAL;
  if (count == 0 || (!size_cap && !run_cap)) return HB_OK;
  DeviceGuard guard(h->device);
  return reserve_log(h, count, groups, size_cap, run_cap);
}

int hb_log_capacity(hb_handle* h, uint32_t group, uint64_t* size_cap, uint64_t* run_cap) {
  if (!h || group >= h->G) return HB_EINVAL;
  if (size_cap) *size_cap = h->h_szx.empty() ? 0 : 1ull << (h->h_szx[group] & LX_TAG);
  if (run_cap) *run_cap = 1ull << (h->h_trx[group] & LX_TAG);
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

int hb_load_timers(hb_handle* h, uint32_t first, uint32_t count, const hb_timer* timers) {
  if (!h || !timers || (uint64_t)first + count > h->G) return HB_EINVAL;
  if (count == 0) return HB_OK;
  std::vector<uint32_t> el(count), pos(count), cfg(count);
  for (uint32_t i = 0; i < count; ++i) {
    if (timers[i].election_tick == 0) return HB_EINVAL;  // r.rand.Int() % 0
    el[i] = timers[i].elapsed;
    pos[i] = timers[i].rand_pos;
    cfg[i] = timers[i].election_tick | ((uint32_t)timers[i].heartbeat_tick << 16);
  }
  DeviceGuard guard(h->device);
  HB_CHECK(hipMemcpyAsync(h->st.elapsed + first, el.data(), count * 4ull, hipMemcpyHostToDevice, h->stream));
  HB_CHECK(hipMemcpyAsync(h->st.rpos + first, pos.data(), count * 4ull, hipMemcpyHostToDevice, h->stream));
  HB_CHECK(hipMemcpyAsync(h->st.tcfg + first, cfg.data(), count * 4ull, hipMemcpyHostToDevice, h->stream));
  HB_CHECK(hipStreamSynchronize(h->stream));
  return HB_OK;
}

int hb_get_timers(hb_handle* h, uint32_t first, uint32_t count, hb_timer* out) {
  if (!h || !out || (uint64_t)first + count > h->G) return HB_EINVAL;
  if (count == 0) return HB_OK;
  std::vector<uint32_t> el(count), pos(count), cfg(count);
  DeviceGuard guard(h->device);
  HB_CHECK(hipMemcpyAsync(el.data(), h->st.elapsed + first, count * 4ull, hipMemcpyDeviceToHost, h->stream));
  HB_CHECK(hipMemcpyAsync(pos.data(), h->st.rpos + first, count * 4ull, hipMemcpyDeviceToHost, h->stream));
  HB_CHECK(hipMemcpyAsync(cfg.data(), h->st.tcfg + first, count * 4ull, hipMemcpyDeviceToHost, h->stream));
  HB_CHECK(hipStreamSynchronize(h->stream));
  for (uint32_t i = 0; i < count; ++i) {
    out[i] = hb_timer{};
    out[i].elapsed = el[i];
    out[i].rand_pos = pos[i];
    out[i].election_tick = (uint16_t)(cfg[i] & 0xFFFFu);
    out[i].heartbeat_tick = (uint16_t)(cfg[i] >> 16);
  }
  return HB_OK;
}

int hb_set_rand(hb_handle* h, uint64_t first, uint64_t count, const uint64_t* draws) {
  if (!h || (count && !draws) || first > h->st.nrnd) return HB_EINVAL;  // no holes
  const uint64_t need = first + count;
  DeviceGuard guard(h->device);
  if (need > h->rnd_cap) {
    const uint64_t cap = need > 2 * h->rnd_cap ? need : 2 * h->rnd_cap;
    uint64_t* p = nullptr;
    HB_CHECK(hipMalloc(&p, cap * 8));
    hipError_t e = hipSuccess;
    if (h->rnd && first) e = hipMemcpyAsync(p, h->rnd, first * 8, hipMemcpyDeviceToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);  // no kernel reads the old table any more
    if (e != hipSuccess) {
      (void)hipFree(p);
      return HB_EDEVICE;
    }
    if (h->rnd) (void)hipFree(h->rnd);
    h->rnd = p;
    h->rnd_cap = cap;
  }
  if (count) {
    HB_CHECK(hipMemcpyAsync(h->rnd + first, draws, count * 8, hipMemcpyHostToDevice, h->stream));
    HB_CHECK(hipStreamSynchronize(h->stream));
  }
  h->st.rnd = h->rnd;
  if (need > h->st.nrnd) h->st.nrnd = need;
  return HB_OK;
}

int hb_load_peers(hb_handle* h, uint32_t first, uint32_t count, const uint64_t* ids) {
  if (!h || (count && !ids) || (uint64_t)first + count > h->G) return HB_EINVAL;
  if (count == 0) return HB_OK;
  DeviceGuard guard(h->device);
  const size_t G = h->G;
  if (!h->peer) {
    HB_CHECK(hipMalloc(&h->peer, G * HB_PEER_ROW * 8));
    HB_CHECK(hipMemsetAsync(h->peer, 0, G * HB_PEER_ROW * 8, h->stream));
  }
  // one 64-byte row per group (k_decode reads it with one gather): slots
  // 0..nmax-1, zeros, then n (k_peer_n)
  std::vector<uint64_t> rows((size_t)count * HB_PEER_ROW, 0);
  for (uint32_t i = 0; i < count; ++i)
    for (uint32_t s = 0; s < h->nmax; ++s) rows[(size_t)i * HB_PEER_ROW + s] = ids[(size_t)i * HB_MAX_REPLICAS + s];
  HB_CHECK(hipMemcpyAsync(h->peer + (size_t)first * HB_PEER_ROW, rows.data(), rows.size() * 8, hipMemcpyHostToDevice,
                          h->stream));
  hipLaunchKernelGGL(k_peer_n, dim3((count + 255) / 256), dim3(256), 0, h->stream, h->peer, h->st.meta, first, count);
  HB_CHECK(hipGetLastError());
  HB_CHECK(hipStreamSynchronize(h->stream));  // rows is freed on return
  return HB_OK;
}

int hb_decode(hb_handle* h, const uint8_t* bytes, const uint64_t* off, const uint32_t* len, const uint32_t* group,
              uint64_t n, const hb_batch* out, uint8_t* status) {
  if (!h || !out) return HB_EINVAL;
  if (n == 0) return HB_OK;
  if (n >= (1ull << 32)) return HB_EINVAL;  // record indices are 32-bit in the pass-2 queue
  if (!bytes || !off || !len || !group || !status || !out->group || !out->info || !out->term || !out->index ||
      !out->hint)
    return HB_EINVAL;
  DeviceGuard guard(h->device);
  DecodeArgs da;
  da.bytes = bytes;
  da.off = off;
  da.len = len;
  da.group = group;
  da.n = n;
  da.meta = h->st.meta;
  da.peer = reinterpret_cast<const uint4*>(h->peer);
  da.G = h->G;
  da.nmax = h->nmax;
  da.o_group = const_cast<uint32_t*>(out->group);
  da.o_info = const_cast<uint32_t*>(out->info);
  da.o_term = const_cast<uint64_t*>(out->term);
  da.o_index = const_cast<uint64_t*>(out->index);
  da.o_hint = const_cast<uint64_t*>(out->hint);
  da.status = status;
  // on the stream the batches come from, so hb_step's prep orders after it
  hipStream_t ds = h->in_stream_set ? h->in_stream : h->stream;
  if (n > h->dec_cap) {  // the pass-2 queue holds up to n record indices
    if (h->dec_q) (void)hipFree(h->dec_q);
    h->dec_q = nullptr;
    h->dec_cap = 0;
    HB_CHECK(hipMalloc(&h->dec_q, n * sizeof(uint32_t)));
    h->dec_cap = n;
  }
  if (!h->dec_qn) {
    HB_CHECK(hipMalloc(&h->dec_qn, 2 * sizeof(uint32_t)));
    HB_CHECK(hipMemsetAsync(h->dec_qn, 0, 2 * sizeof(uint32_t), ds));
  }
  hipLaunchKernelGGL(k_decode, dim3((unsigned)((n + DEC_THREADS - 1) / DEC_THREADS)), dim3(DEC_THREADS), 0, ds, da,
                     h->dec_q, h->dec_qn);
  HB_CHECK(hipGetLastError());
  const uint64_t gb = (n + DEC_THREADS - 1) / DEC_THREADS;
  hipLaunchKernelGGL(k_decode_general, dim3((unsigned)(gb < DEC_GEN_BLOCKS ? gb : DEC_GEN_BLOCKS)), dim3(DEC_THREADS), 0,
                     ds, da, h->dec_q, h->dec_qn);
  HB_CHECK(hipGetLastError());
  return HB_OK;
}

int hb_tick(hb_handle* h, uint32_t flags) {
  if (!h || flags) return HB_EINVAL;
  DeviceGuard guard(h->device);
  hipStream_t st = h->stream;
  const bool two = h->in_stream_set && h->in_stream != h->stream;
  PrepSet& ps = h->set[h->next_set];
  ApplyArgs aa{};
  aa.S = h->st;
  aa.ev = h->ev;
  aa.ev_per_msg = h->ev_per_msg;
  aa.NB = h->NB;
  aa.NBK = h->NBK;
  aa.sis_log = h->sis_log;
  aa.ev_counts = ps.ev_counts;
  aa.ev_off = ps.ev_off;
  aa.stats_shard = h->stats_shard;
  const uint32_t grid = apply_grid(h);
  switch (h->nmax) {
    case 3: hipLaunchKernelGGL(k_tick<3>, dim3(grid), dim3(PART), 0, st, aa); break;
    case 5: hipLaunchKernelGGL(k_tick<5>, dim3(grid), dim3(PART), 0, st, aa); break;
    default: hipLaunchKernelGGL(k_tick<7>, dim3(grid), dim3(PART), 0, st, aa); break;
  }
  hipLaunchKernelGGL(k_finish, dim3(1), dim3(128), 0, st, h->stats_shard, h->stats, h->stats_accum);
  if (two) HB_CHECK(hipEventRecord(ps.applied, st));  // a later prep reusing this set waits for it
  HB_CHECK(hipGetLastError());
  ps.used = true;
  h->cur = h->next_set;
  h->next_set ^= 1;
  h->stepped = true;
  h->kern = 0;
  return HB_OK;
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
  const bool sized = sz_on(h->max_msg_size);  // appended entries carry descriptors
  if (sized && ((b->n && !b->eoff) || (b->props && !b->peoff) || (b->n_edesc && !b->edesc))) return HB_EINVAL;
  // MsgApp entry terms need their per-message offsets, and described entries
  // need terms or descriptors (else a MsgApp's entries would silently vanish)
  if ((b->eterm && b->n && !b->eoff) || (b->n_edesc && !b->eterm && !b->edesc)) return HB_EINVAL;
  if ((flags & HB_STEP_HOST_PTRS) && b->eoff) {  // offsets non-decreasing and within the entries
    uint64_t prev = 0;
    for (uint64_t i = 0; i < b->n; ++i) {
      if (b->eoff[i] < prev || b->eoff[i] > b->n_edesc) return HB_EINVAL;
      prev = b->eoff[i];
    }
  }
  DeviceGuard guard(h->device);
  hipStream_t st = h->stream;  // apply stream
  // prep stream (partition + route): the library's own stream when the caller
  // named a separate input stream, else the apply stream itself (no hops)
  const bool two = h->in_stream_set && h->in_stream != h->stream;
  hipStream_t ps_st = two ? h->prep : st;
  const bool prof = (flags & HB_STEP_PROFILE) != 0;
  const bool prof_apply = prof || (flags & HB_STEP_PROFILE_APPLY) != 0;
  PrepSet& ps = h->set[h->next_set];
  hipEvent_t* ev = h->ph[h->prof_n % hb_handle::PROF_RING];

  // ---- prep inputs.  The prep stream waits for (a) the inputs: the input
  // stream's work so far (default: the apply stream, i.e. no overlap), (b) the
  // last apply that read this prep set (two steps ago).
  BatchDev bd{b->group, b->info, b->term, b->index, b->hint, b->props, b->n};
  const uint32_t* bd_edesc = b->edesc;
  const uint64_t* bd_eoff = b->eoff;
  const uint64_t* bd_peoff = b->peoff;
  const uint64_t* bd_commit = b->commit;
  const uint64_t* bd_eterm = b->eterm;
  if (two) {
    HB_CHECK(hipEventRecord(h->in_ready, h->in_stream));
    HB_CHECK(hipStreamWaitEvent(ps_st, h->in_ready, 0));
    if (ps.used) HB_CHECK(hipStreamWaitEvent(ps_st, ps.applied, 0));
  }
  // Host-pointer batches.  Small ones (the host MultiNode's Ready cycles) are
  // packed into one pinned block and sent with ONE copy; larger ones go
  // array by array into the handle's staging buffers.
  bool packed = false;
  if (flags & HB_STEP_HOST_PTRS) {
    const size_t n = b->n;
    struct Part {
      const void* src;
      size_t bytes;
      size_t off;
    };
    Part parts[11] = {{b->group, n * 4, 0},
                      {b->info, n * 4, 0},
                      {b->term, n * 8, 0},
                      {b->index, n * 8, 0},
                      {b->hint, b->hint ? n * 8 : 0, 0},
                      {b->props, b->props ? (size_t)h->G * 4 : 0, 0},
                      {b->edesc, (sized && b->edesc) ? b->n_edesc * 4 : 0, 0},
                      {b->eterm, b->eterm ? b->n_edesc * 8 : 0, 0},
                      {b->eoff, b->eoff ? n * 8 : 0, 0},
                      {b->commit, b->commit ? n * 8 : 0, 0},
                      {b->peoff, (sized && b->props) ? (size_t)h->G * 8 : 0, 0}};
    size_t total = 0;
    for (Part& q : parts) {
      q.off = total;
      total += (q.src && q.bytes) ? (q.bytes + 255) & ~(size_t)255 : 0;
    }
    if (total > 0 && total <= STAGE_MAX) {
      packed = true;
      if (total > h->hstage_cap) {
        HB_CHECK(hipEventSynchronize(h->hstage_done));
        if (h->hstage) (void)hipHostFree(h->hstage);
        h->hstage = nullptr;
        h->hstage_cap = 0;
        HB_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h->hstage), STAGE_MAX, hipHostMallocDefault));
        h->hstage_cap = STAGE_MAX;
      }
      if (total > ps.dstage_cap) {  // (this set's last reader is done: the prep stream waited for it)
        HB_CHECK(hipStreamSynchronize(st));
        if (ps.dstage) (void)hipFree(ps.dstage);
        ps.dstage = nullptr;
        ps.dstage_cap = 0;
        HB_CHECK(hipMalloc(reinterpret_cast<void**>(&ps.dstage), STAGE_MAX));
        ps.dstage_cap = STAGE_MAX;
      }
      HB_CHECK(hipEventSynchronize(h->hstage_done));  // the previous step's copy has left the block
      for (const Part& q : parts)
        if (q.src && q.bytes) std::memcpy(h->hstage + q.off, q.src, q.bytes);
      HB_CHECK(hipMemcpyAsync(ps.dstage, h->hstage, total, hipMemcpyHostToDevice, ps_st));
      HB_CHECK(hipEventRecord(h->hstage_done, ps_st));
      auto at = [&](int k) { return parts[k].src && parts[k].bytes ? ps.dstage + parts[k].off : nullptr; };
      bd.group = reinterpret_cast<const uint32_t*>(at(0));
      bd.info = reinterpret_cast<const uint32_t*>(at(1));
      bd.term = reinterpret_cast<const uint64_t*>(at(2));
      bd.index = reinterpret_cast<const uint64_t*>(at(3));
      bd.hint = reinterpret_cast<const uint64_t*>(at(4));
      bd.props = reinterpret_cast<const uint32_t*>(at(5));
      bd_edesc = reinterpret_cast<const uint32_t*>(at(6));
      bd_eterm = reinterpret_cast<const uint64_t*>(at(7));
      bd_eoff = reinterpret_cast<const uint64_t*>(at(8));
      bd_commit = reinterpret_cast<const uint64_t*>(at(9));
      bd_peoff = reinterpret_cast<const uint64_t*>(at(10));
    }
  }
  if ((flags & HB_STEP_HOST_PTRS) && !packed) {
    // partition inputs on the prep stream (staging is reused in prep-stream
    // order); props / hint are read by apply, so they go on the apply stream.
    const size_t n = b->n;
    if (n) {
      HB_CHECK(hipMemcpyAsync(h->s_group, b->group, n * 4, hipMemcpyHostToDevice, ps_st));
      HB_CHECK(hipMemcpyAsync(h->s_info, b->info, n * 4, hipMemcpyHostToDevice, ps_st));
      HB_CHECK(hipMemcpyAsync(h->s_term, b->term, n * 8, hipMemcpyHostToDevice, ps_st));
      HB_CHECK(hipMemcpyAsync(h->s_index, b->index, n * 8, hipMemcpyHostToDevice, ps_st));
      if (b->hint) HB_CHECK(hipMemcpyAsync(h->s_hint, b->hint, n * 8, hipMemcpyHostToDevice, st));
    }
    if (b->props) HB_CHECK(hipMemcpyAsync(h->s_props, b->props, (size_t)h->G * 4, hipMemcpyHostToDevice, st));
    bd.group = h->s_group;
    bd.info = h->s_info;
    bd.term = h->s_term;
    bd.index = h->s_index;
    bd.hint = b->hint ? h->s_hint : nullptr;
    bd.props = b->props ? h->s_props : nullptr;
    // entry descriptors / terms, m.Commit: read by apply, so on the apply stream
    auto grow = [&](auto** p, uint64_t* cap, uint64_t need, size_t elem) -> int {
      if (need <= *cap) return HB_OK;
      HB_CHECK(hipStreamSynchronize(st));  // the old staging may still be read
      if (*p) (void)hipFree(*p);
      *p = nullptr;
      *cap = 0;
      HB_CHECK(hipMalloc(reinterpret_cast<void**>(p), need * elem));
      *cap = need;
      return HB_OK;
    };
    if (sized && b->edesc && b->n_edesc) {
      if (grow(&h->s_edesc, &h->s_edesc_cap, b->n_edesc, 4) != HB_OK) return HB_EDEVICE;
      HB_CHECK(hipMemcpyAsync(h->s_edesc, b->edesc, b->n_edesc * 4, hipMemcpyHostToDevice, st));
    }
    if (b->eterm && b->n_edesc) {
      if (grow(&h->s_eterm, &h->s_eterm_cap, b->n_edesc, 8) != HB_OK) return HB_EDEVICE;
      HB_CHECK(hipMemcpyAsync(h->s_eterm, b->eterm, b->n_edesc * 8, hipMemcpyHostToDevice, st));
    }
    if (b->eoff && n) HB_CHECK(hipMemcpyAsync(h->s_eoff, b->eoff, n * 8, hipMemcpyHostToDevice, st));
    if (b->commit && n) HB_CHECK(hipMemcpyAsync(h->s_commit, b->commit, n * 8, hipMemcpyHostToDevice, st));
    if (sized && b->props) HB_CHECK(hipMemcpyAsync(h->s_peoff, b->peoff, (size_t)h->G * 8, hipMemcpyHostToDevice, st));
    bd_edesc = (sized && b->edesc) ? h->s_edesc : nullptr;
    bd_eterm = b->eterm ? h->s_eterm : nullptr;
    bd_eoff = b->eoff ? h->s_eoff : nullptr;
    bd_commit = b->commit ? h->s_commit : nullptr;
    bd_peoff = (sized && b->props) ? h->s_peoff : nullptr;
  }
  if (prof) HB_CHECK(hipEventRecord(ev[0], ps_st));

  // ---- phase 1: partition (prep stream) ---------------------------------------
  const uint32_t NB = h->NB;
  // X mode: a follower-side batch (m.Commit given) carries {hint, commit} with every record
  const bool xmode = bd_commit != nullptr && b->n > 0;
  if (b->n == 0) {
    HB_CHECK(hipMemsetAsync(ps.bk_off, 0, (h->NBK + 1) * 4ull, ps_st));
    HB_CHECK(hipMemsetAsync(ps.bk_fill, 0, h->NBK * 4ull * CTR_STRIDE, ps_st));
    HB_CHECK(hipMemsetAsync(ps.ctr, 0, CTR_WORDS * 4ull, ps_st));
  } else {
    const uint32_t ntiles = (uint32_t)((b->n + RDX_TILE - 1) / RDX_TILE);
    RadixSrc src{bd.group, bd.info, bd.term, bd.index, nullptr, nullptr, ps.side, (uint32_t)b->n,
                 bd.hint, bd_commit, bd_eoff, bd_eterm, b->n_edesc, nullptr};
    const FinalDst fin{ps.rec, ps.recx, ps.bucket, h->passes == 1 ? ps.bk_off : nullptr, h->NBK, h->sis_log};
    uint32_t shift = PART_LOG + h->sis_log;
    if (h->passes == 1 && h->NBK == 1 && ntiles <= SMALL_TILES && !h->no_small) {  // one bucket: a compaction
      if (xmode)
        hipLaunchKernelGGL(k_pack_one<true>, dim3(1), dim3(RDX_THREADS), 0, ps_st, src, fin, h->G, ntiles, ps.bk_fill,
                           h->NBK, ps.ctr, h->n_valid);
      else
        hipLaunchKernelGGL(k_pack_one<false>, dim3(1), dim3(RDX_THREADS), 0, ps_st, src, fin, h->G, ntiles, ps.bk_fill,
                           h->NBK, ps.ctr, h->n_valid);
    } else if (h->passes == 1 && ntiles <= SMALL_TILES && !h->no_small) {  // one launch for the whole partition
      if (xmode)
        hipLaunchKernelGGL(k_radix_small<true>, dim3(1), dim3(RDX_THREADS), 0, ps_st, src, fin, h->G, shift, ntiles,
                           ps.bk_fill, h->NBK, ps.ctr, h->n_valid);
      else
        hipLaunchKernelGGL(k_radix_small<false>, dim3(1), dim3(RDX_THREADS), 0, ps_st, src, fin, h->G, shift, ntiles,
                           ps.bk_fill, h->NBK, ps.ctr, h->n_valid);
    }
    for (uint32_t p = 0; p < h->passes && !(h->passes == 1 && ntiles <= SMALL_TILES && !h->no_small); ++p) {
      const bool last_pass = p + 1 == h->passes;
      const RadixDst& dst = h->tmp[p & 1];
      // two passes split the bucket id's bits evenly (the first takes the low
      // half): 5 + 5 bits for 1,024 buckets write 64-message digit runs in both
      // passes, where 8 + 2 wrote 8-message runs (partial lines) in the first
      const uint32_t b0 = h->bk_bits / 2;
      const uint32_t dbits = h->passes == 1 ? RDX_BITS : p == 0 ? b0 : h->bk_bits - b0;
      const uint32_t dm = h->passes > 1;  // digit-major tile counts (k_scan_rows)
      const uint32_t nhw = (ntiles + HIST_TPB - 1) / HIST_TPB;
      const dim3 sg((ntiles + SCAT_TPW - 1) / SCAT_TPW);
      if (HB_RDX_DIRECT && h->passes == 1) {  // hist + direct scatter: no scan launch
        const uint32_t k = h->sup_k, kn = (k + 1) % SUP_BUFS;
        const size_t bw = (size_t)h->sup_max * RDX_BINS;
        DirectSums dsum{h->hagg, h->hsup + k * bw, h->hsup + kn * bw, h->sup_used[kn] * RDX_BINS,
                        ps.bk_fill, h->NBK, ps.ctr};
        h->sup_used[kn] = 0;
        h->sup_used[k] = (nhw + SB_HW - 1) / SB_HW;
        h->sup_k = kn;
        hipLaunchKernelGGL(k_radix_hist, dim3(nhw), dim3(RDX_THREADS), 0, ps_st, src, h->G, shift, dbits, ntiles, h->hist,
                           0u, dsum);
        if (xmode)
          hipLaunchKernelGGL(k_radix_scatter_d<true>, sg, dim3(RDX_THREADS), 0, ps_st, src, fin, h->G, shift, ntiles,
                             (const uint32_t*)h->hist, (const uint32_t*)h->hagg, (const uint32_t*)dsum.sup, h->n_valid);
        else
          hipLaunchKernelGGL(k_radix_scatter_d<false>, sg, dim3(RDX_THREADS), 0, ps_st, src, fin, h->G, shift, ntiles,
                             (const uint32_t*)h->hist, (const uint32_t*)h->hagg, (const uint32_t*)dsum.sup, h->n_valid);
        break;  // (one pass)
      }
      hipLaunchKernelGGL(k_radix_hist, dim3(nhw), dim3(RDX_THREADS), 0, ps_st, src, h->G, shift, dbits, ntiles, h->hist,
                         dm, DirectSums{});
      hipLaunchKernelGGL(k_scan_rows, dim3(1u << dbits), dim3(1024), 0, ps_st, h->hist, ntiles, dbits, h->totals, ps.bk_fill,
                         h->NBK, ps.ctr, dm);
#define HB_SCATTER(F, X)                                                                                             \
  hipLaunchKernelGGL((k_radix_scatter<F, X>), sg, dim3(RDX_THREADS), 0, ps_st, src, dst, fin, h->G, shift, dbits, ntiles, \
                     (const uint32_t*)h->hist, dm ? ntiles : 1u, dm ? 1u : (1u << dbits), (const uint32_t*)h->totals,    \
                     h->n_valid)
      if (last_pass) {
        if (xmode) HB_SCATTER(true, true);
        else HB_SCATTER(true, false);
      } else {
        if (xmode) HB_SCATTER(false, true);
        else HB_SCATTER(false, false);
      }
#undef HB_SCATTER
      src = RadixSrc{dst.group, nullptr, nullptr, nullptr, dst.rec, h->n_valid, nullptr, (uint32_t)b->n,
                     nullptr, nullptr, nullptr, nullptr, 0, dst.recx};
      shift += dbits;
    }
    if (h->passes > 1)
      hipLaunchKernelGGL(k_bucket_bounds, dim3((h->NBK + 1 + 255) / 256), dim3(256), 0, ps_st,
                         (const uint32_t*)ps.bucket, (const uint32_t*)h->n_valid, h->NBK, ps.bk_off);
  }

  // ---- phase 2: route each partition's messages to its lanes (prep stream) ----
  ApplyArgs aa{};
  aa.S = h->st;
  aa.S.edesc = bd_edesc;
  aa.S.eoff = bd_eoff;
  aa.S.peoff = bd_peoff;
  aa.S.bcommit = bd_commit;
  aa.S.eterm = bd_eterm;
  aa.S.n_ent = b->n_edesc;
  aa.S.bn = b->n;
  aa.ap_cnt = ps.ctr + CTR_AP;
  aa.ap_list = h->ap_list;
  aa.fl_cnt = ps.ctr + CTR_FL;
  aa.fl_list = h->fl_list;
  aa.eflag = h->eflag;
  aa.el_cnt = ps.ctr + CTR_EL;
  aa.el_list = h->el_list;
  aa.grid = apply_grid(h);
  aa.sis_log = h->sis_log;
  aa.done = ps.ctr + CTR_DONE;
  aa.stats = h->stats;
  aa.accum = h->stats_accum;
  aa.rec = ps.rec;
  aa.key = ps.key;
  aa.bk_off = ps.bk_off;
  aa.bk_fill = ps.bk_fill;
  aa.hint = bd.hint;
  aa.props = bd.props;
  aa.ev = h->ev;
  aa.ev_per_msg = h->ev_per_msg;
  aa.props_on = bd.props ? 1u : 0u;
  aa.NB = NB;
  aa.NBK = h->NBK;
  aa.ev_counts = ps.ev_counts;
  aa.ev_off = ps.ev_off;
  aa.stats_shard = h->stats_shard;
  aa.pflag = h->pflag;
  aa.resume = h->resume;
  aa.commit0 = h->commit0;
  aa.kmax = step_kmax(h->nmax, flags);
  aa.cnt = ps.cnt;
  aa.slot = ps.slot;
  aa.side = ps.side;
  aa.recx = ps.recx;
  aa.slotx = xmode ? ps.slotx : nullptr;
  aa.nmax = h->nmax;
  aa.lskip = h->lskip;
  // the route's storm hand-over writes the handle's flags and lists: only when
  // the apply of the previous step is not running beside it (one stream)
  aa.storm = (HB_ROUTE_STORM && h->nmax >= 5 && !two && !xmode && !bd.props) ? h->storm : 0u;
  // n = 3, prep and apply on one stream: the route runs inside the fast
  // kernel's workgroups (k_route_fast; two-pass handles too: cfg5 0.998 ->
  // 0.931 ms/step same box)
  const bool fused = HB_ROUTE_FAST && h->nmax == 3 && !two && (h->fuse >= 2 || (h->fuse == 1 && h->passes == 1)) &&
                     PART_LOG + h->sis_log >= route_fast_rg_log(aa.kmax, xmode);
  switch (h->nmax) {
    case 3:
      if (fused) break;
      if (aa.kmax == 3) launch_route<3>(h, aa, ps_st);
      else launch_route<2>(h, aa, ps_st);
      break;
    case 5: launch_route<route_kmax(5)>(h, aa, ps_st); break;
    default: launch_route<route_kmax(7)>(h, aa, ps_st); break;
  }
  if (prof) HB_CHECK(hipEventRecord(ev[1], ps_st));
  if (two) {
    HB_CHECK(hipEventRecord(ps.prepped, ps_st));
    // ---- phase 3: apply (apply stream, after the previous step's apply) ------
    HB_CHECK(hipStreamWaitEvent(st, ps.prepped, 0));
  }
  switch (h->nmax) {
    case 3: launch_apply<3>(h, aa, prof_apply ? ev : nullptr, prof, fused); break;
    case 5: launch_apply<5>(h, aa, prof_apply ? ev : nullptr, prof); break;
    default: launch_apply<7>(h, aa, prof_apply ? ev : nullptr, prof); break;
  }
  if (prof) HB_CHECK(hipEventRecord(ev[5], st));  // (the finish runs inside k_follow)
  if (two) HB_CHECK(hipEventRecord(ps.applied, st));
  HB_CHECK(hipGetLastError());
  ps.used = true;
  h->cur = h->next_set;
  h->next_set ^= 1;
  if (prof_apply) {
    h->prof_full[h->prof_n % hb_handle::PROF_RING] = prof;
    h->prof_n++;
  }
  h->stepped = true;
  h->kern = (fused ? HB_KERN_ROUTE_FAST : 0u) | (aa.storm >= 2 ? HB_KERN_ROUTE_ELECT : 0u);
  return HB_OK;
}

int hb_events_device(hb_handle* h, const uint64_t** base, const uint64_t** chunk_off, const uint32_t** counts,
                     uint32_t* n_chunks) {
  if (!h || !base || !chunk_off || !counts || !n_chunks) return HB_EINVAL;
  *base = h->ev;
  *chunk_off = h->set[h->cur].ev_off;
  *counts = h->set[h->cur].ev_counts;
  *n_chunks = 2 * h->NB;
  return HB_OK;
}

int hb_copy_events(hb_handle* h, hb_event* out, uint64_t cap, uint64_t* n) {
  if (!h || !n) return HB_EINVAL;
  DeviceGuard guard(h->device);
  HB_CHECK(hipMemcpyAsync(h->stats_pin, h->stats, HB_STAT_COUNT * 8, hipMemcpyDeviceToHost, h->stream));
  HB_CHECK(hipStreamSynchronize(h->stream));
  const uint64_t total = h->stepped ? h->stats_pin[HB_STAT_EVENTS] : 0;
  *n = total;
  if (total == 0) return HB_OK;
  if (!out || cap < total) return HB_EINVAL;
  // expansion scratch (records + per-chunk scan), kept across calls and grown on demand
  const uint64_t need = total * sizeof(hb_event) + 24ull * h->NB;
  if (need > h->evx_cap) {
    if (h->evx) (void)hipFree(h->evx);
    h->evx = nullptr;
    h->evx_cap = 0;
    const uint64_t cap = need + need / 4;
    HB_CHECK(hipMalloc(&h->evx, cap));
    h->evx_cap = cap;
  }
  hb_event* d = reinterpret_cast<hb_event*>(h->evx);
  uint64_t* dst = reinterpret_cast<uint64_t*>(d + total);
  uint32_t* per_chunk = reinterpret_cast<uint32_t*>(dst + 2 * h->NB);
  hipLaunchKernelGGL(k_chunk_events, dim3(2 * h->NB), dim3(256), 0, h->stream, (const uint64_t*)h->ev,
                     (const uint32_t*)h->set[h->cur].ev_counts, (const uint64_t*)h->set[h->cur].ev_off, per_chunk);
  hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, h->stream, (const uint32_t*)per_chunk, 2 * h->NB, dst);
  hipLaunchKernelGGL(k_expand_events, dim3(2 * h->NB), dim3(256), 0, h->stream, (const uint64_t*)h->ev,
                     (const uint32_t*)h->set[h->cur].ev_counts, (const uint64_t*)h->set[h->cur].ev_off, (const uint64_t*)dst, d);
  hipError_t e = hipMemcpyAsync(out, d, total * sizeof(hb_event), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  return e == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_events_to_host(hb_handle* h, uint64_t* words, uint64_t cap, uint32_t* counts, uint64_t* total) {
  if (!h || !counts || !total || (cap && !words)) return HB_EINVAL;
  DeviceGuard guard(h->device);
  void *dw = nullptr, *dc = nullptr, *dt = nullptr;
  if (hipHostGetDevicePointer(&dc, counts, 0) != hipSuccess || hipHostGetDevicePointer(&dt, total, 0) != hipSuccess ||
      (cap && hipHostGetDevicePointer(&dw, words, 0) != hipSuccess))
    return HB_EINVAL;  // not memory from hb_alloc_pinned
  const uint32_t nc = 2 * h->NB;
  if (!h->stepped) {  // no step yet: no events
    HB_CHECK(hipMemsetAsync(dc, 0, nc * 4ull, h->stream));
    HB_CHECK(hipMemsetAsync(dt, 0, 8, h->stream));
    return HB_OK;
  }
  if (h->evw_cap < nc + 1ull) {
    if (h->evw) (void)hipFree(h->evw);
    h->evw = nullptr;
    h->evw_cap = 0;
    HB_CHECK(hipMalloc(&h->evw, (nc + 1ull) * 8));
    h->evw_cap = nc + 1ull;
  }
  const PrepSet& ps = h->set[h->cur];
  if (nc <= WORDS_SMALL && !h->no_small) {
    hipLaunchKernelGGL(k_words_small, dim3(1), dim3(1024), 0, h->stream, (const uint32_t*)ps.ev_counts, nc,
                       (const uint64_t*)h->ev, (const uint64_t*)ps.ev_off, static_cast<uint64_t*>(dw), cap,
                       static_cast<uint32_t*>(dc), static_cast<uint64_t*>(dt));
    return hipGetLastError() == hipSuccess ? HB_OK : HB_EDEVICE;
  }
  hipLaunchKernelGGL(k_scan_words, dim3(1), dim3(1024), 0, h->stream, (const uint32_t*)ps.ev_counts, nc, h->evw,
                     static_cast<uint32_t*>(dc), static_cast<uint64_t*>(dt));
  hipLaunchKernelGGL(k_gather_words, dim3(nc), dim3(256), 0, h->stream, (const uint64_t*)h->ev,
                     (const uint32_t*)ps.ev_counts, (const uint64_t*)ps.ev_off, (const uint64_t*)h->evw,
                     static_cast<uint64_t*>(dw), cap);
  return hipGetLastError() == hipSuccess ? HB_OK : HB_EDEVICE;
}

int hb_event_words_chunks(hb_handle* h, uint32_t* n_chunks, uint32_t* groups_per_chunk) {
  if (!h || !n_chunks) return HB_EINVAL;
  *n_chunks = 2 * h->NB;
  if (groups_per_chunk) *groups_per_chunk = PART;
  return HB_OK;
}

int hb_expand_event_words(const uint64_t* words, uint64_t n_words, const uint32_t* counts, uint32_t n_chunks,
                          hb_event* out, uint64_t cap, uint64_t* n_out) {
  if (!n_out || (n_words && (!words || !counts))) return HB_EINVAL;
  uint64_t k = 0, w = 0;
  for (uint32_t c = 0; c < n_chunks; ++c) {
    const uint64_t end = w + counts[c];
    if (end > n_words) return HB_EINVAL;
    for (; w < end; ++w) {
      const uint64_t x0 = words[w];
      const uint32_t type = (uint32_t)x0 & 0xF;
      if (type == EVC_CONT) continue;
      const uint32_t to = (uint32_t)(x0 >> 4) & 0x7F, aux = (uint32_t)(x0 >> 12) & 0xF;
      const uint32_t group = (c >> 1) * PART + ((uint32_t)(x0 >> 16) & 0xFF);
      uint64_t x = x0 >> 24;
      if (((x0 >> 11) & 1u) && w + 1 < end) x |= (words[w + 1] >> 4) << 40;
      if (type == EVC_BCAST || type == EVC_VBCAST) {
        const uint8_t et = type == EVC_BCAST ? (uint8_t)HB_EV_APP : (uint8_t)HB_EV_VOTE;
        for (uint32_t s = 0; s < 7; ++s)
          if ((to >> s) & 1u) {
            if (out && k < cap) out[k] = hb_event{x, group, et, (uint8_t)s, (uint16_t)aux};
            ++k;
          }
      } else {
        if (out && k < cap) out[k] = hb_event{x, group, (uint8_t)type, (uint8_t)to, (uint16_t)aux};
        ++k;
      }
    }
  }
  *n_out = k;
  return (out && k > cap) ? HB_EINVAL : HB_OK;
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
  HB_CHECK(hipStreamSynchronize(h->prep));
  HB_CHECK(hipStreamSynchronize(h->stream));
  // (start, end) event of each phase in h->ph[k]
  static const int span[HB_PHASE_COUNT][2] = {{0, 1}, {2, 3}, {3, 4}, {4, 5}};
  uint32_t nfull = 0;
  for (uint32_t k = 0; k < n; ++k) nfull += h->prof_full[k] ? 1u : 0u;
  for (uint32_t k = 0; k < n; ++k) {
    for (int i = 0; i < HB_PHASE_COUNT; ++i) {
      if (i != HB_PHASE_APPLY && !h->prof_full[k]) continue;
      float ms = 0.f;
      HB_CHECK(hipEventElapsedTime(&ms, h->ph[k][span[i][0]], h->ph[k][span[i][1]]));
      out[i] += ms / (float)(i == HB_PHASE_APPLY ? n : nfull);
    }
  }
  return HB_OK;
}

int hb_step_kernels(hb_handle* h, uint32_t* mask) {
  if (!h || !mask) return HB_EINVAL;
  *mask = h->kern;
  return HB_OK;
}

int hb_phase_reset(hb_handle* h) {
  if (!h) return HB_EINVAL;
  h->prof_n = 0;
  return HB_OK;
}

int hb_set_stats_accum(hb_handle* h, uint64_t* dev_accum) {
  if (!h) return HB_EINVAL;
  h->stats_accum = dev_accum;
  return HB_OK;
}

int hb_set_input_stream(hb_handle* h, void* stream) {
  if (!h) return HB_EINVAL;
  h->in_stream = reinterpret_cast<hipStream_t>(stream);
  h->in_stream_set = true;
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
