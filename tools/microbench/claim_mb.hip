// Micro-benchmark (not product code): can the cfg2 prep (hist + scan + two-tile
// scatter + route: ~51 us for 2M MsgAppResp over 1M groups) be replaced by a
// DIRECT CLAIM — each message takes its rank among its group's messages with a
// returning atomicAdd on a per-group counter and writes its 16-byte record
// straight into the lane-major slot k of its group (the layout k_apply_fast
// reads)?  VERDICT r04 item 4.  Variants, same 2M messages and 1M groups:
//   copy     read the 24 B SoA batch, write 16 B records in order (the floor)
//   claim    arrival order: atomicAdd(cnt[g]) + slot[k][g] store per message
//   claim_s  the same over a batch pre-sorted by 4096-group bucket (what a
//            scatter tile staged in LDS would issue): stores land in a bucket's
//            64 KB window per slot row
//   claim_l  arrival order, the counter claim done in LDS by a workgroup that
//            owns a 4096-group bucket and reads only its messages (positions
//            precomputed: the route kernel's pattern minus the sorted input)
// Every variant clears the counters first (one memset, timed with it).  Each
// kernel is timed over 50 launches with HIP events.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/claim_mb tools/microbench/claim_mb.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s failed: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                              \
    }                                                       \
  } while (0)

constexpr uint32_t KMAX = 2;

__global__ void k_copy(const uint32_t* grp, const uint32_t* info, const uint64_t* term, const uint64_t* index,
                       uint32_t n, uint4* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t ti = index[i] | (term[i] << 40);
  out[i] = make_uint4(info[i] | ((grp[i] & 255u) << 16), i, (uint32_t)ti, (uint32_t)(ti >> 32));
}

__global__ void k_claim(const uint32_t* grp, const uint32_t* info, const uint64_t* term, const uint64_t* index,
                        uint32_t n, uint32_t G, uint32_t* cnt, uint4* slot) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = grp[i];
  const uint64_t ti = index[i] | (term[i] << 40);
  const uint32_t k = atomicAdd(&cnt[g], 1u);
  if (k < KMAX) slot[(size_t)k * G + g] = make_uint4(info[i] | ((g & 255u) << 16), i, (uint32_t)ti, (uint32_t)(ti >> 32));
}

// one workgroup per 4096-group bucket: its messages' positions in the batch
// (precomputed, arrival order), counters in LDS, slots written per message
__global__ void __launch_bounds__(1024) k_claim_lds(const uint32_t* grp, const uint32_t* info, const uint64_t* term,
                                                    const uint64_t* index, const uint32_t* pos,
                                                    const uint32_t* bk_off, uint32_t G, uint4* slot) {
  __shared__ uint32_t c[4096];
  for (uint32_t j = threadIdx.x; j < 4096; j += blockDim.x) c[j] = 0;
  __syncthreads();
  const uint32_t lo = bk_off[blockIdx.x], hi = bk_off[blockIdx.x + 1];
  for (uint32_t p = lo + threadIdx.x; p < hi; p += blockDim.x) {
    const uint32_t i = pos[p];
    const uint32_t g = grp[i];
    const uint64_t ti = index[i] | (term[i] << 40);
    const uint32_t k = atomicAdd(&c[g & 4095u], 1u);
    if (k < KMAX) slot[(size_t)k * G + g] = make_uint4(info[i] | ((g & 255u) << 16), i, (uint32_t)ti, (uint32_t)(ti >> 32));
  }
}

int main() {
  const uint32_t G = 1u << 20, N = 2u << 20;
  std::mt19937_64 rng(11);
  std::vector<uint32_t> grp(N), info(N, 4u | (1u << 4));
  std::vector<uint64_t> term(N), idx(N);
  {  // every group acked by both followers, in a random permutation (the cfg2 stream)
    std::vector<uint32_t> perm(N);
    std::iota(perm.begin(), perm.end(), 0u);
    std::shuffle(perm.begin(), perm.end(), rng);
    for (uint32_t i = 0; i < N; ++i) grp[i] = perm[i] >> 1;
  }
  for (uint32_t i = 0; i < N; ++i) {
    term[i] = 1 + rng() % 1000;
    idx[i] = 1 + rng() % (1u << 20);
  }
  // bucket-sorted copy (stable) and per-bucket positions
  const uint32_t NB = G >> 12;
  std::vector<uint32_t> bk_off(NB + 1, 0), pos(N);
  for (uint32_t i = 0; i < N; ++i) bk_off[(grp[i] >> 12) + 1]++;
  for (uint32_t b = 0; b < NB; ++b) bk_off[b + 1] += bk_off[b];
  {
    std::vector<uint32_t> fill(bk_off.begin(), bk_off.end() - 1);
    for (uint32_t i = 0; i < N; ++i) pos[fill[grp[i] >> 12]++] = i;
  }
  std::vector<uint32_t> sgrp(N), sinfo(N);
  std::vector<uint64_t> sterm(N), sidx(N);
  for (uint32_t p = 0; p < N; ++p) {
    sgrp[p] = grp[pos[p]];
    sinfo[p] = info[pos[p]];
    sterm[p] = term[pos[p]];
    sidx[p] = idx[pos[p]];
  }
  auto up = [](const auto& v) {
    void* d = nullptr;
    CK(hipMalloc(&d, v.size() * sizeof(v[0])));
    CK(hipMemcpy(d, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice));
    return d;
  };
  auto* dg = (uint32_t*)up(grp);
  auto* di = (uint32_t*)up(info);
  auto* dt = (uint64_t*)up(term);
  auto* dx = (uint64_t*)up(idx);
  auto* sg = (uint32_t*)up(sgrp);
  auto* si = (uint32_t*)up(sinfo);
  auto* st = (uint64_t*)up(sterm);
  auto* sx = (uint64_t*)up(sidx);
  auto* dpos = (uint32_t*)up(pos);
  auto* dbk = (uint32_t*)up(bk_off);
  uint32_t* cnt = nullptr;
  uint4 *slot = nullptr, *out = nullptr;
  CK(hipMalloc(&cnt, G * 4ull));
  CK(hipMalloc(&slot, (size_t)KMAX * G * 16));
  CK(hipMalloc(&out, (size_t)N * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto&& launch) {
    for (int w = 0; w < 5; ++w) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 50; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-8s %8.2f us per step\n", name, ms * 1e3 / 50);
  };
  const uint32_t tb = 256, nbk = (N + tb - 1) / tb;
  timeit("copy", [&] { hipLaunchKernelGGL(k_copy, dim3(nbk), dim3(tb), 0, 0, dg, di, dt, dx, N, out); });
  timeit("memset", [&] { CK(hipMemsetAsync(cnt, 0, G * 4ull)); });
  timeit("claim", [&] {
    CK(hipMemsetAsync(cnt, 0, G * 4ull));
    hipLaunchKernelGGL(k_claim, dim3(nbk), dim3(tb), 0, 0, dg, di, dt, dx, N, G, cnt, slot);
  });
  timeit("claim_s", [&] {
    CK(hipMemsetAsync(cnt, 0, G * 4ull));
    hipLaunchKernelGGL(k_claim, dim3(nbk), dim3(tb), 0, 0, sg, si, st, sx, N, G, cnt, slot);
  });
  timeit("claim_l", [&] {
    hipLaunchKernelGGL(k_claim_lds, dim3(NB), dim3(1024), 0, 0, dg, di, dt, dx, dpos, dbk, G, slot);
  });
  // check: every group's two slots hold its two messages (claim, arrival order input)
  CK(hipMemset(cnt, 0, G * 4ull));
  hipLaunchKernelGGL(k_claim, dim3(nbk), dim3(tb), 0, 0, dg, di, dt, dx, N, G, cnt, slot);
  std::vector<uint32_t> hc(G);
  CK(hipMemcpy(hc.data(), cnt, G * 4ull, hipMemcpyDeviceToHost));
  uint64_t bad = 0;
  for (uint32_t g = 0; g < G; ++g) bad += hc[g] != 2;
  printf("groups with a count other than 2: %llu\n", (unsigned long long)bad);
  return 0;
}
