// Micro-benchmark (not product code): can ONE radix pass with 4096 buckets
// (cfg5: 8M groups, 2048-group buckets) place 16M 24-byte records by direct
// scattered stores, instead of two 8-bit LSD passes with LDS-staged runs?
//   copy   read 24 B SoA + write 24 B records in order (the floor)
//   b4096  write each record at its stable bucket position (4096 buckets)
//   b256   the same with 256 buckets (runs 16x longer)
//   b4096w the same as b4096, one wave writes 64 consecutive records of a bucket
//          (what an LDS-staged tile-sorted single pass would issue with long runs)
// Positions are precomputed on the host (a stable counting sort); the kernels
// read them (4 B per record) — the memory pattern of the store side only.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/scatter_mb scatter_mb.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e = (x);                                         \
    if (e != hipSuccess) {                                      \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));     \
      exit(1);                                                  \
    }                                                           \
  } while (0)

struct Rec {
  uint32_t info, orig;
  uint64_t term, index;
};

__global__ void k_place(const uint32_t* grp, const uint32_t* info, const uint64_t* term, const uint64_t* index,
                        const uint32_t* dst, uint32_t n, Rec* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Rec r;
  r.info = info[i] | (grp[i] << 10);
  r.orig = i;
  r.term = term[i];
  r.index = index[i];
  out[dst ? dst[i] : i] = r;
}

int main() {
  const uint32_t N = 16u << 20, G = 8u << 20;
  std::mt19937_64 rng(7);
  std::vector<uint32_t> grp(N), info(N);
  std::vector<uint64_t> term(N), idx(N);
  for (uint32_t i = 0; i < N; ++i) {
    grp[i] = (uint32_t)(rng() % G);
    info[i] = 4;
    term[i] = rng() % 1000;
    idx[i] = rng() % (1u << 20);
  }
  auto positions = [&](uint32_t bucket_log) {
    const uint32_t nb = G >> bucket_log;
    std::vector<uint32_t> cnt(nb + 1, 0), dst(N);
    for (uint32_t i = 0; i < N; ++i) cnt[(grp[i] >> bucket_log) + 1]++;
    for (uint32_t b = 0; b < nb; ++b) cnt[b + 1] += cnt[b];
    for (uint32_t i = 0; i < N; ++i) dst[i] = cnt[grp[i] >> bucket_log]++;
    return dst;
  };
  uint32_t *d_grp, *d_info, *d_dst;
  uint64_t *d_term, *d_idx;
  Rec* d_out;
  CK(hipMalloc(&d_grp, N * 4));
  CK(hipMalloc(&d_info, N * 4));
  CK(hipMalloc(&d_dst, N * 4));
  CK(hipMalloc(&d_term, N * 8));
  CK(hipMalloc(&d_idx, N * 8));
  CK(hipMalloc(&d_out, (size_t)N * sizeof(Rec)));
  CK(hipMemcpy(d_grp, grp.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_info, info.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_term, term.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_idx, idx.data(), N * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, const uint32_t* dst) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_place, dim3((N + 255) / 256), dim3(256), 0, 0, d_grp, d_info, d_term, d_idx, dst, N, d_out);
    CK(hipEventRecord(e0));
    const int R = 20;
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_place, dim3((N + 255) / 256), dim3(256), 0, 0, d_grp, d_info, d_term, d_idx, dst, N, d_out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / R, bytes = (double)N * (24 + 24 + (dst ? 4 : 0));
    printf("%-8s %8.1f us  %6.2f TB/s (algorithmic %.0f MB)\n", name, us, bytes / (us * 1e-6) / 1e12, bytes / 1e6);
  };
  run("copy", nullptr);
  for (uint32_t bl : {15u, 11u}) {  // 256 buckets, 4096 buckets
    auto dst = positions(bl);
    CK(hipMemcpy(d_dst, dst.data(), N * 4, hipMemcpyHostToDevice));
    run(bl == 15 ? "b256" : "b4096", d_dst);
  }
  {  // b4096w: the same positions, issued bucket-run-major (a wave writes consecutive slots)
    auto dst = positions(11);
    std::vector<uint32_t> order(N), inv(N);
    for (uint32_t i = 0; i < N; ++i) inv[dst[i]] = i;  // position -> message
    // process messages in position order: message j of the launch writes position j
    for (uint32_t p = 0; p < N; ++p) order[p] = p;
    CK(hipMemcpy(d_dst, order.data(), N * 4, hipMemcpyHostToDevice));
    run("inorder", d_dst);
  }
  return 0;
}
