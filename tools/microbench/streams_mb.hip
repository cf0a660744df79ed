// Micro-benchmark (not product code): does the number of separate arrays a
// lane touches bound the apply kernels' HBM rate?  k_apply_fast / k_route_fast
// read ~20 and write ~12 per-group fields, each its own [G] array (SoA), and
// run at ~4 TB/s where a streaming copy reaches ~6 TB/s.  Same bytes per lane
// (160 B read, 96 B written, u64 fields), 1M lanes, 256-lane workgroups:
//   soa1   20 read arrays + 12 written arrays, every load in one round trip
//   soa2   the same, the second 10 loads issued after the first 10 arrived
//          (the fast lane's two round trips)
//   tile1  the same fields, partition-major: [G/256][field][256] (a
//          workgroup's fields are one contiguous 64 KB block), one round trip
//   tile2  tile layout, two round trips
//   copy   a plain copy of 160 B per lane into a 96 B-per-lane output
// Each kernel is timed over 50 launches with HIP events.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/streams_mb tools/microbench/streams_mb.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s failed: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                              \
    }                                                       \
  } while (0)

constexpr uint32_t G = 1u << 20;
constexpr int NR = 20, NW = 12, PARTS = 256;

struct Arr {
  uint64_t* r[NR];
  uint64_t* w[NW];
};

// field f of lane g: SoA -> base[f][g]; tile -> base[(g / 256)][f][g % 256]
template <bool TILE>
__device__ __forceinline__ uint64_t* at(uint64_t* base, int f, int nf, uint32_t g) {
  if (TILE) return base + ((size_t)(g / PARTS) * nf + f) * PARTS + (g % PARTS);
  return base + (size_t)f * G + g;
}

template <bool TILE, bool TWO>
__global__ void __launch_bounds__(256, 4) k_fields(uint64_t* rb, uint64_t* wb, uint64_t key) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  uint64_t v[NR];
#pragma unroll
  for (int f = 0; f < NR / 2; ++f) v[f] = *at<TILE>(rb, f, NR, g);
  uint64_t s = 0;
  if (TWO) {
#pragma unroll
    for (int f = 0; f < NR / 2; ++f) s += v[f];
    if (s == key) return;  // (never: makes the second round depend on the first)
  }
#pragma unroll
  for (int f = NR / 2; f < NR; ++f) v[f] = *at<TILE>(rb, f, NR, g);
#pragma unroll
  for (int f = 0; f < NR; ++f) s ^= v[f] * (f + 1);
#pragma unroll
  for (int f = 0; f < NW; ++f) *at<TILE>(wb, f, NW, g) = s + f;
}

__global__ void __launch_bounds__(256, 4) k_copy(const uint4* in, uint4* out) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  uint4 v[10];
#pragma unroll
  for (int f = 0; f < 10; ++f) v[f] = in[(size_t)f * G + g];
  uint32_t s = 0;
#pragma unroll
  for (int f = 0; f < 10; ++f) s ^= v[f].x + v[f].y + v[f].z + v[f].w;
#pragma unroll
  for (int f = 0; f < 6; ++f) out[(size_t)f * G + g] = make_uint4(s, f, s, f);
}

int main() {
  uint64_t *rb, *wb;
  CK(hipMalloc(&rb, (size_t)NR * G * 8));
  CK(hipMalloc(&wb, (size_t)NW * G * 8));
  CK(hipMemset(rb, 1, (size_t)NR * G * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)G * (NR + NW) * 8;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 5; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 50; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 50;
    printf("%-6s %8.2f us  %7.0f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  const dim3 grid(G / 256), blk(256);
  run("soa1", [&] { hipLaunchKernelGGL((k_fields<false, false>), grid, blk, 0, 0, rb, wb, 7ull); });
  run("soa2", [&] { hipLaunchKernelGGL((k_fields<false, true>), grid, blk, 0, 0, rb, wb, 7ull); });
  run("tile1", [&] { hipLaunchKernelGGL((k_fields<true, false>), grid, blk, 0, 0, rb, wb, 7ull); });
  run("tile2", [&] { hipLaunchKernelGGL((k_fields<true, true>), grid, blk, 0, 0, rb, wb, 7ull); });
  run("copy", [&] {
    hipLaunchKernelGGL(k_copy, grid, blk, 0, 0, reinterpret_cast<const uint4*>(rb), reinterpret_cast<uint4*>(wb));
  });
  CK(hipFree(rb));
  CK(hipFree(wb));
  return 0;
}
