// Micro-benchmark (not product code): costs of placing a batch of 2M random
// messages into per-group slots on MI355X, to choose the prep design.
//   A  returning device-scope atomicAdd per message on cnt[g] + SoA slot stores
//   B  same, AoS 32-byte slot records [g][k] (one 2 x 16-byte store per message)
//   C  AoS records placed by the message's `from` slot (no atomic)
//   D  streaming copy of the batch (read 24 B, write 24 B per message): the floor
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/route_mb route_mb.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));                   \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

struct Rec32 {
  uint32_t info, orig;
  uint64_t term, index, pad;
};

__global__ void kA(const uint32_t* grp, const uint32_t* info, const uint64_t* term, const uint64_t* index, uint32_t n,
                   uint32_t G, uint32_t* cnt, uint32_t* s_info, uint32_t* s_orig, uint64_t* s_term, uint64_t* s_index) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = grp[i];
  const uint32_t r = atomicAdd(&cnt[g], 1u);
  if (r < 2) {
    const size_t o = (size_t)r * G + g;
    s_info[o] = info[i];
    s_orig[o] = i;
    s_term[o] = term[i];
    s_index[o] = index[i];
  }
}

__global__ void kB(const uint32_t* grp, const uint32_t* info, const uint64_t* term, const uint64_t* index, uint32_t n,
                   uint32_t* cnt, Rec32* slots) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = grp[i];
  const uint32_t r = atomicAdd(&cnt[g], 1u);
  if (r < 2) {
    Rec32 x;
    x.info = info[i];
    x.orig = i;
    x.term = term[i];
    x.index = index[i];
    x.pad = 0;
    slots[(size_t)g * 2 + r] = x;
  }
}

__global__ void kC(const uint32_t* grp, const uint32_t* info, const uint64_t* term, const uint64_t* index, uint32_t n,
                   Rec32* slots) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = grp[i];
  const uint32_t f = ((info[i] >> 4) & 0xF) - 1;
  Rec32 x;
  x.info = info[i];
  x.orig = i;
  x.term = term[i];
  x.index = index[i];
  x.pad = 0;
  slots[(size_t)g * 2 + (f & 1)] = x;
}

__global__ void kD(const uint32_t* grp, const uint32_t* info, const uint64_t* term, const uint64_t* index, uint32_t n,
                   uint32_t* o_grp, uint32_t* o_info, uint64_t* o_term, uint64_t* o_index) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o_grp[i] = grp[i];
  o_info[i] = info[i];
  o_term[i] = term[i];
  o_index[i] = index[i];
}

int main(int argc, char** argv) {
  const uint32_t G = argc > 1 ? atoi(argv[1]) : (1u << 20);
  const uint32_t n = 2 * G;
  std::vector<uint32_t> hg(n), hi(n);
  std::vector<uint64_t> ht(n), hx(n);
  for (uint32_t i = 0; i < n; ++i) {
    hg[i] = i / 2;
    hi[i] = 4u | ((1u + (i & 1)) << 4);
  }
  uint64_t s = 12345;
  for (uint32_t i = n - 1; i > 0; --i) {  // shuffle
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t j = (uint32_t)((s >> 33) % (i + 1));
    std::swap(hg[i], hg[j]);
    std::swap(hi[i], hi[j]);
  }
  for (uint32_t i = 0; i < n; ++i) {
    ht[i] = 7;
    hx[i] = 1000 + hg[i];
  }
  uint32_t *dg, *di, *cnt, *si, *so, *og, *oi;
  uint64_t *dt, *dx, *st, *sx, *ot, *ox;
  Rec32* rec;
  CK(hipMalloc(&dg, n * 4));
  CK(hipMalloc(&di, n * 4));
  CK(hipMalloc(&dt, n * 8));
  CK(hipMalloc(&dx, n * 8));
  CK(hipMalloc(&cnt, G * 4));
  CK(hipMalloc(&si, 2ull * G * 4));
  CK(hipMalloc(&so, 2ull * G * 4));
  CK(hipMalloc(&st, 2ull * G * 8));
  CK(hipMalloc(&sx, 2ull * G * 8));
  CK(hipMalloc(&rec, 2ull * G * sizeof(Rec32)));
  CK(hipMalloc(&og, n * 4));
  CK(hipMalloc(&oi, n * 4));
  CK(hipMalloc(&ot, n * 8));
  CK(hipMalloc(&ox, n * 8));
  CK(hipMemcpy(dg, hg.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(di, hi.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, ht.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, hx.data(), n * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 blk(256), grd((n + 255) / 256);
  const int R = 20;
  for (int v = 0; v < 4; ++v) {
    float best = 1e9, sum = 0;
    for (int r = 0; r < R + 3; ++r) {
      if (v < 2) CK(hipMemset(cnt, 0, G * 4));
      CK(hipEventRecord(e0, 0));
      if (v == 0) hipLaunchKernelGGL(kA, grd, blk, 0, 0, dg, di, dt, dx, n, G, cnt, si, so, st, sx);
      if (v == 1) hipLaunchKernelGGL(kB, grd, blk, 0, 0, dg, di, dt, dx, n, cnt, rec);
      if (v == 2) hipLaunchKernelGGL(kC, grd, blk, 0, 0, dg, di, dt, dx, n, rec);
      if (v == 3) hipLaunchKernelGGL(kD, grd, blk, 0, 0, dg, di, dt, dx, n, og, oi, ot, ox);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) {
        sum += ms;
        if (ms < best) best = ms;
      }
    }
    const char* nm[] = {"A atomic+SoA", "B atomic+AoS32", "C from-slot AoS32", "D stream copy"};
    printf("%-20s G=%u n=%u  avg %.1f us  best %.1f us\n", nm[v], G, n, 1e3 * sum / R, 1e3 * best);
  }
  // check A placed every message
  std::vector<uint32_t> hc(G);
  CK(hipMemcpy(hc.data(), cnt, G * 4, hipMemcpyDeviceToHost));
  uint64_t tot = 0;
  for (uint32_t g = 0; g < G; ++g) tot += hc[g];
  printf("check: sum cnt = %llu (n = %u)\n", (unsigned long long)tot, n);
  return 0;
}
