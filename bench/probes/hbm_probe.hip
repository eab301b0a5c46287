// HBM roofline probes (standalone; not part of the dalgo extension).
//
// Anchors the HBM read rate the K1 SSGD gradient (csrc/kernels/lr_grad.hip) is measured
// against, independently of the library: a device-to-device hipMemcpy and a contiguous
// streaming read over >= 8 GB, and the access shape of the SGD minibatch (10 % of the
// 2-KB rows of a 10M x 1024 bf16 matrix, sorted) read by plain / non-temporal loads.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../csrc/include hbm_probe.hip -o hbm_probe
// run:   ./hbm_probe [GB=16]     prints one JSON line per probe (GB/s)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>
#include "dalgo/common.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

namespace dalgo {
// HBM read-roofline probe (diagnostics): every 16 B of [p, p+n16*16) read once with
// dwordx4 loads, UNROLL loads in flight per lane, xor-folded into one word per
// block so the loads cannot be dead-code eliminated.
template <int UNROLL>
__global__ void __launch_bounds__(256)
hbm_read_kernel(const uint4* __restrict__ p, int64_t n16, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) { uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  acc = wave_sum_u32(acc);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

// Probe variant: block b streams its own contiguous region [b*n/G, (b+1)*n/G)
// (the access shape of a row-sharded sweep), UNROLL x 16 B in flight per lane.
template <int UNROLL>
__global__ void __launch_bounds__(256)
hbm_read_blocked_kernel(const uint4* __restrict__ p, int64_t n16, uint32_t* __restrict__ out) {
  const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = min(n16, lo + per);
  uint32_t acc = 0;
  int64_t i = lo + threadIdx.x;
  for (; i + (UNROLL - 1) * 256 < hi; i += UNROLL * 256) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = p[i + u * 256];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < hi; i += 256) { uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  acc = wave_sum_u32(acc);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

// Probe: the access shape of the SGD minibatch (a sorted list of selected 2-KB rows,
// ~10 % of the matrix): each wave streams whole rows, 4 rows (8 KB) in flight per
// wave; the ceiling any K1 design can reach for this pattern.
__global__ void __launch_bounds__(256)
hbm_gather_rows_kernel(const uint4* __restrict__ X, int64_t ld16, const int* __restrict__ idx,
                       int64_t nidx, uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  uint32_t acc = 0;
  for (; w < nidx; w += 4 * nw) {
    uint4 v[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t k = min(w + u * nw, nidx - 1);
      const uint4* row = X + (int64_t)idx[k] * ld16;
      v[u][0] = row[lane];
      v[u][1] = row[64 + lane];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      acc ^= v[u][0].x ^ v[u][0].w ^ v[u][1].y ^ v[u][1].z;
  }
  acc = wave_sum_u32(acc);
  if ((threadIdx.x & 63) == 0) atomicXor(out, acc);
}

// Probe variants of the same access shape: NT = nt loads into registers, and LDS-DMA
// (global_load_lds_dwordx4, nt or default policy) into a per-wave ring of DEPTH rows
// (2 KB each), each row read back from LDS once — the load path a K1 built on LDS-DMA
// would use. Each wave streams a contiguous slice of idx; the slice's row ids are
// staged in LDS first, so no ordinary VMEM load interleaves with the counted DMA waits.
template <bool NT>
__global__ void __launch_bounds__(256)
hbm_gather_rows_nt_kernel(const uint4* __restrict__ X, int64_t ld16, const int* __restrict__ idx,
                          int64_t nidx, uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  uint32_t acc = 0;
  typedef int v4i __attribute__((ext_vector_type(4)));
  for (; w < nidx; w += 4 * nw) {
    v4i v[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t k = min(w + u * nw, nidx - 1);
      const v4i* row = reinterpret_cast<const v4i*>(X + (int64_t)idx[k] * ld16);
      if constexpr (NT) {
        v[u][0] = __builtin_nontemporal_load(row + lane);
        v[u][1] = __builtin_nontemporal_load(row + 64 + lane);
      } else {
        v[u][0] = row[lane];
        v[u][1] = row[64 + lane];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u][0].x ^ v[u][0].w ^ v[u][1].y ^ v[u][1].z;
  }
  acc = wave_sum_u32(acc);
  if ((threadIdx.x & 63) == 0) atomicXor(out, acc);
}

}  // namespace dalgo

using namespace dalgo;

template <class F>
static double time_ms(F f, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();                                   // warm
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 16.0;
  const size_t nbytes = (size_t)(gb * 1e9) / 4096 * 4096;
  void *src = nullptr, *dst = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&src, nbytes));
  CK(hipMalloc(&dst, nbytes / 2));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(src, 1, nbytes));
  const int64_t n16 = nbytes / 16;
  // 1. D2D copy of half the buffer: reads + writes
  double ms = time_ms([&] { CK(hipMemcpyAsync(dst, src, nbytes / 2, hipMemcpyDeviceToDevice, 0)); }, 5);
  printf("{\"probe\": \"hipMemcpy D2D\", \"GB\": %.2f, \"read_GBps\": %.1f, \"rw_GBps\": %.1f}\n",
         nbytes / 2 / 1e9, nbytes / 2 / ms / 1e6, nbytes / ms / 1e6);
  // 2. streaming read, grid-stride and blocked-region forms
  for (int grid : {1024, 2048, 4096, 8192}) {
    ms = time_ms([&] { hipLaunchKernelGGL(hbm_read_kernel<8>, dim3(grid), dim3(256), 0, 0,
                                          (const uint4*)src, n16, out); }, 5);
    printf("{\"probe\": \"read grid-stride\", \"grid\": %d, \"GB\": %.2f, \"GBps\": %.1f}\n", grid,
           nbytes / 1e9, nbytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL(hbm_read_blocked_kernel<8>, dim3(grid), dim3(256), 0, 0,
                                          (const uint4*)src, n16, out); }, 5);
    printf("{\"probe\": \"read blocked\", \"grid\": %d, \"GB\": %.2f, \"GBps\": %.1f}\n", grid,
           nbytes / 1e9, nbytes / ms / 1e6);
  }
  // 3. SGD minibatch shape: sorted 10 % of 2-KB rows (10M x 1024 bf16 = 20.5 GB needs gb >= 20.5;
  //    otherwise as many rows as fit)
  const int64_t rows = std::min<int64_t>(10000000, (int64_t)(nbytes / 2048));
  std::vector<int> sel;
  std::mt19937_64 rng(42);
  for (int64_t r = 0; r < rows; ++r) if ((rng() % 10) == 0) sel.push_back((int)r);
  int* dsel = nullptr;
  CK(hipMalloc(&dsel, sel.size() * sizeof(int)));
  CK(hipMemcpy(dsel, sel.data(), sel.size() * sizeof(int), hipMemcpyHostToDevice));
  const double sel_bytes = (double)sel.size() * 2048;
  for (int grid : {2048, 4096, 8192}) {
    ms = time_ms([&] { hipLaunchKernelGGL(hbm_gather_rows_kernel, dim3(grid), dim3(256), 0, 0,
                                          (const uint4*)src, (int64_t)128, dsel, (int64_t)sel.size(), out); }, 10);
    printf("{\"probe\": \"gather 10%% rows\", \"grid\": %d, \"rows\": %zu, \"GBps\": %.1f}\n", grid,
           sel.size(), sel_bytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL(hbm_gather_rows_nt_kernel<true>, dim3(grid), dim3(256), 0, 0,
                                          (const uint4*)src, (int64_t)128, dsel, (int64_t)sel.size(), out); }, 10);
    printf("{\"probe\": \"gather 10%% rows nt\", \"grid\": %d, \"rows\": %zu, \"GBps\": %.1f}\n", grid,
           sel.size(), sel_bytes / ms / 1e6);
  }
  CK(hipFree(src)); CK(hipFree(dst)); CK(hipFree(out)); CK(hipFree(dsel));
  return 0;
}
