// Counter-based random generation on device:
//   * philox_fill — synthetic data generator (uniform / normal), index-keyed so
//     that a rank generating rows [lo, hi) of a global matrix produces exactly
//     the same values as a single process generating all rows (sharding- and
//     world-size-invariant synthetic datasets; mirrored in dalgo/utils/philox.py).
//   * K6 mc_pi_count — Monte-Carlo pi (randomized_algorithm/monte_carlo.py:17-28):
//     point i = (2u-1, 2v-1) from Philox, count x^2+y^2 <= 1. VALU-bound; wave
//     reduce (permlane swaps + DPP) -> one 64-bit atomic per block.
#include "dalgo/common.h"
#include <algorithm>

namespace dalgo {

enum Dist : int { kUniform = 0, kNormal = 1 };

// value of global element idx
__device__ __forceinline__ float draw_value(uint64_t seed, uint64_t stream, uint64_t idx, int dist,
                                            float a, float b) {
  if (dist == kUniform) {
    u32x4 h = philox_block(seed, stream, idx >> 2);
    uint32_t w = (idx & 3) == 0 ? h.x : ((idx & 3) == 1 ? h.y : ((idx & 3) == 2 ? h.z : h.w));
    return a + (b - a) * u01(w);
  } else {
    u32x4 h = philox_block(seed, stream, idx >> 1);
    uint32_t p = (idx & 1) ? h.z : h.x, q = (idx & 1) ? h.w : h.y;
    float u1 = (float)((p >> 8) + 1) * (1.0f / 16777216.0f);
    float th = 6.283185307179586f * u01(q);
    return a + b * sqrtf(-2.f * logf(u1)) * cosf(th);   // mean a, std b
  }
}

template <bool BF16>
__global__ void __launch_bounds__(256)
philox_fill_kernel(void* out, int64_t nrows, int64_t D, int64_t ld, int64_t row_offset,
                   uint64_t seed, uint64_t stream, int dist, float a, float b) {
  const int64_t total = nrows * ld;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / ld, c = e - r * ld;
    float v = 0.f;
    if (c < D) v = draw_value(seed, stream, (uint64_t)((row_offset + r) * D + c), dist, a, b);
    if (BF16) reinterpret_cast<uint16_t*>(out)[e] = f32_to_bf16(v);
    else reinterpret_cast<float*>(out)[e] = v;
  }
}

__global__ void __launch_bounds__(256)
mc_pi_kernel(uint64_t seed, uint64_t stream, uint64_t offset, uint64_t n,
             unsigned long long* count) {
  // each thread evaluates 2 points per Philox call: (x,y) and (z,w)
  uint32_t local = 0;
  const uint64_t nblk = (n + 1) / 2;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nblk;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i0 = 2 * k;                      // point index (relative)
    u32x4 h = philox_block(seed, stream, (offset + i0) >> 1);
    float x0 = 2.f * u01(h.x) - 1.f, y0 = 2.f * u01(h.y) - 1.f;
    float x1 = 2.f * u01(h.z) - 1.f, y1 = 2.f * u01(h.w) - 1.f;
    local += (x0 * x0 + y0 * y0 <= 1.f) ? 1u : 0u;
    if (i0 + 1 < n) local += (x1 * x1 + y1 * y1 <= 1.f) ? 1u : 0u;
  }
  __shared__ uint32_t s[4];
  uint32_t w = wave_sum_u32(local);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += s[k];
    atomicAdd(count, t);
  }
}

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

}  // namespace dalgo

using namespace dalgo;

extern "C" {

hipError_t dalgo_philox_fill(void* out, int is_bf16, int64_t nrows, int64_t D, int64_t ld,
                             int64_t row_offset, uint64_t seed, uint64_t stream, int dist, float a,
                             float b, hipStream_t st) {
  const int64_t total = nrows * ld;
  if (total == 0) return hipSuccess;
  const int grid = (int)std::min<int64_t>(cdiv(total, 256), 256 * 16);
  if (is_bf16)
    hipLaunchKernelGGL(philox_fill_kernel<true>, dim3(grid), dim3(256), 0, st, out, nrows, D, ld,
                       row_offset, seed, stream, dist, a, b);
  else
    hipLaunchKernelGGL(philox_fill_kernel<false>, dim3(grid), dim3(256), 0, st, out, nrows, D, ld,
                       row_offset, seed, stream, dist, a, b);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_mc_pi(uint64_t seed, uint64_t stream, uint64_t offset, uint64_t n,
                       unsigned long long* count, hipStream_t st) {
  if (offset & 1) return hipErrorInvalidValue;   // point pairs share a Philox block
  const uint64_t nblk = (n + 1) / 2;
  const int grid = (int)std::min<uint64_t>((nblk + 255) / 256, 256 * 8);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(mc_pi_kernel, dim3(grid), dim3(256), 0, st, seed, stream, offset, n, count);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_hbm_gather_rows(const void* X, int64_t ld_bytes, const int* idx, int64_t nidx,
                                 uint32_t* out, int grid, hipStream_t st) {
  if (ld_bytes % 16 || ld_bytes < 2048) return hipErrorInvalidValue;
  hipLaunchKernelGGL(hbm_gather_rows_kernel, dim3(grid), dim3(256), 0, st, (const uint4*)X,
                     ld_bytes / 16, idx, nidx, out);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_hbm_read(const void* p, int64_t nbytes, uint32_t* out, int grid, int unroll,
                          hipStream_t st) {
  const int64_t n16 = nbytes / 16;
  if (unroll < 0) {   // blocked-region variant
    if (unroll <= -8)
      hipLaunchKernelGGL(hbm_read_blocked_kernel<8>, dim3(grid), dim3(256), 0, st, (const uint4*)p, n16, out);
    else
      hipLaunchKernelGGL(hbm_read_blocked_kernel<4>, dim3(grid), dim3(256), 0, st, (const uint4*)p, n16, out);
    DALGO_LAUNCH_CHECK();
    return hipSuccess;
  }
  if (unroll >= 8)
    hipLaunchKernelGGL(hbm_read_kernel<8>, dim3(grid), dim3(256), 0, st, (const uint4*)p, n16, out);
  else
    hipLaunchKernelGGL(hbm_read_kernel<4>, dim3(grid), dim3(256), 0, st, (const uint4*)p, n16, out);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
