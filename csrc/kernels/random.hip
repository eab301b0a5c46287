// Counter-based random generation on device:
//   * philox_fill — synthetic data generator (uniform / normal), index-keyed so
//     that a rank generating rows [lo, hi) of a global matrix produces exactly
//     the same values as a single process generating all rows (sharding- and
//     world-size-invariant synthetic datasets; mirrored in dalgo/utils/philox.py).
//   * K6 mc_pi_count — Monte-Carlo pi (randomized_algorithm/monte_carlo.py:17-28):
//     3 points (21-bit coordinates) per Philox block, count x^2+y^2 <= 1. VALU-bound;
//     wave reduce (permlane swaps + DPP) -> one 64-bit atomic per block.
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

// One thread per aligned group of 4 consecutive GLOBAL element indices: the uniform
// mapping takes all 4 words of one Philox4x32-10 block (idx >> 2), the normal mapping
// the 2 Box-Muller pairs of two blocks (idx >> 1), so every Philox output word is used
// and the (row, column) split costs one 64-bit divide per 4 elements instead of one
// per element (values identical to draw_value / dalgo/utils/philox.py). Groups may
// straddle a row end (any D). Padding columns [D, ld) are zeroed by a second loop.
template <bool BF16>
__device__ __forceinline__ void put(void* out, int64_t off, float v) {
  if (BF16) reinterpret_cast<uint16_t*>(out)[off] = f32_to_bf16(v);
  else reinterpret_cast<float*>(out)[off] = v;
}

template <bool BF16>
__global__ void __launch_bounds__(256)
philox_fill_kernel(void* out, int64_t nrows, int64_t D, int64_t ld, int64_t row_offset,
                   uint64_t seed, uint64_t stream, int dist, float a, float b) {
  const uint64_t g_lo = (uint64_t)row_offset * (uint64_t)D;
  const uint64_t g_hi = g_lo + (uint64_t)nrows * (uint64_t)D;
  const uint64_t k_lo = g_lo >> 2, k_hi = D > 0 ? (g_hi + 3) >> 2 : k_lo;
  for (uint64_t k = k_lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < k_hi;
       k += (uint64_t)gridDim.x * blockDim.x) {
    float v[4];
    if (dist == kUniform) {
      const u32x4 h = philox_block(seed, stream, k);
      v[0] = a + (b - a) * u01(h.x);
      v[1] = a + (b - a) * u01(h.y);
      v[2] = a + (b - a) * u01(h.z);
      v[3] = a + (b - a) * u01(h.w);
    } else {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const u32x4 h = philox_block(seed, stream, 2 * k + half);
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          const uint32_t p = o ? h.z : h.x, q = o ? h.w : h.y;
          const float u1 = (float)((p >> 8) + 1) * (1.0f / 16777216.0f);
          const float th = 6.283185307179586f * u01(q);
          v[2 * half + o] = a + b * sqrtf(-2.f * logf(u1)) * cosf(th);
        }
      }
    }
    uint64_t g = 4 * k;
    uint64_t first = g < g_lo ? g_lo : g;
    int64_t r = (int64_t)((first - g_lo) / (uint64_t)D);
    int64_t c = (int64_t)(first - g_lo) - r * D;
    for (int j = (int)(first - g); j < 4 && g + j < g_hi; ++j) {
      put<BF16>(out, r * ld + c, v[j]);
      if (++c == D) { c = 0; ++r; }
    }
  }
  const int64_t pad = ld - D;
  if (pad > 0) {
    const int64_t total = nrows * pad;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
      const int64_t r = e / pad;
      put<BF16>(out, r * ld + D + (e - r * pad), 0.f);
    }
  }
}

// Point i of the stream = slot i % 3 of Philox block i / 3: the 128 random bits give
// three points with 21-bit coordinates (x0 = w0 >> 11, y0 = w1 >> 11, x1 = w2 >> 11,
// y1 = w3 >> 11, x2 / y2 from the four low 11-bit remainders). 21 bits put the grid bias
// of the disc area at ~1e-6 relative, well below the 1.6e-5 sampling error of 1e10
// points; 3 points per Philox call instead of 2 is 1.5x fewer Philox rounds, which is
// what this kernel's time is made of.
__device__ __forceinline__ uint32_t mc_in(uint32_t xb, uint32_t yb) {
  const float x = ((float)xb + 0.5f) * (2.0f / 2097152.0f) - 1.0f;
  const float y = ((float)yb + 0.5f) * (2.0f / 2097152.0f) - 1.0f;
  return (x * x + y * y <= 1.f) ? 1u : 0u;
}

__global__ void __launch_bounds__(256)
mc_pi_kernel(uint64_t seed, uint64_t stream, uint64_t offset, uint64_t n,
             unsigned long long* count) {
  uint32_t local = 0;
  const uint64_t b0 = offset / 3;                    // offset % 3 == 0 (host check)
  const uint64_t nblk = (n + 2) / 3;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nblk;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 h = philox_block(seed, stream, b0 + k);
    const uint64_t i0 = 3 * k;                       // first point (relative)
    local += mc_in(h.x >> 11, h.y >> 11);
    if (i0 + 1 < n) local += mc_in(h.z >> 11, h.w >> 11);
    if (i0 + 2 < n)
      local += mc_in((h.x & 0x7ffu) | ((h.y & 0x3ffu) << 11), (h.z & 0x7ffu) | ((h.w & 0x3ffu) << 11));
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

}  // namespace dalgo

using namespace dalgo;

extern "C" {

hipError_t dalgo_philox_fill(void* out, int is_bf16, int64_t nrows, int64_t D, int64_t ld,
                             int64_t row_offset, uint64_t seed, uint64_t stream, int dist, float a,
                             float b, hipStream_t st) {
  const int64_t total = nrows * ld;
  if (total == 0) return hipSuccess;
  const int grid = (int)std::min<int64_t>(cdiv(cdiv(total, 4), 256), 256 * 16);
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
  if (offset % 3) return hipErrorInvalidValue;   // point triples share a Philox block
  const uint64_t nblk = (n + 2) / 3;
  const int grid = (int)std::min<uint64_t>((nblk + 255) / 256, 256 * 8);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(mc_pi_kernel, dim3(grid), dim3(256), 0, st, seed, stream, offset, n, count);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
