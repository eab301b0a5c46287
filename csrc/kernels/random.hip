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

typedef __attribute__((address_space(3))) void probe_lds_void;
template <int DEPTH, bool NT>
__global__ void __launch_bounds__(512)
hbm_gather_rows_lds_kernel(const uint4* __restrict__ X, int64_t ld16, const int* __restrict__ idx,
                           int64_t nidx, uint32_t* __restrict__ out) {
  constexpr int NW = 8, IDXB = 512;
  __shared__ __attribute__((aligned(16))) uint4 s_ring[NW * DEPTH * 128];
  __shared__ int s_idx[NW * IDXB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t nwv = (int64_t)gridDim.x * NW;
  const int64_t gw = (int64_t)blockIdx.x * NW + wid;
  const int64_t per = (nidx + nwv - 1) / nwv;
  const int64_t lo = min(nidx, gw * per), hi = min(nidx, lo + per);
  uint32_t acc = 0;
  uint4* ring = s_ring + wid * DEPTH * 128;
  int* sidx = s_idx + wid * IDXB;
  const uint32_t rbase = (uint32_t)(uintptr_t)(probe_lds_void*)ring;
  for (int64_t b0 = lo; b0 < hi; b0 += IDXB) {
    const int nb = (int)min((int64_t)IDXB, hi - b0);
    for (int j = lane; j < nb; j += 64) sidx[j] = idx[b0 + j];
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    auto issue = [&](int i) {
      const int k = min(i, nb - 1);
      const int r = __builtin_amdgcn_readfirstlane(sidx[k]);
      const uint4* row = X + (int64_t)r * ld16;
      const uint32_t m0a = __builtin_amdgcn_readfirstlane(rbase + (uint32_t)((i % DEPTH) * 2048));
      const uint4* s0 = row + lane;
      const uint4* s1 = row + 64 + lane;
      if constexpr (NT) {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt"
                     :: "s"(m0a), "v"(s0) : "memory");
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt"
                     :: "s"(m0a + 1024u), "v"(s1) : "memory");
      } else {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                     :: "s"(m0a), "v"(s0) : "memory");
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                     :: "s"(m0a + 1024u), "v"(s1) : "memory");
      }
    };
    // DEPTH rows always in flight (the tail re-reads the last row: constant counts)
    for (int i = 0; i < DEPTH; ++i) issue(i);
    for (int i = 0; i < nb; ++i) {
      // row i landed: everything but the newest 2 * (DEPTH - 1) DMA instructions
      if constexpr (DEPTH == 4) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (DEPTH == 6) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
      const uint4* sl = ring + (i % DEPTH) * 128;
      const uint4 a = sl[lane], b = sl[64 + lane];
      acc ^= a.x ^ a.w ^ b.y ^ b.z;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // slot read before it is refilled
      issue(i + DEPTH);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  acc = wave_sum_u32(acc);
  if (lane == 0) atomicXor(out, acc);
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

hipError_t dalgo_hbm_gather_rows(const void* X, int64_t ld_bytes, const int* idx, int64_t nidx,
                                 uint32_t* out, int grid, hipStream_t st) {
  if (ld_bytes % 16 || ld_bytes < 2048) return hipErrorInvalidValue;
  // grid >> 20 selects the probe form: 0 registers, 1 registers + nt, 2/3 LDS-DMA depth 4
  // (default / nt), 4/5 depth 6, 6/7 depth 8 (LDS forms: 512-thread blocks, 2 KB rows)
  const int mode = grid >> 20;
  grid &= (1 << 20) - 1;
  const uint4* X4 = (const uint4*)X;
  const int64_t ld16 = ld_bytes / 16;
  if (mode >= 2 && ld_bytes != 2048) return hipErrorInvalidValue;
  switch (mode) {
    case 0: hipLaunchKernelGGL(hbm_gather_rows_kernel, dim3(grid), dim3(256), 0, st, X4, ld16, idx, nidx, out); break;
    case 1: hipLaunchKernelGGL(hbm_gather_rows_nt_kernel<true>, dim3(grid), dim3(256), 0, st, X4, ld16, idx, nidx, out); break;
    case 2: hipLaunchKernelGGL((hbm_gather_rows_lds_kernel<4, false>), dim3(grid), dim3(512), 0, st, X4, ld16, idx, nidx, out); break;
    case 3: hipLaunchKernelGGL((hbm_gather_rows_lds_kernel<4, true>), dim3(grid), dim3(512), 0, st, X4, ld16, idx, nidx, out); break;
    case 4: hipLaunchKernelGGL((hbm_gather_rows_lds_kernel<6, false>), dim3(grid), dim3(512), 0, st, X4, ld16, idx, nidx, out); break;
    case 5: hipLaunchKernelGGL((hbm_gather_rows_lds_kernel<6, true>), dim3(grid), dim3(512), 0, st, X4, ld16, idx, nidx, out); break;
    case 6: hipLaunchKernelGGL((hbm_gather_rows_lds_kernel<8, false>), dim3(grid), dim3(512), 0, st, X4, ld16, idx, nidx, out); break;
    case 7: hipLaunchKernelGGL((hbm_gather_rows_lds_kernel<8, true>), dim3(grid), dim3(512), 0, st, X4, ld16, idx, nidx, out); break;
    default: return hipErrorInvalidValue;
  }
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
