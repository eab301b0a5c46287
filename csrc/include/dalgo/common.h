// dalgo — shared device helpers for the gfx950 (CDNA4) kernels.
//
// Everything here is written for 64-lane wavefronts on MI355X: cross-lane
// reductions use DPP row rotations plus the gfx950 permlane16/32 swaps (no LDS
// round trip), bf16 is unpacked with integer shifts (bf16 is the top half of an
// f32), and the counter-based RNG is Philox4x32-10 so that every sample /
// Monte-Carlo draw is a pure function of (seed, stream, counter) — identical on
// any number of ranks and reproducible by the NumPy reference in
// dalgo/utils/philox.py.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace dalgo {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// launch error plumbing: launchers return hipError_t; the binding layer turns a
// non-success code into a C++ exception with the kernel name.
// ---------------------------------------------------------------------------
#define DALGO_LAUNCH_CHECK() \
  do {                       \
    hipError_t _e = hipGetLastError(); \
    if (_e != hipSuccess) return _e;   \
  } while (0)

// Host-side knob: integer environment variable with a default (read per call; the
// launchers that use it are not on a per-microsecond path).
inline int env_int(const char* name, int dflt) {
  const char* s = getenv(name);
  return (s && *s) ? atoi(s) : dflt;
}

// Non-temporal (`nt`) loads for data streamed exactly once (edge lists, gathered
// X rows): measured +4-8 % on HBM-bound streams (K1 359 -> 333 us at 10M rows).
typedef int dalgo_v4i __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ int4 ld_int4(const int32_t* p) {
  if constexpr (NT) {
    const dalgo_v4i v = __builtin_nontemporal_load(reinterpret_cast<const dalgo_v4i*>(p));
    return make_int4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const int4*>(p);
  }
}
template <bool NT>
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// ---------------------------------------------------------------------------
// bf16 helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf16lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
// round-to-nearest-even f32 -> bf16 (finite inputs; NaN handling not needed here)
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11). counter = (c0,c1,c2,c3), key=(k0,k1).
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * b) >> 32);   // v_mul_hi_u32 on the device
}

__host__ __device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 product per multiplier (v_mad_u64_u32 on the device) instead of a
    // separate mul_hi and mul_lo
    const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// Bernoulli / uniform stream used by every sampler in the library:
// draw(seed, stream, i) = philox(counter = {i>>2 (64 bit), stream (64 bit)},
//                                key = seed (64 bit))[i & 3]
// One Philox call therefore serves 4 consecutive indices.
__host__ __device__ __forceinline__ u32x4 philox_block(uint64_t seed, uint64_t stream, uint64_t block) {
  u32x4 c{(uint32_t)block, (uint32_t)(block >> 32), (uint32_t)stream, (uint32_t)(stream >> 32)};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// ---------------------------------------------------------------------------
// Cross-lane reductions, wave64.
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

// Sum within each 16-lane DPP row; every lane of the row gets the row sum.
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0x128>(v);  // row_ror:8
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x122>(v);  // row_ror:2
  v += dpp_f<0x121>(v);  // row_ror:1
  return v;
}

// Returns (a_lo_half + a_hi_half) in lanes 0-31 and (b_lo + b_hi) in lanes 32-63
// where lo/hi are the lane halves [0,32) and [32,64): v_permlane32_swap.
__device__ __forceinline__ float fold32(float a, float b) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// Same with 16-lane rows: v_permlane16_swap exchanges odd rows of a with even rows of b.
// Result rows: [a0+a1, b0+b1, a2+a3, b2+b3].
__device__ __forceinline__ float fold16(float a, float b) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Full wave sum broadcast to every lane.
__device__ __forceinline__ float wave_sum(float v) {
  v = fold32(v, v);
  v = fold16(v, v);
  return row16_sum(v);
}

// Reduce four per-lane partials d0..d3 (one per row) across the wave with 7
// cross-lane ops. On return lane l holds the full sum for row (l >> 4).
__device__ __forceinline__ float wave_sum4(float d0, float d1, float d2, float d3) {
  float s = fold32(d0, d2);   // lanes 0-31: row0 partial, 32-63: row2
  float t = fold32(d1, d3);   // lanes 0-31: row1 partial, 32-63: row3
  float u = fold16(s, t);     // rows(16-lane blocks): row0,row1,row2,row3
  return row16_sum(u);
}

// Integer wave sum (exact), broadcast to every lane.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  v = a[0] + a[1];
  auto b = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = b[0] + b[1];
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xf, 0xf, false);
  return v;
}

// u32 -> uniform float in [0,1) with 24-bit resolution (mirrored in utils/philox.py)
__device__ __forceinline__ float u01(uint32_t u) { return (float)(u >> 8) * (1.0f / 16777216.0f); }

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Ceil-div and round-up helpers (host + device)
__host__ __device__ constexpr inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ constexpr inline int64_t round_up(int64_t a, int64_t b) { return cdiv(a, b) * b; }

// Bijective XCD-aware block remap (guide T1): consecutive logical tiles land on
// the same XCD (same L2). `orig` = hardware block id, n = grid size.
__device__ __forceinline__ int xcd_remap(int orig, int n) {
  const int nx = 8;
  int q = n / nx, r = n % nx;
  int xcd = orig % nx, idx = orig / nx;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

}  // namespace dalgo
