// K9: linear transitive-closure step as a fused boolean MFMA GEMM.
//
// Reference (graph_computation/transitive_closure.py:31-40): every round joins
// the path set with the reversed edges (shuffle), unions and distinct()s the
// result (shuffle) and count()s it (action) until the count stops changing.
//
// Dense formulation: P[x][z] = 1 iff there is a path x -> z; one round is
//   P <- P OR (A . P)     (A = adjacency, x -> y), boolean semiring.
// We keep T = P^T so that BOTH MFMA operands are contiguous rows:
//   C[x][z] = sum_y A[x][y] * T[z][y]      (A rows = MFMA A operand,
//                                           T rows = MFMA B operand)
// and the epilogue writes T_new[z][x] = T[z][x] | (C[x][z] > 0) — the D layout
// puts z on the lane and 4 consecutive x in each register group, so each lane
// stores 8 contiguous bytes. Values are exact 0/1 in bf16 and the f32
// accumulator counts paths exactly (< 2^24), so the result is exact.
// Columns of P are independent, so ranks partition the targets z: no
// communication besides the int64 count all-reduce of the fixpoint test.
#include "dalgo/common.h"
#include <algorithm>

namespace dalgo {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

// block = 4 waves computing a 64 (x) x 64 (z) tile; wave (wx, wz) a 32x32 tile
__global__ void __launch_bounds__(256)
tc_step_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ Told,
               uint16_t* __restrict__ Tnew, int64_t ldt, int npad,
               unsigned long long* __restrict__ count) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, cl = lane & 31;
  const int x0 = blockIdx.x * 64 + (wid & 1) * 32;
  const int z0 = blockIdx.y * 64 + (wid >> 1) * 32;
  const uint16_t* arow = A + (int64_t)(x0 + cl) * lda + 8 * h;
  const uint16_t* trow = Told + (int64_t)(z0 + cl) * ldt + 8 * h;
  f32x16_t acc = {};
#pragma unroll 4
  for (int y = 0; y < npad; y += 16) {
    const uint4 a = *reinterpret_cast<const uint4*>(arow + y);
    const uint4 b = *reinterpret_cast<const uint4*>(trow + y);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                  __builtin_bit_cast(bf16x8_t, b), acc, 0, 0, 0);
  }
  // epilogue: T_new[z][x..x+3] = T_old | (C > 0)
  const int z = z0 + cl;
  uint32_t ones = 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int x = x0 + 8 * g + 4 * h;
    const uint2 old = *reinterpret_cast<const uint2*>(Told + (int64_t)z * ldt + x);
    const uint16_t o[4] = {(uint16_t)(old.x & 0xffff), (uint16_t)(old.x >> 16),
                           (uint16_t)(old.y & 0xffff), (uint16_t)(old.y >> 16)};
    uint16_t nv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool one = (o[j] != 0) || (acc[4 * g + j] > 0.5f);
      nv[j] = one ? (uint16_t)0x3f80 : (uint16_t)0;   // bf16 1.0
      ones += one ? 1u : 0u;
    }
    *reinterpret_cast<uint2*>(Tnew + (int64_t)z * ldt + x) =
        make_uint2((uint32_t)nv[0] | ((uint32_t)nv[1] << 16), (uint32_t)nv[2] | ((uint32_t)nv[3] << 16));
  }
  ones = wave_sum_u32(ones);
  if (lane == 0 && ones) atomicAdd(count, (unsigned long long)ones);
}

// LDS-tiled version: block = 4 waves computing a 128 (x) x 128 (z) tile, each wave
// 64 x 64 = 2 x 2 MFMA 32x32 tiles; K (= y) staged 32 at a time through double-
// buffered LDS tiles with 80-byte rows (16-B pad -> conflict-free ds_read_b128),
// register-staged so the next stage's global loads overlap the MFMAs.
__global__ void __launch_bounds__(256)
tc_step_lds_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ Told,
                   uint16_t* __restrict__ Tnew, int64_t ldt, int npad,
                   unsigned long long* __restrict__ count) {
  constexpr int RB = 80;                        // LDS row bytes (64 B data + 16 B pad)
  __shared__ __attribute__((aligned(16))) unsigned char sA[2][128 * RB];
  __shared__ __attribute__((aligned(16))) unsigned char sT[2][128 * RB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, cl = lane & 31;
  const int wx = wid & 1, wz = wid >> 1;
  const int x0 = blockIdx.x * 128, z0 = blockIdx.y * 128;
  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16_t{};
  // staging: 128 rows x 4 pieces (16 B) per operand = 512 pieces -> 2 per thread
  uint4 ra[2], rt[2];
  auto load = [&](int y0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int piece = tid + q * 256, row = piece >> 2, pc = piece & 3;
      ra[q] = *reinterpret_cast<const uint4*>(A + (int64_t)(x0 + row) * lda + y0 + pc * 8);
      rt[q] = *reinterpret_cast<const uint4*>(Told + (int64_t)(z0 + row) * ldt + y0 + pc * 8);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int piece = tid + q * 256, row = piece >> 2, pc = piece & 3;
      *reinterpret_cast<uint4*>(&sA[buf][row * RB + pc * 16]) = ra[q];
      *reinterpret_cast<uint4*>(&sT[buf][row * RB + pc * 16]) = rt[q];
    }
  };
  load(0);
  store(0);
  __syncthreads();
  const int nst = npad / 32;
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst) load((st + 1) * 32);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const uint4*>(&sA[cur][(wx * 64 + i * 32 + cl) * RB + ks * 32 + h * 16]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b[j] = *reinterpret_cast<const uint4*>(&sT[cur][(wz * 64 + j * 32 + cl) * RB + ks * 32 + h * 16]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a[i]),
                                                              __builtin_bit_cast(bf16x8_t, b[j]),
                                                              acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nst) store(cur ^ 1);
    __syncthreads();
  }
  uint32_t ones = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int z = z0 + wz * 64 + j * 32 + cl;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int x = x0 + wx * 64 + i * 32 + 8 * g + 4 * h;
        const uint2 old = *reinterpret_cast<const uint2*>(Told + (int64_t)z * ldt + x);
        const uint16_t o[4] = {(uint16_t)(old.x & 0xffff), (uint16_t)(old.x >> 16),
                               (uint16_t)(old.y & 0xffff), (uint16_t)(old.y >> 16)};
        uint16_t nv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool one = (o[e] != 0) || (acc[i][j][4 * g + e] > 0.5f);
          nv[e] = one ? (uint16_t)0x3f80 : (uint16_t)0;
          ones += one ? 1u : 0u;
        }
        *reinterpret_cast<uint2*>(Tnew + (int64_t)z * ldt + x) =
            make_uint2((uint32_t)nv[0] | ((uint32_t)nv[1] << 16), (uint32_t)nv[2] | ((uint32_t)nv[3] << 16));
      }
    }
  ones = wave_sum_u32(ones);
  if (lane == 0 && ones) atomicAdd(count, (unsigned long long)ones);
}

}  // namespace dalgo

using namespace dalgo;

extern "C" {

// A: [npad, lda] bf16 0/1, T_old/T_new: [nz, ldt] bf16 0/1 (nz % 64 == 0,
// npad % 64 == 0, lda/ldt >= npad, multiples of 8).
hipError_t dalgo_tc_step(const void* A, int64_t lda, const void* Told, void* Tnew, int64_t ldt,
                         int npad, int nz, unsigned long long* count, hipStream_t st) {
  if (npad % 64 || nz % 64 || lda % 8 || ldt % 8) return hipErrorInvalidValue;
  if (npad % 128 == 0 && nz % 128 == 0) {
    dim3 grid(npad / 128, nz / 128);
    if (grid.x == 0 || grid.y == 0) return hipSuccess;
    hipLaunchKernelGGL(tc_step_lds_kernel, grid, dim3(256), 0, st, (const uint16_t*)A, lda,
                       (const uint16_t*)Told, (uint16_t*)Tnew, ldt, npad, count);
    DALGO_LAUNCH_CHECK();
    return hipSuccess;
  }
  dim3 grid(npad / 64, nz / 64);
  if (grid.x == 0 || grid.y == 0) return hipSuccess;
  hipLaunchKernelGGL(tc_step_kernel, grid, dim3(256), 0, st, (const uint16_t*)A, lda,
                     (const uint16_t*)Told, (uint16_t*)Tnew, ldt, npad, count);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
