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
// stores one 4-byte word. The matrices are 0/1 bytes and the product runs on the
// int8 MFMA (v_mfma_i32_32x32x32_i8: twice the bf16 rate, half the bytes) with
// exact int32 accumulation, so the result is exact for any n < 2^31.
//
// Tiling: a block of 4 waves owns a 128 (x) x 128 (z) tile, each wave 64 x 64 =
// 2 x 2 MFMA tiles. K (= y) is staged BK bytes at a time with LDS-DMA
// (global_load_lds_dwordx4: no VGPR round trip) into a double-buffered image;
// since LDS-DMA writes lane-linearly, the bank swizzle (16-B chunk ^= (row/RP) &
// (CPR-1)) is applied to the per-lane SOURCE address and undone on the
// ds_read_b128 side, making the fragment reads conflict-free. The next stage's
// loads stay in flight across the compute of the current one (counted vmcnt).
// Columns of P are independent, so ranks partition the targets z: no
// communication besides the int64 count all-reduce of the fixpoint test.
#include "dalgo/common.h"
#include <algorithm>

namespace dalgo {

typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x16_t __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

// TILE x TILE output tile per block: TILE = 128 -> 4 waves of 64 x 64 (2 x 2 MFMA tiles);
// TILE = 256 -> 8 waves of 128 x 64 (4 x 2 MFMA tiles, 128 accumulator VGPRs): half the
// operand bytes per MFMA (the 128 form is bound by L2 / Infinity-Fabric traffic: 38 GB
// of L2 misses per n = 16384 step for 0.5 GB of unique data).
template <int BK, int TILE>
__global__ void __launch_bounds__(TILE == 256 ? 512 : 256)
tc_step_i8_kernel(const uint8_t* __restrict__ A, int64_t lda, const uint8_t* __restrict__ Told,
                  uint8_t* __restrict__ Tnew, int64_t ldt, int npad, int gx,
                  unsigned long long* __restrict__ count) {
  constexpr int NW = TILE == 256 ? 8 : 4;
  constexpr int NT = NW * 64;
  constexpr int WZ = NW / 2;               // waves along z (2 along x)
  constexpr int MI = TILE / 2 / 32;        // MFMA tiles per wave along x
  constexpr int MJ = TILE / WZ / 32;       // ... along z
  constexpr int CPR = BK / 16;             // 16-B chunks per staged row
  constexpr int RP = 256 / BK;             // rows covering the 64 banks once
  constexpr int STAGE = TILE * BK;         // bytes per operand per stage
  constexpr int PPT = STAGE / 16 / NT;     // 16-B pieces per thread per operand
  static_assert(PPT * 16 * NT == STAGE, "whole DMA rounds per stage");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * 2 * STAGE];   // [buf][A | T]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, cl = lane & 31;
  const int wx = wid & 1, wz = wid >> 1;
  // tile order: consecutive block ids walk down x inside a column strip of z tiles so
  // co-resident blocks share their T rows in L2
  const int bid = blockIdx.x;
  const int x0 = (bid % gx) * TILE, z0 = (bid / gx) * TILE;

  const uint8_t* asrc[PPT];
  const uint8_t* tsrc[PPT];
#pragma unroll
  for (int q = 0; q < PPT; ++q) {
    const int p = q * NT + tid, r = p / CPR, pc = p % CPR;
    const int c = pc ^ ((r / RP) & (CPR - 1));
    asrc[q] = A + (int64_t)(x0 + r) * lda + c * 16;
    tsrc[q] = Told + (int64_t)(z0 + r) * ldt + c * 16;
  }
  auto issue = [&](int y0, int buf) {
    uint8_t* base = smem + buf * 2 * STAGE;
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      __builtin_amdgcn_global_load_lds((const void*)(asrc[q] + y0), (lds_void*)(base + (q * NT + wid * 64) * 16), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(tsrc[q] + y0), (lds_void*)(base + STAGE + (q * NT + wid * 64) * 16), 16, 0, 0);
    }
  };

  i32x16_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = i32x16_t{};

  const int nst = npad / BK;
  issue(0, 0);
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst) {
      issue((st + 1) * BK, cur ^ 1);
      wait_vmcnt<2 * PPT>();          // this stage landed; the next one stays in flight
    } else {
      wait_vmcnt<0>();
    }
    // raw barrier: __syncthreads() would add a vmcnt(0) drain of the stage in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const uint8_t* sa = smem + cur * 2 * STAGE;
    const uint8_t* stt = sa + STAGE;
    // fragments of k-step ks+1 are read while the MFMAs of ks run (register double buffer)
    i32x4_t a[2][MI], b[2][MJ];
    auto frags = [&](int ks, i32x4_t (&aa)[MI], i32x4_t (&bb)[MJ]) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int r = wx * (TILE / 2) + i * 32 + cl;
        const int pc = (2 * ks + h) ^ ((r / RP) & (CPR - 1));
        aa[i] = *reinterpret_cast<const i32x4_t*>(sa + r * BK + pc * 16);
      }
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const int r = wz * (TILE / WZ) + j * 32 + cl;
        const int pc = (2 * ks + h) ^ ((r / RP) & (CPR - 1));
        bb[j] = *reinterpret_cast<const i32x4_t*>(stt + r * BK + pc * 16);
      }
    };
    frags(0, a[0], b[0]);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      if (ks + 1 < BK / 32) frags(ks + 1, a[(ks + 1) & 1], b[(ks + 1) & 1]);
      // keep the reads of ks+1 ahead of the MFMAs of ks (hipcc otherwise sinks them to
      // their use and re-uses one register set: a full LDS latency per k-step)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[ks & 1][i], b[ks & 1][j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();     // all reads of `cur` done before it is refilled
    asm volatile("" ::: "memory");
  }

  // epilogue: T_new[z][x..x+3] = T_old | (C > 0)
  uint32_t ones = 0;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int z = z0 + wz * (TILE / WZ) + j * 32 + cl;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int x = x0 + wx * (TILE / 2) + i * 32 + 8 * g + 4 * h;
        const uint32_t old = *reinterpret_cast<const uint32_t*>(Told + (int64_t)z * ldt + x);
        uint32_t nv = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool one = ((old >> (8 * e)) & 0xffu) != 0 || acc[i][j][4 * g + e] > 0;
          nv |= (one ? 1u : 0u) << (8 * e);
          ones += one ? 1u : 0u;
        }
        *reinterpret_cast<uint32_t*>(Tnew + (int64_t)z * ldt + x) = nv;
      }
    }
  ones = wave_sum_u32(ones);
  if (lane == 0 && ones) atomicAdd(count, (unsigned long long)ones);
}

template <int BK, int TILE>
void launch_tc_step(const void* A, int64_t lda, const void* Told, void* Tnew, int64_t ldt, int npad,
                    int gx, int gz, unsigned long long* count, hipStream_t st) {
  hipLaunchKernelGGL((tc_step_i8_kernel<BK, TILE>), dim3(gx * gz), dim3(TILE == 256 ? 512 : 256), 0, st,
                     (const uint8_t*)A, lda, (const uint8_t*)Told, (uint8_t*)Tnew, ldt, npad, gx, count);
}

}  // namespace dalgo

using namespace dalgo;

extern "C" {

// A: [npad, lda] uint8 0/1, T_old/T_new: [nz, ldt] uint8 0/1; npad, nz multiples
// of 128, lda/ldt >= npad and multiples of 16. 256 x 256 tiles (8 waves, 128-B K stages)
// when npad and nz are multiples of 256, else 128 x 128 tiles. The 64-B K-stage forms were
// slower at every size measured (n = 16384: 1.51 / 2.14 vs 1.73 / 2.33 POP/s) and are gone.
hipError_t dalgo_tc_step(const void* A, int64_t lda, const void* Told, void* Tnew, int64_t ldt,
                         int npad, int nz, int variant, unsigned long long* count, hipStream_t st) {
  (void)variant;
  if (npad % 128 || nz % 128 || lda % 16 || ldt % 16) return hipErrorInvalidValue;
  if (npad == 0 || nz == 0) return hipSuccess;
  if (npad % 256 == 0 && nz % 256 == 0)
    launch_tc_step<128, 256>(A, lda, Told, Tnew, ldt, npad, npad / 256, nz / 256, count, st);
  else
    launch_tc_step<128, 128>(A, lda, Told, Tnew, ldt, npad, npad / 128, nz / 128, count, st);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
