// K2 "centre-stationary" form (bf16, DP 64 / 128, kpad = 256 * NCT): the centres stay
// in VGPRs for the whole launch and the points stream through LDS exactly once.
//
// Reference: machine_learning/k-means.py:20-28 (closest_center, an O(k d) scan per
// point, ties to the lowest id by the strict '<' at :25).
//
// Why: the pipelined form (kmeans.hip, variant 52) keeps a block's 384 points in
// VGPRs and re-streams ALL k centres through LDS for every block (8 chunks, one barrier
// each, a fresh point load + start-up per 10 us of MFMA work): 63 % MFMA busy with 36 %
// of wave time parked (profiles/round2/pmc_k2). Here one persistent block per CU
// (8 waves, two per SIMD) holds all kpad centres as MFMA A fragments -- wave w owns
// centre tiles [w * NCT, (w + 1) * NCT), 32 centres each, loaded once -- and streams
// point groups (G tiles of 32 points) through an NBUF-deep ring of LDS images filled by
// LDS-DMA (global_load_lds_dwordx4, no staging VGPRs). Every wave sweeps every point
// tile of a group against its own centres; one barrier per group publishes the group
// and retires the slot being refilled.
//
// Distances: A = -c (sign bits flipped once), B = x, C = 0.5|c|^2 + M (LDS table), so
// acc = 0.5|x - c|^2 + (M - 0.5|x|^2) >= 0 with M = max over the shard of 0.5|x|^2
// (computed once by the caller: the points never change). Non-negative floats order
// like their int bits: per-lane keys (bits & ~31) | r and v_min3 as in variant 52.
// Per wave: the lane's best key over its NCT tiles (strict compare in ascending
// centre order), then the two lane halves (same point, disjoint rows) are merged with
// a permlane32 swap and the wave's (distance bits << 32 | id) is parked in LDS.
// The cross-wave minimum (lowest distance, then lowest id = the reference's tie rule)
// is taken one group later by wave 4 -- waves 0-3 issue the point DMA and never store,
// wave 4 stores the assignments and never issues DMA, so each wave's vmcnt counts one
// kind of operation and the counted waits stay exact.
// SSE: the kernel adds sum over points of 2 (best - M) = |x - c|^2 - |x|^2 to the slots;
// the caller adds the fixed sum of |x|^2. Per-point distances (optional `mind`) use the
// caller's 0.5|x|^2 vector xh.
#include "dalgo/common.h"

namespace dalgo {
namespace {

typedef __bf16 cs_bf16x8 __attribute__((ext_vector_type(8)));
typedef float cs_f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void cs_lds_void;

template <int N>
__device__ __forceinline__ void cs_wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

// wait until at most `ahead` groups of GPT DMA instructions are outstanding
template <int GPT, int MAXA>
__device__ __forceinline__ void cs_wait_groups(int ahead) {
  if constexpr (MAXA >= 5) { if (ahead >= 5) { cs_wait_vmcnt<5 * GPT>(); return; } }
  if constexpr (MAXA >= 4) { if (ahead == 4) { cs_wait_vmcnt<4 * GPT>(); return; } }
  if constexpr (MAXA >= 3) { if (ahead == 3) { cs_wait_vmcnt<3 * GPT>(); return; } }
  if constexpr (MAXA >= 2) { if (ahead == 2) { cs_wait_vmcnt<2 * GPT>(); return; } }
  if constexpr (MAXA >= 1) { if (ahead == 1) { cs_wait_vmcnt<GPT>(); return; } }
  cs_wait_vmcnt<0>();
}

constexpr int kNW = 8;                 // waves per block (two per SIMD)
constexpr int kNT = kNW * 64;
constexpr int kDmaWaves = 4;           // waves 0-3 issue the point DMA
constexpr int kStoreWave = 4;          // wave 4 combines and stores

template <int DP, int NCT, int G, int NBUF>
__global__ void __launch_bounds__(kNW * 64, 1)
kmeans_assign_cs_kernel(const uint16_t* __restrict__ X, int64_t n, int64_t ldx,
                        const uint16_t* __restrict__ Cq, const float* __restrict__ hn,
                        const float* __restrict__ xh, float M, int* __restrict__ assign,
                        float* __restrict__ mind, double* __restrict__ sse, int sse_mask) {
  constexpr int KS = DP / 16;                    // 32x32x16 k-steps
  constexpr int NJ = DP * 2 / 16;                // 16-B pieces per row
  constexpr int SWZ = (NJ >= 16 ? 16 : NJ) - 1;
  constexpr int TILE_P = 32 * NJ;                // pieces per 32-point tile image
  constexpr int GP = G * TILE_P;                 // pieces per group image
  constexpr int GPT = GP / (kDmaWaves * 64);     // DMA instructions per DMA lane per group
  constexpr int KPAD = kNW * NCT * 32;
  constexpr int GPTS = G * 32;                   // points per group
  static_assert(GP % (kDmaWaves * 64) == 0, "group image must split over the DMA waves");
  static_assert(GPTS <= 64, "one combine lane per point of a group");
  __shared__ __attribute__((aligned(16))) uint4 s_img[NBUF * GP];
  __shared__ __attribute__((aligned(16))) float s_hc[KPAD];
  __shared__ unsigned long long s_res[2][kNW][GPTS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, cl = lane & 31;
  const int64_t ntile = (n + 31) / 32;
  const int64_t ngroup = (ntile + G - 1) / G;
  const int64_t nblk = gridDim.x;
  const int64_t iters = ngroup > (int64_t)blockIdx.x ? (ngroup - 1 - blockIdx.x) / nblk + 1 : 0;

  // ---- prologue: this wave's centre fragments (A = -c), the C table, the SSE slot
  uint4 a[NCT][KS];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const uint16_t* crow = Cq + (int64_t)((wid * NCT + ct) * 32 + cl) * DP + h * 8;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const uint4 v = *reinterpret_cast<const uint4*>(crow + 16 * s);
      a[ct][s] = make_uint4(v.x ^ 0x80008000u, v.y ^ 0x80008000u, v.z ^ 0x80008000u,
                            v.w ^ 0x80008000u);
    }
  }
  for (int c = tid; c < KPAD; c += kNT) s_hc[c] = hn[c] + M;
  // every ordinary load retired before the DMA stream starts (the counted waits below
  // are the only vmcnt waits of the DMA waves)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      asm volatile("" : "+v"(a[ct][s].x), "+v"(a[ct][s].y), "+v"(a[ct][s].z), "+v"(a[ct][s].w));

  // DMA: group image slot q = gi * (4 * 64) + dma_lane holds piece (q % NJ) ^ (row & SWZ)
  // of row q / NJ of the group (rows past n are clamped to row n - 1: never stored)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(cs_lds_void*)s_img;
  auto issue = [&](int64_t it) {
    const int64_t grp = (int64_t)blockIdx.x + it * nblk;
    const int64_t p0 = grp * GPTS;
    const uint32_t dst = lds0 + (uint32_t)(((it % NBUF) * GP) * 16);
#pragma unroll
    for (int gi = 0; gi < GPT; ++gi) {
      const int q = gi * (kDmaWaves * 64) + tid;            // tid < 256 on DMA waves
      const int row = q / NJ, jj = (q % NJ) ^ (row & SWZ);
      int64_t p = p0 + row;
      p = p < n ? p : n - 1;
      const uint16_t* src = X + p * ldx + jj * 8;
      const uint32_t m0v = __builtin_amdgcn_readfirstlane(
          dst + (uint32_t)((gi * (kDmaWaves * 64) + wid * 64) * 16));
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                   :: "s"(m0v), "v"(src) : "memory");
    }
  };
  const bool dma_wave = wid < kDmaWaves;
  if (dma_wave) {
    for (int64_t j = 0; j < NBUF - 1 && j < iters; ++j) issue(j);
  }

  int kmask;
  asm volatile("v_mov_b32 %0, 0xffffffe0" : "=v"(kmask));
  double my_sse = 0.0;

  // combine the parked per-wave results of group `it` (wave kStoreWave, one lane per point)
  auto combine = [&](int64_t it) {
    const int64_t grp = (int64_t)blockIdx.x + it * nblk;
    const int64_t p = grp * GPTS + lane;
    if (lane < GPTS && p < n) {
      unsigned long long best = s_res[it & 1][0][lane];
#pragma unroll
      for (int w = 1; w < kNW; ++w) {
        const unsigned long long v = s_res[it & 1][w][lane];
        best = v < best ? v : best;
      }
      const int id = (int)(uint32_t)best;
      assign[p] = id;
      // 2 (best - M) = |x - c|^2 - |x|^2: the caller adds the point set's fixed sum of
      // |x|^2 to the SSE, so no per-point load is needed unless distances are wanted
      const float d = 2.f * (__uint_as_float((uint32_t)(best >> 32)) - M);
      if (mind) mind[p] = fmaxf(d + 2.f * xh[p], 0.f);
      my_sse += (double)d;
    }
  };

  for (int64_t it = 0; it < iters; ++it) {
    if (dma_wave) {
      const int64_t left = iters - 1 - it;
      const int ahead = (int)(left < NBUF - 2 ? left : NBUF - 2);
      cs_wait_groups<GPT, NBUF - 2>(ahead);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // publishes group it; retires every wave's reads of group it-1's slot (refilled
    // next) and its parked results (combined next, slot it-1 & 1)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (dma_wave) {
      if (it + NBUF - 1 < iters) issue(it + NBUF - 1);
    } else if (wid == kStoreWave && it > 0) {
      combine(it - 1);
    }
    const uint4* img = s_img + (it % NBUF) * GP;
#pragma unroll
    for (int t = 0; t < G; ++t) {
      // B fragments of tile t: row cl, piece (2s + h) ^ (cl & SWZ)
      uint4 b[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) b[s] = img[t * TILE_P + cl * NJ + ((2 * s + h) ^ (cl & SWZ))];
      int bkey = 0x7fffffff, bsub = 0;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const int cb = (wid * NCT + ct) * 32;
        cs_f32x16 hc;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 v = *reinterpret_cast<const float4*>(&s_hc[cb + 8 * g4 + 4 * h]);
          hc[4 * g4 + 0] = v.x; hc[4 * g4 + 1] = v.y; hc[4 * g4 + 2] = v.z; hc[4 * g4 + 3] = v.w;
        }
        cs_f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            __builtin_bit_cast(cs_bf16x8, a[ct][0]), __builtin_bit_cast(cs_bf16x8, b[0]), hc, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < KS; ++s)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              __builtin_bit_cast(cs_bf16x8, a[ct][s]), __builtin_bit_cast(cs_bf16x8, b[s]), acc, 0, 0, 0);
        int m = 0x7fffffff;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const int k0 = (__float_as_int(acc[r]) & kmask) | r;
          const int k1 = (__float_as_int(acc[r + 1]) & kmask) | (r + 1);
          m = min(min(m, k0), k1);
        }
        const bool take = m < bkey;          // strict: ties keep the lower tile
        bkey = take ? m : bkey;
        bsub = take ? cb : bsub;
      }
      // decode, merge the two lane halves (same point, disjoint centre rows)
      const int r = bkey & 31;
      const uint32_t dbits = (uint32_t)(bkey & ~31);
      const uint32_t id = (uint32_t)(bsub + (r & 3) + 8 * (r >> 2) + 4 * h);
      const unsigned long long mine = ((unsigned long long)dbits << 32) | id;
      auto sl = __builtin_amdgcn_permlane32_swap((uint32_t)mine, (uint32_t)mine, false, false);
      auto sh = __builtin_amdgcn_permlane32_swap((uint32_t)(mine >> 32), (uint32_t)(mine >> 32),
                                                 false, false);
      const unsigned long long other =
          ((unsigned long long)(h ? sh[0] : sh[1]) << 32) | (h ? sl[0] : sl[1]);
      const unsigned long long best = other < mine ? other : mine;
      if (h == 0) s_res[it & 1][wid][t * 32 + cl] = best;
    }
  }
  // last group: wait for every wave's parked results, then combine
  __syncthreads();
  if (wid == kStoreWave && iters > 0) combine(iters - 1);
  if (sse != nullptr) {
    double s = my_sse;
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
    if (wid == kStoreWave && lane == 0) atomicAdd(sse + (blockIdx.x & sse_mask), s);
  }
}

template <int DP, int NCT>
hipError_t launch_cs(const void* X, int64_t n, int64_t ldx, const void* Cq, const float* hn,
                     const float* xh, float M, int* assign, float* mind, double* sse,
                     int sse_mask, int cus, hipStream_t st) {
  constexpr int G = 2, NBUF = 6;
  const int64_t ngroup = ((n + 31) / 32 + G - 1) / G;
  const int64_t grid = ngroup < cus ? ngroup : cus;
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL((kmeans_assign_cs_kernel<DP, NCT, G, NBUF>), dim3((unsigned)grid),
                     dim3(kNW * 64), 0, st, reinterpret_cast<const uint16_t*>(X), n, ldx,
                     reinterpret_cast<const uint16_t*>(Cq), hn, xh, M, assign, mind, sse, sse_mask);
  return hipGetLastError();
}

}  // namespace
}  // namespace dalgo

extern "C" {

// kpad must be 256, 512 or 1024 (8 waves x NCT 32-centre tiles); DP 64 or 128; bf16
hipError_t dalgo_kmeans_assign_cs(const void* X, int64_t n, int64_t ldx, int DP, const void* Cq,
                                  int kpad, const float* hn, const float* xh, float M, int* assign,
                                  float* mind, double* sse, int sse_mask, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (cus <= 0) cus = 256;
  using namespace dalgo;
#define DALGO_CS(DPV, KP, NCTV)                                                                 \
  if (DP == DPV && kpad == KP)                                                                  \
    return launch_cs<DPV, NCTV>(X, n, ldx, Cq, hn, xh, M, assign, mind, sse, sse_mask, cus, st);
  DALGO_CS(128, 1024, 4)
  DALGO_CS(128, 512, 2)
  DALGO_CS(128, 256, 1)
  DALGO_CS(64, 1024, 4)
  DALGO_CS(64, 512, 2)
  DALGO_CS(64, 256, 1)
#undef DALGO_CS
  return hipErrorInvalidValue;
}

}  // extern "C"
