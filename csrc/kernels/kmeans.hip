// K2 + K3 + centroid update: distributed Lloyd k-means on MFMA.
//
// Reference: machine_learning/k-means.py — closest_center (:20-28) is an O(k*d)
// Python loop per point, reduceByKey (:62-63) sums (point, 1) per cluster and
// the driver replaces non-empty centres (:66-71).
//
// K2 kmeans_assign  — fused distance GEMM + argmin, never materialising N x k:
//   score(x, c) = x.c - 0.5*|c|^2  (argmax score == argmin |x-c|^2).
//   MFMA 32x32x16 bf16 (or 32x32x2 f32): A = 32 centres (rows of D), B = 32 points
//   (columns of D), so each lane owns ONE point and 16 of the 32 centres of the
//   tile in its accumulator registers -> the argmin is a per-lane register scan
//   (no cross-lane work until one final permlane32 swap). The accumulator is
//   initialised with -0.5|c|^2 (row constants as the initial accumulator) so the
//   epilogue is one compare + two selects per element. Centres stream through a
//   double-buffered, XOR-swizzled LDS chunk (32 centres) shared by the block's
//   NW*PT*32 points; point fragments stay in VGPRs for the whole sweep.
//   Ties resolve to the lowest centre id (the reference's strict '<', :25).
// K3 kmeans_accumulate — per-cluster sums and counts without global float
//   atomics per row: block (row-chunk r, cluster-range q) gathers only the rows
//   of chunk r whose cluster lies in range q and accumulates them in an LDS
//   table (ds_add_f32), then adds the table to the global [k x d] sums once.
//   Every X row is read exactly once overall.
// kmeans_update — c = S/n for non-empty clusters, keep the stale centre
//   otherwise (k-means.py:70-71); writes the f32 master, the padded MFMA copy,
//   0.5|c~|^2 of the ROUNDED copy (consistent scores) and the squared shift.
#include <cstdlib>
#include "dalgo/common.h"
#include "launchers.h"
#include <algorithm>

namespace dalgo {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <typename T> struct KTraits;
// bf16: one 16-wide k-step per MFMA, 8 elements (16 B) per lane per k-step
template <> struct KTraits<uint16_t> { static constexpr int ELEMS_PER_LOAD = 8; static constexpr int KSTEPS_PER_LOAD = 1; };
// f32: 2-wide k-steps; a 16-B load (4 floats) feeds 4 k-steps with the permuted
// k order  k(step 4q+u, half h) = 8q + 4h + u  used for BOTH operands
template <> struct KTraits<float>    { static constexpr int ELEMS_PER_LOAD = 4; static constexpr int KSTEPS_PER_LOAD = 4; };

template <typename T, int DP>
struct KGeom {
  static constexpr int ROWB = DP * (int)sizeof(T);       // bytes per centre row
  static constexpr int NJ = ROWB / 16;                    // 16-B pieces per row
  static constexpr int SWZ = (NJ >= 16 ? 16 : NJ) - 1;    // XOR swizzle mask
  static constexpr int CHUNKB = 32 * ROWB;                // one 32-centre chunk
  static constexpr int NLOAD = DP / (2 * KTraits<T>::ELEMS_PER_LOAD);  // 16-B loads per lane per point
};

__device__ __forceinline__ f32x16 mfma_step(const uint4& a, const uint4& b, f32x16 c, uint16_t) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_step(const uint4& a, const uint4& b, f32x16 c, float) {
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.x), __uint_as_float(b.x), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.y), __uint_as_float(b.y), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.z), __uint_as_float(b.z), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.w), __uint_as_float(b.w), c, 0, 0, 0);
  return c;
}

__device__ __forceinline__ float sq_sum(const uint4& v, uint16_t) {
  float s = 0.f, f;
  f = bf16lo(v.x); s = fmaf(f, f, s); f = bf16hi(v.x); s = fmaf(f, f, s);
  f = bf16lo(v.y); s = fmaf(f, f, s); f = bf16hi(v.y); s = fmaf(f, f, s);
  f = bf16lo(v.z); s = fmaf(f, f, s); f = bf16hi(v.z); s = fmaf(f, f, s);
  f = bf16lo(v.w); s = fmaf(f, f, s); f = bf16hi(v.w); s = fmaf(f, f, s);
  return s;
}
__device__ __forceinline__ float sq_sum(const uint4& v, float) {
  float a = __uint_as_float(v.x), b = __uint_as_float(v.y), c = __uint_as_float(v.z),
        d = __uint_as_float(v.w);
  return a * a + b * b + c * c + d * d;
}

// X: [n, ldx] (columns [d, DP) must be zero), Cq: [kpad, DP] (rows >= k zero),
// hn: [kpad] = 0.5|c|^2 (1e30 for padding centres).
// NSUB 32-centre sub-tiles are staged per barrier (chunk = 32*NSUB centres);
// kpad must be a multiple of 32*NSUB.
template <typename T, int DP, int PT, int NW, int NSUB, int MINW>
__global__ void __launch_bounds__(NW * 64, MINW)
kmeans_assign_kernel(const T* __restrict__ X, int64_t n, int64_t ldx, const T* __restrict__ Cq,
                     const float* __restrict__ hn, int kpad, int* __restrict__ assign,
                     float* __restrict__ mind, double* __restrict__ sse, int sse_mask) {
  using G = KGeom<T, DP>;
  constexpr int NT = NW * 64;
  constexpr int CH = 32 * NSUB;
  constexpr int CHUNKB = NSUB * G::CHUNKB;
  constexpr int NPIECE = CHUNKB / 16;
  constexpr int PER_T = (NPIECE + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) unsigned char s_c[2][CHUNKB];
  __shared__ __attribute__((aligned(16))) float s_hn[2][CH];
  __shared__ double s_sse[NW];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, cl = lane & 31;
  const int64_t pbase = ((int64_t)blockIdx.x * NW + wid) * (PT * 32);

  // ---- point fragments (B operand) resident in VGPRs for the whole sweep
  uint4 bf[PT][G::NLOAD];
  float xn[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    const int64_t p = pbase + t * 32 + cl;
    xn[t] = 0.f;
#pragma unroll
    for (int s = 0; s < G::NLOAD; ++s) {
      if (p < n) {
        bf[t][s] = *reinterpret_cast<const uint4*>(X + p * ldx + (2 * s + h) * KTraits<T>::ELEMS_PER_LOAD);
      } else {
        bf[t][s] = make_uint4(0u, 0u, 0u, 0u);
      }
      xn[t] += sq_sum(bf[t][s], T{});
    }
  }

  float best[PT];
  int bidx[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) { best[t] = -3.0e38f; bidx[t] = 0; }

  const int nchunk = kpad / CH;
  const unsigned char* Cb = reinterpret_cast<const unsigned char*>(Cq);
  uint4 stg[PER_T];
  float stg_h = 0.f;
  auto stage_load = [&](int ch) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int piece = tid + i * NT;
      if (piece < NPIECE)
        stg[i] = *reinterpret_cast<const uint4*>(Cb + (int64_t)ch * CHUNKB + piece * 16);
    }
    if (tid < CH) stg_h = hn[ch * CH + tid];
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int piece = tid + i * NT;
      if (piece < NPIECE) {
        const int cc = piece / G::NJ, j = piece % G::NJ;   // centre within chunk (row-major: sub-tiles contiguous)
        *reinterpret_cast<uint4*>(&s_c[buf][cc * G::ROWB + ((j ^ (cc & G::SWZ)) << 4)]) = stg[i];
      }
    }
    if (tid < CH) s_hn[buf][tid] = stg_h;
  };

  stage_load(0);
  stage_store(0);
  __syncthreads();
  for (int ch = 0; ch < nchunk; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nchunk) stage_load(ch + 1);   // in flight under the MFMAs
#pragma unroll
    for (int sub = 0; sub < NSUB; ++sub) {
      // accumulator init = -0.5|c|^2 of the centre each register holds
      f32x16 acc[PT];
      {
        float4 h4[4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
          h4[g] = *reinterpret_cast<const float4*>(&s_hn[buf][32 * sub + 8 * g + 4 * h]);
#pragma unroll
        for (int t = 0; t < PT; ++t) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            acc[t][4 * g + 0] = -h4[g].x; acc[t][4 * g + 1] = -h4[g].y;
            acc[t][4 * g + 2] = -h4[g].z; acc[t][4 * g + 3] = -h4[g].w;
          }
        }
      }
      const unsigned char* sub_base = &s_c[buf][sub * G::CHUNKB];
#pragma unroll
      for (int s = 0; s < G::NLOAD; ++s) {
        const int j = 2 * s + h;
        const uint4 a = *reinterpret_cast<const uint4*>(&sub_base[cl * G::ROWB + ((j ^ (cl & G::SWZ)) << 4)]);
#pragma unroll
        for (int t = 0; t < PT; ++t) acc[t] = mfma_step(a, bf[t][s], acc[t], T{});
      }
      // running argmax over this lane's 16 centres, ascending centre order
#pragma unroll
      for (int t = 0; t < PT; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = ch * CH + sub * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float v = acc[t][r];
          const bool take = v > best[t];
          best[t] = take ? v : best[t];
          bidx[t] = take ? c : bidx[t];
        }
      }
    }
    if (ch + 1 < nchunk) {
      stage_store(buf ^ 1);
    }
    __syncthreads();
  }

  // ---- combine the two lane halves (same point, disjoint centre subsets)
  double my_sse = 0.0;
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    auto rb = __builtin_amdgcn_permlane32_swap(__float_as_uint(best[t]), __float_as_uint(best[t]), false, false);
    auto ri = __builtin_amdgcn_permlane32_swap((uint32_t)bidx[t], (uint32_t)bidx[t], false, false);
    auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(xn[t]), __float_as_uint(xn[t]), false, false);
    const float pb = __uint_as_float(h ? rb[0] : rb[1]);
    const int pi = (int)(h ? ri[0] : ri[1]);
    const float px = __uint_as_float(h ? rx[0] : rx[1]);
    float b = best[t];
    int bi = bidx[t];
    if (pb > b || (pb == b && pi < bi)) { b = pb; bi = pi; }
    const float x2 = xn[t] + px;
    const int64_t p = pbase + t * 32 + cl;
    if (h == 0 && p < n) {
      const float dist = fmaxf(x2 - 2.f * b, 0.f);
      assign[p] = bi;
      if (mind) mind[p] = dist;
      my_sse += (double)dist;
    }
  }
  if (sse) {
    // wave sum in f64 via two f32 halves is overkill; a plain LDS pass is enough
    __shared__ double s_part[NW * 64];
    s_part[tid] = my_sse;
    __syncthreads();
    if (lane == 0) {
      double s = 0.0;
      for (int i = 0; i < 64; ++i) s += s_part[wid * 64 + i];
      s_sse[wid] = s;
    }
    __syncthreads();
    if (tid == 0) {
      double s = 0.0;
      for (int w = 0; w < NW; ++w) s += s_sse[w];
      atomicAdd(sse + (blockIdx.x & sse_mask), s);
    }
  }
}

// ---------------------------------------------------------------------------
// K2 "pipelined" form (bf16): distance keys + LDS-DMA centre chunks, built so the
// MFMA pipe is not starved by LDS waits, barriers or a long VALU epilogue:
//  * centre chunks (32*NSUB rows) go global -> LDS by LDS-DMA (global_load_lds_dwordx4,
//    no staging VGPRs), triple-buffered: chunk ch+2 is in flight while ch is consumed,
//    and one raw s_barrier per chunk both publishes chunk ch and retires chunk ch-1;
//  * the MFMA produces a shifted half-distance directly: B = -x (sign bits flipped
//    once), C = 0.5|c|^2 + M with M = max over the block's points of 0.5|x|^2, so
//    acc = 0.5|x - c|^2 + (M - 0.5|x|^2) >= 0 for every (point, centre) of the block;
//    C comes from an LDS-resident copy of 0.5|c|^2 + M (no accumulator-init moves);
//  * non-negative floats order like their int bits, so the per-sub-tile argmin is an
//    integer min over keys (bits & ~31) | r: one v_and_or + half a v_min3 per
//    distance (the compare / two-select form costs 3 VALU); the 5 dropped bits are
//    2^-18 relative, far below the bf16 operand rounding. A strict compare per
//    sub-tile keeps ties at the lowest id (ascending centre order per lane);
//  * the next sub-tile's A fragments and C values are read under the current MFMAs.
// Two 4-wave blocks per CU (launch_bounds min 2 -> 256 VGPRs, 2 waves/SIMD): one
// block's point loads and first chunk overlap the other block's MFMAs.
// The source side of the LDS-DMA carries the XOR swizzle (the LDS image is written
// lane-linear): slot (row, jj) holds piece jj ^ (row & SWZ) of centre `row`.
template <int N>
__device__ __forceinline__ void km_wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}
typedef __attribute__((address_space(3))) void km_lds_void;

// SWP (software-pipelined argmin): the MFMA chains of sub-tile s run in the same basic
// block as the argmin VALU of sub-tile s-1 (its accumulators stay live one sub-tile
// longer), so the key/min work of the LAST sub-tile of a chunk no longer runs MFMA-less
// after the chunk's final MFMA (s_nop hazard pad + ~50 VALU + DMA issue + barrier + LDS
// fragment latency per chunk in the plain form): it fills the issue gaps of the next
// chunk's first MFMAs instead. Only the last point tile's reduction is deferred (16
// accumulator VGPRs instead of 16 * PT); the earlier tiles' reductions overlap the later
// tiles' MFMA chains.
// TOP2 (bound-filtered Lloyd): also keep each point's second-smallest key and write the
// second-best distance (a lower bound: keys are truncated downwards) to mind2.
//
// Work distribution: the grid walks "block tiles" of NW * PT * 32 points, block b taking
// tiles b, b + gridDim.x, ... (one tile per block when the launcher sizes the grid to the
// tile count). The number of rows may live on the device (`mcount`, the bound filter's
// active count): the launcher then sizes a resident grid (blocks per CU x CUs) for the
// worst case and no host sync is needed to launch.
// Optional outputs of a full pass (the first bound-filtered iteration): xh[row] = 0.5|x|^2
// and *xmax = max over the rows of 0.5|x|^2 (float bits, non-negative: integer max).
// LOOP (the filtered iterations) also fuses the bound update that followed K2: instead
// of mind / mind2 it writes u = sqrt(dist + tol) rounded up and l = sqrt(dist2 - tol)
// rounded down (tol on the device), and appends the rows whose cluster differs from
// a_prev[row] to `changed` through a per-block LDS buffer (one global atomic per flush).
struct KmAux {
  const unsigned long long* mcount;   // device row count (LOOP)
  float* xh;                          // full pass: 0.5|x|^2 per row
  unsigned* xmax;                     // full pass: max 0.5|x|^2 (float bits)
  const int* a_prev;                  // LOOP: cluster before this iteration
  const float* tol;                   // LOOP: slack of a kernel distance
  float2* ul;                         // LOOP: (u, l) per row: upper bound of the distance
                                      //       to the centre, lower bound of every other
  int* changed;                       // LOOP: rows whose cluster changed ...
  unsigned long long* n_changed;      //       ... and their number
  long long cap;                      //       capacity of `changed`
  int* chg_new;                       // LOOP (optional): their new and previous cluster,
  int* chg_old;                       //       aligned with `changed` (the moved-row sort
                                      //       then reads them sequentially)
  const int* acl;                     // LOOP (optional, no a_prev): previous cluster of the
                                      //       active row at list position p (the filter's
                                      //       output order); neither: assign[row] itself
  // CAND (candidate-pruned LOOP): the active rows sorted by cluster (idx), tiles that never
  // straddle two clusters, and each centre's neighbour lists (km_centre_nbrs_kernel)
  const int4* tiles;                  // tile t: (cluster, first, end position in idx, -)
  const unsigned long long* n_tiles;  // device tile count
  const float* hnb;                   // [k][kpad]: 0.5|c|^2 in neighbour order of centre a
  const int32_t* nb;                  // [k][kpad]: their ids
  const float* nd;                    // [k][kpad]: |c - c_a| rounded down, ascending
  int extend;                         // CAND: stream more chunks where l would be loose
  // CAND + DRIFT: per list entry (aligned with nb) its distance to c_a (rounded down) and
  // its centre's shift since the last iteration (rounded up)
  const float* ndb;
  const float* dnb;
  const float* tau_cap;               // DRIFT (device, nullable): largest pruning threshold
  int drift_ball;                     // DRIFT: also drop the centres outside the ball R (their
                                      // bound nd_first - ua is loose where ua is small)
};
constexpr int kChgBuf = 512;          // changed rows buffered per block (LDS)

__device__ __forceinline__ float km_up1(float x) { return nextafterf(x, __builtin_inff()); }
__device__ __forceinline__ float km_dn1(float x) { return nextafterf(x, -__builtin_inff()); }

#ifdef KM_XP_TIMING
// timing experiment: per-tile phase clocks of the first blocks (wave 0, lane 0)
constexpr int kDbgBlocks = 64, kDbgTiles = 64, kDbgSlots = 16;
__device__ unsigned long long g_km_dbg[kDbgBlocks * kDbgTiles * kDbgSlots];
#define KM_TS(slot)                                                                          \
  if (CAND && lane == 0 && (wid == 0 || wid == NW - 1) && blockIdx.x < kDbgBlocks &&        \
      dbg_it < kDbgTiles)                                                                    \
    g_km_dbg[((int)blockIdx.x * kDbgTiles + dbg_it) * kDbgSlots + (slot) + (wid == 0 ? 0 : 8)] = \
        __builtin_amdgcn_s_memtime();
#else
#define KM_TS(slot)
#endif

template <int DP, int NW, int PT, int NSUB, int MINB, int NBUF, bool PF, bool TOP2 = false,
          bool LOOP = false, bool CAND = false, bool DRIFT = false>
__global__ void __launch_bounds__(NW * 64, MINB)
kmeans_assign_pipe_kernel(const uint16_t* __restrict__ X, int64_t n, int64_t ldx,
                          const uint16_t* __restrict__ Cq, const float* __restrict__ hn, int kpad,
                          int* __restrict__ assign, float* __restrict__ mind,
                          double* __restrict__ sse, int sse_mask,
                          const int32_t* __restrict__ idx, float* __restrict__ mind2,
                          const KmAux aux) {
  static_assert(!LOOP || TOP2, "the fused bound update needs the second-best distance");
  static_assert(!CAND || LOOP, "candidate pruning is a form of the filtered iteration");
  static_assert(!DRIFT || CAND, "drift pruning refines the candidate lists");
  // idx (optional): the block's point j is row idx[j] of X (and of assign / mind), j < n
  // -- the bound-filtered form of Lloyd only re-assigns the points the filter keeps
  constexpr int KS = DP / 16;                  // 32x32x16 k-steps per centre row
  constexpr int NJ = DP * 2 / 16;              // 16-B pieces per row (= 2 KS)
  constexpr int SWZ = (NJ >= 16 ? 16 : NJ) - 1;
  constexpr int CH = 32 * NSUB;
  constexpr int NT = NW * 64;
  constexpr int CHP = CH * NJ;                 // 16-B pieces per chunk
  constexpr int GPT = CHP / NT;                // LDS-DMA instructions per thread per chunk
  constexpr int TILE = NW * PT * 32;           // points per block tile
  static_assert(CHP % NT == 0, "chunk must be a whole number of block-wide DMA rounds");
  static_assert((NT / NJ) % (SWZ + 1) == 0, "DMA swizzle must repeat every block-wide round");
  static_assert(NBUF >= 2 && NBUF <= 4, "double, triple or quadruple buffered chunks");
  __shared__ __attribute__((aligned(16))) uint4 s_c[NBUF * CHP];
  extern __shared__ __attribute__((aligned(16))) float s_hn[];   // [kpad]: 0.5|c|^2 + M
  __shared__ float s_m[NW];
  __shared__ float s_r[NW];
  __shared__ int s_ext[NW];
  __shared__ float s_tau[DRIFT ? NW : 1];
  __shared__ int s_kc[DRIFT ? NW : 1];
  __shared__ float s_kd[DRIFT ? NW : 1], s_kf[DRIFT ? NW : 1];
  // DRIFT: every tile row's l (read again by the epilogue: not held in VGPRs over the sweep)
  __shared__ float s_lold[DRIFT ? NW * PT * 32 : 1];
  __shared__ double s_sse[NW];

  __shared__ int s_chg[LOOP ? kChgBuf : 1];
  __shared__ uint16_t s_chgn[LOOP ? kChgBuf : 1], s_chgo[LOOP ? kChgBuf : 1];
  // CAND: the tile cluster's neighbour list (ids, k <= 1024), double-buffered by tile parity
  // so a tile can stage its list before the barrier that ends the previous tile's reads
  __shared__ uint16_t s_nb[CAND ? 2 : 1][CAND ? 1024 : 1];
  // CAND: the tile cluster's centre c_acl, one copy per wave (each wave DMAs its own: no
  // barrier before its reads)
  __shared__ __attribute__((aligned(16))) uint4 s_ca[CAND ? NW : 1][CAND ? NJ : 1];
  int par = 0;
#ifdef KM_XP_TIMING
  int dbg_it = 0;
#endif
  __shared__ int s_nchg;
  __shared__ unsigned long long s_chg_base;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, cl = lane & 31;
  const int nchunk = kpad / CH;
  if (aux.mcount != nullptr) n = min(n, (int64_t)*aux.mcount);
  float tol = 0.f;
  if constexpr (LOOP) {
    tol = *aux.tol;
    if (tid == 0) s_nchg = 0;
  }
  // LOOP: move the buffered changed rows to the global list (block-uniform call)
  auto flush_changed = [&]() {
    __syncthreads();
    const int c = s_nchg;
    if (c > 0) {
      if (tid == 0) s_chg_base = atomicAdd(aux.n_changed, (unsigned long long)c);
      __syncthreads();
      const long long b = (long long)s_chg_base;
      for (int j = tid; j < c; j += NT)
        if (b + j < aux.cap) {
          aux.changed[b + j] = s_chg[j];
          if (aux.chg_new) {
            aux.chg_new[b + j] = s_chgn[j];
            aux.chg_old[b + j] = s_chgo[j];
          }
        }
      __syncthreads();
      if (tid == 0) s_nchg = 0;
    }
    __syncthreads();
  };
  const int64_t ntile = CAND ? (int64_t)*aux.n_tiles : (n + TILE - 1) / TILE;

  // per-thread DMA sources: slot q = g*NT + tid of the chunk image
  int src_off[GPT];
#pragma unroll
  for (int g = 0; g < GPT; ++g) {
    const int q = g * NT + tid, row = q / NJ, jj = q % NJ;
    src_off[g] = row * DP + (jj ^ (row & SWZ)) * 8;
  }
  // Issued as inline asm: with the builtin, hipcc cannot tell the DMA target from the
  // chunk being read and drains vmcnt(0) before every ds_read (the chunk in flight
  // would then never overlap compute). The counted waits below are the only waits.
  const uint32_t lds0 = (uint32_t)(uintptr_t)(km_lds_void*)s_c;
  auto issue = [&](int ch) {
    const uint16_t* base = Cq + (int64_t)ch * CH * DP;
    const uint32_t dst = lds0 + (uint32_t)(((ch % NBUF) * CHP) * 16);
#pragma unroll
    for (int g = 0; g < GPT; ++g) {
      const uint32_t m0v = __builtin_amdgcn_readfirstlane(dst + (uint32_t)((g * NT + wid * 64) * 16));
      if constexpr (CAND) {
        // gather: chunk row r of the tile's stream is centre s_nb[par][ch * CH + r] of Cq
        // (L2-resident); src_off[g] = r * DP + piece offset. SGPR base + 32-bit offset
        // (NT / NJ is a multiple of SWZ + 1: the swizzled piece is the same for every g)
        const int rr = tid / NJ, r = g * (NT / NJ) + rr;
        const uint32_t pz = (uint32_t)(((tid % NJ) ^ (rr & SWZ)) * 8);
        const uint32_t off = ((uint32_t)s_nb[par][ch * CH + r] * DP + pz) * 2u;
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                     :: "s"(m0v), "v"(off), "s"(Cq) : "memory");
      } else {
        const uint16_t* src = base + src_off[g];
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                     :: "s"(m0v), "v"(src) : "memory");
      }
    }
  };
  int kmask;   // key mask in a VGPR so each pack is ONE v_and_or_b32 (VGPR mask, inline r)
  asm volatile("v_mov_b32 %0, 0xffffffe0" : "=v"(kmask));
  // lane's A-row base inside a chunk image: row = sub*32 + cl, piece (2s + h) ^ (cl & SWZ)
  const int arow = cl * NJ;
  const int asw = cl & SWZ;
  double my_sse = 0.0;
  float my_xmax = 0.f;

  // CAND: the next tile's record (with the current tile's set-up loads) and row ids (after
  // the current tile's chunk-0 DMA) are loaded during the current tile, so a tile starts
  // with its point loads instead of a chain of three
  int4 trn = make_int4(0, 0, 0, 0);
  int idxn[CAND ? PT : 1];
  auto load_rec = [&](int64_t bt) {
    if constexpr (CAND) trn = bt < ntile ? aux.tiles[bt] : make_int4(0, 0, 0, 0);
  };
  auto load_ids = [&]() {
    if constexpr (CAND) {
      // always PT loads per lane (clamped): the chunk-0 wait counts them
      const int64_t hi = trn.z > trn.y ? (int64_t)trn.z - 1 : 0;
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        const int64_t p = min((int64_t)trn.y + wid * (PT * 32) + t * 32 + cl, hi);
        idxn[t] = idx[p];
      }
    }
  };
  // one block tile (a lambda so the single-tile launch compiles to straight-line code:
  // the loop form costs registers the 3-tile plain form does not have)
  auto tile = [&](const int64_t bt) {
  KM_TS(0)
#ifdef KM_XP_TIMING
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  KM_TS(7)
#endif
  // CAND: tile bt = up to TILE positions of one cluster's run in idx
  int acl = 0;
  int64_t pbase, pend = n;
  const float* hbase = hn;
  if constexpr (CAND) {
    const int4 tr = trn;
    acl = tr.x;
    pend = tr.z;
    pbase = (int64_t)tr.y + (int64_t)wid * (PT * 32);
    hbase = aux.hnb + (int64_t)acl * kpad;
    par ^= 1;
  } else {
    pbase = (bt * NW + wid) * (PT * 32);
  }

  // ---- points (B operand, negated), resident for the whole sweep; rows past n are zero
  uint4 bf[PT][KS];
  float x2[PT];                                // |x|^2 of the lane's point (both halves)
  float ua[CAND ? PT : 1];                     // CAND: bound on |x - c_acl| (from chunk 0)
  uint32_t pmask[CAND ? 1 : PT];               // !CAND: ~0 for the lane's rows inside the tile
  int rowk[CAND ? PT : 1];                     // CAND: the lane's rows (kept for the epilogue:
                                               // no second, dependent idx read there)
  if constexpr (CAND) {
    // The tile's rows are scattered over X. Loaded straight into the fragment layout, each
    // wave-instruction would touch 32 rows (32 B of each): the per-line cost of those
    // gathers made the load the longest phase of a tile. Instead they are gathered into
    // LDS (the chunk buffers, free until chunk 0 is issued after the set-up barrier) by
    // LDS-DMA in whole-row pieces -- NJ lanes per row, 64 / NJ rows per instruction, the
    // XOR swizzle on the source side -- and read back as B fragments below.
    static_assert(NW * PT * 32 * NJ <= NBUF * CHP, "the point tile must fit the chunk buffers");
    constexpr int RPI = 64 / NJ;                 // rows per wave-instruction
    // the row ids (prefetched during the previous tile) are consumed here, before the
    // first DMA: the compiler does not see the DMAs (inline asm), and a wait it placed
    // for an id inside the DMA loop would also drain the DMAs issued before it
#pragma unroll
    for (int t = 0; t < PT; ++t) rowk[t] = idxn[t];
    asm volatile("" :: "v"(rowk[0]), "v"(rowk[PT - 1]));
    __syncthreads();                             // every wave is past the last tile's chunk reads
    {
      // c_acl first (the lane term opaque per tile, so its address is not a hoisted,
      // spilled loop invariant whose reload would wait for the point DMAs)
      int lq = lane;
      asm volatile("" : "+v"(lq));
      if (lq < NJ) {
        const uint16_t* src = Cq + ((int64_t)acl * DP + lq * 8);
        const uint32_t m0v = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(km_lds_void*)&s_ca[wid][0]);
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                     :: "s"(m0v), "v"(src) : "memory");
      }
    }
    const int rsub = lane / NJ, q = lane % NJ;
    const uint32_t wbase = lds0 + (uint32_t)(wid * PT * 32 * NJ * 16);
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int idt = rowk[t];
      // (not unrolled: 16 precomputed 64-bit addresses would spill the fragment registers)
#pragma unroll 1
      for (int g = 0; g < 32 / RPI; ++g) {
        const int rc = g * RPI + rsub;           // lane of the row's id in idxn[t]
        const int rl = t * 32 + rc;              // the wave's row
        const int rid = __shfl(idt, rc);
        const bool ok = pbase + rl < pend;
        const uint16_t* src = X + (int64_t)(ok ? rid : 0) * ldx + (q ^ (rl & SWZ)) * 8;
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(wbase + (uint32_t)(rl - rsub) * (NJ * 16));
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                     :: "s"(m0v), "v"(src) : "memory");
      }
    }
  } else {
    // unconditional loads (rows past the end read row 0), masked after the prologue wait
    // below: with a select, hipcc sank every load into its own branch and waited for it
    // there (24 serialized memory latencies per tile)
    // (the row ids first: a wait for one of them between two rows' loads would also
    // wait for the loads before it)
    int64_t rowv[CAND ? 1 : PT];
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int64_t p = pbase + t * 32 + cl;
      const bool ok = p < pend;
      pmask[t] = ok ? 0xffffffffu : 0u;
      rowv[t] = ok ? (idx ? (int64_t)idx[min(p, pend - 1)] : p) : 0;
    }
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const uint16_t* src = X + rowv[t] * ldx + h * 8;
#pragma unroll
      for (int s = 0; s < KS; ++s) bf[t][s] = *reinterpret_cast<const uint4*>(src + 16 * s);
    }
  }
  // CAND: everything the tile's set-up reads is loaded here, under the point loads (one
  // memory latency per tile instead of a chain): c_acl, the first distance of every
  // chunk of acl's list (lane j: nd[acl][j * CH]) and the list's 0.5|c|^2
  constexpr int KH = CAND ? 1024 / NT : 1;
  float thrv = __builtin_inff();
  float hv[KH];
  int nbv[KH];
  float hna = 0.f;                             // CAND: 0.5|c_acl|^2
  // DRIFT: entry p = KH tid + j of acl's list (consecutive per thread: one scan over the
  // threads compacts the list) -- its distance to c_acl and its centre's shift; and the
  // lower bound l of every tile row (vs the previous centres, from the last iteration)
  float ndv[DRIFT ? KH : 1], dnv[DRIFT ? KH : 1], lold[DRIFT ? PT : 1];
  if constexpr (CAND) {
    hna = hn[acl];
    if constexpr (DRIFT) {
      static_assert(KH == 4, "DRIFT: four consecutive list entries per thread");
      const bool in = tid * KH < kpad;
      const int64_t o = (int64_t)acl * kpad + tid * KH;
      const int4 i4 = in ? *reinterpret_cast<const int4*>(aux.nb + o) : make_int4(0, 0, 0, 0);
      const float4 h4 = in ? *reinterpret_cast<const float4*>(hbase + tid * KH) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float inf = __builtin_inff();
      const float4 n4 = in ? *reinterpret_cast<const float4*>(aux.ndb + o) : make_float4(inf, inf, inf, inf);
      const float4 d4 = in ? *reinterpret_cast<const float4*>(aux.dnb + o) : make_float4(0.f, 0.f, 0.f, 0.f);
      nbv[0] = i4.x; nbv[1] = i4.y; nbv[2] = i4.z; nbv[3] = i4.w;
      hv[0] = h4.x; hv[1] = h4.y; hv[2] = h4.z; hv[3] = h4.w;
      ndv[0] = n4.x; ndv[1] = n4.y; ndv[2] = n4.z; ndv[3] = n4.w;
      dnv[0] = d4.x; dnv[1] = d4.y; dnv[2] = d4.z; dnv[3] = d4.w;
      const float* ulf = reinterpret_cast<const float*>(aux.ul);
#pragma unroll
      for (int t = 0; t < PT; ++t) lold[t] = ulf[2 * (int64_t)rowk[t] + 1];
    } else {
      if (lane < nchunk) thrv = aux.nd[(int64_t)acl * kpad + lane * CH];
#pragma unroll
      for (int j = 0; j < KH; ++j) {
        const bool in = tid + j * NT < kpad;
        hv[j] = in ? hbase[tid + j * NT] : 0.f;
        nbv[j] = in ? aux.nb[(int64_t)acl * kpad + tid + j * NT] : 0;
      }
    }
    load_rec(bt + gridDim.x);            // the next tile's record (tr holds this one's)
  }
  // all ordinary loads retired before the DMA stream starts, and the fragments pinned
  // here, so the compiler's own waits never drain a chunk in flight (vmcnt(0) in-loop)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  KM_TS(1)
  // the next record is consumed here (retired above), so that the compiler's own wait
  // for it is not placed after the chunk-0 DMA, where it would drain that DMA
  if constexpr (CAND) asm volatile("" :: "v"(trn.y), "v"(trn.z));
  if constexpr (!CAND) {
#pragma unroll
    for (int t = 0; t < PT; ++t)
#pragma unroll
      for (int s = 0; s < KS; ++s)
        bf[t][s] = make_uint4(bf[t][s].x & pmask[t], bf[t][s].y & pmask[t], bf[t][s].z & pmask[t],
                              bf[t][s].w & pmask[t]);
  }
  if constexpr (CAND) {
    // the wave's own rows (its DMA, retired above): no barrier needed before the reads.
    // Branch-free (unconditional reads, masked), and the swizzle term made opaque per
    // tile: hoisted out of the tile loop, the 16 read addresses were spilled, and each
    // read waited for its own scratch reload
    const uint4* img = s_c + wid * PT * 32 * NJ;
    int sw = cl & SWZ;                           // (t * 32 + cl) & SWZ
    asm volatile("" : "+v"(sw));
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int rl = t * 32 + cl;
      const uint32_t m = pbase + rl < pend ? 0xffffffffu : 0u;
      const uint4* rowp = img + rl * NJ;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const uint4 v = rowp[(2 * s + h) ^ sw];
        bf[t][s] = make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
      }
    }
    if constexpr (DRIFT) {
      // chunk 0 (acl and its CH - 1 nearest, always streamed) now; the rest of the list
      // is compacted after the tile's bounds are known
#pragma unroll
      for (int j = 0; j < KH; ++j)
        if (tid * KH + j < CH) s_nb[par][tid * KH + j] = (uint16_t)nbv[j];
    } else {
#pragma unroll
      for (int j = 0; j < KH; ++j)
        if (tid + j * NT < kpad) s_nb[par][tid + j * NT] = (uint16_t)nbv[j];
    }
    // every wave has its fragments (the chunk buffers are free again) and the list is
    // staged: chunk 0 -- always streamed -- goes out now, under the set-up below
    __syncthreads();
    issue(0);
    load_ids();                          // PT loads after the DMA: chunk 0 waits vmcnt(PT)
  }
  float mx = 0.f;
  // CAND: the lane's half of c_acl (same k layout as the point fragments, from the wave's
  // LDS copy one k-step at a time), for the exact distance of every tile point to its
  // cluster's centre (v_dot2 on the bf16 pairs)
  float qs[PT], dts[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) { qs[t] = 0.f; dts[t] = 0.f; }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    uint4 cas = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (CAND) cas = s_ca[wid][2 * s + h];
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      asm volatile("" : "+v"(bf[t][s].x), "+v"(bf[t][s].y), "+v"(bf[t][s].z), "+v"(bf[t][s].w));
      qs[t] += sq_sum(bf[t][s], uint16_t{});
      if constexpr (CAND) {
        const uint32_t xw[4] = {bf[t][s].x, bf[t][s].y, bf[t][s].z, bf[t][s].w};
        const uint32_t cw[4] = {cas.x, cas.y, cas.z, cas.w};
#pragma unroll
        for (int w = 0; w < 4; ++w)
          dts[t] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, xw[w]),
                                                   __builtin_bit_cast(bf16x2, cw[w]), dts[t], false);
      }
      bf[t][s] = make_uint4(bf[t][s].x ^ 0x80008000u, bf[t][s].y ^ 0x80008000u,
                            bf[t][s].z ^ 0x80008000u, bf[t][s].w ^ 0x80008000u);
    }
  }
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    const float q = qs[t], dt = dts[t];
    auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(q), __float_as_uint(q), false, false);
    x2[t] = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    mx = fmaxf(mx, 0.5f * x2[t]);
    if constexpr (CAND) {
      auto sd = __builtin_amdgcn_permlane32_swap(__float_as_uint(dt), __float_as_uint(dt), false, false);
      const float dot = __uint_as_float(sd[0]) + __uint_as_float(sd[1]);
      // |x - c|^2 = |x|^2 - 2 x.c + 2 hn (f32 error far below tol: the K2 slack)
      const float dist = fmaxf(x2[t] - 2.f * dot + 2.f * hna, 0.f);
      ua[t] = km_up1(sqrtf(km_up1(dist + tol)));
    }
  }
  for (int off = 32; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  my_xmax = fmaxf(my_xmax, mx);
  // the previous tile's waves are past every read of s_m / s_hn / the chunk buffers
  // (each crossed this tile's chunk barriers' predecessor: the last chunk barrier of the
  // previous tile precedes all of its reads), so the block barrier below orders the
  // rewrite after them
  float um = 0.f;
  float tv = __builtin_inff();                 // DRIFT: min over the tile rows of l - u
  if constexpr (CAND) {
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      if (pbase + t * 32 + cl < pend) {
        um = fmaxf(um, ua[t]);
        if constexpr (DRIFT) tv = fminf(tv, km_dn1(lold[t] - ua[t]));
      }
      // (the previous tile's epilogue reads of s_lold precede this tile's first barrier)
      if constexpr (DRIFT) if (h == 0) s_lold[(wid * PT + t) * 32 + cl] = lold[t];
    }
    for (int off = 32; off >= 1; off >>= 1) {
      um = fmaxf(um, __shfl_xor(um, off));
      if constexpr (DRIFT) tv = fminf(tv, __shfl_xor(tv, off));
    }
  }
  if (lane == 0) {
    s_m[wid] = mx;
    if constexpr (CAND) s_r[wid] = um;
    if constexpr (DRIFT) s_tau[wid] = tv;
  }
  __syncthreads();
  // CAND: the tile's centre stream is cluster acl's neighbour list. ua >= |x - c_acl| for
  // every tile point, so only centres c with |c - c_acl| <= R = 2 max ua can be the
  // nearest of one (|x - c| >= |c - c_acl| - |x - c_acl| > |x - c_acl| otherwise); nd is
  // ascending, so they are a prefix of the list: nch_t whole chunks of it. Every wave
  // finds the count by a two-level search of nd (all agree: no barrier)
  KM_TS(2)
  int nch_t = nchunk;
  float nd_first = __builtin_inff();   // CAND: smallest distance of a pruned centre
  float dmp = -__builtin_inff();       // DRIFT: largest shift of a drift-pruned centre
  int kept = 0;                        // DRIFT: list entries kept past chunk 0
  int sp[DRIFT ? KH : 1];              // DRIFT: stream position of the thread's entries
  if constexpr (CAND) {
    float R = s_r[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) R = fmaxf(R, s_r[w]);
    R = km_up1(2.f * R);
    if constexpr (DRIFT) {
      // Past chunk 0 an entry c of the list is streamed iff |c - c_acl| <= R (the ball) AND
      // its shift delta_c >= tau = min over the tile rows of (l - ua): l <= |x - c_prev| for
      // every c other than acl (last iteration's centres), so a centre with delta_c < tau has
      // |x - c| >= l - delta_c > ua >= |x - c_acl| for every tile row and cannot be the
      // nearest. The kept entries are compacted (block scan) behind chunk 0; the pruned
      // ones bound l by nd_first - ua (ball) and l - dmp (drift)
      float tau = s_tau[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) tau = fminf(tau, s_tau[w]);
      // a pruned centre costs the rows up to tau of their lower bound l (the next filter
      // tests l - maxd): the threshold is capped so only the slow centres are dropped
      if (aux.tau_cap != nullptr) tau = fminf(tau, *aux.tau_cap);
      int c = 0;
      float dm = -__builtin_inff(), nf = __builtin_inff();
      bool keep[KH];
#pragma unroll
      for (int j = 0; j < KH; ++j) {
        const int p = tid * KH + j;
        const bool tail = p >= CH && p < kpad;
        const bool ball = !aux.drift_ball || ndv[j] <= R;
        keep[j] = tail && ball && dnv[j] >= tau;
        c += keep[j] ? 1 : 0;
        // every dropped centre c has |x - c| >= l - delta_c (drift bound) and, outside the
        // ball, also >= |c - c_acl| - ua: the slow ones (delta_c < tau) enter the new l
        // through l - dmp, the fast ones outside the ball through nd_first - ua (the first
        // distance among them only, not among every dropped centre: tight l where ua is small)
        if (tail && !keep[j]) {
          if (dnv[j] < tau) dm = fmaxf(dm, dnv[j]);
          else nf = fminf(nf, ndv[j]);
        }
      }
      int x = c;
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      for (int off = 32; off >= 1; off >>= 1) {
        dm = fmaxf(dm, __shfl_xor(dm, off));
        nf = fminf(nf, __shfl_xor(nf, off));
      }
      if (lane == 63) s_kc[wid] = x;
      if (lane == 0) { s_kd[wid] = dm; s_kf[wid] = nf; }
      __syncthreads();
      int pre = x - c;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        if (w < wid) pre += s_kc[w];
        kept += s_kc[w];
        dmp = fmaxf(dmp, s_kd[w]);
        nd_first = fminf(nd_first, s_kf[w]);
      }
      nch_t = 1 + (kept + CH - 1) / CH;
#pragma unroll
      for (int j = 0; j < KH; ++j) {
        sp[j] = keep[j] ? CH + pre : -1;
        if (keep[j]) s_nb[par][CH + pre++] = (uint16_t)nbv[j];
      }
    } else {
      // chunk j >= 1 is needed iff its first (smallest) distance is <= R; chunk 0 always
      nch_t = 1 + __popcll(__ballot(lane >= 1 && lane < nchunk && thrv <= R));
    }
  }
  if constexpr (LOOP) {
    // every wave is past the previous tile's appends: room for this tile's (<= TILE)?
    if (s_nchg > kChgBuf - TILE) flush_changed();
  }
  float M = s_m[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) M = fmaxf(M, s_m[w]);
  // slack so that rounding of the MFMA sum cannot push a near-zero distance negative
  M = M * 1.0001f + 1e-6f;
  if constexpr (DRIFT) {
    // 0.5|c|^2 + M in stream order: chunk 0 as listed, the kept entries at their compacted
    // places (sp, from the scan), then padding up to whole chunks (acl, never the nearest:
    // 1e30 as hn's padding centres)
#pragma unroll
    for (int j = 0; j < KH; ++j) {
      const int p = tid * KH + j;
      if (p < CH) s_hn[p] = hv[j] + M;
      else if (sp[j] >= 0) s_hn[sp[j]] = hv[j] + M;
    }
    for (int q = CH + kept + tid; q < nch_t * CH; q += NT) {
      s_hn[q] = 1e30f + M;
      s_nb[par][q] = (uint16_t)acl;
    }
  } else if constexpr (CAND) {
#pragma unroll
    for (int j = 0; j < KH; ++j)
      if (tid + j * NT < kpad) s_hn[tid + j * NT] = hv[j] + M;   // extensions read past nch_t
  } else {
    for (int c = tid; c < kpad; c += NT) s_hn[c] = hbase[c] + M;
  }

  int bkey[PT], bsub[PT], bkey2[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) { bkey[t] = 0x7fffffff; bsub[t] = 0; bkey2[t] = 0x7fffffff; }

  auto load_frag = [&](const uint4* img, int sub, int cb, uint4 (&a)[KS], f32x16& hc) {
#pragma unroll
    for (int s = 0; s < KS; ++s) a[s] = img[sub * 32 * NJ + arow + ((2 * s + h) ^ asw)];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 v = *reinterpret_cast<const float4*>(&s_hn[cb + 8 * g + 4 * h]);
      hc[4 * g + 0] = v.x; hc[4 * g + 1] = v.y; hc[4 * g + 2] = v.z; hc[4 * g + 3] = v.w;
    }
  };

  // accumulators of the last point tile, reduced one sub-tile late. Initial keys are NaN
  // bits (0x7fffffe0 | r after masking): larger than any finite distance key, so the
  // dummy first reduction is displaced by the first real one.
  constexpr int T0 = PT - 1;                   // the deferred tile
  f32x16 pacc;
#pragma unroll
  for (int r = 0; r < 16; ++r) pacc[r] = __int_as_float(0x7fffffff);
  int pcb = 0;
  auto reduce_tile = [&](const f32x16& acc, int t, int cb) {
    int m = 0x7fffffff;
    if constexpr (TOP2) {
      // running pair (m <= m2) fed two keys at a time: with (x, y) new,
      //   m' = min3(m, x, y),  m2' = min(m2, med3(m, x, y))
      // (the second smallest of {m, m2, x, y}: if m2 is it, the median of {m, x, y}
      // -- the second of a set missing it -- is >= m2; otherwise both of the two
      // smallest are in {m, x, y} and their second is the median): 1.5 VALU per key
      // instead of 2 (med3 + min per key)
      int m2 = 0x7fffffff;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const int k0 = (__float_as_int(acc[r]) & kmask) | r;
        const int k1 = (__float_as_int(acc[r + 1]) & kmask) | (r + 1);
        int md;
        asm volatile("v_med3_i32 %0, %1, %2, %3" : "=v"(md) : "v"(m), "v"(k0), "v"(k1));
        m2 = min(m2, md);
        m = min(min(m, k0), k1);   // v_min3_i32
      }
      // merge with the running pair (bkey <= bkey2): second smallest of the four
      bkey2[t] = min(max(bkey[t], m), min(bkey2[t], m2));
    } else {
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const int k0 = (__float_as_int(acc[r]) & kmask) | r;
        const int k1 = (__float_as_int(acc[r + 1]) & kmask) | (r + 1);
        m = min(min(m, k0), k1);   // one v_min3_i32 per pair
      }
    }
    // strict: an equal key of a later sub-tile (higher ids) never displaces
    const bool take = m < bkey[t];
    bkey[t] = take ? m : bkey[t];
    bsub[t] = take ? cb : bsub[t];
  };

  if constexpr (!CAND) issue(0);
  if (NBUF >= 3 && nch_t > 1) issue(1);
  if (NBUF >= 4 && nch_t > 2) issue(2);
  for (int ch = 0; ch < nch_t; ++ch) {
    // chunk ch landed; chunks ch+1 .. ch+NBUF-2 stay in flight
    const int ahead = NBUF >= 3 ? min(NBUF - 2, nch_t - 1 - ch) : 0;
    if constexpr (NBUF >= 4) {
      if (ahead >= 2) km_wait_vmcnt<2 * GPT>();
      else if (ahead == 1) km_wait_vmcnt<GPT>();
      else km_wait_vmcnt<0>();
    } else if constexpr (NBUF == 3) {
      if (ahead >= 1) km_wait_vmcnt<GPT>();
      else km_wait_vmcnt<0>();
    } else {
      if constexpr (CAND) {
        if (ch == 0) km_wait_vmcnt<PT>();   // the next tile's row ids stay in flight
        else km_wait_vmcnt<0>();
      } else {
        km_wait_vmcnt<0>();
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // s_hn stores (first chunk)
    // publishes chunk ch to every wave AND retires everyone's reads of chunk ch-1,
    // whose buffer is refilled next (triple: chunk ch+2 after this chunk's MFMAs;
    // double: chunk ch+1 right away)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#ifdef KM_XP_TIMING
    if (ch == 0) { KM_TS(3) }
#endif
    if (NBUF == 2 && ch + 1 < nch_t) issue(ch + 1);
    const uint4* img = s_c + (ch % NBUF) * CHP;
    uint4 a[KS];
    f32x16 hc;
    load_frag(img, 0, ch * CH, a, hc);
#pragma unroll
    for (int sub = 0; sub < NSUB; ++sub) {
      const int cb = ch * CH + sub * 32;
      uint4 an[KS];
      f32x16 hn_next;
      if (PF && sub + 1 < NSUB) load_frag(img, sub + 1, cb + 32, an, hn_next);
      f32x16 cacc;
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            __builtin_bit_cast(bf16x8, a[0]), __builtin_bit_cast(bf16x8, bf[t][0]), hc, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < KS; ++s)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              __builtin_bit_cast(bf16x8, a[s]), __builtin_bit_cast(bf16x8, bf[t][s]), acc, 0, 0, 0);
        if (t == T0) cacc = acc;
        else reduce_tile(acc, t, cb);
      }
      // argmin of the previous sub-tile's last tile: independent of the MFMAs above
      reduce_tile(pacc, T0, pcb);
      pacc = cacc;
      pcb = cb;
      // pin the interleave: one MFMA, then a few argmin VALU ops, for every MFMA of
      // this sub-tile (hipcc otherwise clusters the MFMAs and sinks the VALU after them)
#pragma unroll
      for (int i = 0; i < PT * KS; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // VALU
      }
      if (sub + 1 < NSUB) {
        if constexpr (PF) {
#pragma unroll
          for (int s = 0; s < KS; ++s) a[s] = an[s];
          hc = hn_next;
        } else {
          load_frag(img, sub + 1, cb + 32, a, hc);
        }
      }
    }
    if (NBUF >= 3 && ch + NBUF - 1 < nch_t) issue(ch + NBUF - 1);
    if constexpr (CAND) {
      if (!DRIFT && aux.extend && ch == nch_t - 1 && nch_t < nchunk) {
        // The pruned centres bound l from below by nd_first - ua only. Where that is below
        // a point's second-best distance so far, its l (and the next iteration's filter)
        // would be loose: then the tile streams one more chunk (block-uniform decision)
        reduce_tile(pacc, T0, pcb);
#pragma unroll
        for (int r = 0; r < 16; ++r) pacc[r] = __int_as_float(0x7fffffff);
        const float nf = __shfl(thrv, nch_t);
        bool need = false;
#pragma unroll
        for (int t = 0; t < PT; ++t) {
          const float v = __int_as_float(bkey[t] & ~31), v2 = __int_as_float(bkey2[t] & ~31);
          auto s1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
          auto s2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v2), __float_as_uint(v2), false, false);
          const float pv = __uint_as_float(h ? s1[0] : s1[1]);
          const float pv2 = __uint_as_float(h ? s2[0] : s2[1]);
          const float sec = fminf(fmaxf(v, pv), fminf(v2, pv2));
          const float d2 = 2.f * (sec - M) + x2[t];
          const float lp = nf - ua[t];
          need |= pbase + t * 32 + cl < pend && (lp < 0.f || lp * lp < d2);
        }
        if (lane == 0) s_ext[wid] = __ballot(need) != 0ull;
        __syncthreads();
        int ext = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) ext |= s_ext[w];
        if (ext) {
          // (prefetching past the planned prefix instead measured slower: 1.6 ms over the
          // 5-iteration job, the unused chunks' L2 reads outweigh the exposed DMA)
          ++nch_t;
          if (NBUF == 2) issue(ch + 1);   // buffer (ch + 1) % 2: chunk ch - 1 retired
        }
      }
    }
  }
  reduce_tile(pacc, T0, pcb);
  KM_TS(4)
  // (warming L2 with the next tile's rows by throw-away LDS-DMA here measured no gain:
  // 17.92 vs 17.86 ms per iteration of the benchmark job)
  if constexpr (CAND && !DRIFT)
    if (nch_t < nchunk) nd_first = __shfl(thrv, nch_t);

  // ---- decode, combine the two lane halves (same point, disjoint centre rows)
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    const int r = bkey[t] & 31;
    const float v = __int_as_float(bkey[t] & ~31);
    int mi = bsub[t] + (r & 3) + 8 * (r >> 2) + 4 * h;
    if constexpr (CAND) mi = s_nb[par][mi];   // list position -> id
    auto sv = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    auto si = __builtin_amdgcn_permlane32_swap((uint32_t)mi, (uint32_t)mi, false, false);
    const float pv = __uint_as_float(h ? sv[0] : sv[1]);
    const int pi = (int)(h ? si[0] : si[1]);
    float bv = v;
    int bi = mi;
    if (pv < bv || (pv == bv && pi < bi)) { bv = pv; bi = pi; }
    float bv2 = 0.f;
    if constexpr (TOP2) {
      // second best over both halves: second smallest of {v, v2, pv, pv2}
      const float v2 = __int_as_float(bkey2[t] & ~31);
      auto s2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v2), __float_as_uint(v2), false, false);
      const float pv2 = __uint_as_float(h ? s2[0] : s2[1]);
      bv2 = fminf(fmaxf(v, pv), fminf(v2, pv2));
    }
    const int64_t p = pbase + t * 32 + cl;
    bool chg = false;
    int64_t row = 0;
    int old_c = 0;
    if (h == 0 && p < pend) {
      // acc = 0.5|x-c|^2 + M - 0.5|x|^2
      const float dist = fmaxf(2.f * (bv - M) + x2[t], 0.f);
      if constexpr (CAND) row = rowk[t];
      else row = idx ? (int64_t)idx[p] : p;
      if constexpr (LOOP) {
        const float dist2 = fmaxf(2.f * (bv2 - M) + x2[t], 0.f);
        float lo2 = km_dn1(sqrtf(fmaxf(km_dn1(dist2 - tol), 0.f)));
        // CAND: every pruned centre is >= nd_first - |x - c_acl| from x
        if constexpr (CAND) lo2 = fminf(lo2, km_dn1(nd_first - ua[t]));
        // DRIFT: every drift-pruned centre is >= l - dmp from x (dmp = -inf: none pruned)
        if constexpr (DRIFT) lo2 = fminf(lo2, km_dn1(s_lold[(wid * PT + t) * 32 + cl] - dmp));
        // the rows are scattered over X, so each store is a separate partial line write
        // (the kernel's largest cost after the MFMAs): u and l go out as one 8-byte pair,
        // and assign only where the cluster changed (assign[row] holds old_c otherwise)
        aux.ul[row] = make_float2(km_up1(sqrtf(km_up1(dist + tol))), fmaxf(lo2, 0.f));
        // CAND: the tile's rows were sorted by their previous cluster, acl
        old_c = CAND ? acl : (aux.a_prev ? aux.a_prev[row] : (aux.acl ? aux.acl[p] : assign[row]));
        chg = bi != old_c;
        if (chg) assign[row] = bi;
      } else {
        assign[row] = bi;
        if (mind) mind[row] = dist;
        if constexpr (TOP2) mind2[row] = fmaxf(2.f * (bv2 - M) + x2[t], 0.f);
        if (aux.xh) aux.xh[row] = 0.5f * x2[t];
      }
      my_sse += (double)dist;
    }
    if constexpr (LOOP) {
      const uint64_t cm = __ballot(chg);
      if (cm != 0ull) {
        int base = 0;
        if (lane == 0) base = atomicAdd(&s_nchg, __popcll(cm));
        base = __shfl(base, 0);
        if (chg) {
          const int slot = base + __popcll(cm & ((1ull << lane) - 1ull));
          s_chg[slot] = (int)row;
          s_chgn[slot] = (uint16_t)bi;
          s_chgo[slot] = (uint16_t)old_c;
        }
      }
    }
  }
#ifdef KM_XP_TIMING
  KM_TS(5)
  if (CAND && tid == 0 && blockIdx.x < kDbgBlocks && dbg_it < kDbgTiles)
    g_km_dbg[((int)blockIdx.x * kDbgTiles + dbg_it) * kDbgSlots + 6] = (unsigned long long)nch_t;
  ++dbg_it;
#endif
  };   // tile
  if constexpr (LOOP) {
    load_rec(blockIdx.x);
    load_ids();
    for (int64_t bt = blockIdx.x; bt < ntile; bt += gridDim.x) tile(bt);
    flush_changed();
  } else {
    if ((int64_t)blockIdx.x < ntile) tile(blockIdx.x);
  }

  if (aux.xmax && lane == 0) atomicMax(aux.xmax, __float_as_uint(my_xmax));
  if (sse) {
    double s = my_sse;
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) s_sse[wid] = s;
    __syncthreads();
    if (tid == 0) {
      double tot = 0.0;
      for (int w = 0; w < NW; ++w) tot += s_sse[w];
      atomicAdd(sse + (blockIdx.x & sse_mask), tot);
    }
  }
}

// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
kmeans_update_kernel(float* __restrict__ C, const float* __restrict__ S,
                     const unsigned long long* __restrict__ cnt,
                     int k, int d, int DP, T* __restrict__ Cq, float* __restrict__ hn, int kpad,
                     float* __restrict__ shift2) {
  // one wave per centre
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (c >= kpad) return;
  float nrm = 0.f, sh = 0.f;
  const float nc = (c < k) ? (float)cnt[c] : 0.f;
  for (int j = lane; j < DP; j += 64) {
    float v = 0.f;
    if (c < k && j < d) {
      const float old = C[(int64_t)c * d + j];
      v = nc > 0.f ? S[(int64_t)c * DP + j] / nc : old;
      sh += (v - old) * (v - old);
      C[(int64_t)c * d + j] = v;
    }
    float vr;
    if constexpr (sizeof(T) == 2) {
      const uint16_t b = f32_to_bf16(v);
      Cq[(int64_t)c * DP + j] = b;
      vr = bf16_to_f32(b);
    } else {
      Cq[(int64_t)c * DP + j] = v;
      vr = v;
    }
    nrm = fmaf(vr, vr, nrm);
  }
  nrm = wave_sum(nrm);
  sh = wave_sum(sh);
  if (lane == 0) {
    hn[c] = (c < k) ? 0.5f * nrm : 1.0e30f;
    if (shift2 && c < k) atomicAdd(shift2, sh);
  }
}

// ---------------------------------------------------------------------------
// K3 (sort-based, default): counting sort of the rows by cluster, then every
// wave sums a contiguous run of <= SEG rows of one cluster in registers and adds
// that partial row once to S. Global float atomics: one d-vector per segment
// (~N/SEG + k of them) instead of one per row; every X row is gathered once.
//   hist    : per row-chunk LDS histogram -> block_counts[b][c]
//   scan    : per cluster, exclusive offsets over chunks; cluster starts; segments
//   scatter : LDS cursors -> perm[pos] = row
//   segsum  : per segment register accumulation -> atomicAdd into S[c]
// Device-resident entry count (the incremental pass: 2 signed entries per moved row,
// counted on the device by the bound filter / diff): every kernel of the sort derives the
// same geometry from it -- n = mul * *ndev entries over B = clamp(ceil(n / chunk), 1,
// bmax) chunks of rpc rows -- so the launches need no host sync; blocks past B exit.
struct SortGeom { int64_t n, rpc; int B; };
__device__ __forceinline__ SortGeom sort_geom(int64_t n, int64_t rpc, int B,
                                              const unsigned long long* ndev, int mul,
                                              int64_t chunk) {
  if (ndev == nullptr) return {n, rpc, B};
  const int64_t nn = (int64_t)mul * (int64_t)*ndev;
  const int64_t b = min((int64_t)B, max((int64_t)1, (nn + chunk - 1) / chunk));
  return {nn, max((int64_t)1, (nn + b - 1) / b), (int)b};
}

__global__ void __launch_bounds__(256)
kmeans_hist_kernel(const int* __restrict__ assign, int64_t n_, int64_t rpc_, int k,
                   int* __restrict__ block_counts, const unsigned long long* __restrict__ ndev,
                   int mul, int64_t chunk) {
  const SortGeom g = sort_geom(n_, rpc_, gridDim.x, ndev, mul, chunk);
  if ((int)blockIdx.x >= g.B) return;
  const int64_t n = g.n, rpc = g.rpc;
  extern __shared__ int hist[];
  for (int c = threadIdx.x; c < k; c += blockDim.x) hist[c] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rpc, r1 = min(n, r0 + rpc);
  // kHB loads in flight per thread (clamped, unconditional) before their LDS atomics
  constexpr int kHB = 8;
  for (int64_t q = r0 + threadIdx.x; q < r1; q += (int64_t)kHB * blockDim.x) {
    int c[kHB];
#pragma unroll
    for (int b = 0; b < kHB; ++b) c[b] = assign[min(q + (int64_t)b * blockDim.x, r1 - 1)];
#pragma unroll
    for (int b = 0; b < kHB; ++b)
      if (q + (int64_t)b * blockDim.x < r1) atomicAdd(&hist[c[b]], 1);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < k; c += blockDim.x) block_counts[(int64_t)blockIdx.x * k + c] = hist[c];
}

// Column pass of the sort scan: block_counts[b][c] -> exclusive prefix over b, column
// totals -> colsum[c] (the cluster_start array, overwritten by kmeans_scan_kernel).
// 64 columns per block, 16 row ranges per column: 16x the memory parallelism of one
// block walking every column (that walk was load-latency bound: ~96 us at B=1100, k=1024).
constexpr int kCsCols = 64, kCsParts = 16, kCsBat = 16;
__global__ void __launch_bounds__(kCsCols * kCsParts)
kmeans_colscan_kernel(int* __restrict__ block_counts, int B_, int k, int64_t* __restrict__ colsum,
                      unsigned long long* __restrict__ cnt_out,
                      const unsigned long long* __restrict__ ndev, int mul, int64_t chunk) {
  const int B = sort_geom(0, 1, B_, ndev, mul, chunk).B;
  __shared__ int s_sum[kCsParts][kCsCols];
  const int col = threadIdx.x % kCsCols, p = threadIdx.x / kCsCols;
  const int c = blockIdx.x * kCsCols + col;
  const bool okc = c < k;
  const int cc = okc ? c : k - 1;
  const int rp = (B + kCsParts - 1) / kCsParts;
  const int b0 = min(B, p * rp), b1 = min(B, b0 + rp);
  int sum = 0;
  for (int b = b0; b < b1; b += kCsBat) {
    int v[kCsBat];
#pragma unroll
    for (int j = 0; j < kCsBat; ++j) v[j] = block_counts[(int64_t)min(b + j, b1 - 1) * k + cc];
#pragma unroll
    for (int j = 0; j < kCsBat; ++j) sum += b + j < b1 ? v[j] : 0;
  }
  s_sum[p][col] = sum;
  __syncthreads();
  int run = 0;
  for (int q = 0; q < p; ++q) run += s_sum[q][col];
  for (int b = b0; b < b1; b += kCsBat) {
    int v[kCsBat];
#pragma unroll
    for (int j = 0; j < kCsBat; ++j) v[j] = block_counts[(int64_t)min(b + j, b1 - 1) * k + cc];
#pragma unroll
    for (int j = 0; j < kCsBat; ++j)
      if (okc && b + j < b1) { block_counts[(int64_t)(b + j) * k + c] = run; run += v[j]; }
  }
  if (okc && p == kCsParts - 1) {
    colsum[c] = run;
    if (cnt_out) cnt_out[c] += (unsigned long long)run;
  }
}

// Cross-cluster scan: colsum[c] (kmeans_colscan_kernel's totals, in cluster_start) ->
// cluster_start / seg_start exclusive prefixes.
__global__ void __launch_bounds__(1024)
kmeans_scan_kernel(int k, int seg, int64_t* __restrict__ cluster_start,
                   int64_t* __restrict__ seg_start) {
  // [2k] int32 (n < 2^31 is checked by the launcher): counts, then segment counts;
  // 8 B per cluster keeps k = 16384 inside the 160 KB LDS (128 KB dynamic)
  extern __shared__ int tot[];
  __shared__ int64_t s_part[2][1024 / 64];
  for (int c = threadIdx.x; c < k; c += blockDim.x) {
    const int run = (int)cluster_start[c];
    tot[c] = run;
    tot[k + c] = (run + seg - 1) / seg;
  }
  __syncthreads();
  // exclusive scans of tot[0..k) and tot[k..2k) by a single thread per chunk of k/1024
  const int per = (k + blockDim.x - 1) / blockDim.x;
  const int c0 = threadIdx.x * per, c1 = min(k, c0 + per);
  int64_t a = 0, b = 0;
  for (int c = c0; c < c1; ++c) { a += tot[c]; b += tot[k + c]; }
  // block-wide exclusive scan of (a, b) via LDS (wave partials)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t ia = a, ib = b;
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t ta = __shfl_up(ia, off), tb = __shfl_up(ib, off);
    if (lane >= off) { ia += ta; ib += tb; }
  }
  if (lane == 63) { s_part[0][wid] = ia; s_part[1][wid] = ib; }
  __syncthreads();
  int64_t wa = 0, wb = 0;
  for (int w = 0; w < wid; ++w) { wa += s_part[0][w]; wb += s_part[1][w]; }
  int64_t ra = wa + ia - a, rb = wb + ib - b;    // exclusive prefix for c0
  for (int c = c0; c < c1; ++c) {
    cluster_start[c] = ra;
    seg_start[c] = rb;
    ra += tot[c];
    rb += tot[k + c];
  }
  if (c1 == k && c0 < k) { cluster_start[k] = ra; seg_start[k] = rb; }
  if (k == 0 && threadIdx.x == 0) { cluster_start[0] = 0; seg_start[0] = 0; }
}

__global__ void __launch_bounds__(256)
kmeans_scatter_kernel(const int* __restrict__ assign, int64_t n, int64_t rpc, int k,
                      const int* __restrict__ block_offsets, const int64_t* __restrict__ cluster_start,
                      int* __restrict__ perm) {
  // (k > kScKmax only; host-known counts)
  extern __shared__ int cursor[];
  for (int c = threadIdx.x; c < k; c += blockDim.x)
    cursor[c] = (int)(cluster_start[c] + block_offsets[(int64_t)blockIdx.x * k + c]);
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rpc, r1 = min(n, r0 + rpc);
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const int pos = atomicAdd(&cursor[assign[r]], 1);
    perm[pos] = (int)r;
  }
}

// Coalesced scatter (default for k <= kScKmax): the block's rows are handled in
// chunks of CH rows; each chunk is counting-sorted by cluster in LDS first (local
// ranks by LDS atomics, block scan of the local counts, one packed (cluster, row
// offset) word per slot), then slot i is written to cursor[c] + (i - lstart[c]):
// consecutive lanes store consecutive perm entries of one cluster run (~CH/k
// rows per run) instead of 64 unrelated 4-byte locations per store instruction.
// CH / KMAX: chunk rows / cluster bound; <16384, 1024> (76 KB LDS) runs 2 blocks per CU
// where k <= 1024, so one block's scan and barriers overlap the other's memory phases.
constexpr int kScKmax = 2048, kScNT = 1024;
template <int CH, int KMAX>
__global__ void __launch_bounds__(kScNT)
kmeans_scatter_chunked_kernel(const int* __restrict__ assign, int64_t n_, int64_t rpc_, int k,
                              const int* __restrict__ block_offsets,
                              const int64_t* __restrict__ cluster_start, int* __restrict__ perm,
                              const unsigned long long* __restrict__ ndev, int mul, int64_t chunk,
                              const int* __restrict__ vals = nullptr) {
  // vals (optional): store vals[entry] instead of the entry index
  const SortGeom g = sort_geom(n_, rpc_, gridDim.x, ndev, mul, chunk);
  if ((int)blockIdx.x >= g.B) return;
  const int64_t n = g.n, rpc = g.rpc;
  constexpr int kScPer = CH / kScNT;
  __shared__ int stage[CH];
  __shared__ int cursor[KMAX], lcnt[KMAX], lstart[KMAX];
  __shared__ int s_wsum[kScNT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int c = tid; c < k; c += kScNT)
    cursor[c] = (int)(cluster_start[c] + block_offsets[(int64_t)blockIdx.x * k + c]);
  const int64_t r0 = (int64_t)blockIdx.x * rpc, r1 = min(n, r0 + rpc);
  const int per = (k + kScNT - 1) / kScNT;        // scan entries per thread
  for (int64_t q0 = r0; q0 < r1; q0 += CH) {
    const int m = (int)min((int64_t)CH, r1 - q0);
    for (int c = tid; c < k; c += kScNT) lcnt[c] = 0;
    __syncthreads();
    int packed[kScPer];                            // (cluster << 15) | local rank
#pragma unroll
    for (int j = 0; j < kScPer; ++j) {
      const int o = j * kScNT + tid;
      packed[j] = -1;
      if (o < m) {
        const int c = assign[q0 + o];
        packed[j] = (c << 15) | atomicAdd(&lcnt[c], 1);
      }
    }
    __syncthreads();
    // exclusive scan of lcnt -> lstart (per thread: `per` consecutive clusters)
    const int c0 = tid * per, c1 = min(k, c0 + per);
    int a = 0;
    for (int c = c0; c < c1; ++c) a += lcnt[c];
    int ia = a;
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(ia, off);
      if (lane >= off) ia += t;
    }
    if (lane == 63) s_wsum[wid] = ia;
    __syncthreads();
    int run = ia - a;
    for (int w = 0; w < wid; ++w) run += s_wsum[w];
    for (int c = c0; c < c1; ++c) { lstart[c] = run; run += lcnt[c]; }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kScPer; ++j) {
      if (packed[j] >= 0) {
        const int c = packed[j] >> 15;
        stage[lstart[c] + (packed[j] & 0x7fff)] = (c << 15) | (j * kScNT + tid);
      }
    }
    __syncthreads();
    // (batching the vals[e] gathers 16 deep measured no faster, profiles/round4/r4_42:
    // the chunk's vals window is L2-resident after its first touches)
    for (int i = tid; i < m; i += kScNT) {
      const int v = stage[i];
      const int c = v >> 15;
      const int64_t e = q0 + (v & 0x7fff);
      perm[cursor[c] + (i - lstart[c])] = vals ? vals[e] : (int)e;
    }
    __syncthreads();
    for (int c = tid; c < k; c += kScNT) cursor[c] += lcnt[c];
    __syncthreads();
  }
}

// the sort scan: column pass (multi-block) then the cross-cluster pass (one block)
static void launch_sort_scan(int* block_counts, int B, int k, int seg, int64_t* cluster_start,
                             int64_t* seg_start, unsigned long long* cnt,
                             const unsigned long long* ndev, int mul, int64_t chunk, size_t lds,
                             hipStream_t st) {
  hipLaunchKernelGGL(kmeans_colscan_kernel, dim3((k + kCsCols - 1) / kCsCols), dim3(kCsCols * kCsParts),
                     0, st, block_counts, B, k, cluster_start, cnt, ndev, mul, chunk);
  hipLaunchKernelGGL(kmeans_scan_kernel, dim3(1), dim3(1024), lds, st, k, seg, cluster_start, seg_start);
}

template <typename... A>
static void launch_scatter_chunked(int k, int B, hipStream_t st, A... a) {
#ifndef KM_XP_SC1
  if (k <= 1024) {
    hipLaunchKernelGGL((kmeans_scatter_chunked_kernel<16384, 1024>), dim3(B), dim3(kScNT), 0, st, a...);
    return;
  }
#endif
  hipLaunchKernelGGL((kmeans_scatter_chunked_kernel<32768, kScKmax>), dim3(B), dim3(kScNT), 0, st, a...);
}

template <typename T, int DP, int NW, bool NT>
__global__ void __launch_bounds__(NW * 64)
kmeans_segsum_kernel(const T* __restrict__ X, int64_t ldx, const int* __restrict__ perm,
                     const int64_t* __restrict__ cluster_start, const int64_t* __restrict__ seg_start,
                     int k, int seg, float* __restrict__ S) {
  constexpr int EPL = DP >= 64 ? DP / 64 : 1;
  const int lane = threadIdx.x & 63;
  const int64_t nseg = seg_start[k];
  const bool lane_on = (DP >= 64) || (lane < DP);
  for (int64_t sid = (int64_t)blockIdx.x * NW + (threadIdx.x >> 6); sid < nseg;
       sid += (int64_t)gridDim.x * NW) {
    // cluster of this segment: last c with seg_start[c] <= sid
    int lo = 0, hi = k - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (seg_start[mid] <= sid) lo = mid; else hi = mid - 1;
    }
    const int c = lo;
    const int64_t r0 = cluster_start[c] + (sid - seg_start[c]) * (int64_t)seg;
    const int64_t r1 = min(cluster_start[c + 1], r0 + seg);
    float acc[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
    // 64 row ids per coalesced load (next block prefetched), 16 rows in flight
    int idx = (r0 + lane < r1) ? perm[r0 + lane] : -1;
    for (int64_t i = r0; i < r1; i += 64) {
      const int nxt = (i + 64 + lane < r1) ? perm[i + 64 + lane] : -1;
#pragma unroll
      for (int u0 = 0; u0 < 64; u0 += 16) {
        float v[16][EPL];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int row = __builtin_amdgcn_readlane(idx, u0 + u);
          const T* rp = X + (int64_t)(row < 0 ? 0 : row) * ldx + lane * EPL;
          if constexpr (sizeof(T) == 2 && EPL % 2 == 0) {
            // rows are gathered exactly once per iteration: nt loads
#pragma unroll
            for (int e = 0; e < EPL; e += 2) {
              const uint32_t w2 = ld_u32<NT>(reinterpret_cast<const uint32_t*>(rp) + e / 2);
              v[u][e] = (lane_on && row >= 0) ? bf16lo(w2) : 0.f;
              v[u][e + 1] = (lane_on && row >= 0) ? bf16hi(w2) : 0.f;
            }
          } else {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
              float x = 0.f;
              if constexpr (sizeof(T) == 2) x = bf16_to_f32(reinterpret_cast<const uint16_t*>(rp)[e]);
              else x = reinterpret_cast<const float*>(rp)[e];
              v[u][e] = (lane_on && row >= 0) ? x : 0.f;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int e = 0; e < EPL; ++e) acc[e] += v[u][e];
      }
      idx = nxt;
    }
    if (lane_on) {
#pragma unroll
      for (int e = 0; e < EPL; ++e) atomicAdd(&S[(int64_t)c * DP + lane * EPL + e], acc[e]);
    }
  }
}

// Incremental K3, sort-based (moved rows only). Entry e < m adds row changed[e] to its
// new cluster, entry m + e subtracts it from its old one. The entries are counting-sorted
// by cluster with the K3 kernels above, then every wave sums a run of <= SEG entries of
// one cluster in f64 registers (signed) and adds it once to S64 / cnt / Q: ~(2m/SEG + k)
// d-vector atomics instead of 2 per moved row and feature (km_move, kmeans_inc.hip).
__global__ void __launch_bounds__(256)
km_dexpand_kernel(const int32_t* __restrict__ changed, int64_t m, const int32_t* __restrict__ a_new,
                  const int32_t* __restrict__ a_old, int* __restrict__ ec, int* __restrict__ er,
                  const unsigned long long* __restrict__ mdev, const int32_t* __restrict__ cnew,
                  const int32_t* __restrict__ cold) {
  // cnew / cold (optional): the clusters aligned with `changed` (written by the K2
  // epilogue): sequential reads instead of two gathers per moved row
  if (mdev != nullptr) m = min(m, (int64_t)*mdev);
  const int64_t n2 = 2 * m;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n2;
       e += (int64_t)gridDim.x * blockDim.x) {
    const bool add = e < m;
    const int row = changed[add ? e : e - m];
    if (cnew) ec[e] = add ? cnew[e] : cold[e - m];
    else ec[e] = add ? a_new[row] : a_old[row];
    er[e] = add ? row : ~row;          // negative: subtract
  }
}

// Candidate-pruned K2 tiles: cluster c's run [cs[c], cs[c+1]) of the cluster-sorted active
// rows is cut into ceil(run / tile) tiles; tile t -> (cluster, first position). One block
// (k <= 2048): per-thread clusters, block exclusive scan of their tile counts.
__global__ void __launch_bounds__(1024)
km_tiles_kernel(const int64_t* __restrict__ cs, int k, int tile, int4* __restrict__ tiles,
                unsigned long long* __restrict__ n_tiles, int64_t max_tiles) {
  // every block scans the (k <= 2048) tile counts itself, then writes its share of the
  // records: tile t's cluster by binary search in LDS (coalesced record stores)
  __shared__ int64_t s_part[1024 / 64];
  __shared__ int s_toff[2049];                     // first tile of cluster c
  __shared__ int s_cs[2049];                       // cluster runs (positions < 2^31)
  const int per = (k + blockDim.x - 1) / blockDim.x;
  const int c0 = threadIdx.x * per, c1 = min(k, c0 + per);
  for (int c = threadIdx.x; c <= k; c += blockDim.x) s_cs[c] = (int)cs[c];
  __syncthreads();
  int64_t a = 0;
  for (int c = c0; c < c1; ++c) a += (s_cs[c + 1] - s_cs[c] + tile - 1) / tile;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t ia = a;
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t t = __shfl_up(ia, off);
    if (lane >= off) ia += t;
  }
  if (lane == 63) s_part[wid] = ia;
  __syncthreads();
  int64_t t0 = ia - a;
  for (int w = 0; w < wid; ++w) t0 += s_part[w];
  for (int c = c0; c < c1; ++c) {
    s_toff[c] = (int)t0;
    t0 += (s_cs[c + 1] - s_cs[c] + tile - 1) / tile;
  }
  if (c1 == k && c0 < k) {
    s_toff[k] = (int)t0;
    if (blockIdx.x == 0) *n_tiles = (unsigned long long)min(t0, max_tiles);
  }
  __syncthreads();
  const int total = (int)min((int64_t)s_toff[k], max_tiles);
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    int lo = 0, hi = k - 1;                        // last c with s_toff[c] <= t
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_toff[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const int first = s_cs[lo] + (t - s_toff[lo]) * tile;
    tiles[t] = make_int4(lo, first, min(s_cs[lo + 1], first + tile), 0);
  }
}

template <typename T, int DP, int NW>
__global__ void __launch_bounds__(NW * 64)
km_dsegsum_kernel(const T* __restrict__ X, int64_t ldx, const int* __restrict__ perm,
                  const int* __restrict__ er, const int64_t* __restrict__ cluster_start,
                  const int64_t* __restrict__ seg_start, int k, int seg, double* __restrict__ S,
                  unsigned long long* __restrict__ cnt, const float* __restrict__ xh,
                  double* __restrict__ Q) {
  constexpr int EPL = DP >= 64 ? DP / 64 : 1;
  constexpr int kNone = (int)0x80000000;
  const int lane = threadIdx.x & 63;
  const int64_t nseg = seg_start[k];
  const bool lane_on = (DP >= 64) || (lane < DP);
  for (int64_t sid = (int64_t)blockIdx.x * NW + (threadIdx.x >> 6); sid < nseg;
       sid += (int64_t)gridDim.x * NW) {
    int lo = 0, hi = k - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (seg_start[mid] <= sid) lo = mid; else hi = mid - 1;
    }
    const int c = lo;
    const int64_t r0 = cluster_start[c] + (sid - seg_start[c]) * (int64_t)seg;
    const int64_t r1 = min(cluster_start[c + 1], r0 + seg);
    double acc[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) acc[e] = 0.0;
    int csum = 0;
    double qsum = 0.0;
    int code = (r0 + lane < r1) ? er[perm[r0 + lane]] : kNone;
    for (int64_t i = r0; i < r1; i += 64) {
      const int nxt = (i + 64 + lane < r1) ? er[perm[i + 64 + lane]] : kNone;
      if (code != kNone) {
        const int row = code < 0 ? ~code : code;
        csum += code < 0 ? -1 : 1;
        if (Q != nullptr) qsum += (code < 0 ? -2.0 : 2.0) * (double)xh[row];
      }
#pragma unroll
      for (int u0 = 0; u0 < 64; u0 += 16) {
        float v[16][EPL];
        float sg[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int cu = __builtin_amdgcn_readlane(code, u0 + u);
          const int row = cu == kNone ? 0 : (cu < 0 ? ~cu : cu);
          sg[u] = cu == kNone ? 0.f : (cu < 0 ? -1.f : 1.f);
          const T* rp = X + (int64_t)row * ldx + lane * EPL;
          if constexpr (sizeof(T) == 2 && EPL == 2) {
            // both bf16 of the lane in one dword load (4-B aligned: ldx is a multiple of 8)
            const uint32_t w = ld_u32<true>(reinterpret_cast<const uint32_t*>(rp));   // nt: read once
            v[u][0] = bf16lo(w);
            v[u][1] = bf16hi(w);
          } else {
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
              float x = 0.f;
              if constexpr (sizeof(T) == 2) x = bf16_to_f32(reinterpret_cast<const uint16_t*>(rp)[e]);
              else x = reinterpret_cast<const float*>(rp)[e];
              v[u][e] = lane_on ? x : 0.f;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int e = 0; e < EPL; ++e) acc[e] += (double)(sg[u] * v[u][e]);
      }
      code = nxt;
    }
    if (lane_on) {
#pragma unroll
      for (int e = 0; e < EPL; ++e)
        if (acc[e] != 0.0) atomicAdd(&S[(int64_t)c * DP + lane * EPL + e], acc[e]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      csum += __shfl_xor(csum, o, 64);
      qsum += __shfl_xor(qsum, o, 64);
    }
    if (lane == 0) {
      if (csum != 0) atomicAdd(&cnt[c], (unsigned long long)(long long)csum);
      if (Q != nullptr && qsum != 0.0) atomicAdd(&Q[c], qsum);
    }
  }
}

}  // namespace dalgo

using namespace dalgo;

template <typename T, int DP, int NW, int NSUB, int PTB = 2, int MINW = 1>
static hipError_t launch_assign_v(const void* X, int64_t n, int64_t ldx, const void* Cq,
                                  const float* hn, int kpad, int* assign, float* mind, double* sse, int sse_mask,
                                  hipStream_t st) {
  constexpr int PT = sizeof(T) == 2 ? PTB : 1;
  if (kpad % (32 * NSUB)) return hipErrorInvalidValue;
  const int64_t per_block = NW * PT * 32;
  const int64_t grid = cdiv(n, per_block);
  if (grid == 0) return hipSuccess;
  if (grid > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL((kmeans_assign_kernel<T, DP, PT, NW, NSUB, MINW>), dim3((unsigned)grid),
                     dim3(NW * 64), 0, st, (const T*)X, n, ldx, (const T*)Cq, hn, kpad, assign,
                     mind, sse, sse_mask);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

static int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cached[dev] = v;
  }
  return cached[dev];
}

// pipelined K2 (bf16, DP >= 64). Host-known row count: one block tile per block.
// Device-resident count (mcount, n = its upper bound): a resident grid (MINB blocks per
// CU) walks the tiles, so the launch needs no host sync.
template <int DP, int NW, int PT, int NSUB, int MINB, int NBUF, bool PF, bool TOP2 = false,
          bool LOOP = false, bool CAND = false, bool DRIFT = false>
static hipError_t launch_assign_pipe(const void* X, int64_t n, int64_t ldx, const void* Cq,
                                     const float* hn, int kpad, int* assign, float* mind,
                                     double* sse, int sse_mask, hipStream_t st,
                                     const int32_t* idx = nullptr, float* mind2 = nullptr,
                                     const KmAux& aux = KmAux{}) {
  constexpr int CH = 32 * NSUB;
  constexpr size_t kStatic = NBUF * (size_t)CH * DP * 2;
  if (kpad % CH) return hipErrorInvalidValue;
  const size_t dyn = (size_t)kpad * sizeof(float);
  if (kStatic + dyn + 1024 > 160 * 1024) return hipErrorInvalidValue;
  int64_t grid = cdiv(n, (int64_t)NW * PT * 32);
  if (grid == 0) return hipSuccess;
  if ((aux.mcount != nullptr) != LOOP) return hipErrorInvalidValue;
  // previous clusters: the Hamerly-only form reads a_prev[row], acl[p] or assign[row]; the
  // candidate form has them per tile
  if (LOOP && (aux.tol == nullptr || aux.ul == nullptr || aux.changed == nullptr ||
               aux.n_changed == nullptr || (!CAND && aux.acl != nullptr && idx == nullptr)))
    return hipErrorInvalidValue;
  if (CAND && (kpad > 1024 || aux.tiles == nullptr || aux.n_tiles == nullptr || aux.hnb == nullptr ||
               aux.nb == nullptr || aux.nd == nullptr || idx == nullptr))
    return hipErrorInvalidValue;
  if (DRIFT && (aux.ndb == nullptr || aux.dnb == nullptr || kpad % 4 != 0)) return hipErrorInvalidValue;
  // CAND: up to n / TILE + k tiles (device count) -> always the resident grid
  if (CAND) grid = (int64_t)device_cus() * MINB;
  else if (LOOP) grid = std::min<int64_t>(grid, (int64_t)device_cus() * MINB);
  if (grid > 0x7fffffffLL) return hipErrorInvalidValue;
  auto kfn = kmeans_assign_pipe_kernel<DP, NW, PT, NSUB, MINB, NBUF, PF, TOP2, LOOP, CAND, DRIFT>;
  static size_t attr_set = 0;   // largest dynamic size this instantiation was enabled for
  if (dyn > attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)dyn);
    if (e != hipSuccess) return e;
    attr_set = dyn;
  }
  hipLaunchKernelGGL(kfn, dim3((unsigned)grid), dim3(NW * 64), dyn, st, (const uint16_t*)X, n, ldx,
                     (const uint16_t*)Cq, hn, kpad, assign, mind, sse, sse_mask, idx, mind2, aux);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// ---------------------------------------------------------------------------
// K2 on 16x16x32 MFMAs (bf16, DP = 128): the same distance keys as the pipelined form,
// tiled for v_mfma_f32_16x16x32_bf16, which sustains ~12 % more FLOP/s than the 32x32x16
// form next to an argmin VALU load (profiles/round4/r4_36: a power / clock effect). A wave
// holds PG groups of 16 points (B operand; lane l: point l % 16, dims 32 s + 8 (l / 16)
// .. +8 of k-step s); a 128-centre chunk (the same swizzled LDS-DMA image as the 32x32
// form) is 8 sub-tiles of 16 centres (A: lane l reads centre l % 16, piece 4 s + l / 16).
// The accumulator starts at -(0.5|c|^2 + M), so acc = -(0.5|x - c|^2 + M - 0.5|x|^2) < 0
// and the signed-integer order of its bits is the distance order; lane l holds centres
// 4 (l / 16) + r of the sub-tile for point l % 16: key = bits & ~31 | (sub * 4 + r) keeps
// the lowest id among equal keys of a chunk, chunks compare on the value bits only
// (strict), and the four lane groups of a point are merged at the end.
// BND (the dense form of a bound-filtered iteration): the rows are idx[0, *aux.mcount)
// (device count; blocks past it exit at once), every lane also keeps its second-smallest
// key (v_med3 per key pair, merged over chunks and lane groups), and the epilogue is the
// filtered iteration's: u / l per row, assign and the moved-row list where the cluster
// differs from the previous one (aux.acl[p], else aux.a_prev[row], else assign[row]).
// CND (the candidate-pruned form on the same tiling, BND implied): block b is tile b of the
// cluster-sorted active rows (<= TILE rows of one cluster acl; blocks past the device tile
// count exit), the centre stream is acl's neighbour list (gathered by LDS-DMA through the
// staged ids, 0.5|c|^2 from hnb in list order), and only its first nc chunks are streamed:
// the chunks whose first distance to c_acl is <= R = 2 max over the tile of ua, ua >= |x -
// c_acl| (exact v_dot2 distance in the prologue, rounded up) -- a centre farther than R
// from c_acl is farther than c_acl from every tile point. The pruned centres bound the new
// l by nd_first - ua; the previous cluster of every row is acl.
// CND + DRIFT (drift-aware lists, as the pipelined form's DRIFT): past chunk 0 a list entry
// is streamed iff it is inside the ball AND its centre moved by >= tau = min over the tile
// rows of (l - ua) (capped): a slower centre is farther than c_acl from every tile row. The
// kept entries are compacted behind chunk 0 (block scan); the dropped ones bound the new l
// by l - (largest dropped shift) and nd_first - ua.
template <int NW, int PG, int MINB, bool BND = false, bool CND = false, bool DRIFT = false>
__global__ void __launch_bounds__(NW * 64, MINB)
kmeans_assign16_kernel(const uint16_t* __restrict__ X, int64_t n, int64_t ldx,
                       const uint16_t* __restrict__ Cq, const float* __restrict__ hn, int kpad,
                       int* __restrict__ assign, float* __restrict__ mind,
                       double* __restrict__ sse, int sse_mask, float* __restrict__ xh,
                       unsigned* __restrict__ xmax, const int32_t* __restrict__ idx, const KmAux aux) {
  constexpr int DP = 128, KS = DP / 32;        // 16x16x32 k-steps per centre row
  constexpr int NJ = DP * 2 / 16;              // 16-B pieces per row
  constexpr int SWZ = 15;
  constexpr int CH = 128, NSUB = CH / 16;
  constexpr int NT = NW * 64;
  constexpr int CHP = CH * NJ;
  constexpr int GPT = CHP / NT;
  constexpr int NBUF = 2;
  constexpr int TILE = NW * PG * 16;
  static_assert(CHP % NT == 0 && (NT / NJ) % (SWZ + 1) == 0, "DMA layout");
  static_assert(!CND || BND, "the candidate form is a form of the filtered iteration");
  static_assert(!DRIFT || CND, "drift pruning refines the candidate lists");
  constexpr int KH = DRIFT ? 1024 / (NW * 64) : 1;   // list entries per thread (consecutive)
  __shared__ __attribute__((aligned(16))) uint4 s_c[NBUF * CHP];
  extern __shared__ __attribute__((aligned(16))) float s_hn16[];   // [kpad]: 0.5|c|^2 + M
  __shared__ float s_m[NW];
  __shared__ double s_sse[NW];
  __shared__ float s_x2[NW][PG * 16];           // |x|^2 per point (read in the epilogue)
  __shared__ int s_row[BND ? NW : 1][BND ? PG * 16 : 1];   // BND: row and previous cluster
  __shared__ int s_old[BND && !CND ? NW : 1][BND && !CND ? PG * 16 : 1];   //      per point
  __shared__ uint16_t s_nbl[CND ? 1024 : 1];   // CND: the tile cluster's neighbour list
  __shared__ float s_ur[CND ? NW : 1];         // CND: per-wave max of ua
  // CND / DRIFT: every point's ua and last l, read again by the epilogue (LDS rather than
  // 12 VGPRs held over the chunk loop: the register file is full there)
  __shared__ float s_ua[CND ? NW : 1][CND ? PG * 16 : 1];
  __shared__ float s_lold[DRIFT ? NW : 1][DRIFT ? PG * 16 : 1];
  __shared__ float s_tau[DRIFT ? NW : 1];      // DRIFT: per-wave min of l - ua
  __shared__ int s_kc[DRIFT ? NW : 1];         // DRIFT: kept entries per wave
  __shared__ float s_kd[DRIFT ? NW : 1], s_kf[DRIFT ? NW : 1];
  // BND: the block's moved rows (row, new, previous cluster), appended to the global list
  // with ONE atomic per block: a device-scope atomic per wave on the single counter
  // serialised the launch (55 vs 19 ms at 14M moved rows, profiles/round5/r5_13)
  __shared__ int s_mv[BND ? TILE : 1];
  __shared__ uint16_t s_mvn[BND ? TILE : 1], s_mvo[BND ? TILE : 1];   // clusters < 2^16
  __shared__ int s_nmv;
  __shared__ unsigned long long s_mvbase;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lg = lane >> 4, pl = lane & 15;
  const int nchunk = kpad / CH;
  int64_t pbase = ((int64_t)blockIdx.x * NW + wid) * (PG * 16);
  float tol = 0.f;
  int acl = 0;
  if constexpr (CND) {
    if ((int64_t)blockIdx.x >= (int64_t)*aux.n_tiles) return;   // block-uniform
    const int4 tr = aux.tiles[blockIdx.x];
    acl = tr.x;
    n = tr.z;
    pbase = (int64_t)tr.y + (int64_t)wid * (PG * 16);
    tol = *aux.tol;
    if (tid == 0) s_nmv = 0;
  } else if constexpr (BND) {
    n = min(n, (int64_t)*aux.mcount);
    if ((int64_t)blockIdx.x * TILE >= n) return;   // block-uniform, before any barrier
    tol = *aux.tol;
    if (tid == 0) s_nmv = 0;                       // published by the first barrier below
  }

  // ---- points: rows past n read a valid row and are zeroed after the wait (last wave only)
  uint4 bf[PG][KS];
  const bool full = pbase + PG * 16 <= n;
  int rowv[BND ? PG : 1], oldv[BND ? PG : 1];
  if constexpr (BND) {
#pragma unroll
    for (int g = 0; g < PG; ++g) {
      const int64_t p = pbase + g * 16 + pl;
      rowv[g] = idx[p < n ? p : n - 1];
    }
  }
#pragma unroll
  for (int g = 0; g < PG; ++g) {
    const int64_t p = pbase + g * 16 + pl;
    const int64_t row = BND ? (int64_t)rowv[g] : (full || p < n ? p : 0);
    const uint16_t* src = X + row * ldx + 8 * lg;
#pragma unroll
    for (int s = 0; s < KS; ++s) bf[g][s] = *reinterpret_cast<const uint4*>(src + 32 * s);
  }
  if constexpr (BND && !CND) {
#pragma unroll
    for (int g = 0; g < PG; ++g) {
      const int64_t p = pbase + g * 16 + pl;
      oldv[g] = aux.acl ? aux.acl[p < n ? p : n - 1] : (aux.a_prev ? aux.a_prev[rowv[g]] : assign[rowv[g]]);
    }
  }
  // CND: c_acl in the points' k layout (lane: dims 32 s + 8 lg .. + 8), the list's first
  // distance of every chunk (lane j: chunk j), the list itself (ids -> LDS)
  uint4 ca[CND ? KS : 1];
  float thrv = __builtin_inff(), hna = 0.f;
  // DRIFT: entries p = KH tid + j of acl's list (ids, 0.5|c|^2, distance to c_acl, shift)
  // and every point's l from the last iteration
  int nbv[KH];
  float hv[KH], ndv[KH], dnv[KH], lold[DRIFT ? PG : 1];
  if constexpr (CND) {
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) ca[s2] = *reinterpret_cast<const uint4*>(Cq + (int64_t)acl * DP + 32 * s2 + 8 * lg);
    if (lane < nchunk) thrv = aux.nd[(int64_t)acl * kpad + lane * CH];
    hna = hn[acl];
    if constexpr (DRIFT) {
      static_assert(KH == 4, "DRIFT: four consecutive list entries per thread");
      const bool in = tid * KH < kpad;
      const int64_t o = (int64_t)acl * kpad + tid * KH;
      const float inf = __builtin_inff();
      const int4 i4 = in ? *reinterpret_cast<const int4*>(aux.nb + o) : make_int4(0, 0, 0, 0);
      const float4 h4v = in ? *reinterpret_cast<const float4*>(aux.hnb + o) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 n4 = in ? *reinterpret_cast<const float4*>(aux.ndb + o) : make_float4(inf, inf, inf, inf);
      const float4 d4 = in ? *reinterpret_cast<const float4*>(aux.dnb + o) : make_float4(0.f, 0.f, 0.f, 0.f);
      nbv[0] = i4.x; nbv[1] = i4.y; nbv[2] = i4.z; nbv[3] = i4.w;
      hv[0] = h4v.x; hv[1] = h4v.y; hv[2] = h4v.z; hv[3] = h4v.w;
      ndv[0] = n4.x; ndv[1] = n4.y; ndv[2] = n4.z; ndv[3] = n4.w;
      dnv[0] = d4.x; dnv[1] = d4.y; dnv[2] = d4.z; dnv[3] = d4.w;
      const float* ulf = reinterpret_cast<const float*>(aux.ul);
#pragma unroll
      for (int g = 0; g < PG; ++g) lold[g] = ulf[2 * (int64_t)rowv[g] + 1];
    } else {
      for (int i = tid; i < kpad; i += NT) s_nbl[i] = (uint16_t)aux.nb[(int64_t)acl * kpad + i];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!full) {
#pragma unroll
    for (int g = 0; g < PG; ++g)
      if (pbase + g * 16 + pl >= n)
#pragma unroll
        for (int s = 0; s < KS; ++s) bf[g][s] = make_uint4(0u, 0u, 0u, 0u);
  }
  if constexpr (BND) {
    if (lg == 0) {
#pragma unroll
      for (int g = 0; g < PG; ++g) {
        s_row[wid][g * 16 + pl] = rowv[g];
        if constexpr (!CND) s_old[wid][g * 16 + pl] = oldv[g];
      }
    }
  }
  float mx = 0.f;
  float ua[CND ? PG : 1];
  float um = 0.f;
  float tv = __builtin_inff();                 // DRIFT: min over the tile rows of l - ua
#pragma unroll
  for (int g = 0; g < PG; ++g) {
    // |x|^2 by v_dot2c_f32_bf16 (two bf16 products per instruction, f32 accumulate)
    float q = 0.f, dt = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const uint32_t w[4] = {bf[g][s].x, bf[g][s].y, bf[g][s].z, bf[g][s].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x2 h = __builtin_bit_cast(bf16x2, w[j]);
        q = __builtin_amdgcn_fdot2_f32_bf16(h, h, q, false);
      }
      if constexpr (CND) {
        const uint32_t cw[4] = {ca[s].x, ca[s].y, ca[s].z, ca[s].w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          dt = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, w[j]), __builtin_bit_cast(bf16x2, cw[j]),
                                               dt, false);
      }
    }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    if (lg == 0) s_x2[wid][g * 16 + pl] = q;
    mx = fmaxf(mx, 0.5f * q);
    if constexpr (CND) {
      dt += __shfl_xor(dt, 16, 64);
      dt += __shfl_xor(dt, 32, 64);
      // |x - c_acl|^2 = |x|^2 - 2 x.c + 2 hn (f32 error far below tol: the K2 slack)
      const float dist = fmaxf(q - 2.f * dt + 2.f * hna, 0.f);
      ua[g] = km_up1(sqrtf(km_up1(dist + tol)));
      if (pbase + g * 16 + pl < n) {
        um = fmaxf(um, ua[g]);
        if constexpr (DRIFT) tv = fminf(tv, km_dn1(lold[g] - ua[g]));
      }
      if (lg == 0) {
        s_ua[wid][g * 16 + pl] = ua[g];
        if constexpr (DRIFT) s_lold[wid][g * 16 + pl] = lold[g];
      }
    }
  }
  for (int off = 32; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  if (lane == 0) s_m[wid] = mx;
  if constexpr (CND) {
    for (int off = 32; off >= 1; off >>= 1) {
      um = fmaxf(um, __shfl_xor(um, off));
      if constexpr (DRIFT) tv = fminf(tv, __shfl_xor(tv, off));
    }
    if (lane == 0) {
      s_ur[wid] = um;
      if constexpr (DRIFT) s_tau[wid] = tv;
    }
  }

  // ---- chunk DMA (the 32x32 form's image: slot (row, jj) holds piece jj ^ (row & SWZ));
  // the global address is an SGPR base (the chunk) + a loop-invariant VGPR offset, the
  // LDS destination an SGPR (m0): no per-chunk vector address arithmetic
  // slot qq = g * NT + tid: row = qq / NJ, piece jj = qq % NJ = tid % NJ; NT / NJ rows per
  // round is a multiple of SWZ + 1, so the swizzle term (row & SWZ) does not depend on g:
  // round g is the same VGPR offset + g * (NT / NJ) rows, added to the SGPR base
  static_assert((NT / NJ) % (SWZ + 1) == 0 && NT % NJ == 0, "DMA offset layout");
  const uint32_t src_off = (uint32_t)((tid / NJ) * DP + ((tid % NJ) ^ ((tid / NJ) & SWZ)) * 8) * 2u;
  const uint32_t lds_w = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(km_lds_void*)s_c + (uint32_t)(wid * 64 * 16));
  // CND: chunk row r of the stream is centre s_nbl[ch * CH + r] (L2-resident Cq), same
  // swizzled piece (the row & SWZ term does not depend on the round g)
  const uint32_t pz = (uint32_t)(((tid % NJ) ^ ((tid / NJ) & SWZ)) * 8) * 2u;
  auto issue_to = [&](int ch, int buf) {
    const uint16_t* base = Cq + (int64_t)ch * CH * DP;
    const uint32_t dst = lds_w + (uint32_t)((buf * CHP) * 16);
#pragma unroll
    for (int g = 0; g < GPT; ++g) {
      const uint32_t m0v = dst + (uint32_t)(g * NT * 16);
      if constexpr (CND) {
        const uint32_t off = (uint32_t)s_nbl[ch * CH + g * (NT / NJ) + tid / NJ] * (uint32_t)(DP * 2) + pz;
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                     :: "s"(m0v), "v"(off), "s"(Cq) : "memory");
      } else {
        const uint16_t* bg = base + g * (NT / NJ) * DP;
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                     :: "s"(m0v), "v"(src_off), "s"(bg) : "memory");
      }
    }
  };
  auto issue = [&](int ch) { issue_to(ch, ch % NBUF); };
  __syncthreads();
  float M = s_m[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) M = fmaxf(M, s_m[w]);
  M = M * 1.0001f + 1e-6f;
  // the accumulators start at -(0.5|c|^2 + M) and add c.x (B = the points as loaded):
  // acc = -(0.5|x - c|^2 + M - 0.5|x|^2) < 0, and for negative floats the SIGNED integer
  // order of the bits is the reverse of the value order, so the smallest key is the
  // largest acc = the nearest centre (padding centres, -1e30, have the largest keys)
  int nc = nchunk;                    // chunks streamed (CND: the list prefix within R)
  float nd_first = __builtin_inff();  // CND: first distance of a pruned centre to c_acl
  float dmp = -__builtin_inff();      // DRIFT: largest shift of a drift-pruned centre
  if constexpr (DRIFT) {
    float R = s_ur[0], tau = s_tau[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      R = fmaxf(R, s_ur[w]);
      tau = fminf(tau, s_tau[w]);
    }
    R = km_up1(2.f * R);
    // a dropped centre costs the rows up to tau of their l (the next filter tests
    // l - maxd): the threshold is capped so only the slow centres are dropped
    if (aux.tau_cap != nullptr) tau = fminf(tau, *aux.tau_cap);
    int c = 0;
    float dm = -__builtin_inff(), nf = __builtin_inff();
    bool keep[KH];
#pragma unroll
    for (int j = 0; j < KH; ++j) {
      const int p = tid * KH + j;
      const bool tail = p >= CH && p < kpad;
      const bool ball = !aux.drift_ball || ndv[j] <= R;
      keep[j] = tail && ball && dnv[j] >= tau;
      c += keep[j] ? 1 : 0;
      if (tail && !keep[j]) {
        if (dnv[j] < tau) dm = fmaxf(dm, dnv[j]);   // slow: bounds l through l - dmp
        else nf = fminf(nf, ndv[j]);               // fast, outside the ball: nd_first - ua
      }
    }
    int x = c;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    for (int off = 32; off >= 1; off >>= 1) {
      dm = fmaxf(dm, __shfl_xor(dm, off));
      nf = fminf(nf, __shfl_xor(nf, off));
    }
    if (lane == 63) s_kc[wid] = x;
    if (lane == 0) { s_kd[wid] = dm; s_kf[wid] = nf; }
    __syncthreads();
    int pre = x - c, kept = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      if (w < wid) pre += s_kc[w];
      kept += s_kc[w];
      dmp = fmaxf(dmp, s_kd[w]);
      nd_first = fminf(nd_first, s_kf[w]);
    }
    nc = 1 + (kept + CH - 1) / CH;
    // stream order: chunk 0 as listed, the kept entries compacted behind it, then padding
    // up to whole chunks (acl with 0.5|c|^2 = 1e30: never the nearest)
#pragma unroll
    for (int j = 0; j < KH; ++j) {
      const int p = tid * KH + j;
      int q = -1;
      if (p < CH) q = p;
      else if (keep[j]) q = CH + pre++;
      if (q >= 0) {
        s_nbl[q] = (uint16_t)nbv[j];
        s_hn16[q] = -(hv[j] + M);
      }
    }
    for (int q = CH + kept + tid; q < nc * CH; q += NT) {
      s_nbl[q] = (uint16_t)acl;
      s_hn16[q] = -(1e30f + M);
    }
    __syncthreads();                            // the stream's ids staged for the DMA
  } else if constexpr (CND) {
    float R = s_ur[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) R = fmaxf(R, s_ur[w]);
    R = km_up1(2.f * R);
    // chunk j >= 1 is needed iff its first (smallest) distance is <= R; chunk 0 always
    nc = 1 + __popcll(__ballot(lane >= 1 && lane < nchunk && thrv <= R));
    if (nc < nchunk) nd_first = __shfl(thrv, nc);
    const float* hb = aux.hnb + (int64_t)acl * kpad;
    for (int c = tid; c < kpad; c += NT) s_hn16[c] = -(hb[c] + M);
  } else {
    for (int c = tid; c < kpad; c += NT) s_hn16[c] = -(hn[c] + M);
  }
  issue(0);

  int bkey[PG], bch[PG], cm[PG];
  int bkey2[BND ? PG : 1], cm2[BND ? PG : 1];   // BND: second-smallest keys
#pragma unroll
  for (int g = 0; g < PG; ++g) { bkey[g] = 0x7fffffff; bch[g] = 0; cm[g] = 0x7fffffff; }
  if constexpr (BND) {
#pragma unroll
    for (int g = 0; g < PG; ++g) { bkey2[g] = 0x7fffffff; cm2[g] = 0x7fffffff; }
  }
  const int kmask = ~31;
  // software pipeline over the 8 sub-tiles of a chunk: sub-tile s accumulates into set
  // s & 1 while the argmin of sub-tile s - 1 reads the other set, so the argmin VALU runs
  // between the MFMAs instead of after them (sched_group_barrier pins the interleave);
  // sub-tile 7's argmin and the chunk merge run under the next chunk's sub-tile 0. The
  // pending set starts as +huge keys, so the first chunk's merge of "chunk -1" is inert.
  f32x4 acc[2][PG];
#pragma unroll
  for (int g = 0; g < PG; ++g) {
    const float big = __int_as_float(0x7f7fffff);
    acc[1][g] = {big, big, big, big};
  }
  auto load_frag = [&](const uint4* img, int ch, int sub, uint4 (&af)[KS], float4& h4) {
    const int row = sub * 16 + pl;
    h4 = *reinterpret_cast<const float4*>(&s_hn16[ch * CH + sub * 16 + 4 * lg]);
#pragma unroll
    for (int s = 0; s < KS; ++s) af[s] = img[row * NJ + ((4 * s + lg) ^ (row & SWZ))];
  };
  auto mfma_sub = [&](f32x4 (&ac)[PG], const uint4 (&af)[KS], const float4& h4) {
    const f32x4 c0 = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
    for (int g = 0; g < PG; ++g)
      ac[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[0]),
                                                      __builtin_bit_cast(bf16x8, bf[g][0]), c0, 0, 0, 0);
#pragma unroll
    for (int s = 1; s < KS; ++s)
#pragma unroll
      for (int g = 0; g < PG; ++g)
        ac[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[s]),
                                                        __builtin_bit_cast(bf16x8, bf[g][s]), ac[g], 0, 0, 0);
  };
  // keys = value bits & ~31 | (sub * 4 + r): the lowest id wins among equal keys of a chunk.
  // BND: with (x, y) new, the running pair (m <= m2) becomes m' = min3(m, x, y),
  // m2' = min(m2, med3(m, x, y)) (see reduce_tile of the pipelined form)
  auto med3 = [](int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
  };
  auto argmin_sub = [&](const f32x4 (&ac)[PG], int sub) {
#pragma unroll
    for (int g = 0; g < PG; ++g) {
      const int k0 = (__float_as_int(ac[g][0]) & kmask) | (sub * 4 + 0);
      const int k1 = (__float_as_int(ac[g][1]) & kmask) | (sub * 4 + 1);
      const int k2 = (__float_as_int(ac[g][2]) & kmask) | (sub * 4 + 2);
      const int k3 = (__float_as_int(ac[g][3]) & kmask) | (sub * 4 + 3);
      if constexpr (BND) {
        // second smallest of {cm, cm2, k0..k3}: min3(cm2, med3(cm, k0, k1), med3(cm', k2, k3))
        const int md1 = med3(cm[g], k0, k1);
        cm[g] = min(min(cm[g], k0), k1);
        const int md2 = med3(cm[g], k2, k3);
        cm[g] = min(min(cm[g], k2), k3);
        cm2[g] = min(min(cm2[g], md1), md2);
      } else {
        cm[g] = min(min(cm[g], k0), k1);
        cm[g] = min(min(cm[g], k2), k3);
      }
    }
  };
  // chunk merge: across chunks on the value bits only (strict: the earlier chunk keeps a
  // tie); BND: second smallest of {bkey, bkey2, cm, cm2}
  auto merge_chunk = [&](int chp) {
#pragma unroll
    for (int g = 0; g < PG; ++g) {
      if constexpr (BND) bkey2[g] = min(max(bkey[g], cm[g]), min(bkey2[g], cm2[g]));
      const bool take = (cm[g] & kmask) < (bkey[g] & kmask);
      bkey[g] = take ? cm[g] : bkey[g];
      bch[g] = take ? chp : bch[g];
      cm[g] = 0x7fffffff;
      if constexpr (BND) cm2[g] = 0x7fffffff;
    }
  };
  // interleave: 24 MFMAs of this sub-tile, the previous sub-tile's argmin VALU ops (36,
  // 1.5 per MFMA: inside the 8 issue cycles a 16x16x32 MFMA leaves free; BND: 60), and the
  // next sub-tile's fragment reads each right after the MFMAs that last read the register
  // it replaces (k-step s of all PG groups, then fragment s is dead): the next C values and
  // fragment 0 after MFMA 6, fragment 1 after 12, 2 after 18, 3 after 24 -- the two
  // fragment sets share registers instead of both living through the whole sub-tile
  auto pin = [&]() {
#ifndef KM_XP_NOPIN
#pragma unroll
    for (int i = 0; i < KS * PG; i += 2) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                 // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, BND ? 3 : 2, 0);       // VALU
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, BND ? 2 : 1, 0);
      if (i + 2 == PG) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS read
      else if ((i + 2) % PG == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
#endif
  };
  uint4 a[KS], an[KS];
  float4 h4, hn4;
  km_wait_vmcnt<0>();
  __syncthreads();                             // chunk 0 landed, s_hn16 written
  if (nc > 1) issue(1);
  load_frag(s_c, 0, 0, a, h4);
  for (int ch = 0; ch < nc; ++ch) {
    const uint4* img = s_c + (ch % NBUF) * CHP;
    const uint4* img_next = s_c + ((ch + 1) % NBUF) * CHP;
    // sub-tile 0 under the previous chunk's sub-tile 7 argmin, then the merge of that chunk
    load_frag(img, ch, 1, an, hn4);
    mfma_sub(acc[0], a, h4);
    argmin_sub(acc[1], 7);
    pin();
    __builtin_amdgcn_sched_barrier(0);
    merge_chunk(ch - 1);
#pragma unroll
    for (int sub = 1; sub < NSUB; ++sub) {
#pragma unroll
      for (int s = 0; s < KS; ++s) a[s] = an[s];
      h4 = hn4;
      // (branch-free: the last chunk re-reads its own first fragments, unused)
      if (sub + 1 < NSUB) load_frag(img, ch, sub + 1, an, hn4);
      else load_frag(ch + 1 < nc ? img_next : img, ch + 1 < nc ? ch + 1 : ch, 0, an, hn4);
      mfma_sub(acc[sub & 1], a, h4);
      argmin_sub(acc[(sub - 1) & 1], sub - 1);
      pin();
      __builtin_amdgcn_sched_barrier(0);
      if (sub == NSUB - 2) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        km_wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();          // chunk ch + 1 landed; chunk ch retired
        asm volatile("" ::: "memory");
        {
          // branch-free (a branch here splits the unrolled body and spills): past the
          // end the last chunk is loaded again into buffer (ch + 2) % 2, which no wave reads
          // again (chunk ch's, all of whose reads precede the barrier) or which already
          // holds those same bytes (the last chunk's own)
          const int c2 = ch + 2 < nc ? ch + 2 : nc - 1;
          issue_to(c2, (ch + 2) % NBUF);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) a[s] = an[s];
    h4 = hn4;
  }
  km_wait_vmcnt<0>();                          // the redundant last DMAs landed
  // the last chunk's sub-tile 7 and merge
  argmin_sub(acc[1], 7);
  merge_chunk(nc - 1);

  // ---- merge the 4 lane groups of each point, write the outputs
  double my_sse = 0.0;
#pragma unroll
  for (int g = 0; g < PG; ++g) {
    float v = -__int_as_float(bkey[g] & kmask);
    float v2 = 0.f;
    if constexpr (BND) v2 = -__int_as_float(bkey2[g] & kmask);
    const int ix = bkey[g] & 31;
    int id = bch[g] * CH + (ix >> 2) * 16 + 4 * lg + (ix & 3);
    if constexpr (CND) id = s_nbl[id];           // list position -> centre id
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float pv = __shfl_xor(v, o, 64);
      const int pi = __shfl_xor(id, o, 64);
      if constexpr (BND) {
        // second best over both: second smallest of {v, v2, pv, pv2}
        const float pv2 = __shfl_xor(v2, o, 64);
        v2 = fminf(fmaxf(v, pv), fminf(v2, pv2));
      }
      if (pv < v || (pv == v && pi < id)) { v = pv; id = pi; }
    }
    const int64_t p = pbase + g * 16 + pl;
    if constexpr (BND) {
      bool chg = false;
      int row = 0, old_c = 0;
      if (lg == 0 && p < n) {
        const float x2 = s_x2[wid][g * 16 + pl];
        row = s_row[wid][g * 16 + pl];
        if constexpr (CND) old_c = acl;
        else old_c = s_old[wid][g * 16 + pl];
        const float dist = fmaxf(2.f * (v - M) + x2, 0.f);
        const float dist2 = fmaxf(2.f * (v2 - M) + x2, 0.f);
        // u rounded up, l rounded down (the keys are truncated towards smaller distances)
        float lo2 = km_dn1(sqrtf(fmaxf(km_dn1(dist2 - tol), 0.f)));
        // CND: every pruned centre is >= nd_first - |x - c_acl| from x
        if constexpr (CND) lo2 = fminf(lo2, km_dn1(nd_first - s_ua[wid][g * 16 + pl]));
        // DRIFT: every drift-pruned centre is >= l - dmp from x (dmp = -inf: none pruned)
        if constexpr (DRIFT) lo2 = fminf(lo2, km_dn1(s_lold[wid][g * 16 + pl] - dmp));
        aux.ul[row] = make_float2(km_up1(sqrtf(km_up1(dist + tol))), fmaxf(lo2, 0.f));
        chg = id != old_c;
        if (chg) assign[row] = id;
        my_sse += (double)dist;
      }
      // moved rows -> the block's LDS list (one LDS atomic per wave and point group)
      const uint64_t cmk = __ballot(chg);
      if (cmk != 0ull) {
        int base = 0;
        if (lane == 0) base = atomicAdd(&s_nmv, __popcll(cmk));
        base = __shfl(base, 0);
        if (chg) {
          const int slot = base + __popcll(cmk & ((1ull << lane) - 1ull));
          s_mv[slot] = row;
          s_mvn[slot] = (uint16_t)id;
          s_mvo[slot] = (uint16_t)old_c;
        }
      }
    } else {
      if (lg == 0 && p < n) {
        const float x2 = s_x2[wid][g * 16 + pl];
        const float dist = fmaxf(2.f * (v - M) + x2, 0.f);
        assign[p] = id;
        if (mind) mind[p] = dist;
        if (xh) xh[p] = 0.5f * x2;
        my_sse += (double)dist;
      }
    }
  }
  if constexpr (BND) {
    // the block's moved rows -> the global list at one reserved range (coalesced writes)
    __syncthreads();
    const int c = s_nmv;
    if (c > 0) {
      if (tid == 0) s_mvbase = atomicAdd(aux.n_changed, (unsigned long long)c);
      __syncthreads();
      const long long b = (long long)s_mvbase;
      for (int j = tid; j < c; j += NT)
        if (b + j < aux.cap) {
          aux.changed[b + j] = s_mv[j];
          if (aux.chg_new) {
            aux.chg_new[b + j] = s_mvn[j];
            aux.chg_old[b + j] = s_mvo[j];
          }
        }
    }
  }
  if (xmax && lane == 0) atomicMax(xmax, __float_as_uint(mx));
  if (sse) {
    double s = my_sse;
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) s_sse[wid] = s;
    __syncthreads();
    if (tid == 0) {
      double tot = 0.0;
      for (int w = 0; w < NW; ++w) tot += s_sse[w];
      atomicAdd(sse + (blockIdx.x & sse_mask), tot);
    }
  }
}

// the 16x16x32 form holds two 32 KB centre chunks plus 0.5|c|^2 for every centre in LDS
// and runs two blocks per CU: it takes kpad <= 3456 (BND, with the per-point row /
// previous-cluster tables and the moved-row list: <= 2304); larger k goes to the
// pipelined form
static bool assign16_fits(int kpad, bool bnd = false, bool cnd = false) {
  // static: 2 chunk buffers (64 KB) + |x|^2 of the 384 points (+ BND: 5 x 384 words; CND:
  // 6 x 384 words + the 1024-entry u16 list) + small
  // (CND: the compiler's static size is 76944 B with DRIFT; 256 B of small arrays)
  return kpad % 128 == 0 && (!cnd || kpad <= 1024) &&
         2 * 128 * 128 * 2 + (bnd ? (cnd ? 6 : 5) : 1) * 4 * 6 * 16 * 4 + (cnd ? 2048 + 256 : 1024) +
                 (size_t)kpad * sizeof(float) <=
             80 * 1024;
}

template <bool BND, bool CND = false, bool DRIFT = false>
static hipError_t launch_assign16(const void* X, int64_t n, int64_t ldx, const void* Cq,
                                  const float* hn, int kpad, int* assign, float* mind, double* sse,
                                  int sse_mask, float* xh, unsigned* xmax, hipStream_t st,
                                  const int32_t* idx = nullptr, const KmAux& aux = KmAux{}) {
  // (one 8-wave block per CU -- half the centre-chunk traffic per point -- measured 2 %
  // slower: 20.5-20.7 vs 20.1-20.2 ms on one box, profiles/round5/r5_22)
  constexpr int NW = 4, PG = 6, MINB = 2;
  if (!assign16_fits(kpad, BND, CND)) return hipErrorInvalidValue;
  if (CND && (aux.tiles == nullptr || aux.n_tiles == nullptr || aux.nb == nullptr || aux.hnb == nullptr ||
              aux.nd == nullptr))
    return hipErrorInvalidValue;
  if (BND && (idx == nullptr || aux.mcount == nullptr || aux.tol == nullptr || aux.ul == nullptr ||
              aux.changed == nullptr || aux.n_changed == nullptr ||
              (aux.chg_new == nullptr) != (aux.chg_old == nullptr)))
    return hipErrorInvalidValue;
  const size_t dyn = (size_t)kpad * sizeof(float);
  // BND: n = the host's upper bound of the device count (blocks past the count exit)
  const int64_t grid = cdiv(n, (int64_t)NW * PG * 16);
  if (grid == 0) return hipSuccess;
  if (grid > 0x7fffffffLL) return hipErrorInvalidValue;
  auto kfn = kmeans_assign16_kernel<NW, PG, MINB, BND, CND, DRIFT>;
  static size_t attr_set = 0;
  if (dyn > attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)dyn);
    if (e != hipSuccess) return e;
    attr_set = dyn;
  }
  hipLaunchKernelGGL(kfn, dim3((unsigned)grid), dim3(NW * 64), dyn, st, (const uint16_t*)X, n, ldx,
                     (const uint16_t*)Cq, hn, kpad, assign, mind, sse, sse_mask, xh, xmax, idx, aux);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// K2 dispatch. bf16 with DP = 128: the 16x16x32 form above (kmeans_assign16_kernel).
// bf16 with DP = 64 (and the indexed forms): the pipelined distance-key form (4-wave blocks, two
// per CU, 3 point tiles per wave, 128-centre chunks double-buffered by LDS-DMA, next
// fragments prefetched, last tile's argmin software-pipelined): 1.20-1.25 PF/s at
// 20M-100M x 128 x 1024. f32, and bf16 with DP < 64: the generic form (8-wave blocks,
// 32-centre chunks staged through VGPRs, 128-VGPR cap, 4 blocks per CU).
// Measured and removed (numbers in profiles/round2/README.md, profiles/round3/README.md):
// 26 other tilings of the pipelined form (1 / 2 / 4 point tiles, 8-wave blocks, 64- and
// 256-centre chunks, triple / quadruple buffering, with and without prefetch or the
// software-pipelined argmin), a resident-centre form (centres in LDS for the whole
// launch, points streamed), a centre-stationary form (centres in VGPRs, points through
// an LDS-DMA ring: 23.4 vs 22.8 ms at 100M), a persistent form looping over point groups
// with next-group L2 prefetch (2-4 % slower), s_setprio on alternate blocks (within 1 %)
// and one 4-wave block per CU with 4-8 point tiles (5.0-5.5 vs 4.14 ms at 20M).
template <typename T, int DP>
static hipError_t launch_assign_dp(const void* X, int64_t n, int64_t ldx, const void* Cq,
                                   const float* hn, int kpad, int* assign, float* mind, double* sse,
                                   int sse_mask, hipStream_t st) {
#ifndef KM_XP_NO16
  if constexpr (sizeof(T) == 2 && DP == 128)
    if (assign16_fits(kpad))
      return launch_assign16<false>(X, n, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, nullptr, nullptr, st);
#endif
  if constexpr (sizeof(T) == 2 && DP >= 64)
    if (kpad % 128 == 0)
      return launch_assign_pipe<DP, 4, 3, 4, 2, 2, true>(X, n, ldx, Cq, hn, kpad, assign, mind, sse,
                                                         sse_mask, st);
  return launch_assign_v<T, DP, 8, 1, 2, 4>(X, n, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, st);
}

template <typename T>
static hipError_t launch_assign(int DP, const void* X, int64_t n, int64_t ldx, const void* Cq,
                                const float* hn, int kpad, int* assign, float* mind, double* sse, int sse_mask,
                                hipStream_t st) {
  switch (DP) {
    case 16: return launch_assign_dp<T, 16>(X, n, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, st);
    case 32: return launch_assign_dp<T, 32>(X, n, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, st);
    case 64: return launch_assign_dp<T, 64>(X, n, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, st);
    case 128: return launch_assign_dp<T, 128>(X, n, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, st);
    default: return hipErrorInvalidValue;
  }
}

template <typename T, int DP>
static hipError_t launch_segsum_dp(const void* X, int64_t ldx, const int* perm, const int64_t* cs,
                                   const int64_t* ss, int k, int seg, int64_t max_segs, float* S,
                                   hipStream_t st) {
  constexpr int NW = 4;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(max_segs, NW), 256 * 16));
  hipLaunchKernelGGL((kmeans_segsum_kernel<T, DP, NW, true>), dim3(grid), dim3(NW * 64), 0, st,
                     (const T*)X, ldx, perm, cs, ss, k, seg, S);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

template <typename T>
static hipError_t launch_segsum(int DP, const void* X, int64_t ldx, const int* perm,
                                const int64_t* cs, const int64_t* ss, int k, int seg,
                                int64_t max_segs, float* S, hipStream_t st) {
  switch (DP) {
    case 16: return launch_segsum_dp<T, 16>(X, ldx, perm, cs, ss, k, seg, max_segs, S, st);
    case 32: return launch_segsum_dp<T, 32>(X, ldx, perm, cs, ss, k, seg, max_segs, S, st);
    case 64: return launch_segsum_dp<T, 64>(X, ldx, perm, cs, ss, k, seg, max_segs, S, st);
    case 128: return launch_segsum_dp<T, 128>(X, ldx, perm, cs, ss, k, seg, max_segs, S, st);
    default: return hipErrorInvalidValue;
  }
}

extern "C" {
#ifdef KM_XP_TIMING
hipError_t dalgo_km_dbg_read(void* host, size_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dalgo::g_km_dbg), bytes, 0, hipMemcpyDeviceToHost);
}
#endif

// Sort-based K3. Workspace: block_counts int32[B*k], cluster_start/seg_start
// int64[k+1], perm int32[n]. B = number of row chunks (any >= 1).
hipError_t dalgo_kmeans_accumulate_sorted(const void* X, int is_bf16, int64_t n, int64_t ldx, int DP,
                                          const int* assign, int k, int B, int seg, int* block_counts,
                                          int64_t* cluster_start, int64_t* seg_start, int* perm,
                                          float* S, unsigned long long* cnt, hipStream_t st) {
  if (k < 1 || k > 16384 || B < 1 || seg < 1 || n >= (int64_t)0x7fffffff) return hipErrorInvalidValue;
  const int64_t rpc = cdiv(std::max<int64_t>(n, 1), B);
  const size_t lds_k = (size_t)k * sizeof(int);
  hipLaunchKernelGGL(kmeans_hist_kernel, dim3(B), dim3(256), lds_k, st, assign, n, rpc, k, block_counts,
                     (const unsigned long long*)nullptr, 1, (int64_t)1);
  DALGO_LAUNCH_CHECK();
  const size_t scan_lds = 2 * (size_t)k * sizeof(int);
  if (scan_lds > 64 * 1024) {
    static size_t scan_attr = 0;   // largest dynamic size enabled so far (k > 8192)
    if (scan_lds > scan_attr) {
      hipError_t e = hipFuncSetAttribute((const void*)kmeans_scan_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)scan_lds);
      if (e != hipSuccess) return e;
      scan_attr = scan_lds;
    }
  }
  launch_sort_scan(block_counts, B, k, seg, cluster_start, seg_start, cnt, nullptr, 1, 1, scan_lds, st);
  DALGO_LAUNCH_CHECK();
  if (k <= kScKmax)   // per-row LDS-cursor scatter only where the chunked form's LDS ends
    launch_scatter_chunked(k, B, st, assign, n, rpc, k,
                       (const int*)block_counts, (const int64_t*)cluster_start, perm,
                       (const unsigned long long*)nullptr, 1, (int64_t)1);
  else
    hipLaunchKernelGGL(kmeans_scatter_kernel, dim3(B), dim3(256), lds_k, st, assign, n, rpc, k,
                       (const int*)block_counts, (const int64_t*)cluster_start, perm);
  DALGO_LAUNCH_CHECK();
  const int64_t max_segs = cdiv(n, seg) + k;
  return is_bf16 ? launch_segsum<uint16_t>(DP, X, ldx, perm, cluster_start, seg_start, k, seg, max_segs, S, st)
                 : launch_segsum<float>(DP, X, ldx, perm, cluster_start, seg_start, k, seg, max_segs, S, st);
}

// Sort-based incremental K3 over the moved rows (2 signed entries each). m = the host's
// upper bound of the moved rows; mdev (optional) = the device-resident count (<= m).
// Workspace: ec / er / perm int32[2m], block_counts int32[B*k], cluster_start /
// seg_start int64[k+1]; B = the chunk count for 2m entries (chunks of `chunk` entries).
hipError_t dalgo_kmeans_move_sorted(const void* X, int is_bf16, int64_t ldx, int DP,
                                    const int32_t* changed, int64_t m, const int32_t* a_new,
                                    const int32_t* a_old, int k, int B, int seg, int* ec, int* er,
                                    int* block_counts, int64_t* cluster_start, int64_t* seg_start,
                                    int* perm, double* S, unsigned long long* cnt, const float* xh,
                                    double* Q, const unsigned long long* mdev, int64_t chunk,
                                    const int32_t* cnew, const int32_t* cold, hipStream_t st) {
  if (m <= 0) return hipSuccess;
  const int64_t n2 = 2 * m;
  if (k < 1 || k > kScKmax || B < 1 || seg < 1 || chunk < 1 || n2 >= (int64_t)0x7fffffff)
    return hipErrorInvalidValue;
  const int g = (int)std::min<int64_t>(cdiv(n2, 256), 4096);
  if ((cnew == nullptr) != (cold == nullptr)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(km_dexpand_kernel, dim3(g), dim3(256), 0, st, changed, m, a_new, a_old, ec, er, mdev,
                     cnew, cold);
  DALGO_LAUNCH_CHECK();
  const int64_t rpc = cdiv(n2, B);
  const size_t lds_k = (size_t)k * sizeof(int);
  hipLaunchKernelGGL(kmeans_hist_kernel, dim3(B), dim3(256), lds_k, st, (const int*)ec, n2, rpc, k,
                     block_counts, mdev, 2, chunk);
  DALGO_LAUNCH_CHECK();
  launch_sort_scan(block_counts, B, k, seg, cluster_start, seg_start, nullptr, mdev, 2, chunk, 2 * lds_k,
                   st);
  DALGO_LAUNCH_CHECK();
  launch_scatter_chunked(k, B, st, (const int*)ec, n2,
                     rpc, k, (const int*)block_counts, (const int64_t*)cluster_start, perm, mdev, 2,
                     chunk);
  DALGO_LAUNCH_CHECK();
  constexpr int NW = 4;
  const int64_t max_segs = cdiv(n2, seg) + k;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(max_segs, NW), 256 * 16));
#define KM_DSEG_LAUNCH(TT, D)                                                                        \
  hipLaunchKernelGGL((km_dsegsum_kernel<TT, D, NW>), dim3(grid), dim3(NW * 64), 0, st,           \
                     (const TT*)X, ldx, (const int*)perm, (const int*)er, (const int64_t*)cluster_start, \
                     (const int64_t*)seg_start, k, seg, S, cnt, xh, Q)
  switch (DP) {
    case 16: if (is_bf16) KM_DSEG_LAUNCH(uint16_t, 16); else KM_DSEG_LAUNCH(float, 16); break;
    case 32: if (is_bf16) KM_DSEG_LAUNCH(uint16_t, 32); else KM_DSEG_LAUNCH(float, 32); break;
    case 64: if (is_bf16) KM_DSEG_LAUNCH(uint16_t, 64); else KM_DSEG_LAUNCH(float, 64); break;
    case 128: if (is_bf16) KM_DSEG_LAUNCH(uint16_t, 128); else KM_DSEG_LAUNCH(float, 128); break;
    default: return hipErrorInvalidValue;
  }
#undef KM_DSEG_LAUNCH
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_kmeans_assign(const void* X, int is_bf16, int64_t n, int64_t ldx, int DP,
                               const void* Cq, const float* hn, int kpad, int* assign, float* mind,
                               double* sse, int sse_mask, hipStream_t st) {
  if (kpad % 32 != 0) return hipErrorInvalidValue;
  return is_bf16 ? launch_assign<uint16_t>(DP, X, n, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, st)
                 : launch_assign<float>(DP, X, n, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, st);
}

// K2 (pipelined form) over the rows idx[0, m) of X only (bound-filtered Lloyd iteration).
// idx may be null (rows 0 .. m); mind2 non-null selects the top-2 form (second-best
// distance per row, a lower bound for the bound filter); xh / xmax: 0.5|x|^2 per row and
// its maximum (full pass). post != null: the filtered-iteration form -- the row count is
// *post->mcount (device; m its upper bound), a resident grid walks the tiles and the
// bound update (u, l, changed rows vs a_prev) is fused into the epilogue.
hipError_t dalgo_kmeans_assign_idx(const void* X, int64_t m, int64_t ldx, int DP, const void* Cq,
                                   const float* hn, int kpad, const int32_t* idx, int* assign,
                                   float* mind, float* mind2, double* sse, int sse_mask, float* xh,
                                   unsigned* xmax, const DalgoKmPost* post, const DalgoKmCand* cand,
                                   hipStream_t st) {
  if (m <= 0) return hipSuccess;
  if (kpad % 128 != 0) return hipErrorInvalidValue;
  KmAux aux{};
  aux.xh = xh;
  aux.xmax = xmax;
  if (cand != nullptr && post == nullptr) return hipErrorInvalidValue;
  if (post != nullptr) {
    aux.mcount = post->mcount; aux.a_prev = post->a_prev; aux.tol = post->tol;
    aux.ul = reinterpret_cast<float2*>(post->ul); aux.changed = post->changed; aux.n_changed = post->n_changed;
    aux.cap = post->cap; aux.chg_new = post->chg_new; aux.chg_old = post->chg_old; aux.acl = post->acl;
    if ((aux.chg_new == nullptr) != (aux.chg_old == nullptr)) return hipErrorInvalidValue;
    if (cand != nullptr) {
      // idx = the active rows sorted by cluster (dalgo_kmeans_sort_active)
      aux.tiles = reinterpret_cast<const int4*>(cand->tiles);
      aux.n_tiles = cand->n_tiles; aux.hnb = cand->hnb;
      aux.nb = cand->nb; aux.nd = cand->nd; aux.extend = cand->extend;
      aux.ndb = cand->ndb; aux.dnb = cand->dnb; aux.tau_cap = cand->tau_cap;
      aux.drift_ball = cand->extend;   // (no extension chunks in the drift form)
      if (cand->tile16) {
        // the 16x16x32 tiling with the list prefix / the drift-compacted list (tiles of
        // <= 384 rows)
        if (DP != 128 || idx == nullptr) return hipErrorInvalidValue;
        if (cand->ndb != nullptr)
          return launch_assign16<true, true, true>(X, cand->max_tiles * 384, ldx, Cq, hn, kpad, assign, nullptr,
                                                   sse, sse_mask, nullptr, nullptr, st, idx, aux);
        return launch_assign16<true, true>(X, cand->max_tiles * 384, ldx, Cq, hn, kpad, assign, nullptr, sse,
                                           sse_mask, nullptr, nullptr, st, idx, aux);
      }
      if (cand->ndb != nullptr) {   // drift-aware candidate lists
        if (DP == 128)
          return launch_assign_pipe<128, 4, 2, 4, 2, 2, false, true, true, true, true>(
              X, m, ldx, Cq, hn, kpad, assign, nullptr, sse, sse_mask, st, idx, nullptr, aux);
        if (DP == 64)
          return launch_assign_pipe<64, 4, 2, 4, 2, 2, false, true, true, true, true>(
              X, m, ldx, Cq, hn, kpad, assign, nullptr, sse, sse_mask, st, idx, nullptr, aux);
        return hipErrorInvalidValue;
      }
      if (DP == 128)
        return launch_assign_pipe<128, 4, 2, 4, 2, 2, false, true, true, true>(
            X, m, ldx, Cq, hn, kpad, assign, nullptr, sse, sse_mask, st, idx, nullptr, aux);
      if (DP == 64)
        return launch_assign_pipe<64, 4, 2, 4, 2, 2, false, true, true, true>(
            X, m, ldx, Cq, hn, kpad, assign, nullptr, sse, sse_mask, st, idx, nullptr, aux);
      return hipErrorInvalidValue;
    }
#ifndef KM_XP_NO16
    // the dense form of the filtered iteration: 16x16x32 MFMAs, top-2 keys, no pruning
    if (DP == 128 && assign16_fits(kpad, true) && idx != nullptr)
      return launch_assign16<true>(X, m, ldx, Cq, hn, kpad, assign, nullptr, sse, sse_mask, nullptr, nullptr,
                                   st, idx, aux);
#endif
    if (cand == nullptr && aux.a_prev == nullptr && aux.acl == nullptr && idx == nullptr)
      return hipErrorInvalidValue;
    // top-2: 2 point tiles per wave (3 would spill past 256 VGPRs in the tile loop)
    if (DP == 128)
      return launch_assign_pipe<128, 4, 2, 4, 2, 2, false, true, true>(
          X, m, ldx, Cq, hn, kpad, assign, nullptr, sse, sse_mask, st, idx, nullptr, aux);
    if (DP == 64)
      return launch_assign_pipe<64, 4, 2, 4, 2, 2, false, true, true>(
          X, m, ldx, Cq, hn, kpad, assign, nullptr, sse, sse_mask, st, idx, nullptr, aux);
    return hipErrorInvalidValue;
  }
  if (mind2 != nullptr) {
    if (DP == 128)
      return launch_assign_pipe<128, 4, 2, 4, 2, 2, false, true>(
          X, m, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, st, idx, mind2, aux);
    if (DP == 64)
      return launch_assign_pipe<64, 4, 2, 4, 2, 2, false, true>(
          X, m, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, st, idx, mind2, aux);
    return hipErrorInvalidValue;
  }
#ifndef KM_XP_NO16
  if (DP == 128 && idx == nullptr && assign16_fits(kpad))
    return launch_assign16<false>(X, m, ldx, Cq, hn, kpad, assign, mind, sse, sse_mask, aux.xh, aux.xmax, st);
#endif
  if (DP == 128)
    return launch_assign_pipe<128, 4, 3, 4, 2, 2, true>(X, m, ldx, Cq, hn, kpad, assign, mind, sse,
                                                        sse_mask, st, idx, nullptr, aux);
  if (DP == 64)
    return launch_assign_pipe<64, 4, 3, 4, 2, 2, true>(X, m, ldx, Cq, hn, kpad, assign, mind, sse,
                                                       sse_mask, st, idx, nullptr, aux);
  return hipErrorInvalidValue;
}

hipError_t dalgo_kmeans_update(float* C, const float* S, const unsigned long long* cnt, int k,
                               int d, int DP,
                               void* Cq, int is_bf16, float* hn, int kpad, float* shift2,
                               hipStream_t st) {
  const int grid = (int)cdiv(kpad, 4);
  if (is_bf16)
    hipLaunchKernelGGL(kmeans_update_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, C, S, cnt, k,
                       d, DP, (uint16_t*)Cq, hn, kpad, shift2);
  else
    hipLaunchKernelGGL(kmeans_update_kernel<float>, dim3(grid), dim3(256), 0, st, C, S, cnt, k, d,
                       DP, (float*)Cq, hn, kpad, shift2);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// Candidate-pruned K2 preparation: the active rows idx[0, *n_active) (cluster acl[e] each)
// counting-sorted by cluster into rows_sorted, their cluster runs cstart[0..k], and the
// tile table (tile -> cluster, first position; tiles of `tile` rows never straddle two
// clusters). cap = the capacity of idx; B = the chunk bound of the sort (entries per chunk
// `chunk`). No host sync: every launch derives its geometry from the device count.
hipError_t dalgo_kmeans_sort_active(const int32_t* acl, const int32_t* idx, int64_t cap,
                                    const unsigned long long* n_active, int k, int B, int64_t chunk,
                                    int* block_counts, int64_t* cstart, int64_t* seg_start,
                                    int32_t* rows_sorted, int tile, int32_t* tiles,
                                    unsigned long long* n_tiles,
                                    int64_t max_tiles, hipStream_t st) {
  if (cap <= 0) return hipSuccess;
  if (k < 1 || k > kScKmax || B < 1 || chunk < 1 || tile < 1 || cap >= (int64_t)0x7fffffff ||
      n_active == nullptr)
    return hipErrorInvalidValue;
  const int64_t rpc = cdiv(cap, B);
  const size_t lds_k = (size_t)k * sizeof(int);
  hipLaunchKernelGGL(kmeans_hist_kernel, dim3(B), dim3(256), lds_k, st, (const int*)acl, cap, rpc, k,
                     block_counts, n_active, 1, chunk);
  DALGO_LAUNCH_CHECK();
  launch_sort_scan(block_counts, B, k, 1 << 20, cstart, seg_start, nullptr, n_active, 1, chunk, 2 * lds_k,
                   st);
  DALGO_LAUNCH_CHECK();
  launch_scatter_chunked(k, B, st, (const int*)acl, cap,
                     rpc, k, (const int*)block_counts, (const int64_t*)cstart, (int*)rows_sorted,
                     n_active, 1, chunk, (const int*)idx);
  DALGO_LAUNCH_CHECK();
  hipLaunchKernelGGL(km_tiles_kernel, dim3(64), dim3(1024), 0, st, (const int64_t*)cstart, k, tile,
                     reinterpret_cast<int4*>(tiles), n_tiles, max_tiles);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
