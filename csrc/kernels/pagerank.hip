// K4: PageRank on a destination-partitioned edge list (pull), plus an on-device
// R-MAT (Graph500-style) power-law edge generator.
//
// Reference (graph_computation/pagerank.py): adjacency lists via
// distinct().groupByKey() (:41), N = number of source vertices (:44), ranks
// 1/N (:47), then 10 x [join + flatMap(computeContribs) (:52-54) ->
// reduceByKey(add).mapValues(q/N + (1-q)*r) (:57)] — two shuffles per iteration.
//
// Here each rank owns destination vertices [v_lo, v_hi) and exactly their
// in-edges, sorted by (dst, src) and deduplicated (= distinct()). One iteration:
//   c_full = all_gather(c_slice)                 (RCCL, N floats)
//   pr_spmv : acc[v] = sum_{u->v} c[u]           (segmented wave reduction)
//   pr_update: r[v] = q/N + (1-q)*acc[v]; c[v] = r[v]/outdeg[v]   (fused epilogue)
// pr_spmv streams src/dst once (8 B/edge, 16-B vector loads, 4 edges per lane)
// and gathers c[src] (the random part, Infinity-Cache sensitive). Each wave walks
// 256-edge windows; per-lane runs are summed sequentially, then a 6-step
// segmented scan over lane aggregates (key = destination) finishes the window.
// Rows that begin and end inside a window are written with plain stores; only
// window-crossing rows use float atomics, so heavy (power-law) rows are split
// across waves automatically and the work per wave is edge-balanced.
//
// "reference" semantics reproduce the join-based formulation exactly: c[u] < 0
// marks a vertex that is absent from the ranks RDD (no contribution record); a
// destination is present after an iteration iff it received >= 1 record.
// "standard" semantics: every vertex present, dangling mass redistributed.
#include "dalgo/common.h"
#include <algorithm>

namespace dalgo {

// ---------------------------------------------------------------------------
// R-MAT edge generator: edge e of stream (seed, 7): 2 Philox calls -> 8 x 32-bit
// words; each byte picks one quadrant level (8-bit probabilities).
__device__ __forceinline__ uint32_t scramble(uint32_t v, int scale, uint32_t k0, uint32_t k1) {
  const uint32_t mask = (scale >= 32) ? 0xffffffffu : ((1u << scale) - 1u);
  v = (v * (k0 | 1u)) & mask;
  v ^= (v >> (scale / 2 + 1));
  v = (v * (k1 | 1u)) & mask;
  v ^= (v >> (scale / 3 + 1));
  v = (v * 0x9E3779B1u) & mask;
  return v;
}

__global__ void __launch_bounds__(256)
rmat_kernel(uint64_t seed, int scale, int64_t e_off, int64_t n, uint32_t pa, uint32_t pab,
            uint32_t pabc, int do_scramble, int32_t* __restrict__ src, int32_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = (uint64_t)(e_off + i);
    u32x4 h0 = philox_block(seed, 7, 2 * e), h1 = philox_block(seed, 7, 2 * e + 1);
    const uint32_t w[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    uint32_t s = 0, d = 0;
#pragma unroll
    for (int l = 0; l < 32; ++l) {
      if (l < scale) {
        const uint32_t u = (w[l >> 2] >> (8 * (l & 3))) & 0xffu;
        const uint32_t sb = (u >= pab) ? 1u : 0u;
        const uint32_t db = (u >= pabc) ? 1u : ((u >= pa && u < pab) ? 1u : 0u);
        s = (s << 1) | sb;
        d = (d << 1) | db;
      }
    }
    if (do_scramble) {
      s = scramble(s, scale, (uint32_t)seed ^ 0x5bd1e995u, (uint32_t)(seed >> 32) ^ 0x27d4eb2fu);
      d = scramble(d, scale, (uint32_t)seed ^ 0x5bd1e995u, (uint32_t)(seed >> 32) ^ 0x27d4eb2fu);
    }
    src[i] = (int32_t)s;
    dst[i] = (int32_t)d;
  }
}

// ---------------------------------------------------------------------------
// pull SpMV over a (dst, src)-sorted local edge list (reduce-by-key per wave)
// ACC: a second pass over another edge subset of the same rows (overlapped ghost exchange):
// complete rows add to acc / set pres instead of overwriting them
template <bool ACC>
__device__ __forceinline__ void flush_run(float* acc, int32_t* pres, int key, float v, int f,
                                          bool partial) {
  if (key < 0) return;
  if (partial) {
    atomicAdd(&acc[key], v);
    if (f) atomicOr(&pres[key], 1);
  } else if constexpr (ACC) {
    acc[key] += v;
    if (f) pres[key] = 1;
  } else {
    acc[key] = v;
    pres[key] = f;
  }
}

// The gather c[src] bounds this kernel on the vector-memory address path, not on bytes:
// measured and removed (profiles/round3/pmc_pagerank.md, profiles/round3/logs): an
// XCD-partitioned form with the edges split by source line over the 8 L2s (fabric reads
// 62 -> 21 GB, time unchanged), a hot-source LDS table and a software-pipelined edge
// stream (both within 3 % or slower). The blocked form (pr_binned.hip) removes the
// random gather altogether and is the default.
template <int NW, bool NT, bool ACC>
__global__ void __launch_bounds__(NW * 64)
pr_spmv_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dstl, int64_t E,
               const float* __restrict__ c, float* __restrict__ acc, int32_t* __restrict__ pres) {
  // dstl: destination as LOCAL row index. E is padded to a multiple of 4 with
  // (src = -1, dst = -1) edges. Windows of 256 edges, 4 consecutive per lane.
  const int lane = threadIdx.x & 63;
  const int64_t nwin = (E + 255) / 256;
  const int64_t wave = (int64_t)blockIdx.x * NW + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * NW;
  for (int64_t wi = wave; wi < nwin; wi += nwaves) {
    const int64_t e0 = wi * 256 + 4 * lane;
    int4 s4 = make_int4(-1, -1, -1, -1), d4 = make_int4(-1, -1, -1, -1);
    if (e0 < E) {
      s4 = ld_int4<NT>(src + e0);
      d4 = ld_int4<NT>(dstl + e0);
    }
    const int sv[4] = {s4.x, s4.y, s4.z, s4.w};
    const int dv[4] = {d4.x, d4.y, d4.z, d4.w};
    float cv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) cv[j] = (sv[j] >= 0) ? c[sv[j]] : -1.f;
    // keys of the edges just outside the window (row continuation tests)
    int dprev = -2, dnext = -2;
    if (lane == 0 && wi > 0) dprev = dstl[wi * 256 - 1];
    if (lane == 63 && wi * 256 + 256 < E) dnext = dstl[wi * 256 + 256];
    dprev = __builtin_amdgcn_readlane(dprev, 0);
    dnext = __builtin_amdgcn_readlane(dnext, 63);
    const int wk_first = __builtin_amdgcn_readlane(dv[0], 0);    // key of the window's first edge
    const int wk_last = __builtin_amdgcn_readlane(dv[3], 63);    // key of the window's last edge
    auto partial_key = [&](int key) {
      return (key == wk_first && key == dprev) || (key == wk_last && key == dnext);
    };

    // ---- per-lane runs: head (first run), tail (last run), interior runs flushed now
    const int k0 = dv[0];
    int key = k0;
    float run = 0.f;
    int runf = 0;
    float head = 0.f;
    int headf = 0;
    bool single = true;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (dv[j] != key) {
        if (single) { head = run; headf = runf; single = false; }
        else flush_run<ACC>(acc, pres, key, run, runf, false);   // interior: complete row
        key = dv[j];
        run = 0.f;
        runf = 0;
      }
      const float v = cv[j];
      run += (v > 0.f) ? v : 0.f;
      runf |= (v >= 0.f) ? 1 : 0;
    }
    const int kt = key;   // tail key (== k0 when single)

    // ---- segmented inclusive scan of tail values across lanes
    // element L: (tail_L, flag_L) with flag = run starts in lane L
    const int kt_left = __shfl_up(kt, 1);
    int flag = (!single || lane == 0 || kt_left != k0) ? 1 : 0;
    float sv_ = run;
    int sf_ = runf;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float v2 = __shfl_up(sv_, off);
      const int f2 = __shfl_up(sf_, off);
      const int g2 = __shfl_up(flag, off);
      if (lane >= off && !flag) {
        sv_ += v2;
        sf_ |= f2;
        flag |= g2;
      }
    }
    // S_L = sv_: complete (within-window) sum of the run ending at lane L's right edge
    const float S_left = __shfl_up(sv_, 1);
    const int F_left = __shfl_up(sf_, 1);
    const bool cont_left = (lane > 0) && (kt_left == k0);
    const int k0_right = __shfl_down(k0, 1);
    const bool cont_right = (lane < 63) && (k0_right == kt);

    if (!single) {
      // head run ends inside this lane
      const float hv = head + (cont_left ? S_left : 0.f);
      const int hf = headf | (cont_left ? F_left : 0);
      flush_run<ACC>(acc, pres, k0, hv, hf, partial_key(k0));
    }
    if (!cont_right) flush_run<ACC>(acc, pres, kt, sv_, sf_, partial_key(kt));
  }
}


// ---------------------------------------------------------------------------
// fused epilogue: ranks, next contributions, dangling mass
//   mode 0 (reference): r = pres ? q/N + (1-q)*acc : absent(-1);
//                       c = (pres && outdeg > 0) ? r/outdeg : -1
//   mode 1 (standard):  r = q/N + (1-q)*(acc + dangling/N); c = outdeg > 0 ? r/outdeg : 0;
//                       dangling_next += (outdeg == 0) ? r : 0
__global__ void __launch_bounds__(256)
pr_update_kernel(const float* __restrict__ acc, const int32_t* __restrict__ pres,
                 const int32_t* __restrict__ outdeg, int64_t n, float q, float invN, int mode,
                 const float* __restrict__ dangling_in, float* __restrict__ r,
                 float* __restrict__ c, float* __restrict__ dangling_out) {
  float dl = 0.f;
  const float dang = (mode == 1 && dangling_in) ? dangling_in[0] : 0.f;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
       v += (int64_t)gridDim.x * blockDim.x) {
    const int od = outdeg[v];
    if (mode == 0) {
      const bool p = pres[v] != 0;
      const float rv = p ? q * invN + (1.f - q) * acc[v] : -1.f;
      r[v] = rv;
      c[v] = (p && od > 0) ? rv / (float)od : -1.f;
    } else {
      const float rv = q * invN + (1.f - q) * (acc[v] + dang * invN);
      r[v] = rv;
      c[v] = od > 0 ? rv / (float)od : 0.f;
      if (od == 0) dl += rv;
    }
  }
  if (mode == 1 && dangling_out) {
    dl = wave_sum(dl);
    if ((threadIdx.x & 63) == 0 && dl != 0.f) atomicAdd(dangling_out, dl);
  }
}

}  // namespace dalgo

using namespace dalgo;

extern "C" {

hipError_t dalgo_rmat(uint64_t seed, int scale, int64_t e_off, int64_t n, float a, float b, float c,
                      int do_scramble, int32_t* src, int32_t* dst, hipStream_t st) {
  if (scale < 1 || scale > 31) return hipErrorInvalidValue;
  const uint32_t pa = (uint32_t)(a * 256.f + 0.5f);
  const uint32_t pab = (uint32_t)((a + b) * 256.f + 0.5f);
  const uint32_t pabc = (uint32_t)((a + b + c) * 256.f + 0.5f);
  const int grid = (int)std::min<int64_t>(cdiv(n, 256), 256 * 16);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(rmat_kernel, dim3(grid), dim3(256), 0, st, seed, scale, e_off, n, pa, pab,
                     pabc, do_scramble, src, dst);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_pr_spmv(const int32_t* src, const int32_t* dstl, int64_t E, const float* c,
                         int64_t n_c, float* acc, int32_t* pres, int accumulate, hipStream_t st) {
  if (E % 4 != 0) return hipErrorInvalidValue;
  constexpr int NW = 4;
  const int64_t nwin = cdiv(E, 256);
  const int grid = (int)std::min<int64_t>(cdiv(nwin, NW), 256 * 16);
  if (grid == 0) return hipSuccess;
  // edge stream read once per iteration: non-temporal loads
  if (accumulate)
    hipLaunchKernelGGL((pr_spmv_kernel<NW, true, true>), dim3(grid), dim3(NW * 64), 0, st, src, dstl,
                       E, c, acc, pres);
  else
    hipLaunchKernelGGL((pr_spmv_kernel<NW, true, false>), dim3(grid), dim3(NW * 64), 0, st, src, dstl,
                       E, c, acc, pres);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_pr_update(const float* acc, const int32_t* pres, const int32_t* outdeg, int64_t n,
                           float q, float invN, int mode, const float* dangling_in, float* r,
                           float* c, float* dangling_out, hipStream_t st) {
  const int grid = (int)std::min<int64_t>(cdiv(n, 256), 256 * 8);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(pr_update_kernel, dim3(grid), dim3(256), 0, st, acc, pres, outdeg, n, q, invN,
                     mode, dangling_in, r, c, dangling_out);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
