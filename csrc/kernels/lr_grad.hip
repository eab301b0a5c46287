// K1 + K7 + K10: fused Bernoulli-sampled logistic-regression gradient and eval.
//
// Replaces the reference's per-record Python hot loop
//   points.sample(False, f, 42+t).map(gradient).treeAggregate(...)
// (optimization/ssgd.py:97-103, gradient at ssgd.py:27-33, logistic_f at
// ssgd.py:23-24; per-partition mean at optimization/ma.py:39-43) with ONE pass over
// the sampled rows of X held in HBM:
//   sel(row)  = philox(seed, step, global_row) < frac * 2^32        (K7, in-register)
//   z         = x . w (+ bias)                                      (row GEMV)
//   r         = sigma(z) - y,  sigma = 1/(exp(-z) + 1 + eps)
//   g        += r * x,  g_bias += r,  cnt += 1                      (rank-1 accumulate)
// The gradient is GEMV-shaped (about 1 FLOP/B) so the roofline is HBM bandwidth:
// each selected row is read exactly once with 16-byte vector loads, four rows per
// wave in flight, the per-row dot product reduced across the 64 lanes with 7
// cross-lane ops (permlane32/permlane16 swaps + DPP row rotations, no LDS), and
// the gradient accumulated in VGPRs (each lane owns a fixed set of columns, so
// g never crosses lanes). Per-block partials go to a slab and are combined by a
// deterministic two-level last-arriver reduction (agent-scope release/acquire,
// fixed summation order) — no float atomics, bitwise reproducible.
//
// Segments: rows [seg_lo[s], seg_lo[s+1]) use model s (MA/BMUF/EASGD keep one
// local model per logical worker, ma.py:86-87); SSGD uses a single segment.
#include "dalgo/common.h"

namespace dalgo {

struct LrParams {
  const void* X;        // [n_local, ld] row-major, T = bf16 or f32
  const float* y;       // [n_local] labels in {0,1}
  const float* W;       // [n_seg, ldw]  (w[0..D) features, w[D] bias if has_bias)
  const int64_t* seg;   // [n_seg + 1] local row bounds (device)
  int64_t ld;           // row stride of X in elements (multiple of the 16-B vector)
  int64_t row_offset;   // global index of local row 0 (sampling is keyed by global row)
  int D;                // feature count (columns [D, ld) are ignored: zero weights, no writes)
  int ldw;              // row stride of W / G
  int has_bias;
  float eps;            // 0 (ssgd.py:24) or 1e-6 (ma.py:26)
  uint64_t seed, step;  // sampling stream
  uint32_t thr;         // Bernoulli threshold: select iff u32 < thr
  int full;             // 1: every row selected (full-batch GD)
  int rows_per_block;   // multiple of 256
  // grad outputs
  float* slab;          // [n_seg * gx, S]
  float* gslab;         // [n_seg * ngroups, S]
  unsigned* cnt1;       // [n_seg * ngroups]   arrival counters (zeroed)
  unsigned* cnt2;       // [n_seg]
  float* G;             // [n_seg, ldw] gradient sum
  float* C;             // [n_seg] selected-row count
  int S;                // slab row stride (>= ldw + 1)
  // eval outputs
  unsigned long long* correct;  // [n_seg] (eval mode)
  float* loss;                  // [n_seg] sum of log-loss (eval mode)
};

constexpr int kGroup = 16;   // blocks per first-level reduction group

template <typename T> struct VecTraits;
template <> struct VecTraits<uint16_t> { static constexpr int VEC = 8; };
template <> struct VecTraits<float>    { static constexpr int VEC = 4; };

template <typename T>
__device__ __forceinline__ void unpack(const uint4& v, float (&o)[VecTraits<T>::VEC]);
template <>
__device__ __forceinline__ void unpack<uint16_t>(const uint4& v, float (&o)[8]) {
  o[0] = bf16lo(v.x); o[1] = bf16hi(v.x); o[2] = bf16lo(v.y); o[3] = bf16hi(v.y);
  o[4] = bf16lo(v.z); o[5] = bf16hi(v.z); o[6] = bf16lo(v.w); o[7] = bf16hi(v.w);
}
template <>
__device__ __forceinline__ void unpack<float>(const uint4& v, float (&o)[4]) {
  o[0] = __uint_as_float(v.x); o[1] = __uint_as_float(v.y);
  o[2] = __uint_as_float(v.z); o[3] = __uint_as_float(v.w);
}

__device__ __forceinline__ void publish_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void acquire_fence() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// EVAL=false: gradient; EVAL=true: accuracy + log-loss over every row.
template <typename T, int NC, bool EVAL, int NW>
__global__ void __launch_bounds__(NW * 64)
lr_rows_kernel(LrParams p) {
  constexpr int VEC = VecTraits<T>::VEC;
  constexpr int COLS = NC * 64 * VEC;  // columns covered per lane-set
  __shared__ int s_list[NW][256];      // per-wave list of selected rows (local idx)
  __shared__ float s_red[NW][COLS + 2 + 2];
  __shared__ int s_flag;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int seg = blockIdx.y;
  const int bx = blockIdx.x;
  const int gx = gridDim.x;
  const int64_t seg_lo = p.seg[seg], seg_hi = p.seg[seg + 1];
  const int64_t lo = seg_lo + (int64_t)bx * p.rows_per_block;
  const int64_t hi = max(lo, min(seg_hi, lo + (int64_t)p.rows_per_block));
  const int nchunks = (int)(p.ld / VEC);

  // model fragment in registers
  const float* w = p.W + (int64_t)seg * p.ldw;
  float wr[NC][VEC];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      int col = (c * 64 + lane) * VEC + e;
      wr[c][e] = (col < p.D) ? w[col] : 0.f;
    }
  const float wb = p.has_bias ? w[p.D] : 0.f;

  float g[NC][VEC];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < VEC; ++e) g[c][e] = 0.f;
  float gb = 0.f;      // bias gradient (sum r), identical in every lane
  float cntf = 0.f;    // selected rows
  float lossf = 0.f;   // eval: log-loss sum
  unsigned correct = 0;

  const T* X = reinterpret_cast<const T*>(p.X);
  // group walk in global-row space, 256 rows per group, 4 rows per lane
  const int64_t glo = p.row_offset + lo, ghi = p.row_offset + hi;
  const int64_t gstart = glo & ~(int64_t)3;
  int* list = s_list[wid];

  for (int64_t g0 = gstart + (int64_t)wid * 256; g0 < ghi; g0 += (int64_t)NW * 256) {
    // ---- K7: Bernoulli selection, compacted into the wave's LDS list
    const int64_t r0 = g0 + 4 * lane;
    u32x4 h{0u, 0u, 0u, 0u};
    if (!p.full && !EVAL && r0 < ghi) h = philox_block(p.seed, p.step, (uint64_t)r0 >> 2);
    const uint32_t hv[4] = {h.x, h.y, h.z, h.w};
    int base = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gr = r0 + j;
      const bool sel = (gr >= glo) && (gr < ghi) && (EVAL || p.full || hv[j] < p.thr);
      const uint64_t m = __ballot(sel);
      const int pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (sel) list[pos] = (int)(gr - p.row_offset - lo);
      base += __popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int n = base;

    // ---- row batches of 4: loads first, then dot, reduce, sigmoid, accumulate
    for (int i = 0; i < n; i += 4) {
      const int k1 = min(i + 1, n - 1), k2 = min(i + 2, n - 1), k3 = min(i + 3, n - 1);
      const int64_t ra = lo + __builtin_amdgcn_readfirstlane(list[i]);
      const int64_t rb = lo + __builtin_amdgcn_readfirstlane(list[k1]);
      const int64_t rc = lo + __builtin_amdgcn_readfirstlane(list[k2]);
      const int64_t rd = lo + __builtin_amdgcn_readfirstlane(list[k3]);
      const float va = 1.f, vb = (i + 1 < n) ? 1.f : 0.f, vc = (i + 2 < n) ? 1.f : 0.f,
                  vd = (i + 3 < n) ? 1.f : 0.f;
      uint4 xa[NC], xb[NC], xc[NC], xd[NC];
      const T* pa = X + ra * p.ld;
      const T* pb = X + rb * p.ld;
      const T* pc = X + rc * p.ld;
      const T* pd = X + rd * p.ld;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = c * 64 + lane;
        if (ch < nchunks) {
          xa[c] = *reinterpret_cast<const uint4*>(pa + (int64_t)ch * VEC);
          xb[c] = *reinterpret_cast<const uint4*>(pb + (int64_t)ch * VEC);
          xc[c] = *reinterpret_cast<const uint4*>(pc + (int64_t)ch * VEC);
          xd[c] = *reinterpret_cast<const uint4*>(pd + (int64_t)ch * VEC);
        } else {
          xa[c] = xb[c] = xc[c] = xd[c] = make_uint4(0u, 0u, 0u, 0u);
        }
      }
      // labels: lane l serves row (l >> 4)
      const int q = lane >> 4;
      const int64_t rq = q == 0 ? ra : (q == 1 ? rb : (q == 2 ? rc : rd));
      const float yq = p.y[rq];

      float da = 0.f, db = 0.f, dc = 0.f, dd = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        float fa[VEC], fb[VEC], fc[VEC], fd[VEC];
        unpack<T>(xa[c], fa); unpack<T>(xb[c], fb); unpack<T>(xc[c], fc); unpack<T>(xd[c], fd);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          da = fmaf(fa[e], wr[c][e], da);
          db = fmaf(fb[e], wr[c][e], db);
          dc = fmaf(fc[e], wr[c][e], dc);
          dd = fmaf(fd[e], wr[c][e], dd);
        }
      }
      const float z = wave_sum4(da, db, dc, dd) + wb;
      const float sig = 1.f / (__expf(-z) + 1.f + p.eps);
      const float vq = q == 0 ? va : (q == 1 ? vb : (q == 2 ? vc : vd));
      if constexpr (EVAL) {
        // pred = sigma < 0.5 ? 0 : 1  (ssgd.py:108-109)
        const float pred = sig < 0.5f ? 0.f : 1.f;
        const float ok = (pred == yq) ? 1.f : 0.f;
        const float sc = fminf(fmaxf(sig, 1e-7f), 1.f - 1e-7f);
        const float l = -(yq * __logf(sc) + (1.f - yq) * __logf(1.f - sc));
        // one lane per row-block contributes
        const float oka = readlane_f(ok * vq, 0) + readlane_f(ok * vq, 16) +
                          readlane_f(ok * vq, 32) + readlane_f(ok * vq, 48);
        lossf += readlane_f(l * vq, 0) + readlane_f(l * vq, 16) + readlane_f(l * vq, 32) +
                 readlane_f(l * vq, 48);
        correct += (unsigned)oka;
      } else {
        const float r = (sig - yq) * vq;
        const float ra_ = readlane_f(r, 0), rb_ = readlane_f(r, 16), rc_ = readlane_f(r, 32),
                    rd_ = readlane_f(r, 48);
        gb += (ra_ + rb_) + (rc_ + rd_);
        cntf += va + vb + vc + vd;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          float fa[VEC], fb[VEC], fc[VEC], fd[VEC];
          unpack<T>(xa[c], fa); unpack<T>(xb[c], fb); unpack<T>(xc[c], fc); unpack<T>(xd[c], fd);
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            float acc = g[c][e];
            acc = fmaf(ra_, fa[e], acc);
            acc = fmaf(rb_, fb[e], acc);
            acc = fmaf(rc_, fc[e], acc);
            acc = fmaf(rd_, fd[e], acc);
            g[c][e] = acc;
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  if constexpr (EVAL) {
    __shared__ float s_ev[NW][2];
    if (lane == 0) { s_ev[wid][0] = (float)correct; s_ev[wid][1] = lossf; }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long c = 0; float l = 0.f;
      for (int k = 0; k < NW; ++k) { c += (unsigned long long)s_ev[k][0]; l += s_ev[k][1]; }
      atomicAdd(&p.correct[seg], c);
      atomicAdd(&p.loss[seg], l);
    }
    return;
  } else {
    // ---- block reduction across waves (fixed order)
    float* red = s_red[wid];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int e = 0; e < VEC; ++e) red[(c * 64 + lane) * VEC + e] = g[c][e];
    if (lane == 0) { red[COLS] = gb; red[COLS + 1] = cntf; }
    __syncthreads();
    const int S = p.S;
    const int D = p.D;
    float* my = p.slab + ((int64_t)seg * gx + bx) * S;
    for (int col = threadIdx.x; col < D; col += NW * 64) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < NW; ++k) s += s_red[k][col];
      my[col] = s;
    }
    if (threadIdx.x == 0) {
      float sb = 0.f, sc = 0.f;
      for (int k = 0; k < NW; ++k) { sb += s_red[k][COLS]; sc += s_red[k][COLS + 1]; }
      my[D] = sb;       // bias grad slot
      my[D + 1] = sc;   // count slot
    }
    // ---- level 1: last arriver of each 16-block group sums the group's slabs
    const int ngroups = (gx + kGroup - 1) / kGroup;
    const int grp = bx / kGroup;
    const int gsize = min(kGroup, gx - grp * kGroup);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      publish_fence();
      unsigned t = __hip_atomic_fetch_add(&p.cnt1[seg * ngroups + grp], 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
      s_flag = (t == (unsigned)(gsize - 1));
    }
    __syncthreads();
    if (!s_flag) return;
    if (threadIdx.x == 0) acquire_fence();
    __syncthreads();
    const int nv = D + 2;
    {
      const float* src = p.slab + ((int64_t)seg * gx + grp * kGroup) * S;
      float* dst = p.gslab + ((int64_t)seg * ngroups + grp) * S;
      for (int col = threadIdx.x; col < nv; col += NW * 64) {
        float s = 0.f;
        for (int k = 0; k < gsize; ++k) s += src[(int64_t)k * S + col];
        dst[col] = s;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      p.cnt1[seg * ngroups + grp] = 0u;   // re-arm for the next launch
      publish_fence();
      unsigned t = __hip_atomic_fetch_add(&p.cnt2[seg], 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
      s_flag = (t == (unsigned)(ngroups - 1));
    }
    __syncthreads();
    if (!s_flag) return;
    if (threadIdx.x == 0) acquire_fence();
    __syncthreads();
    // ---- level 2: sum group slabs in order -> G[seg], C[seg]
    {
      const float* src = p.gslab + (int64_t)seg * ngroups * S;
      float* Gs = p.G + (int64_t)seg * p.ldw;
      for (int col = threadIdx.x; col < nv; col += NW * 64) {
        float s = 0.f;
        for (int k = 0; k < ngroups; ++k) s += src[(int64_t)k * S + col];
        if (col < D) Gs[col] = s;
        else if (col == D) { if (p.has_bias) Gs[D] = s; }
        else p.C[seg] = s;
      }
    }
    if (threadIdx.x == 0) p.cnt2[seg] = 0u;
  }
}

}  // namespace dalgo

using namespace dalgo;

template <typename T, int NC, bool EVAL>
static hipError_t launch_lr(const LrParams& p, int gx, int nseg, hipStream_t st) {
  constexpr int NW = 8;
  dim3 grid(gx, nseg), block(NW * 64);
  hipLaunchKernelGGL((lr_rows_kernel<T, NC, EVAL, NW>), grid, block, 0, st, p);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

template <bool EVAL>
static hipError_t dispatch_lr(const LrParams& p, int is_bf16, int gx, int nseg, hipStream_t st) {
  const int vec = is_bf16 ? 8 : 4;
  const int64_t nchunks = p.ld / vec;
  const int nc = (int)cdiv(nchunks, 64);
  if (is_bf16) {
    switch (nc) {
      case 1: return launch_lr<uint16_t, 1, EVAL>(p, gx, nseg, st);
      case 2: return launch_lr<uint16_t, 2, EVAL>(p, gx, nseg, st);
      case 3: case 4: return launch_lr<uint16_t, 4, EVAL>(p, gx, nseg, st);
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (nc) {
      case 1: return launch_lr<float, 1, EVAL>(p, gx, nseg, st);
      case 2: return launch_lr<float, 2, EVAL>(p, gx, nseg, st);
      case 3: case 4: return launch_lr<float, 4, EVAL>(p, gx, nseg, st);
      default: return hipErrorInvalidValue;
    }
  }
}

extern "C" {

// Maximum supported row stride: 4 chunks/lane -> 2048 bf16 or 1024 f32 columns.
int dalgo_lr_max_cols(int is_bf16) { return is_bf16 ? 2048 : 1024; }

hipError_t dalgo_lr_grad(const void* X, const float* y, const float* W, const int64_t* seg,
                         int64_t ld, int64_t row_offset, int D, int ldw, int has_bias, float eps,
                         uint64_t seed, uint64_t step, uint32_t thr, int full, int is_bf16,
                         int gx, int nseg, int rows_per_block, float* slab, float* gslab,
                         unsigned* cnt1, unsigned* cnt2, float* G, float* C, int S,
                         hipStream_t st) {
  LrParams p{};
  p.X = X; p.y = y; p.W = W; p.seg = seg; p.ld = ld; p.row_offset = row_offset; p.D = D;
  p.ldw = ldw; p.has_bias = has_bias; p.eps = eps; p.seed = seed; p.step = step; p.thr = thr;
  p.full = full; p.rows_per_block = rows_per_block; p.slab = slab; p.gslab = gslab;
  p.cnt1 = cnt1; p.cnt2 = cnt2; p.G = G; p.C = C; p.S = S;
  return dispatch_lr<false>(p, is_bf16, gx, nseg, st);
}

hipError_t dalgo_lr_eval(const void* X, const float* y, const float* W, const int64_t* seg,
                         int64_t ld, int D, int ldw, int has_bias, float eps, int is_bf16, int gx,
                         int nseg, int rows_per_block, unsigned long long* correct, float* loss,
                         hipStream_t st) {
  LrParams p{};
  p.X = X; p.y = y; p.W = W; p.seg = seg; p.ld = ld; p.row_offset = 0; p.D = D; p.ldw = ldw;
  p.has_bias = has_bias; p.eps = eps; p.full = 1; p.rows_per_block = rows_per_block;
  p.correct = correct; p.loss = loss;
  return dispatch_lr<true>(p, is_bf16, gx, nseg, st);
}

}  // extern "C"
