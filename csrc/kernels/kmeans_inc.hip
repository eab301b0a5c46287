// K3 incremental form: per-cluster sums maintained across Lloyd iterations by
// moving only the points whose assignment changed.
//
// Reference: machine_learning/k-means.py:62-63 recomputes (sum, count) per cluster
// from every point each iteration (reduceByKey). The sums are linear in the
// assignment, so with the previous iteration's local sums S (f64, exact for any
// realistic n) and its assignment a_old,
//     S[c] = S_old[c] + sum_{a_new(x)=c, a_old(x)!=c} x - sum_{a_old(x)=c, a_new(x)!=c} x
// is the same (sum, count) table the full pass would produce (up to f64 rounding
// order). On clustered data the changed share drops below 1 % after the first
// iteration (0.86 % -> 0.06 % on the 1024-blob benchmark data), so the
// 25.6 GB re-read of X in the full K3 pass becomes a pass over the two
// assignment vectors (0.8 GB) plus ~1-2 KB of f64 atomics per moved point.
// The caller falls back to the full pass when the changed share is large (25 %).
//
//   km_diff    : compare a_new / a_old, append the changed row ids through a
//                per-block LDS buffer (one global atomic per block flush)
//   the moved rows then go through the counting-sorted form in kmeans.hip (km_dexpand
//                / km_dsegsum: ~0.1 ms per million signed entries; a per-row f64-atomic
//                form, ~3 ms per million moved rows at 100M points, was removed)
//   km_filter / km_bounds_init / km_centre_bounds: the bound-filtered (Hamerly) iteration
//                (the post-K2 bound update is fused into the K2 epilogue, kmeans.hip).
// Every count (changed rows, active rows) stays on the device: the launches that
// consume it read it there, so an iteration needs no host sync.
#include "dalgo/common.h"

namespace dalgo {
namespace {

constexpr int kDiffThreads = 256;
constexpr int kDiffBuf = 4096;      // changed row ids buffered per block in LDS
constexpr int kEpt = 8;             // rows per thread and step (filter / post)

// one ulp outward after a round-to-nearest result: >= / <= the exact value (the RN error
// is at most half an ulp), so bounds built from them stay valid bounds
__device__ __forceinline__ float up1(float x) { return nextafterf(x, __builtin_inff()); }
__device__ __forceinline__ float dn1(float x) { return nextafterf(x, -__builtin_inff()); }

// One block per contiguous row range. Changed rows are appended to an LDS buffer with
// LDS atomics (one per wave and step) and flushed to the global list with ONE global
// atomic per flush -- a global counter hit by every wave serialises (~88 atomics/us on
// one word: 5 ms for 1.3M changed rows at 100M points, measured).
__global__ void __launch_bounds__(kDiffThreads)
km_diff_kernel(const int32_t* __restrict__ a_new, const int32_t* __restrict__ a_old, int64_t n,
               int32_t* __restrict__ changed, unsigned long long* __restrict__ n_changed,
               int64_t cap) {
  __shared__ int32_t s_buf[kDiffBuf];
  __shared__ int s_cnt;
  __shared__ unsigned long long s_base;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = lo + per < n ? lo + per : n;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  auto flush = [&]() {
    const int m = s_cnt;                       // read after a barrier: stable
    if (m == 0) return;
    if (threadIdx.x == 0) s_base = atomicAdd(n_changed, (unsigned long long)m);
    __syncthreads();
    const int64_t b = (int64_t)s_base;
    for (int j = threadIdx.x; j < m; j += kDiffThreads)
      if (b + j < cap) changed[b + j] = s_buf[j];
    __syncthreads();
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
  };
  for (int64_t base = lo; base < hi; base += kDiffThreads) {
    const int64_t i = base + threadIdx.x;
    const bool ch = i < hi && a_new[i] != a_old[i];
    const uint64_t mask = __ballot(ch);
    if (mask != 0) {
      const int lane = __lane_id();
      const int leader = __ffsll((long long)mask) - 1;
      int b = 0;
      if (lane == leader) b = atomicAdd(&s_cnt, __popcll(mask));
      b = __shfl(b, leader);
      if (ch) {
        const uint64_t below = lane == 0 ? 0ull : (mask & (~0ull >> (64 - lane)));
        s_buf[b + __popcll(below)] = (int32_t)i;
      }
    }
    __syncthreads();
    if (s_cnt > kDiffBuf - kDiffThreads) flush();   // room for one more step
  }
  flush();
}

// ---------------------------------------------------------------------------
// Bound-filtered Lloyd (Hamerly, exact): u[i] >= |x_i - c_a| and l[i] <= min over the
// other centres of |x_i - c| for the centres of the last assignment. The centre of x_i
// moved by delta[a] since and no centre moved more than maxd, so u + delta[a] bounds
// the distance to its centre from above and l - maxd every other distance from below;
// if u + delta[a] < max(s[a], l - maxd) (s[a] = half the distance from c_a to its
// nearest other centre) c_a is still strictly the closest centre (triangle inequality)
// and x_i is skipped (u, l updated); otherwise its row id is appended to the active
// list and its assignment saved in a_prev.
// maxd = max over the k centre shifts, reduced by every block from delta (k floats from
// L2: cheaper than a separate reduction launch).
__global__ void __launch_bounds__(kDiffThreads)
km_filter_kernel(const int32_t* __restrict__ assign, float2* __restrict__ ul,
                 const float* __restrict__ delta, const float* __restrict__ s, int k, int64_t n,
                 int32_t* __restrict__ a_prev, int32_t* __restrict__ idx,
                 unsigned long long* __restrict__ n_active, int64_t cap,
                 int32_t* __restrict__ acl) {
  // acl (optional): cluster of every appended row, in list order (the candidate-pruned
  // K2 sorts the active rows by it)
  __shared__ int32_t s_buf[kDiffBuf];
  __shared__ int32_t s_cl[kDiffBuf];
  __shared__ int s_cnt;
  __shared__ unsigned long long s_base;
  __shared__ float s_md[kDiffThreads / 64];
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = lo + per < n ? lo + per : n;
  float mdl = 0.f;
  for (int c = threadIdx.x; c < k; c += kDiffThreads) mdl = fmaxf(mdl, delta[c]);
  for (int off = 32; off >= 1; off >>= 1) mdl = fmaxf(mdl, __shfl_xor(mdl, off));
  if ((threadIdx.x & 63) == 0) s_md[threadIdx.x >> 6] = mdl;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  float md = s_md[0];
#pragma unroll
  for (int w = 1; w < kDiffThreads / 64; ++w) md = fmaxf(md, s_md[w]);
  auto flush = [&]() {
    const int m = s_cnt;
    if (m == 0) return;
    if (threadIdx.x == 0) s_base = atomicAdd(n_active, (unsigned long long)m);
    __syncthreads();
    const int64_t b = (int64_t)s_base;
    for (int j = threadIdx.x; j < m; j += kDiffThreads)
      if (b + j < cap) {
        idx[b + j] = s_buf[j];
        if (acl) acl[b + j] = s_cl[j];
      }
    __syncthreads();
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
  };
  // kEpt rows per thread per step, all loads issued before the dependent gathers
  // (one row per thread and step left the pass latency bound: 0.59 ms at 100M rows)
  for (int64_t base = lo; base < hi; base += (int64_t)kDiffThreads * kEpt) {
    int a[kEpt];
    float uu[kEpt], ll[kEpt];
#pragma unroll
    for (int e = 0; e < kEpt; ++e) {
      const int64_t i = base + threadIdx.x + (int64_t)kDiffThreads * e;
      const bool in = i < hi;
      a[e] = in ? assign[i] : 0;
      const float2 b = in ? ul[i] : make_float2(0.f, 0.f);
      uu[e] = b.x;
      ll[e] = b.y;
    }
    // bounds rounded outward (u up, l down): a skipped point's bounds stay valid over any
    // number of consecutive skipped iterations, independent of the f32 rounding of u / l
    float ub[kEpt], lb[kEpt], bound[kEpt];
#pragma unroll
    for (int e = 0; e < kEpt; ++e) {
      ub[e] = up1(uu[e] + delta[a[e]]);
      lb[e] = dn1(ll[e] - md);
      bound[e] = fmaxf(s[a[e]], lb[e]);
    }
#pragma unroll
    for (int e = 0; e < kEpt; ++e) {
      const int64_t i = base + threadIdx.x + (int64_t)kDiffThreads * e;
      const bool in = i < hi;
      const bool act = in && !(ub[e] < bound[e]);
      if (in && !act) {
        ul[i] = make_float2(ub[e], lb[e]);
      } else if (act && a_prev) {
        a_prev[i] = a[e];
      }
      const uint64_t mask = __ballot(act);
      if (mask != 0) {
        const int lane = __lane_id();
        const int leader = __ffsll((long long)mask) - 1;
        int b = 0;
        if (lane == leader) b = atomicAdd(&s_cnt, __popcll(mask));
        b = __shfl(b, leader);
        if (act) {
          const uint64_t below = lane == 0 ? 0ull : (mask & (~0ull >> (64 - lane)));
          s_buf[b + __popcll(below)] = (int32_t)i;
          s_cl[b + __popcll(below)] = a[e];
        }
      }
    }
    __syncthreads();
    if (s_cnt > kDiffBuf - kDiffThreads * kEpt) flush();   // room for one more step
  }
  flush();
}

// Q[c] = sum over rows assigned to c of |x|^2 = 2 xh (f64; LDS histogram per block,
// k <= 2048, then one global add per cluster and block)
__global__ void __launch_bounds__(256)
km_qsum_kernel(const int32_t* __restrict__ assign, const float* __restrict__ xh, int64_t n, int k,
               double* __restrict__ Q) {
  __shared__ double s_q[2048];
  for (int c = threadIdx.x; c < k; c += 256) s_q[c] = 0.0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    atomicAdd(&s_q[assign[i]], 2.0 * (double)xh[i]);
  __syncthreads();
  for (int c = threadIdx.x; c < k; c += 256)
    if (s_q[c] != 0.0) atomicAdd(&Q[c], s_q[c]);
}

// Bound-filter geometry of the new centres (f64 on the ROUNDED centres the assign kernel
// uses, one block per centre): delta[c] = |c_now - c_prev| rounded up (relative 1e-6 +
// absolute 1e-6 margin, then f32 round-up), s[c] = half the distance to the nearest
// other centre rounded down (relative 1e-6 margin, f32 round-down); k == 1: s = inf.
// Replaces a torch cdist + norm + min chain (8 launches and a library first use).
template <typename T>
__global__ void __launch_bounds__(256)
km_centre_bounds_kernel(const T* __restrict__ cnow, const T* __restrict__ cprev, int k, int d,
                        int DP, float* __restrict__ delta, float* __restrict__ sout) {
  __shared__ double s_c[128];
  __shared__ double s_red[2][4];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  auto val = [](const T* p) -> double {
    if constexpr (sizeof(T) == 2) return (double)bf16_to_f32(*reinterpret_cast<const uint16_t*>(p));
    else return (double)*p;
  };
  double dd = 0.0;
  for (int j = tid; j < d; j += 256) {
    const double a = val(cnow + (int64_t)c * DP + j);
    s_c[j] = a;
    const double b = a - val(cprev + (int64_t)c * DP + j);
    dd += b * b;
  }
  __syncthreads();
  double best = __builtin_inf();
  for (int o = tid; o < k; o += 256) {
    if (o == c) continue;
    const T* row = cnow + (int64_t)o * DP;
    double acc = 0.0;
    for (int j = 0; j < d; ++j) {
      const double t = s_c[j] - val(row + j);
      acc = fma(t, t, acc);
    }
    best = fmin(best, acc);
  }
  for (int off = 32; off >= 1; off >>= 1) {
    dd += __shfl_xor(dd, off);
    best = fmin(best, __shfl_xor(best, off));
  }
  if (lane == 0) { s_red[0][wid] = dd; s_red[1][wid] = best; }
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, b = __builtin_inf();
    for (int w = 0; w < 4; ++w) { a += s_red[0][w]; b = fmin(b, s_red[1][w]); }
    delta[c] = up1((float)(sqrt(a) * (1.0 + 1e-6) + 1e-6));
    sout[c] = k == 1 ? __builtin_inff() : dn1((float)(0.5 * sqrt(b) * (1.0 - 1e-6)));
  }
}

// Candidate lists of the pruned K2 (one block per centre a, kpad <= 2048, d <= 128, f64 on
// the ROUNDED centres the assign kernel uses): nd[a][j] = the j-th smallest |c - c_a|
// rounded down (relative 1e-6 margin, f32 round-down; +inf for the padding centres),
// nb[a][.] = the same centres with each aligned group of 32 re-ordered by id (a group of
// the list is one 32-centre sub-tile of K2, so any processed prefix of whole sub-tiles is
// the same set as the distance order's), hnb = their 0.5|c|^2. Also delta[a] and s[a] as
// km_centre_bounds_kernel (one launch per iteration instead of two).
__global__ void __launch_bounds__(256)
km_centre_nbrs_kernel(const uint16_t* __restrict__ cq, const uint16_t* __restrict__ cprev,
                      const float* __restrict__ hn, int k, int kpad, int d, int DP,
                      float* __restrict__ delta, float* __restrict__ sout, float* __restrict__ nd,
                      int32_t* __restrict__ nb, float* __restrict__ hnb, float* __restrict__ ndb) {
  __shared__ double s_c[128];
  __shared__ float s_d[2048];
  __shared__ int32_t s_i[2048];
  __shared__ int32_t s_g[2048];
  __shared__ float s_gd[2048];
  __shared__ double s_red[2][4];
  const int a = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double dd = 0.0;
  for (int j = tid; j < d; j += 256) {
    const double v = (double)bf16_to_f32(cq[(int64_t)a * DP + j]);
    s_c[j] = v;
    const double b = v - (double)bf16_to_f32(cprev[(int64_t)a * DP + j]);
    dd += b * b;
  }
  __syncthreads();
  int P = 32;
  while (P < kpad) P <<= 1;
  double best = __builtin_inf();
  for (int o = tid; o < P; o += 256) {
    float dv = __builtin_inff();
    if (o < k) {
      const uint16_t* row = cq + (int64_t)o * DP;
      double acc = 0.0;
      for (int j = 0; j < d; ++j) {
        const double t = s_c[j] - (double)bf16_to_f32(row[j]);
        acc = fma(t, t, acc);
      }
      if (o != a) best = fmin(best, acc);
      dv = o == a ? 0.f : dn1((float)(sqrt(acc) * (1.0 - 1e-6)));
    }
    s_d[o] = dv;
    s_i[o] = o;
  }
  for (int off = 32; off >= 1; off >>= 1) {
    dd += __shfl_xor(dd, off);
    best = fmin(best, __shfl_xor(best, off));
  }
  if (lane == 0) { s_red[0][wid] = dd; s_red[1][wid] = best; }
  __syncthreads();
  if (tid == 0) {
    double x = 0.0, y = __builtin_inf();
    for (int w = 0; w < 4; ++w) { x += s_red[0][w]; y = fmin(y, s_red[1][w]); }
    delta[a] = up1((float)(sqrt(x) * (1.0 + 1e-6) + 1e-6));
    sout[a] = k == 1 ? __builtin_inff() : dn1((float)(0.5 * sqrt(y) * (1.0 - 1e-6)));
  }
  // bitonic sort of (distance, id) ascending (ties by id: deterministic)
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = tid; i < P / 2; i += 256) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const float d0 = s_d[lo], d1 = s_d[hi];
        const int i0 = s_i[lo], i1 = s_i[hi];
        const bool gt = d0 > d1 || (d0 == d1 && i0 > i1);
        if (gt == up) { s_d[lo] = d1; s_d[hi] = d0; s_i[lo] = i1; s_i[hi] = i0; }
      }
    }
  }
  __syncthreads();
  // regroup: position of entry j inside its aligned group of 32 = its id rank there
  const int64_t base = (int64_t)a * kpad;
  for (int j = tid; j < kpad; j += 256) {
    const int g0 = j & ~31, id = s_i[j];
    int rank = 0;
    for (int q = 0; q < 32; ++q) rank += s_i[g0 + q] < id ? 1 : 0;
    s_g[g0 + rank] = id;
    s_gd[g0 + rank] = s_d[j];
    nd[base + j] = s_d[j];
  }
  __syncthreads();
  for (int j = tid; j < kpad; j += 256) {
    nb[base + j] = s_g[j];
    hnb[base + j] = hn[s_g[j]];
    if (ndb) ndb[base + j] = s_gd[j];
  }
}

// drift-aware lists: dnb[a][j] = delta[nb[a][j]] (every centre's shift, after the launch
// that computes them; padding entries: 0)
__global__ void __launch_bounds__(256)
km_nbr_drift_kernel(const int32_t* __restrict__ nb, const float* __restrict__ delta, int k, int64_t total,
                    float* __restrict__ dnb) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = nb[i];
    dnb[i] = c < k ? delta[c] : 0.f;
  }
}

// Bounds after the full first pass: tol = 2 M 2^-14 with M = max 0.5|x|^2 * 1.0001 + 1e-6
// (slack of a truncated kernel distance; xmax = the float bits K2 max-reduced),
// u = sqrt(dist + tol) rounded up, l = sqrt(dist2 - tol) rounded down. One pass.
__global__ void __launch_bounds__(256)
km_bounds_init_kernel(const float* __restrict__ mind, const float* __restrict__ mind2,
                      const unsigned* __restrict__ xmax, int64_t n, float2* __restrict__ ul,
                      float* __restrict__ tol_out) {
  const float M = __uint_as_float(*xmax) * 1.0001f + 1e-6f;
  const float tol = up1(2.f * M * 6.103515625e-05f);   // 2^-14
  if (blockIdx.x == 0 && threadIdx.x == 0) *tol_out = tol;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    ul[i] = make_float2(up1(sqrtf(up1(fmaxf(mind[i], 0.f) + tol))),
                        fmaxf(dn1(sqrtf(fmaxf(dn1(mind2[i] - tol), 0.f))), 0.f));
  }
}

}  // namespace
}  // namespace dalgo

extern "C" {

hipError_t dalgo_km_diff(const int32_t* a_new, const int32_t* a_old, int64_t n, int32_t* changed,
                         unsigned long long* n_changed, int64_t cap, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t g = (n + dalgo::kDiffThreads - 1) / dalgo::kDiffThreads;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(dalgo::km_diff_kernel, dim3((unsigned)g), dim3(dalgo::kDiffThreads), 0, st,
                     a_new, a_old, n, changed, n_changed, cap);
  return hipGetLastError();
}

hipError_t dalgo_km_filter(const int32_t* assign, float* ul, const float* delta,
                           const float* s, int k, int64_t n, int32_t* a_prev, int32_t* idx,
                           unsigned long long* n_active, int64_t cap, int32_t* acl,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t g = (n + dalgo::kDiffThreads - 1) / dalgo::kDiffThreads;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(dalgo::km_filter_kernel, dim3((unsigned)g), dim3(dalgo::kDiffThreads), 0, st,
                     assign, reinterpret_cast<float2*>(ul), delta, s, k, n, a_prev, idx, n_active, cap, acl);
  return hipGetLastError();
}

hipError_t dalgo_km_bounds_init(const float* mind, const float* mind2, const unsigned* xmax,
                                int64_t n, float* ul, float* tol, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(dalgo::km_bounds_init_kernel, dim3((unsigned)g), dim3(256), 0, st, mind, mind2,
                     xmax, n, reinterpret_cast<float2*>(ul), tol);
  return hipGetLastError();
}

hipError_t dalgo_km_centre_bounds(const void* cnow, const void* cprev, int is_bf16, int k, int d,
                                  int DP, float* delta, float* s, hipStream_t st) {
  if (k <= 0) return hipSuccess;
  if (d > 128 || d > DP) return hipErrorInvalidValue;
  if (is_bf16)
    hipLaunchKernelGGL(dalgo::km_centre_bounds_kernel<uint16_t>, dim3(k), dim3(256), 0, st,
                       (const uint16_t*)cnow, (const uint16_t*)cprev, k, d, DP, delta, s);
  else
    hipLaunchKernelGGL(dalgo::km_centre_bounds_kernel<float>, dim3(k), dim3(256), 0, st,
                       (const float*)cnow, (const float*)cprev, k, d, DP, delta, s);
  return hipGetLastError();
}

hipError_t dalgo_km_centre_nbrs(const void* cq, const void* cprev, const float* hn, int k, int kpad,
                                int d, int DP, float* delta, float* s, float* nd, int32_t* nb,
                                float* hnb, float* ndb, float* dnb, hipStream_t st) {
  if (k <= 0) return hipSuccess;
  if (d > 128 || d > DP || kpad > 2048 || kpad < k || kpad % 32 != 0 || DP % 8 != 0)
    return hipErrorInvalidValue;
  if ((ndb == nullptr) != (dnb == nullptr)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dalgo::km_centre_nbrs_kernel, dim3(k), dim3(256), 0, st,
                     (const uint16_t*)cq, (const uint16_t*)cprev, hn, k, kpad, d, DP, delta, s, nd,
                     nb, hnb, ndb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || dnb == nullptr) return e;
  const int64_t total = (int64_t)k * kpad;
  hipLaunchKernelGGL(dalgo::km_nbr_drift_kernel, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 4096)),
                     dim3(256), 0, st, nb, delta, k, total, dnb);
  return hipGetLastError();
}

hipError_t dalgo_km_qsum(const int32_t* assign, const float* xh, int64_t n, int k, double* Q,
                         hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (k > 2048) return hipErrorInvalidValue;
  int64_t g = (n + 255) / 256;
  if (g > 512) g = 512;
  hipLaunchKernelGGL(dalgo::km_qsum_kernel, dim3((unsigned)g), dim3(256), 0, st, assign, xh, n, k, Q);
  return hipGetLastError();
}

}  // extern "C"
