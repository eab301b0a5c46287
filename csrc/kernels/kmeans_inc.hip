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
//   km_move    : one wave per changed row: the row's DP features (bf16 / f32, one
//                256-B or 512-B coalesced read) are added to S[a_new] and
//                subtracted from S[a_old] with f64 atomics shaped as contiguous
//                512-B wave instructions; lane 0 moves the counts. Used below 16k
//                moved rows: at 100M points its 2 * DP device-scope f64 atomics per
//                row cost ~3 ms per million moved rows, so larger moves go through
//                the counting-sorted form in kmeans.hip (km_dexpand / km_dsegsum:
//                ~0.1 ms per million signed entries).
#include "dalgo/common.h"

namespace dalgo {
namespace {

constexpr int kDiffThreads = 256;
constexpr int kDiffBuf = 4096;      // changed row ids buffered per block in LDS
constexpr int kEpt = 8;             // rows per thread and step (filter / post)

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

template <typename T, int DP>
__global__ void __launch_bounds__(256)
km_move_kernel(const T* __restrict__ X, int64_t ldx, const int32_t* __restrict__ changed,
               int64_t m, const int32_t* __restrict__ a_new, const int32_t* __restrict__ a_old,
               double* __restrict__ S, unsigned long long* __restrict__ cnt,
               const float* __restrict__ xh, double* __restrict__ Q) {
  constexpr int PER = (DP + 63) / 64;     // features per lane
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = wave; w < m; w += nwaves) {
    const int64_t row = changed[w];
    const int cn = a_new[row], co = a_old[row];
    const T* xr = X + row * ldx;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int j = q * 64 + lane;        // one wave instruction = 64 consecutive f64
      if (j < DP) {
        float v;
        if constexpr (sizeof(T) == 2) v = bf16_to_f32(reinterpret_cast<const uint16_t*>(xr)[j]);
        else v = reinterpret_cast<const float*>(xr)[j];
        if (v != 0.f) {
          atomicAdd(&S[(int64_t)cn * DP + j], (double)v);
          atomicAdd(&S[(int64_t)co * DP + j], -(double)v);
        }
      }
    }
    if (lane == 0) {
      atomicAdd(&cnt[cn], 1ull);
      atomicAdd(&cnt[co], ~0ull);   // -1 (two's complement)
      if (Q != nullptr) {           // per-cluster sum of |x|^2 (SSE identity)
        const double q = 2.0 * (double)xh[row];
        atomicAdd(&Q[cn], q);
        atomicAdd(&Q[co], -q);
      }
    }
  }
}

template <typename T, int DP>
hipError_t launch_move(const void* X, int64_t ldx, const int32_t* changed, int64_t m,
                       const int32_t* a_new, const int32_t* a_old, double* S,
                       unsigned long long* cnt, const float* xh, double* Q, hipStream_t st) {
  int64_t g = (m + 3) / 4;                 // 4 waves per 256-thread block
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL((km_move_kernel<T, DP>), dim3((unsigned)g), dim3(256), 0, st,
                     reinterpret_cast<const T*>(X), ldx, changed, m, a_new, a_old, S, cnt, xh, Q);
  return hipGetLastError();
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
__global__ void __launch_bounds__(kDiffThreads)
km_filter_kernel(const int32_t* __restrict__ assign, float* __restrict__ u, float* __restrict__ l,
                 const float* __restrict__ delta, const float* __restrict__ s,
                 const float* __restrict__ maxd, int64_t n,
                 int32_t* __restrict__ a_prev, int32_t* __restrict__ idx,
                 unsigned long long* __restrict__ n_active, int64_t cap) {
  __shared__ int32_t s_buf[kDiffBuf];
  __shared__ int s_cnt;
  __shared__ unsigned long long s_base;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = lo + per < n ? lo + per : n;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const float md = maxd[0];
  auto flush = [&]() {
    const int m = s_cnt;
    if (m == 0) return;
    if (threadIdx.x == 0) s_base = atomicAdd(n_active, (unsigned long long)m);
    __syncthreads();
    const int64_t b = (int64_t)s_base;
    for (int j = threadIdx.x; j < m; j += kDiffThreads)
      if (b + j < cap) idx[b + j] = s_buf[j];
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
      uu[e] = in ? u[i] : 0.f;
      ll[e] = in ? l[i] : 0.f;
    }
    float ub[kEpt], bound[kEpt];
#pragma unroll
    for (int e = 0; e < kEpt; ++e) {
      ub[e] = uu[e] + delta[a[e]];
      bound[e] = fmaxf(s[a[e]], ll[e] - md);
    }
#pragma unroll
    for (int e = 0; e < kEpt; ++e) {
      const int64_t i = base + threadIdx.x + (int64_t)kDiffThreads * e;
      const bool in = i < hi;
      const bool act = in && !(ub[e] < bound[e]);
      if (in && !act) {
        u[i] = ub[e];
        l[i] = ll[e] - md;
      } else if (act) {
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
        }
      }
    }
    __syncthreads();
    if (s_cnt > kDiffBuf - kDiffThreads * kEpt) flush();   // room for one more step
  }
  flush();
}

// After K2 re-assigned the active rows: u = sqrt(dist + tol) (an upper bound of the
// distance to the assigned centre, tol covering the kernel's key truncation) and the
// rows whose cluster changed appended to `changed` (LDS-buffered, as km_diff).
__global__ void __launch_bounds__(kDiffThreads)
km_post_kernel(const int32_t* __restrict__ idx, int64_t m, const int32_t* __restrict__ assign,
               const int32_t* __restrict__ a_prev, const float* __restrict__ mind,
               const float* __restrict__ mind2, float tol, float* __restrict__ u,
               float* __restrict__ l, int32_t* __restrict__ changed,
               unsigned long long* __restrict__ n_changed, int64_t cap) {
  __shared__ int32_t s_buf[kDiffBuf];
  __shared__ int s_cnt;
  __shared__ unsigned long long s_base;
  const int64_t per = (m + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = lo + per < m ? lo + per : m;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  auto flush = [&]() {
    const int c = s_cnt;
    if (c == 0) return;
    if (threadIdx.x == 0) s_base = atomicAdd(n_changed, (unsigned long long)c);
    __syncthreads();
    const int64_t b = (int64_t)s_base;
    for (int j = threadIdx.x; j < c; j += kDiffThreads)
      if (b + j < cap) changed[b + j] = s_buf[j];
    __syncthreads();
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
  };
  for (int64_t base = lo; base < hi; base += (int64_t)kDiffThreads * kEpt) {
    int32_t row[kEpt];
#pragma unroll
    for (int e = 0; e < kEpt; ++e) {
      const int64_t j = base + threadIdx.x + (int64_t)kDiffThreads * e;
      row[e] = j < hi ? idx[j] : -1;
    }
    float d1[kEpt], d2[kEpt];
    int an[kEpt], ap[kEpt];
#pragma unroll
    for (int e = 0; e < kEpt; ++e) {
      const int r = max(row[e], 0);
      d1[e] = mind[r];
      d2[e] = mind2[r];
      an[e] = assign[r];
      ap[e] = a_prev[r];
    }
#pragma unroll
    for (int e = 0; e < kEpt; ++e) {
      bool ch = false;
      if (row[e] >= 0) {
        u[row[e]] = sqrtf(fmaxf(d1[e], 0.f) + tol);
        l[row[e]] = sqrtf(fmaxf(d2[e] - tol, 0.f));
        ch = an[e] != ap[e];
      }
      const uint64_t mask = __ballot(ch);
      if (mask != 0) {
        const int lane = __lane_id();
        const int leader = __ffsll((long long)mask) - 1;
        int b = 0;
        if (lane == leader) b = atomicAdd(&s_cnt, __popcll(mask));
        b = __shfl(b, leader);
        if (ch) {
          const uint64_t below = lane == 0 ? 0ull : (mask & (~0ull >> (64 - lane)));
          s_buf[b + __popcll(below)] = row[e];
        }
      }
    }
    __syncthreads();
    if (s_cnt > kDiffBuf - kDiffThreads * kEpt) flush();
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

hipError_t dalgo_km_move(const void* X, int is_bf16, int64_t ldx, int DP, const int32_t* changed,
                         int64_t m, const int32_t* a_new, const int32_t* a_old, double* S,
                         unsigned long long* cnt, const float* xh, double* Q, hipStream_t st) {
  if (m <= 0) return hipSuccess;
  using namespace dalgo;
#define DALGO_KM_MOVE(DPV)                                                                   \
  if (DP == DPV)                                                                             \
    return is_bf16 ? launch_move<uint16_t, DPV>(X, ldx, changed, m, a_new, a_old, S, cnt, xh, Q, st) \
                   : launch_move<float, DPV>(X, ldx, changed, m, a_new, a_old, S, cnt, xh, Q, st);
  DALGO_KM_MOVE(16)
  DALGO_KM_MOVE(32)
  DALGO_KM_MOVE(64)
  DALGO_KM_MOVE(128)
#undef DALGO_KM_MOVE
  return hipErrorInvalidValue;
}

hipError_t dalgo_km_filter(const int32_t* assign, float* u, float* l, const float* delta,
                           const float* s, const float* maxd, int64_t n, int32_t* a_prev,
                           int32_t* idx, unsigned long long* n_active, int64_t cap, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t g = (n + dalgo::kDiffThreads - 1) / dalgo::kDiffThreads;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(dalgo::km_filter_kernel, dim3((unsigned)g), dim3(dalgo::kDiffThreads), 0, st,
                     assign, u, l, delta, s, maxd, n, a_prev, idx, n_active, cap);
  return hipGetLastError();
}

hipError_t dalgo_km_post(const int32_t* idx, int64_t m, const int32_t* assign, const int32_t* a_prev,
                         const float* mind, const float* mind2, float tol, float* u, float* l,
                         int32_t* changed, unsigned long long* n_changed, int64_t cap,
                         hipStream_t st) {
  if (m <= 0) return hipSuccess;
  int64_t g = (m + dalgo::kDiffThreads - 1) / dalgo::kDiffThreads;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(dalgo::km_post_kernel, dim3((unsigned)g), dim3(dalgo::kDiffThreads), 0, st,
                     idx, m, assign, a_prev, mind, mind2, tol, u, l, changed, n_changed, cap);
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
