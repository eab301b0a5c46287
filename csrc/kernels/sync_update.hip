// K8: fused model-update / synchronisation rules of the parallel-SGD family.
//
// The reference runs these as driver-side NumPy after every treeAggregate:
//   SSGD        w -= eta * (g/|B| + lam * reg(w))            optimization/ssgd.py:105, reg ssgd.py:36-47
//   full GD     w -= eta * g           (sum, not mean)      machine_learning/logistic_regression.py:85
//   MA local    w_i -= eta * mean_B(g_i)                     optimization/ma.py:39-43
//   EASGD local x_i -= eta * mean_B(g_i) + alpha (x_i - w~)  optimization/easgd.py:41-45
//   MA sync     w = (1/P) sum_i w_i                          optimization/ma.py:104-106
//   BMUF sync   D = mu D + zeta (w_avg - w); w += D          optimization/bmuf.py:109-114
//   EASGD sync  w~ = (1-beta) w~ + beta (1/P) sum_i x_i       optimization/easgd.py:104-106
// Here each is one launch over the (D+1)-vector (or the [P_local, D+1] block of
// local models) — launch-bound, so everything per step is fused into a single
// grid and every rank applies the identical rule to replicated state (no driver).
#include "dalgo/common.h"
#include <algorithm>

namespace dalgo {

enum UpdateMode : int {
  kSSGD = 0,        // w -= eta*(g/cnt + lam*reg(w))
  kGDSum = 1,       // w -= eta*g
  kLocalMean = 2,   // W[i] -= eta*G[i]/cnt[i]                 (MA / BMUF local step)
  kLocalElastic = 3,// W[i] -= eta*G[i]/cnt[i] + alpha*(W[i]-c)  (EASGD local step)
  kAverage = 4,     // w = S/P                                   (MA sync)
  kBMUF = 5,        // wavg=S/P; Dl = mu*Dl + zeta*(wavg-w); w += Dl
  kElasticCenter = 6// w = (1-beta) w + beta*S/P
};

enum RegType : int { kRegNone = 0, kRegL2 = 1, kRegL1 = 2, kRegElastic = 3 };

struct UpdParams {
  float* W;            // [nrow, ld]  model(s) updated in place
  float* G;            // [nrow, ld]  gradient sums  (local modes / SSGD)
  float* C;            // [nrow]      counts
  const float* center; // [ld]        EASGD centre variable (local elastic)
  const float* S;      // [ld]        all-reduced sum of models (sync modes)
  float* Dl;           // [ld]        BMUF block-momentum buffer
  double* count_acc;   // optional: += sum of C[row] over the rows (throughput accounting
                       //    without a host sync; the local modes add every local model's count)
  int n, ld, nrow;
  int mode, reg;
  float eta, lam, alpha, reg_alpha, mu, zeta, beta, inv_p;
  int zero_grad;       // 1: leave G[row] and C[row] zeroed after use (one block per row):
                       //    the next atomic-epilogue gradient launch accumulates into them
};

__device__ __forceinline__ float reg_grad(float w, int reg, float a) {
  switch (reg) {
    case kRegL2: return w;
    case kRegL1: return (w > 0.f) ? 1.f : (w < 0.f ? -1.f : 0.f);
    case kRegElastic: {
      float s = (w > 0.f) ? 1.f : (w < 0.f ? -1.f : 0.f);
      return a * s + (1.f - a) * w;
    }
    default: return 0.f;
  }
}

__global__ void __launch_bounds__(1024) sync_update_kernel(UpdParams p) {
  const int row = blockIdx.y;
  if (p.count_acc && blockIdx.x == 0 && threadIdx.x == 0) {
    if (p.nrow == 1) p.count_acc[0] += (double)p.C[0];
    else atomicAdd(p.count_acc, (double)p.C[row]);
  }
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < p.n; j += gridDim.x * blockDim.x) {
    const int64_t o = (int64_t)row * p.ld + j;
    float w = p.W[o];
    switch (p.mode) {
      case kSSGD: {
        const float c = p.C[row];
        const float gm = c > 0.f ? p.G[o] / c : 0.f;   // empty minibatch: no gradient step
        w -= p.eta * (gm + p.lam * reg_grad(w, p.reg, p.reg_alpha));
        break;
      }
      case kGDSum: w -= p.eta * p.G[o]; break;
      case kLocalMean: {
        const float c = p.C[row];
        if (c > 0.f) w -= p.eta * (p.G[o] / c);
        break;
      }
      case kLocalElastic: {
        const float c = p.C[row];
        const float gm = c > 0.f ? p.G[o] / c : 0.f;
        w = w - p.eta * gm - p.alpha * (w - p.center[j]);
        break;
      }
      default: break;
      case kAverage: w = p.S[j] * p.inv_p; break;
      case kBMUF: {
        const float wavg = p.S[j] * p.inv_p;
        const float d = p.mu * p.Dl[j] + p.zeta * (wavg - w);
        p.Dl[j] = d;
        w += d;
        break;
      }
      case kElasticCenter: w = (1.f - p.beta) * w + p.beta * (p.S[j] * p.inv_p); break;
    }
    p.W[o] = w;
    if (p.zero_grad) p.G[o] = 0.f;
  }
  if (p.zero_grad) {
    __syncthreads();   // every thread of this row's (single) block has read C[row]
    if (threadIdx.x == 0 && p.C) p.C[row] = 0.f;
  }
}

// Sum the rows of a [nrow, ld] block of local models into out[ld] (fixed order),
// optionally also broadcasting `src` into every row (MA/BMUF "reset locals to w",
// ma.py:96). Used before the cross-rank all-reduce of the local-SGD family.
__global__ void __launch_bounds__(256)
rows_sum_kernel(const float* __restrict__ W, int nrow, int ld, int n, float* __restrict__ out) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int r = 0; r < nrow; ++r) s += W[(int64_t)r * ld + j];
    out[j] = s;
  }
}

__global__ void __launch_bounds__(256)
rows_broadcast_kernel(float* __restrict__ W, int nrow, int ld, int n, const float* __restrict__ src) {
  const int row = blockIdx.y;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    W[(int64_t)row * ld + j] = src[j];
}

}  // namespace dalgo

using namespace dalgo;

extern "C" {

hipError_t dalgo_sync_update(float* W, float* G, float* C, const float* center,
                             const float* S, float* Dl, double* count_acc, int n, int ld, int nrow,
                             int mode, int reg, float eta, float lam, float alpha, float reg_alpha,
                             float mu, float zeta, float beta, float inv_p, int zero_grad,
                             hipStream_t st) {
  zero_grad = (zero_grad && G != nullptr && mode <= kLocalElastic) ? 1 : 0;
  UpdParams p{W, G, C, center, S, Dl, count_acc, n, ld, nrow, mode, reg,
              eta, lam, alpha, reg_alpha, mu, zeta, beta, inv_p, zero_grad};
  // zero_grad needs one block per row (C[row] is cleared after a block barrier):
  // give that block 1024 threads so the ~1k-float vector is one pass
  const int bx = zero_grad ? 1 : (int)std::min<int64_t>(cdiv(n, 256), 64);
  const int nt = zero_grad ? 1024 : 256;
  hipLaunchKernelGGL(sync_update_kernel, dim3(bx, nrow), dim3(nt), 0, st, p);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_rows_sum(const float* W, int nrow, int ld, int n, float* out, hipStream_t st) {
  const int bx = (int)std::min<int64_t>(cdiv(n, 256), 64);
  hipLaunchKernelGGL(rows_sum_kernel, dim3(bx), dim3(256), 0, st, W, nrow, ld, n, out);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_rows_broadcast(float* W, int nrow, int ld, int n, const float* src,
                                hipStream_t st) {
  const int bx = (int)std::min<int64_t>(cdiv(n, 256), 64);
  hipLaunchKernelGGL(rows_broadcast_kernel, dim3(bx, nrow), dim3(256), 0, st, W, nrow, ld, n, src);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
