// K5 (ALS solve): ridge-regularised SPD inverse of the k x k Gram matrix.
//
// Reference matrix_computation/matrix_decomposition.py:24-33 — `update` rebuilds
// XtX = mat^T mat (+ lam * X_dim on the diagonal) and calls np.linalg.solve for
// EVERY row of U (and of V): m (n) identical Gram builds + LU factorisations per
// half-sweep. Here the Gram is built once per half-sweep (one GEMM), inverted
// once by this kernel, and all rows are solved together as one GEMM:
//     U_rows = (R_rows . V) . (V^T V + lam*X_dim*I)^-1
// The inversion runs in f64 in LDS (in-place Gauss-Jordan, no pivoting — the
// matrix is symmetric positive definite thanks to the ridge), one workgroup,
// k <= 128; the f32 result feeds the MFMA GEMMs.
#include "dalgo/common.h"

namespace dalgo {

__global__ void __launch_bounds__(1024)
spd_inverse_kernel(const float* __restrict__ G, int k, int ldg, float ridge, float* __restrict__ out,
                   int ldo, int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double a[];   // k * k
  __shared__ double s_pivot;
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int e = tid; e < k * k; e += nt) {
    const int i = e / k, j = e % k;
    double v = (double)G[(int64_t)i * ldg + j];
    if (i == j) v += (double)ridge;
    a[e] = v;
  }
  __syncthreads();
  int bad = 0;
  for (int p = 0; p < k; ++p) {
    if (tid == 0) s_pivot = a[p * k + p];
    __syncthreads();
    const double piv = s_pivot;
    if (!(piv > 0.0)) bad = 1;   // not SPD (never with a positive ridge)
    const double inv = 1.0 / piv;
    // scale pivot row (column p becomes 1/piv)
    for (int j = tid; j < k; j += nt) a[p * k + j] = (j == p) ? inv : a[p * k + j] * inv;
    __syncthreads();
    // eliminate column p from every other row
    for (int e = tid; e < k * k; e += nt) {
      const int i = e / k, j = e % k;
      if (i == p) continue;
      const double f = a[i * k + p];
      if (j == p) continue;
      a[e] -= f * a[p * k + j];
    }
    __syncthreads();
    for (int i = tid; i < k; i += nt)
      if (i != p) a[i * k + p] = -a[i * k + p] * inv;
    __syncthreads();
  }
  for (int e = tid; e < k * k; e += nt) out[(int64_t)(e / k) * ldo + (e % k)] = (float)a[e];
  if (status && tid == 0) status[0] = bad;
}

}  // namespace dalgo

using namespace dalgo;

extern "C" {

hipError_t dalgo_spd_inverse(const float* G, int k, int ldg, float ridge, float* out, int ldo,
                             int* status, hipStream_t st) {
  if (k < 1 || k > 128) return hipErrorInvalidValue;
  const size_t lds = (size_t)k * k * sizeof(double);
  const int threads = k * k >= 1024 ? 1024 : ((k * k + 63) / 64) * 64;
  hipLaunchKernelGGL(spd_inverse_kernel, dim3(1), dim3(threads), lds, st, G, k, ldg, ridge, out, ldo,
                     status);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
