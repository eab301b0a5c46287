// extern "C" entry points of the gfx950 kernels (csrc/kernels/*.hip).
// Host-only header: the torch binding layer (bindings.cpp) and the native
// C++ tests include it; no torch or device code here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

// ---- K1/K7/K10 logistic regression (lr_grad.hip)
int dalgo_lr_max_cols(int is_bf16);
hipError_t dalgo_lr_grad(const void* X, const float* y, const float* W, const int64_t* seg,
                         int64_t ld, int64_t row_offset, int D, int ldw, int has_bias, float eps,
                         uint64_t seed, uint64_t step, uint32_t thr, int full, int is_bf16,
                         int gx, int nseg, int rows_per_block, float* slab, float* gslab,
                         unsigned* cnt1, unsigned* cnt2, float* G, float* C, int S, int variant,
                         hipStream_t st);
hipError_t dalgo_lr_eval(const void* X, const float* y, const float* W, const int64_t* seg,
                         int64_t ld, int D, int ldw, int has_bias, float eps, int is_bf16, int gx,
                         int nseg, int rows_per_block, unsigned long long* correct, float* loss,
                         int variant, hipStream_t st);

// ---- K8 sync/update rules (sync_update.hip)
hipError_t dalgo_sync_update(float* W, const float* G, const float* C, const float* center,
                             const float* S, float* Dl, double* count_acc, int n, int ld, int nrow,
                             int mode, int reg, float eta, float lam, float alpha, float reg_alpha,
                             float mu, float zeta, float beta, float inv_p, hipStream_t st);
hipError_t dalgo_rows_sum(const float* W, int nrow, int ld, int n, float* out, hipStream_t st);
hipError_t dalgo_rows_broadcast(float* W, int nrow, int ld, int n, const float* src,
                                hipStream_t st);

// ---- random generation + K6 Monte-Carlo pi (random.hip)
hipError_t dalgo_philox_fill(void* out, int is_bf16, int64_t nrows, int64_t D, int64_t ld,
                             int64_t row_offset, uint64_t seed, uint64_t stream, int dist, float a,
                             float b, hipStream_t st);
hipError_t dalgo_hbm_read(const void* p, int64_t nbytes, uint32_t* out, int grid, int unroll,
                          hipStream_t st);
hipError_t dalgo_mc_pi(uint64_t seed, uint64_t stream, uint64_t offset, uint64_t n,
                       unsigned long long* count, hipStream_t st);

}  // extern "C"
