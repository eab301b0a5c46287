// K5 (ALS row solve): U_rows = (R_rows . F) . (F^T F + lam*X_dim*I)^-1
//
// Reference matrix_computation/matrix_decomposition.py:24-33 — `update` rebuilds
// XtX = mat^T mat (+ lam * X_dim on the diagonal) and calls np.linalg.solve for
// EVERY row of U (and of V): m (n) identical Gram builds + LU factorisations per
// half-sweep, called per row at :52-54 / :60-62. Here one half-sweep is
//   1. G = F^T F once (tiny GEMM, torch), inverted once by spd_inverse_kernel
//      (f64 Gauss-Jordan in LDS, one workgroup, k <= 128);
//   2. als_pack_f16_kernel: F (n x k f32) -> MFMA A-fragments of F^T, split into a bf16
//      hi part and a bf16 residual (lo) part, laid out so that each wave's fragment
//      load is 1 KB contiguous;
//   3. als_rf16_kernel: B = R_rows . F for all local rows at once on the bf16 MFMA
//      (v_mfma_f32_16x16x32_bf16, R rows as the B operand) with a 3-product split
//          R.F ~= Rhi.Fhi + Rhi.Flo + Rlo.Fhi        (dropped Rlo.Flo: 2^-16 relative)
//      R is f32 and streamed from HBM exactly once (split into hi/lo in registers with
//      v_cvt_pk_bf16_f32); the GEMM is HBM-bound (k <= 128 outputs per R element), so
//      the 3x MFMA work is free while giving ~f32 accuracy (the f32-input MFMA would
//      run at 1/16 of the bf16 rate and be compute-bound). The K (= n) dimension is
//      split over blocks (split-major, XCD-grouped block order, so the blocks sharing an
//      L2 share F ranges); partials go to a workspace. The 32x32x16 form
//      (als_pack_f_kernel + als_rf_kernel) is kept as a variant: its B-operand loads
//      cover 32 rows x 2 x 16 B per instruction and stream R ~10 % slower;
//   4. als_reduce_solve_kernel: sums the K-split partials of each row (fixed order:
//      deterministic) and multiplies by G^-1 in the epilogue.
// 100k x 50k x 64 (bench/als_bench.py, 1 x MI355X): 3.90 ms = 5.13 TB/s of R, against
// 5.64 ms for torch.matmul(torch.matmul(R, F), Ginv) (hipBLASLt).
#include "dalgo/common.h"
#include <algorithm>

namespace dalgo {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

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

// ---------------------------------------------------------------------------
// f32 pair -> packed bf16 (round to nearest even; the compiler emits v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const bf16x2 v = __builtin_convertvector((f32x2){a, b}, bf16x2);
  return __builtin_bit_cast(uint32_t, v);
}
// hi = bf16(v), lo = bf16(v - hi) for 2 consecutive elements
__device__ __forceinline__ void split_pair(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pk_bf16(a, b);
  lo = pk_bf16(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u));
}
__device__ __forceinline__ void split8(const float4& p, const float4& q, uint4& hi, uint4& lo) {
  split_pair(p.x, p.y, hi.x, lo.x);
  split_pair(p.z, p.w, hi.y, lo.y);
  split_pair(q.x, q.y, hi.z, lo.z);
  split_pair(q.z, q.w, hi.w, lo.w);
}

// Fq[((ks * NC + c) * 2 + p) * 64 + lane] = 8 bf16: element j = part p of
// F[W S + 8 SS h + 8 s' + j][32 c + r]   with ks = S SS + s' (super-step S of W = 16 SS
// columns, sub-step s'), r = lane & 31, h = lane >> 5; zero outside n x k.
// This is the A-operand fragment of the F^T tile (rows = factor columns) in the K order
// the R loads use (see als_rf_kernel): the contraction is over a permuted K, the same
// permutation on both operands.
__global__ void __launch_bounds__(256)
als_pack_f_kernel(const float* __restrict__ F, int64_t n, int k, int64_t ldf, int NC, int SS,
                  uint4* __restrict__ Fq, int64_t nks) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // (ks, c, lane)
  const int64_t total = nks * NC * 64;
  if (gid >= total) return;
  const int lane = (int)(gid & 63), r = lane & 31, h = lane >> 5;
  const int64_t t = gid >> 6;
  const int c = (int)(t % NC);
  const int64_t ks = t / NC;
  const int64_t S = ks / SS, sub = ks % SS;
  const int64_t kb = S * 16 * SS + 8 * SS * h + 8 * sub;
  const int col = 32 * c + r;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t K = kb + j;
    v[j] = (K < n && col < k) ? F[K * ldf + col] : 0.f;
  }
  uint4 hi, lo;
  split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), hi, lo);
  Fq[(t * 2 + 0) * 64 + lane] = hi;
  Fq[(t * 2 + 1) * 64 + lane] = lo;
}

// R loads keep the default cache policy: a K-step uses only part of each row's 128-B
// line and the next K-step the rest, and with `nt` loads the line is gone by then
// (bench/probes/row_tile_probe.hip: this access shape 2.85 TB/s with nt, 4.98 without)
__device__ __forceinline__ float4 ld_f4(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}

// B = R . F partials. Block = NW waves x RT row tiles of 32 rows; lane (r, h) of row
// tile t owns R row row0 + 32 t + r. K runs in super-steps of W = 16 SS columns: in
// super-step S the lane loads the 8 SS contiguous floats [W S + 8 SS h, +8 SS) of its
// row (2 SS dwordx4), so each row is visited W * 4 bytes at a time (a 64-B visit per
// row, SS = 1, leaves HBM at ~2.6 TB/s: the 100k rows of a sweep are 200 KB apart);
// sub-step s' feeds elements [8 s', +8) as the B-operand fragment of R^T for K-step
// S SS + s' (the F fragments are packed in the same K order). MFMA: D[factor col][R row]
// += F^T . R^T, lane (r, h) ends with R row r, factor columns (i&3) + 8(i>>2) + 4h.
// Register double buffer: the F and R loads of super-step S+1 are issued (F first)
// before the MFMAs of S, so in-order vmcnt waits never drain them.
template <int RT, int NC, int SS, int NW, int MINB>
__global__ void __launch_bounds__(NW * 64, MINB)
als_rf_kernel(const float* __restrict__ R, int64_t m, int64_t n, int64_t ldr,
              const uint4* __restrict__ Fq, int nrb, int nsplit, int ss_per_split,
              float* __restrict__ P, int kpad) {
  constexpr int ROWS = NW * RT * 32;
  constexpr int W = 16 * SS;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  // split-major logical order, consecutive logical blocks on one XCD (shared F range in L2)
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int sp = L / nrb, rb = L % nrb;
  const int64_t nss_full = n / W;                      // super-steps entirely inside n
  const int64_t nss = (n + W - 1) / W;
  const int64_t S0 = (int64_t)sp * ss_per_split;
  const int64_t S1 = std::min<int64_t>(nss, S0 + ss_per_split);
  const int64_t row0 = (int64_t)rb * ROWS + (int64_t)wid * (RT * 32);

  const float* rp[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int64_t row = row0 + 32 * t + r;
    rp[t] = R + (row < m ? row : 0) * ldr + 8 * SS * h;   // rows past m read row 0, never stored
  }
  f32x16 acc[RT][NC];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][c][i] = 0.f;

  auto load_f = [&](uint4 (&fv)[SS][NC][2], int64_t S) {
    const uint4* fp = Fq + (S * SS * NC * 2) * 64 + lane;
#pragma unroll
    for (int u = 0; u < SS; ++u)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        fv[u][c][0] = fp[((u * NC + c) * 2) * 64];
        fv[u][c][1] = fp[((u * NC + c) * 2 + 1) * 64];
      }
  };
  auto load = [&](float4 (&rv)[RT][2 * SS], uint4 (&fv)[SS][NC][2], int64_t S) {
    load_f(fv, S);
    const int64_t c0 = S * W;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int q = 0; q < 2 * SS; ++q) rv[t][q] = ld_f4(rp[t] + c0 + 4 * q);
  };
  auto compute = [&](const float4 (&rv)[RT][2 * SS], const uint4 (&fv)[SS][NC][2]) {
#pragma unroll
    for (int u = 0; u < SS; ++u)
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        uint4 rh, rl;
        split8(rv[t][2 * u], rv[t][2 * u + 1], rh, rl);
        const bf16x8 bh = __builtin_bit_cast(bf16x8, rh), bl = __builtin_bit_cast(bf16x8, rl);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const bf16x8 fh = __builtin_bit_cast(bf16x8, fv[u][c][0]);
          const bf16x8 fl = __builtin_bit_cast(bf16x8, fv[u][c][1]);
          acc[t][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fh, bh, acc[t][c], 0, 0, 0);
          acc[t][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fl, bh, acc[t][c], 0, 0, 0);
          acc[t][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fh, bl, acc[t][c], 0, 0, 0);
        }
      }
  };

  float4 ra[RT][2 * SS], rb2[RT][2 * SS];
  uint4 fa[SS][NC][2], fb[SS][NC][2];
  const int64_t send = std::min<int64_t>(S1, nss_full);
  int64_t S = S0;
  // sched_barrier: keep each prefetch issued BEFORE the MFMAs of the current super-step
  // (hipcc otherwise sinks the loads to the end of the compute block, which leaves no
  // overlap: measured 2.3 TB/s)
  if (S < send) load(ra, fa, S);
  for (; S + 1 < send; S += 2) {
    load(rb2, fb, S + 1);
    __builtin_amdgcn_sched_barrier(0);
    compute(ra, fa);
    __builtin_amdgcn_sched_barrier(0);
    if (S + 2 < send) load(ra, fa, S + 2);
    __builtin_amdgcn_sched_barrier(0);
    compute(rb2, fb);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (S < send) { compute(ra, fa); ++S; }
  if (S < S1) {
    // tail super-step (n % W != 0): element-wise guarded loads, zeros past n
    const int64_t c0 = S * W;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int q = 0; q < 2 * SS; ++q) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] = (c0 + 8 * SS * h + 4 * q + e < n) ? rp[t][c0 + 4 * q + e] : 0.f;
        ra[t][q] = make_float4(v[0], v[1], v[2], v[3]);
      }
    load_f(fa, S);
    compute(ra, fa);
  }

  // partial P[sp][row][kpad]: registers 4g..4g+3 = factor columns 32c + 8g + 4h + 0..3
  float* Ps = P + (int64_t)sp * m * kpad;
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int64_t row = row0 + 32 * t + r;
    if (row >= m) continue;
    float* dst = Ps + row * kpad + 4 * h;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(dst + 32 * c + 8 * g) =
            make_float4(acc[t][c][4 * g], acc[t][c][4 * g + 1], acc[t][c][4 * g + 2],
                        acc[t][c][4 * g + 3]);
  }
}

// ---- 16x16x32 form: R rows as the B operand of v_mfma_f32_16x16x32_bf16 (lane l holds
// B[k = 8 (l>>4) + j][col l&15] = R[row l&15][.]), so ONE wave-instruction reads 16 rows x
// 64 contiguous bytes (4 lanes per row) instead of 32 rows x 2 x 16 B: measured 5.9-6.0 TB/s
// for this shape against 4.9-5.4 for the 32x32x16 B-operand shape (row_tile_probe.hip).
// K order (same permutation on both operands): in super-step S (32 SS columns), K-step
// u, lane group g = l >> 4, element j <-> physical column
//     32 SS S + 16 (2u + (j >> 2)) + 4 g + (j & 3)
// i.e. load instruction q = 2u + (j >> 2) covers columns [16 q, 16 q + 16) of every row.
__device__ __forceinline__ int64_t als16_col(int64_t S, int SS, int u, int g, int j) {
  return 32 * (int64_t)SS * S + 16 * (2 * u + (j >> 2)) + 4 * g + (j & 3);
}

// Fq16[((ks * NC + c) * 2 + p) * 64 + lane] = 8 bf16: element j = part p of
// F[als16_col(S, SS, u, g, j)][16 c + (lane & 15)],  ks = S SS + u (A-operand fragment of
// the F^T tile: rows = 16 factor columns)
__global__ void __launch_bounds__(256)
als_pack_f16_kernel(const float* __restrict__ F, int64_t n, int k, int64_t ldf, int NC, int SS,
                    uint4* __restrict__ Fq, int64_t nks) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // (ks, c, lane)
  const int64_t total = nks * NC * 64;
  if (gid >= total) return;
  const int lane = (int)(gid & 63), g = lane >> 4;
  const int64_t t = gid >> 6;
  const int c = (int)(t % NC);
  const int64_t ks = t / NC;
  const int64_t S = ks / SS;
  const int u = (int)(ks % SS);
  const int col = 16 * c + (lane & 15);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t K = als16_col(S, SS, u, g, j);
    v[j] = (K < n && col < k) ? F[K * ldf + col] : 0.f;
  }
  uint4 hi, lo;
  split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), hi, lo);
  Fq[(t * 2 + 0) * 64 + lane] = hi;
  Fq[(t * 2 + 1) * 64 + lane] = lo;
}

// B = R . F partials, 16x16x32 form. Block = NW waves x RT row tiles of 16 rows; lane l
// of row tile t owns R row row0 + 16 t + (l & 15). Per super-step the lane loads 2 SS
// float4 (instruction q: columns 16 q + 4 g of its row). MFMA D[factor col][R row] +=
// F^T . R^T: lane l ends with R row (l & 15), factor columns 16 c + 4 g + i (i < 4) of
// col tile c -> one float4 store per (tile, col tile).
template <int RT, int NC, int SS, int NW, int MINB, int NBUF>
__global__ void __launch_bounds__(NW * 64, MINB)
als_rf16_kernel(const float* __restrict__ R, int64_t m, int64_t n, int64_t ldr,
                const uint4* __restrict__ Fq, int nrb, int nsplit, int ss_per_split,
                float* __restrict__ P, int kpad) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int ROWS = NW * RT * 16;
  constexpr int W = 32 * SS;
  constexpr int NQ = 2 * SS;                           // float4 loads per row per super-step
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, rr = lane & 15, g = lane >> 4;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int sp = L / nrb, rb = L % nrb;
  const int64_t nss_full = n / W;
  const int64_t nss = (n + W - 1) / W;
  const int64_t S0 = (int64_t)sp * ss_per_split;
  const int64_t S1 = std::min<int64_t>(nss, S0 + ss_per_split);
  const int64_t row0 = (int64_t)rb * ROWS + (int64_t)wid * (RT * 16);

  const float* rp[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int64_t row = row0 + 16 * t + rr;
    rp[t] = R + (row < m ? row : 0) * ldr + 4 * g;       // rows past m read row 0, never stored
  }
  f32x4 acc[RT][NC];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[t][c] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto load_f = [&](uint4 (&fv)[SS][NC][2], int64_t S) {
    const uint4* fp = Fq + (S * SS * NC * 2) * 64 + lane;
#pragma unroll
    for (int u = 0; u < SS; ++u)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        fv[u][c][0] = fp[((u * NC + c) * 2) * 64];
        fv[u][c][1] = fp[((u * NC + c) * 2 + 1) * 64];
      }
  };
  auto load = [&](float4 (&rv)[RT][NQ], uint4 (&fv)[SS][NC][2], int64_t S) {
    load_f(fv, S);
    const int64_t c0 = S * W;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int q = 0; q < NQ; ++q) rv[t][q] = ld_f4(rp[t] + c0 + 16 * q);
  };
  auto compute = [&](const float4 (&rv)[RT][NQ], const uint4 (&fv)[SS][NC][2]) {
#pragma unroll
    for (int u = 0; u < SS; ++u)
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        uint4 rh, rl;
        split8(rv[t][2 * u], rv[t][2 * u + 1], rh, rl);
        const bf16x8 bh = __builtin_bit_cast(bf16x8, rh), bl = __builtin_bit_cast(bf16x8, rl);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const bf16x8 fh = __builtin_bit_cast(bf16x8, fv[u][c][0]);
          const bf16x8 fl = __builtin_bit_cast(bf16x8, fv[u][c][1]);
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh, bh, acc[t][c], 0, 0, 0);
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl, bh, acc[t][c], 0, 0, 0);
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh, bl, acc[t][c], 0, 0, 0);
        }
      }
  };

  // NBUF-deep register ring: the loads of super-step S + NBUF - 1 are issued before the
  // MFMAs of S (sched_barrier keeps hipcc from sinking them), so NBUF - 1 super-steps of
  // R (RT x 16 rows x 128 SS bytes each) are in flight per wave
  float4 rv[NBUF][RT][NQ];
  uint4 fv[NBUF][SS][NC][2];
  const int64_t send = std::min<int64_t>(S1, nss_full);
#pragma unroll
  for (int b = 0; b + 1 < NBUF; ++b)
    if (S0 + b < send) load(rv[b], fv[b], S0 + b);
  int64_t S = S0;
  for (; S < send; S += NBUF) {
#pragma unroll
    for (int b = 0; b < NBUF; ++b) {
      if (S + b < send) {
        const int64_t Sn = S + b + NBUF - 1;
        if (Sn < send) load(rv[(b + NBUF - 1) % NBUF], fv[(b + NBUF - 1) % NBUF], Sn);
        __builtin_amdgcn_sched_barrier(0);
        compute(rv[b], fv[b]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  S = send;
  if (S < S1) {
    // tail super-step (n % W != 0): element-wise guarded loads, zeros past n
    const int64_t c0 = S * W;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] = (c0 + 16 * q + 4 * g + e < n) ? rp[t][c0 + 16 * q + e] : 0.f;
        rv[0][t][q] = make_float4(v[0], v[1], v[2], v[3]);
      }
    load_f(fv[0], S);
    compute(rv[0], fv[0]);
  }

  float* Ps = P + (int64_t)sp * m * kpad;
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int64_t row = row0 + 16 * t + rr;
    if (row >= m) continue;
    float* dst = Ps + row * kpad + 4 * g;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      *reinterpret_cast<float4*>(dst + 16 * c) =
          make_float4(acc[t][c][0], acc[t][c][1], acc[t][c][2], acc[t][c][3]);
  }
}

// ---- residual sum of squares  sum_ij (R_ij - U_i . V_j)^2  (the ALS RMSE of
// matrix_decomposition.py:19-21) in one pass over R, never forming U V^T: the closed form
// ||R||^2 - 2<U, R V> + <U^T U, V^T V> cancels ~5 significant digits at 100k x 50k, where
// an f32 R V (even with the hi/lo split) moves the RMSE by 0.5 %; here every residual is
// formed in f32 from an f32-accurate U V^T tile and squared, so nothing cancels.
// 16x16x32 MFMA with A = V^T tile (16 V rows = columns of R, Vq packed hi/lo fragments),
// B = U^T tile (16 U rows = rows of R, resident hi/lo fragments): lane l ends with R row
// (l & 15) and columns 4 (l >> 4) + i, i < 4 — one float4 of R per lane per tile pair.
// Vq[((ct * KS + s) * 2 + p) * 64 + lane] = part p of V[16 ct + (lane & 15)][32 s + 8 (lane >> 4) + j]
__global__ void __launch_bounds__(256)
als_pack_v_kernel(const float* __restrict__ V, int64_t n, int k, int64_t ldv, int KS,
                  uint4* __restrict__ Vq, int64_t nct) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // (ct, s, lane)
  if (gid >= nct * KS * 64) return;
  const int lane = (int)(gid & 63);
  const int64_t t = gid >> 6;
  const int sidx = (int)(t % KS);
  const int64_t ct = t / KS;
  const int64_t row = 16 * ct + (lane & 15);
  const int k0 = 32 * sidx + 8 * (lane >> 4);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (row < n && k0 + j < k) ? V[row * ldv + k0 + j] : 0.f;
  uint4 hi, lo;
  split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), hi, lo);
  Vq[(t * 2 + 0) * 64 + lane] = hi;
  Vq[(t * 2 + 1) * 64 + lane] = lo;
}

template <int RT, int KS>
__global__ void __launch_bounds__(256, 1)
als_residual_kernel(const float* __restrict__ R, int64_t m, int64_t n, int64_t ldr,
                    const float* __restrict__ U, int k, int64_t ldu, const uint4* __restrict__ Vq,
                    int nrb, int64_t ct_per_split, double* __restrict__ part) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int NW = 4;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, rr = lane & 15, g = lane >> 4;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int sp = L / nrb, rb = L % nrb;
  const int64_t nct = (n + 15) / 16;
  const int64_t ct0 = (int64_t)sp * ct_per_split;
  const int64_t ct1 = std::min<int64_t>(nct, ct0 + ct_per_split);
  const int64_t row0 = ((int64_t)rb * NW + wid) * (RT * 16);
  // resident U^T fragments (B operand): row row0 + 16 t + rr, k = 32 s + 8 g + j
  bf16x8 uh[RT][KS], ul[RT][KS];
  const float* rp[RT];
  bool rok[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int64_t row = row0 + 16 * t + rr;
    rok[t] = row < m;
    const int64_t rs = rok[t] ? row : 0;
    rp[t] = R + rs * ldr + 4 * g;
#pragma unroll
    for (int sidx = 0; sidx < KS; ++sidx) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = 32 * sidx + 8 * g + j;
        v[j] = (kk < k) ? U[rs * ldu + kk] : 0.f;
      }
      uint4 hi, lo;
      split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), hi, lo);
      uh[t][sidx] = __builtin_bit_cast(bf16x8, hi);
      ul[t][sidx] = __builtin_bit_cast(bf16x8, lo);
    }
  }
  auto load_v = [&](uint4 (&vf)[KS][2], int64_t ct) {
    const uint4* vp = Vq + (ct * KS * 2) * 64 + lane;
#pragma unroll
    for (int sidx = 0; sidx < KS; ++sidx) {
      vf[sidx][0] = vp[(2 * sidx) * 64];
      vf[sidx][1] = vp[(2 * sidx + 1) * 64];
    }
  };
  const bool full_cols = (n % 16) == 0;
  auto load_r = [&](float4 (&rv)[RT], int64_t ct) {
    const int64_t c = 16 * ct + 4 * g;
    if (full_cols || c + 4 <= n) {
#pragma unroll
      for (int t = 0; t < RT; ++t) rv[t] = *reinterpret_cast<const float4*>(rp[t] + 16 * ct);
    } else {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (c + e < n) ? rp[t][16 * ct + e] : 0.f;
        rv[t] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  double dsum = 0.0;
  float fsum = 0.f;
  int nacc = 0;
  auto tile = [&](const float4 (&rv)[RT], const uint4 (&vf)[KS][2], int64_t ct) {
    const int64_t c = 16 * ct + 4 * g;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      f32x4 d = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sidx = 0; sidx < KS; ++sidx) {
        const bf16x8 vh = __builtin_bit_cast(bf16x8, vf[sidx][0]);
        const bf16x8 vl = __builtin_bit_cast(bf16x8, vf[sidx][1]);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, uh[t][sidx], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vl, uh[t][sidx], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, ul[t][sidx], d, 0, 0, 0);
      }
      const float r0 = rv[t].x - d[0], r1 = rv[t].y - d[1], r2 = rv[t].z - d[2], r3 = rv[t].w - d[3];
      float q = 0.f;
      if (rok[t]) {
        q = (c + 0 < n ? r0 * r0 : 0.f) + (c + 1 < n ? r1 * r1 : 0.f) +
            (c + 2 < n ? r2 * r2 : 0.f) + (c + 3 < n ? r3 * r3 : 0.f);
      }
      fsum += q;
    }
    if (++nacc == 32) { dsum += (double)fsum; fsum = 0.f; nacc = 0; }
  };

  float4 ra[RT], rb2[RT];
  uint4 va[KS][2], vb[KS][2];
  int64_t ct = ct0;
  if (ct < ct1) { load_v(va, ct); load_r(ra, ct); }
  for (; ct + 1 < ct1; ct += 2) {
    load_v(vb, ct + 1);
    load_r(rb2, ct + 1);
    __builtin_amdgcn_sched_barrier(0);
    tile(ra, va, ct);
    __builtin_amdgcn_sched_barrier(0);
    if (ct + 2 < ct1) { load_v(va, ct + 2); load_r(ra, ct + 2); }
    __builtin_amdgcn_sched_barrier(0);
    tile(rb2, vb, ct + 1);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (ct < ct1) tile(ra, va, ct);
  dsum += (double)fsum;
  // block sum (wave shuffles in f64, then LDS), one partial per block
  for (int off = 32; off >= 1; off >>= 1) dsum += __shfl_xor(dsum, off);
  __shared__ double s_w[NW];
  if (lane == 0) s_w[wid] = dsum;
  __syncthreads();
  if (tid == 0) {
    double tot = 0.0;
    for (int w = 0; w < NW; ++w) tot += s_w[w];
    part[blockIdx.x] = tot;
  }
}

// out[i, :k] = (sum_s P[s][i, :]) . Ginv   — 32 rows per block, fixed split order
__global__ void __launch_bounds__(256)
als_reduce_solve_kernel(const float* __restrict__ P, int nsplit, int64_t m, int kpad,
                        const float* __restrict__ Ginv, int k, int ldg, float* __restrict__ out,
                        int64_t ldo) {
  extern __shared__ __attribute__((aligned(16))) float s_mem[];
  float* s_g = s_mem;                         // [k][k]
  float* s_b = s_mem + k * k;                 // [32][kpad + 1]
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * 32;
  const int nr = (int)std::min<int64_t>(32, m - r0);
  for (int e = tid; e < k * k; e += 256) s_g[e] = Ginv[(int64_t)(e / k) * ldg + (e % k)];
  for (int e = tid; e < nr * kpad; e += 256) {
    const int i = e / kpad, c = e % kpad;
    const float* p = P + (r0 + i) * kpad + c;
    float s = 0.f;
    for (int q = 0; q < nsplit; ++q) s += p[(int64_t)q * m * kpad];
    s_b[i * (kpad + 1) + c] = s;
  }
  __syncthreads();
  for (int e = tid; e < nr * k; e += 256) {
    const int i = e / k, j = e % k;
    const float* b = s_b + i * (kpad + 1);
    float s = 0.f;
    for (int c = 0; c < k; ++c) s = fmaf(b[c], s_g[c * k + j], s);
    out[(r0 + i) * ldo + j] = s;
  }
}

// Gram matrix G = F^T F of an n x k factor (k <= 128), once per half-sweep. The library
// GEMM runs this skinny shape (M = N = k, K = n = 50k) on a handful of workgroups (280 us
// in the round-2 profile); here n is split over up to 256 blocks, each stages 32 rows at a
// time in LDS and accumulates its k*k partial in registers (thread t owns entries t,
// t+256, ...), and a second kernel sums the partials in block order (deterministic).
__global__ void __launch_bounds__(256)
als_gram_partial_kernel(const float* __restrict__ F, int64_t n, int k, int64_t ldf,
                        int64_t rows_per_block, float* __restrict__ part) {
  constexpr int RB = 32;
  __shared__ float s_f[RB * 128];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = std::min<int64_t>(n, r0 + rows_per_block);
  const int kk = k * k;
  float acc[64];
  int ei[64], ej[64];
  const int ne = (kk + 255) / 256;             // entries per thread (<= 64 for k <= 128)
#pragma unroll
  for (int q = 0; q < 64; ++q) {
    acc[q] = 0.f;
    const int e = tid + 256 * q;
    ei[q] = e < kk ? e / k : 0;
    ej[q] = e < kk ? e % k : 0;
  }
  for (int64_t rb = r0; rb < r1; rb += RB) {
    const int nr = (int)std::min<int64_t>(RB, r1 - rb);
    __syncthreads();
    for (int e = tid; e < nr * k; e += 256) {
      const int i = e / k, j = e % k;
      s_f[i * k + j] = F[(rb + i) * ldf + j];
    }
    __syncthreads();
    for (int i = 0; i < nr; ++i) {
      const float* row = s_f + i * k;
#pragma unroll
      for (int q = 0; q < 64; ++q)
        if (q < ne) acc[q] = fmaf(row[ei[q]], row[ej[q]], acc[q]);
    }
  }
  float* out = part + (int64_t)blockIdx.x * kk;
#pragma unroll
  for (int q = 0; q < 64; ++q) {
    const int e = tid + 256 * q;
    if (q < ne && e < kk) out[e] = acc[q];
  }
}

__global__ void __launch_bounds__(256)
als_gram_sum_kernel(const float* __restrict__ part, int nb, int k, float* __restrict__ G, int ldg) {
  const int kk = k * k;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < kk; e += gridDim.x * 256) {
    float s = 0.f;
    for (int b = 0; b < nb; ++b) s += part[(int64_t)b * kk + e];
    G[(int64_t)(e / k) * ldg + (e % k)] = s;
  }
}

static int als_device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    cached[dev] = v;
  }
  return cached[dev];
}

// Launch configuration by factor count k (DALGO_ALS_VARIANT = 1 selects the fallback):
//   form 16 (default): als_rf16_kernel, 16-row tiles, NC = factor tiles of 16 (k padded
//                      to 16/32/64/128), 8 row tiles per wave (4 at k > 64), 3 F buffers;
//   form 32 (fallback): als_rf_kernel, 32-row tiles, NC = factor tiles of 32.
// rt = row tiles per wave, ss = K-steps per super-step, minb = blocks per CU (4 waves each).
// The other launch shapes measured in rounds 2-4 (8-wave LDS-shared F, 2 / 4 F buffers,
// 2 blocks per CU) were slower and are gone (profiles/round4/README.md).
struct AlsCfg { int form, nc, rt, ss, minb, nbuf; };
static int als_variant() { return env_int("DALGO_ALS_VARIANT", 0); }
static AlsCfg als_cfg(int k, int variant) {
  const int nc16 = k <= 16 ? 1 : k <= 32 ? 2 : k <= 64 ? 4 : 8;
  const int nc32 = (k + 31) / 32;
  if (variant == 1) return {32, nc32, nc32 <= 2 ? 4 : 2, 2, 1, 2};
  return {16, nc16, nc16 <= 4 ? 8 : 4, 1, 1, 3};
}
static int als_waves(const AlsCfg&) { return 4; }
static int als_tile(const AlsCfg& c) { return c.form == 32 ? 32 : 16; }
static int64_t als_rows_per_block(const AlsCfg& c) { return (int64_t)als_waves(c) * c.rt * als_tile(c); }
static int64_t als_ks_width(const AlsCfg& c) { return c.form == 32 ? 16 : 32; }   // columns per K-step
static int als_kpad(const AlsCfg& c) { return c.nc * als_tile(c); }

template <int FORM, int RT, int NC, int SS, int MINB, int NBUF>
static hipError_t launch_rf(const float* R, int64_t m, int64_t n, int64_t ldr, const uint4* Fq,
                            int nsplit, int ssps, float* P, int kpad, hipStream_t st) {
  constexpr int NW = 4;
  const int nrb = (int)cdiv(m, NW * RT * (FORM == 32 ? 32 : 16));
  if constexpr (FORM == 16) {
    hipLaunchKernelGGL((als_rf16_kernel<RT, NC, SS, NW, MINB, NBUF>), dim3(nrb * nsplit), dim3(NW * 64), 0,
                       st, R, m, n, ldr, Fq, nrb, nsplit, ssps, P, kpad);
  } else {
    hipLaunchKernelGGL((als_rf_kernel<RT, NC, SS, NW, MINB>), dim3(nrb * nsplit), dim3(NW * 64), 0, st,
                       R, m, n, ldr, Fq, nrb, nsplit, ssps, P, kpad);
  }
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

static hipError_t dispatch_rf(const AlsCfg& cf, const float* R, int64_t m, int64_t n, int64_t ldr,
                              const uint4* Fq, int nsplit, int ssps, float* P, int kpad,
                              hipStream_t st) {
#define ALS_RF_CASE(FM_, RT_, NC_, SS_, MB_, NB_)                                             \
  if (cf.form == FM_ && cf.rt == RT_ && cf.nc == NC_ && cf.ss == SS_ && cf.minb == MB_ &&        \
      cf.nbuf == NB_)                                                                            \
    return launch_rf<FM_, RT_, NC_, SS_, MB_, NB_>(R, m, n, ldr, Fq, nsplit, ssps, P, kpad, st);
  ALS_RF_CASE(16, 8, 1, 1, 1, 3) ALS_RF_CASE(16, 8, 2, 1, 1, 3) ALS_RF_CASE(16, 8, 4, 1, 1, 3)
  ALS_RF_CASE(16, 4, 8, 1, 1, 3)
  ALS_RF_CASE(32, 4, 1, 2, 1, 2) ALS_RF_CASE(32, 4, 2, 2, 1, 2) ALS_RF_CASE(32, 2, 3, 2, 1, 2)
  ALS_RF_CASE(32, 2, 4, 2, 1, 2)
#undef ALS_RF_CASE
  return hipErrorInvalidValue;
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

// G[k x k] = F^T F (F: n x k f32, k <= 128); part: dalgo_als_gram_blocks(n) * k * k floats
int dalgo_als_gram_blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(256, cdiv(n, 64))); }
hipError_t dalgo_als_gram(const float* F, int64_t n, int k, int64_t ldf, float* G, int ldg, float* part,
                          hipStream_t st) {
  if (k < 1 || k > 128 || n < 0) return hipErrorInvalidValue;
  const int nb = dalgo_als_gram_blocks(n);
  const int64_t rpb = std::max<int64_t>(1, cdiv(n, nb));
  hipLaunchKernelGGL(als_gram_partial_kernel, dim3(nb), dim3(256), 0, st, F, n, k, ldf, rpb, part);
  DALGO_LAUNCH_CHECK();
  hipLaunchKernelGGL(als_gram_sum_kernel, dim3((unsigned)cdiv((int64_t)k * k, 256)), dim3(256), 0, st, part,
                     nb, k, G, ldg);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// sum_ij (R_ij - U_i . V_j)^2 over R (m x n f32, ldr % 4 == 0, 16-B aligned), U (m x k),
// V (n x k), k <= 128. Vq: dalgo_als_residual_vq_bytes(n, k) bytes; part: one double per
// block, dalgo_als_residual_blocks(m, n) of them (the caller sums them in order).
static void als_residual_grid(int64_t m, int64_t n, int* nrb, int* nsp, int64_t* ctps) {
  const int64_t rows = 4 * 8 * 16;
  *nrb = (int)std::max<int64_t>(1, cdiv(m, rows));
  const int64_t nct = std::max<int64_t>(1, cdiv(n, 16));
  const int64_t want = std::max<int64_t>(1, cdiv(4 * (int64_t)als_device_cus(), *nrb));
  const int64_t s = std::min<int64_t>(want, nct);
  *ctps = cdiv(nct, s);
  *nsp = (int)cdiv(nct, *ctps);
}
int64_t dalgo_als_residual_vq_bytes(int64_t n, int k) {
  return std::max<int64_t>(1, cdiv(n, 16)) * ((k + 31) / 32) * 2 * 64 * 16;
}
int dalgo_als_residual_blocks(int64_t m, int64_t n) {
  int nrb, nsp;
  int64_t ctps;
  als_residual_grid(m, n, &nrb, &nsp, &ctps);
  return nrb * nsp;
}
hipError_t dalgo_als_residual(const float* R, int64_t m, int64_t n, int64_t ldr, const float* U,
                              int64_t ldu, const float* V, int64_t ldv, int k, void* Vq, double* part,
                              hipStream_t st) {
  if (k < 1 || k > 128 || m < 1 || n < 1 || (ldr & 3)) return hipErrorInvalidValue;
  if (((uintptr_t)R & 15) || ((uintptr_t)Vq & 15)) return hipErrorInvalidValue;
  const int KS = (k + 31) / 32;
  const int64_t nct = cdiv(n, 16);
  {
    const int64_t total = nct * KS * 64;
    hipLaunchKernelGGL(als_pack_v_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, st, V, n, k, ldv,
                       KS, reinterpret_cast<uint4*>(Vq), nct);
    DALGO_LAUNCH_CHECK();
  }
  int nrb, nsp;
  int64_t ctps;
  als_residual_grid(m, n, &nrb, &nsp, &ctps);
  const uint4* vq = reinterpret_cast<const uint4*>(Vq);
  const dim3 grid(nrb * nsp), blk(256);
  switch (KS) {
    case 1: hipLaunchKernelGGL((als_residual_kernel<8, 1>), grid, blk, 0, st, R, m, n, ldr, U, k, ldu, vq, nrb, ctps, part); break;
    case 2: hipLaunchKernelGGL((als_residual_kernel<8, 2>), grid, blk, 0, st, R, m, n, ldr, U, k, ldu, vq, nrb, ctps, part); break;
    case 3: hipLaunchKernelGGL((als_residual_kernel<8, 3>), grid, blk, 0, st, R, m, n, ldr, U, k, ldu, vq, nrb, ctps, part); break;
    default: hipLaunchKernelGGL((als_residual_kernel<8, 4>), grid, blk, 0, st, R, m, n, ldr, U, k, ldu, vq, nrb, ctps, part); break;
  }
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// Workspace sizes for dalgo_als_solve (same DALGO_ALS_VARIANT as the solve): Fq bytes,
// the K-split count and the padded factor width of the partials P[nsplit][m][kpad].
int64_t dalgo_als_fq_bytes(int64_t n, int k) {
  const AlsCfg cf = als_cfg(k, als_variant());
  const int64_t w = als_ks_width(cf) * cf.ss;
  return cdiv(n, w) * cf.ss * cf.nc * 2 * 64 * 16;
}
int dalgo_als_kpad(int k) { return als_kpad(als_cfg(k, als_variant())); }
// K-split count: balances the block rounds over the CUs against the partial traffic
int dalgo_als_nsplit(int64_t m, int64_t n, int k) {
  const AlsCfg cf = als_cfg(k, als_variant());
  const int64_t nrb = cdiv(m, als_rows_per_block(cf));
  const int64_t nss = cdiv(n, als_ks_width(cf) * cf.ss);
  const int64_t slots = (int64_t)als_device_cus() * cf.minb;
  const double rbytes = (double)m * n * 4.0;
  int best = 1;
  double best_cost = 1e300;
  for (int s = 1; s <= 64; ++s) {
    if (s > 1 && cdiv(nss, s) * cf.ss * als_ks_width(cf) < 256) break;   // >= 256 columns per split
    const int64_t ssps = cdiv(nss, s);
    const int64_t used = cdiv(nss, ssps);              // splits that get work
    const int64_t blocks = nrb * used;
    const double rounds = (double)cdiv(blocks, slots);
    const double waste = rounds * slots / (double)blocks;
    const double cost = rbytes * std::max(1.0, waste) + 1.2 * (double)used * m * als_kpad(cf) * 8.0;
    if (cost < best_cost * 0.999) { best_cost = cost; best = (int)used; }
  }
  return best;
}

// out[m x k] = (R[m x n] . F[n x k]) . Ginv[k x k];  R f32 (ldr % 4 == 0, 16-B aligned),
// k <= 128. Fq: dalgo_als_fq_bytes(n, k) bytes; P: nsplit * m * dalgo_als_kpad(k) floats,
// nsplit = dalgo_als_nsplit(m, n, k) (all three under the same DALGO_ALS_VARIANT).
hipError_t dalgo_als_solve(const float* R, int64_t m, int64_t n, int64_t ldr, const float* F,
                           int64_t ldf, int k, const float* Ginv, int ldg, float* out, int64_t ldo,
                           void* Fq, float* P, int nsplit, hipStream_t st) {
  if (k < 1 || k > 128 || m < 1 || n < 1 || (ldr & 3) || nsplit < 1) return hipErrorInvalidValue;
  if (((uintptr_t)R & 15) || ((uintptr_t)Fq & 15) || ((uintptr_t)P & 15)) return hipErrorInvalidValue;
  const AlsCfg cf = als_cfg(k, als_variant());
  const int kpad = als_kpad(cf);
  const int64_t nss = cdiv(n, als_ks_width(cf) * cf.ss);
  const int ssps = (int)cdiv(nss, nsplit);
  if (cdiv(nss, ssps) != nsplit) return hipErrorInvalidValue;   // caller: dalgo_als_nsplit()
  {
    const int64_t nks = nss * cf.ss;
    const int64_t total = nks * cf.nc * 64;
    if (cf.form != 32)
      hipLaunchKernelGGL(als_pack_f16_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, st, F, n, k,
                         ldf, cf.nc, cf.ss, reinterpret_cast<uint4*>(Fq), nks);
    else
      hipLaunchKernelGGL(als_pack_f_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, st, F, n, k,
                         ldf, cf.nc, cf.ss, reinterpret_cast<uint4*>(Fq), nks);
    DALGO_LAUNCH_CHECK();
  }
  const hipError_t e = dispatch_rf(cf, R, m, n, ldr, reinterpret_cast<const uint4*>(Fq), nsplit, ssps,
                                   P, kpad, st);
  if (e != hipSuccess) return e;
  const size_t lds = ((size_t)k * k + 32 * (size_t)(kpad + 1)) * sizeof(float);
  hipLaunchKernelGGL(als_reduce_solve_kernel, dim3((unsigned)cdiv(m, 32)), dim3(256), lds, st, P,
                     nsplit, m, kpad, Ginv, k, ldg, out, ldo);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
