// Read-pattern probe for the K5 ALS GEMM (R: m x n f32, row-major, rows 200 KB apart).
// Each kernel only loads R and folds it into a register (no MFMA), so the time is the
// memory system's cost of the access shape:
//   lanes  : per-lane rows — lane (r, h) of a wave reads row r, 2*SS consecutive 16-B
//            pieces starting at 8*SS*h (the MFMA B-operand layout; RT row tiles per wave)
//   rowsNB : coalesced — one wave-instruction reads R rows as 1 KB / (64 / LPR lanes) ...
//            i.e. LPR lanes per row, 16 B each, so each instruction covers 64/LPR rows x
//            16*LPR bytes
//   stream : plain contiguous stream (ceiling)
// Build: hipcc --offload-arch=gfx950 -O3 -o row_tile_probe row_tile_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f4v ld(const float* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
  else return *reinterpret_cast<const f4v*>(p);
}

// per-lane rows: grid = (row blocks) x (K splits); block = 4 waves x RT*32 rows; K range per split
template <int RT, int SS, bool NT>
__global__ void __launch_bounds__(256) lanes_kernel(const float* R, int64_t m, int64_t n, int64_t ld_,
                                                    int nrb, int ssps, float* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int sp = blockIdx.x / nrb, rb = blockIdx.x % nrb;
  constexpr int W = 16 * SS;
  const int64_t nss = n / W;
  const int64_t S0 = (int64_t)sp * ssps, S1 = S0 + ssps < nss ? S0 + ssps : nss;
  const float* rp[RT];
  for (int t = 0; t < RT; ++t) {
    int64_t row = (int64_t)rb * (4 * RT * 32) + wid * RT * 32 + t * 32 + r;
    if (row >= m) row = 0;
    rp[t] = R + row * ld_ + 8 * SS * h;
  }
  f4v acc = {0, 0, 0, 0};
  for (int64_t S = S0; S < S1; ++S) {
    f4v v[RT][2 * SS];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int q = 0; q < 2 * SS; ++q) v[t][q] = ld<NT>(rp[t] + S * W + 4 * q);
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int q = 0; q < 2 * SS; ++q) acc += v[t][q];
  }
  if (acc.x == 1234.5f) out[threadIdx.x] = acc.y + acc.z + acc.w;
}

// coalesced: LPR lanes per row; one instruction covers 64/LPR rows x 16*LPR bytes; each
// wave owns RPW rows and walks its K range UNR instructions at a time
template <int LPR, int RPW, int UNR, bool NT>
__global__ void __launch_bounds__(256) rows_kernel(const float* R, int64_t m, int64_t n, int64_t ld_,
                                                   int nrb, int cols_per_split, float* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int RPI = 64 / LPR;          // rows per instruction
  constexpr int G = RPW / RPI;           // instruction groups covering the wave's rows
  const int sp = blockIdx.x / nrb, rb = blockIdx.x % nrb;
  const int64_t c0 = (int64_t)sp * cols_per_split;
  int64_t c1 = c0 + cols_per_split;
  if (c1 > n) c1 = n;
  const int sub = lane / LPR, l = lane % LPR;
  const float* rp[G];
  for (int g = 0; g < G; ++g) {
    int64_t row = (int64_t)rb * (4 * RPW) + wid * RPW + g * RPI + sub;
    if (row >= m) row = 0;
    rp[g] = R + row * ld_ + 4 * l;
  }
  f4v acc = {0, 0, 0, 0};
  constexpr int STEP = 4 * LPR;          // columns per instruction per row
  for (int64_t c = c0; c + UNR * STEP <= c1; c += UNR * STEP) {
    f4v v[G][UNR];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int u = 0; u < UNR; ++u) v[g][u] = ld<NT>(rp[g] + c + u * STEP);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int u = 0; u < UNR; ++u) acc += v[g][u];
  }
  if (acc.x == 1234.5f) out[threadIdx.x] = acc.y + acc.z + acc.w;
}

__global__ void __launch_bounds__(256) stream_kernel(const float* R, int64_t nf, float* out) {
  f4v acc = {0, 0, 0, 0};
  const int64_t nv = nf / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (int64_t)gridDim.x * 256 * 4) {
    f4v a = ld<true>(R + 4 * i), b = {0,0,0,0}, c = {0,0,0,0}, d = {0,0,0,0};
    if (i + (int64_t)gridDim.x * 256 < nv) b = ld<true>(R + 4 * (i + (int64_t)gridDim.x * 256));
    if (i + 2 * (int64_t)gridDim.x * 256 < nv) c = ld<true>(R + 4 * (i + 2 * (int64_t)gridDim.x * 256));
    if (i + 3 * (int64_t)gridDim.x * 256 < nv) d = ld<true>(R + 4 * (i + 3 * (int64_t)gridDim.x * 256));
    acc += a + b + c + d;
  }
  if (acc.x == 1234.5f) out[threadIdx.x] = acc.y;
}

static float time_it(void (*launch)(void*), void* ctx, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  launch(ctx);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch(ctx);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

struct Ctx { const float* R; int64_t m, n; float* out; };
static Ctx g;

template <int RT, int SS, bool NT>
static void run_lanes(void*) {
  const int rows = 4 * RT * 32;
  const int nrb = (int)((g.m + rows - 1) / rows);
  const int64_t nss = g.n / (16 * SS);
  int splits = 1;
  while ((int64_t)nrb * splits < 2048 && splits < 64) ++splits;
  const int ssps = (int)((nss + splits - 1) / splits);
  hipLaunchKernelGGL((lanes_kernel<RT, SS, NT>), dim3(nrb * splits), dim3(256), 0, 0, g.R, g.m, g.n, g.n, nrb,
                     ssps, g.out);
}
template <int LPR, int RPW, int UNR, bool NT>
static void run_rows(void*) {
  const int nrb = (int)((g.m + 4 * RPW - 1) / (4 * RPW));
  int splits = 1;
  while ((int64_t)nrb * splits < 2048 && splits < 256) ++splits;
  const int step = 4 * LPR * UNR;
  int cps = (int)((g.n + splits - 1) / splits);
  cps = (cps + step - 1) / step * step;
  hipLaunchKernelGGL((rows_kernel<LPR, RPW, UNR, NT>), dim3(nrb * splits), dim3(256), 0, 0, g.R, g.m, g.n, g.n,
                     nrb, cps, g.out);
}
static void run_stream(void*) {
  hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, 0, g.R, g.m * g.n, g.out);
}

int main(int argc, char** argv) {
  g.m = argc > 1 ? atoll(argv[1]) : 100000;
  g.n = argc > 2 ? atoll(argv[2]) : 50000;
  float* R;
  CK(hipMalloc(&R, g.m * g.n * 4));
  CK(hipMemset(R, 0, g.m * g.n * 4));
  CK(hipMalloc(&g.out, 4096));
  g.R = R;
  const double gb = g.m * g.n * 4 / 1e9;
  struct E { const char* name; void (*f)(void*); };
  std::vector<E> es = {
      {"stream", run_stream},
      {"lanes RT4 SS1", run_lanes<4, 1, false>},
      {"lanes RT2 SS2", run_lanes<2, 2, false>},
      {"lanes RT4 SS2", run_lanes<4, 2, false>},
      {"lanes RT2 SS4", run_lanes<2, 4, false>},
      {"rows LPR4 RPW64 UNR2", run_rows<4, 64, 2, false>},
      {"rows LPR4 RPW64 UNR4", run_rows<4, 64, 4, false>},
      {"rows LPR4 RPW128 UNR2", run_rows<4, 128, 2, false>},
      {"rows LPR4 RPW32 UNR4", run_rows<4, 32, 4, false>},
      {"rows LPR8 RPW32 UNR4", run_rows<8, 32, 4, false>},
      {"rows LPR8 RPW64 UNR2", run_rows<8, 64, 2, false>},
      {"rows LPR16 RPW16 UNR4", run_rows<16, 16, 4, false>},
      {"rows LPR16 RPW64 UNR1", run_rows<16, 64, 1, false>},
      {"rows LPR16 RPW16 UNR4 nt", run_rows<16, 16, 4, true>},
  };
  for (int round = 0; round < 2; ++round)
    for (auto& e : es) {
      float ms = time_it(e.f, nullptr, 5);
      printf("%-28s %8.3f ms  %6.2f TB/s\n", e.name, ms, gb / ms);
      fflush(stdout);
    }
  return 0;
}
