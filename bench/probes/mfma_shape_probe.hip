// Standalone probe: sustained bf16 MFMA rate of v_mfma_f32_32x32x16_bf16 vs
// v_mfma_f32_16x16x32_bf16 at K2-like occupancy (2 waves per SIMD, 2048 waves), with and
// without a K2-like VALU side load (min/med3 on the accumulators every iteration).
// Timing only. Build and run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 bench/probes/mfma_shape_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 20000;

template <bool VALU>
__global__ void __launch_bounds__(256, 2) k32(float* out, int seed) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(float)((threadIdx.x + i + seed) & 7);
    b[i] = (__bf16)(float)((threadIdx.x * 3 + i) & 7);
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  int m = 0x7fffffff;
  for (int it = 0; it < kIters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    if (VALU) {
#pragma unroll
      for (int r = 0; r < 16; r += 2)
        m = min(min(m, __float_as_int(c0[r]) & ~31), __float_as_int(c1[r + 1]) | r);
    }
  }
  float s = m * 1e-30f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <bool VALU>
__global__ void __launch_bounds__(256, 2) k16(float* out, int seed) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(float)((threadIdx.x + i + seed) & 7);
    b[i] = (__bf16)(float)((threadIdx.x * 3 + i) & 7);
  }
  f32x4 c[16] = {};
  int m = 0x7fffffff;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[j], 0, 0, 0);
    if (VALU) {
#pragma unroll
      for (int j = 0; j < 8; j += 2)
        m = min(min(m, __float_as_int(c[j][0]) & ~31), __float_as_int(c[j + 1][1]) | j);
    }
  }
  float s = m * 1e-30f;
  for (int j = 0; j < 8; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static double run(K kern, float* out, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1);   // warm-up
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  // both kernels: 65536 MACs per wave-iteration
  const double flops = 3.0 * blocks * 4.0 * kIters * 65536.0 * 2.0;
  return flops / (ms * 1e-3) / 1e12;
}

int main() {
  const int blocks = 256 * 2;                 // 2 blocks of 4 waves per CU
  float* out;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  for (int rep = 0; rep < 2; ++rep) {
    printf("32x32x16: %.0f TF/s   16x16x32: %.0f TF/s   (MFMA only)\n", run(k32<false>, out, blocks),
           run(k16<false>, out, blocks));
    printf("32x32x16: %.0f TF/s   16x16x32: %.0f TF/s   (with a VALU side load)\n",
           run(k32<true>, out, blocks), run(k16<true>, out, blocks));
  }
  hipFree(out);
  return 0;
}
