// LDS atomic throughput probe (gfx950): ds_add_f32 / ds_add_u32 with random or
// conflict-free addresses, 1024-thread blocks, one 128 KB accumulator per block.
// Build: hipcc --offload-arch=gfx950 -O3 lds_atomic_probe.hip -o lds_atomic_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE, int BW>
__global__ void __launch_bounds__(1024) probe(float* out, int iters, uint32_t seed) {
  __shared__ float s[BW];
  for (int i = threadIdx.x; i < BW; i += 1024) s[i] = 0.f;
  __syncthreads();
  uint32_t x = seed ^ (blockIdx.x * 1024 + threadIdx.x) * 2654435761u;
  const float v = 1.0f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      x = x * 1664525u + 1013904223u;
      uint32_t a;
      if (MODE == 0) a = (x >> 8) & (BW - 1);                    // random
      else if (MODE == 1) a = ((threadIdx.x & 63) + 64 * u + 1024 * (threadIdx.x >> 6)) & (BW - 1);  // conflict-free
      else a = (x >> 8) & 31;                                     // 32 hot addresses
      if (MODE == 4) {
        atomicAdd(reinterpret_cast<unsigned long long*>(&s[2 * ((x >> 8) & (BW / 2 - 1))]), 1ull);
      } else if (MODE == 3) {
        atomicAdd(reinterpret_cast<uint32_t*>(&s[(x >> 8) & (BW - 1)]), 1u);
      } else {
        atomicAdd(&s[a], v);
      }
    }
  }
  __syncthreads();
  float t = 0.f;
  for (int i = threadIdx.x; i < BW; i += 1024) t += s[i];
  if (t == 12345.f) out[0] = t;
}

template <int MODE>
void run(const char* name, float* d, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  probe<MODE, 32768><<<blocks, 1024>>>(d, iters, 1);
  hipEventRecord(a);
  probe<MODE, 32768><<<blocks, 1024>>>(d, iters, 2);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  const double ops = (double)blocks * 1024 * iters * 16;
  printf("%-28s %8.3f ms  %8.1f G lane-atomics/s  %.3f per CU-cycle (2.4 GHz, 256 CU)\n", name, ms,
         ops / ms / 1e6, ops / (ms * 1e-3) / (256 * 2.4e9));
}

int main() {
  float* d; hipMalloc(&d, 4);
  const int blocks = 256 * 4, iters = 256;
  run<0>("f32 random", d, blocks, iters);
  run<1>("f32 conflict-free", d, blocks, iters);
  run<2>("f32 32 hot addresses", d, blocks, iters);
  run<3>("u32 random", d, blocks, iters);
  run<4>("u64 random", d, blocks, iters);
  return 0;
}
