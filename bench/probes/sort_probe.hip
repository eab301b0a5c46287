// Probe: rocPRIM onesweep radix sort of N 64-bit keys over their low B bits, with the
// default gfx950 config (8 bits per place) and wider / narrower digits -- the adjacency
// build's key sort (csrc/kernels/graph_build.hip dalgo_gb_sort) is its largest phase.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 sort_probe.hip -o sort_probe
// Run:   ./sort_probe [N=1060000000] [B=52]
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

__global__ void fill_keys(uint64_t* k, int64_t n, int bits, uint64_t seed) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 33;
    // skewed top bits (R-MAT-like block sizes): square a uniform in [0, 1) for the high 13
    const uint64_t hi = (uint64_t)(((double)(x >> 40) / (double)(1ull << 24)) *
                                   ((double)(x >> 40) / (double)(1ull << 24)) * (1 << 13));
    k[i] = ((hi << (bits - 13)) | (x & ((1ull << (bits - 13)) - 1)));
  }
}

template <class Cfg>
static float run(const char* name, uint64_t* in, uint64_t* out, int64_t n, int bits) {
  size_t bytes = 0;
  CK(rocprim::radix_sort_keys<Cfg>(nullptr, bytes, in, out, (size_t)n, 0u, (unsigned)bits, 0));
  void* tmp = nullptr;
  CK(hipMalloc(&tmp, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 4; ++r) {
    CK(hipEventRecord(a, 0));
    CK(rocprim::radix_sort_keys<Cfg>(tmp, bytes, in, out, (size_t)n, 0u, (unsigned)bits, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r > 0 && ms < best) best = ms;
  }
  CK(hipFree(tmp));
  std::printf("%-34s n=%lld bits=%d  %.2f ms\n", name, (long long)n, bits, best);
  std::fflush(stdout);
  return best;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 1060000000LL;
  const int bits = argc > 2 ? std::atoi(argv[2]) : 52;
  uint64_t *in = nullptr, *out = nullptr;
  CK(hipMalloc(&in, n * 8));
  CK(hipMalloc(&out, n * 8));
  hipLaunchKernelGGL(fill_keys, dim3(4096), dim3(256), 0, 0, in, n, bits, 12345ull);
  CK(hipDeviceSynchronize());
  using namespace rocprim;
  run<default_config>("default (gfx950: 8 bits/place)", in, out, n, bits);
  run<radix_sort_config<default_config, default_config,
                        radix_sort_onesweep_config<kernel_config<256, 12>, kernel_config<1024, 8>, 10,
                                                   block_radix_rank_algorithm::match>>>(
      "onesweep 10 bits, 1024x8", in, out, n, bits);
  run<radix_sort_config<default_config, default_config,
                        radix_sort_onesweep_config<kernel_config<256, 12>, kernel_config<1024, 12>, 9,
                                                   block_radix_rank_algorithm::match>>>(
      "onesweep 9 bits, 1024x12", in, out, n, bits);
  run<radix_sort_config<default_config, default_config,
                        radix_sort_onesweep_config<kernel_config<512, 16>, kernel_config<1024, 16>, 8,
                                                   block_radix_rank_algorithm::match>>>(
      "onesweep 8 bits, 1024x16", in, out, n, bits);
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
