// Host-side checks of the native layer, built with AddressSanitizer + UBSan
// (tests/test_native_host.py): the Philox generator shared by every sampler
// (known-answer test + values supplied by the NumPy mirror on argv/stdin), and
// the argument validation of the extern "C" launchers, which must reject bad
// shapes before any HIP call (so this runs on a machine without a GPU).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "dalgo/common.h"
#include "launchers.h"

using namespace dalgo;

static int failures = 0;
#define CHECK(cond)                                                     \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #cond, __LINE__); \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

int main() {
  // Philox4x32-10 known answer (Salmon et al. / Random123 kat vector 0)
  u32x4 r = philox4x32_10(u32x4{0, 0, 0, 0}, 0, 0);
  CHECK(r.x == 0x6627e8d5u && r.y == 0xe169c58du && r.z == 0xbc57ac4cu && r.w == 0x9b00dbd8u);
  // stream of (seed, stream, block) triples from stdin: print the 4 words each
  unsigned long long seed, stream, block;
  while (std::scanf("%llu %llu %llu", &seed, &stream, &block) == 3) {
    u32x4 v = philox_block(seed, stream, block);
    std::printf("%u %u %u %u\n", v.x, v.y, v.z, v.w);
  }
  // launcher validation: rejected before touching the device
  unsigned long long cnt = 0;
  CHECK(dalgo_tc_step(nullptr, 128, nullptr, nullptr, 128, 100, 128, 0, &cnt, nullptr) ==
        hipErrorInvalidValue);                                 // npad not a multiple of 128
  CHECK(dalgo_tc_step(nullptr, 120, nullptr, nullptr, 128, 128, 128, 0, &cnt, nullptr) ==
        hipErrorInvalidValue);                                 // lda not a multiple of 16
  void* bufs[9] = {};
  uint32_t* ep = reinterpret_cast<uint32_t*>(&cnt);             // never dereferenced: rejected first
  CHECK(dalgo_xgmi_allreduce(nullptr, nullptr, 10, 0, 9, bufs, 16, ep, nullptr, 1.0, nullptr, 0, 0, 0, 0, 0.f, 0.f, 0.f, nullptr, nullptr) ==
        hipErrorInvalidValue);                                 // > 8 ranks
  CHECK(dalgo_xgmi_allreduce(nullptr, nullptr, 10, 0, 2, bufs, 16, nullptr, nullptr, 1.0, nullptr, 0, 0, 0, 0, 0.f, 0.f, 0.f, nullptr, nullptr) ==
        hipErrorInvalidValue);                                 // no device epoch counter
  CHECK(dalgo_xgmi_allreduce(nullptr, nullptr, 32, 0, 2, bufs, 16, ep, nullptr, 1.0, nullptr, 0, 0, 0, 0, 0.f, 0.f, 0.f, nullptr, nullptr) ==
        hipErrorInvalidValue);                                 // vector larger than the slot
  CHECK(dalgo_xgmi_allreduce(nullptr, nullptr, 8, 0, 2, bufs, 16, ep, nullptr, 1.0, nullptr, 0, 0, 0, 0, 0.f, 0.f, 0.f, nullptr, nullptr) ==
        hipErrorInvalidValue);                                 // unmapped peer buffer
  CHECK(dalgo_xgmi_buffer_bytes(4096) == 256 + 2 * 8 * 4096 * sizeof(float));
  CHECK(dalgo_lr_max_cols(1) == 2048 && dalgo_lr_max_cols(0) == 1024);
  if (failures) {
    std::fprintf(stderr, "%d host check(s) failed\n", failures);
    return 1;
  }
  std::fprintf(stderr, "host checks passed\n");
  return 0;
}
