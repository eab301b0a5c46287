// K11: one-shot all-reduce of small f32 vectors over xGMI peer memory.
//
// Replaces the treeAggregate / reduce call sites of the SGD family
// (optimization/ssgd.py:99-103, ma.py:104, bmuf.py:109, easgd.py:104) for the
// latency-bound case: the SSGD bucket [g || count] is ~4 KB, where a ring
// all-reduce pays 2(W-1) link latencies. xGMI on MI355X is point-to-point (every
// GPU has a direct link to each of its 7 peers), so one hop suffices:
//
//   1. every rank PUSHES its vector into slot [phase][rank] of every rank's
//      exchange buffer (remote stores travel the direct link; all 7 links busy),
//   2. system-scope fence, then one flag word per destination: flags[phase][rank]
//      = epoch,
//   3. wait for the W flags of this epoch in the LOCAL buffer, then sum the W slots
//      in rank order — every rank adds the same numbers in the same order, so the
//      result is bitwise identical on all ranks (replicated-model invariant).
//
// The exchange buffers are allocated uncached (hipDeviceMallocUncached) and shared
// with hipIpcGetMemHandle / hipIpcOpenMemHandle, so remote stores land in the
// owner's HBM and the owner's loads never hit a stale cache line. Two phases
// (epoch & 1) make back-to-back calls safe: a rank can run at most one call
// ahead of a peer, and that call writes the other phase. Epochs start at 1 and
// only ever increase, so flags need no reset. The wait is bounded (wall clock):
// on timeout the kernel sets *err and finishes, never hangs the GPU.
#include "dalgo/common.h"
#include <cstring>

namespace dalgo {

constexpr int kXgMaxRanks = 8;
constexpr int kXgHeaderBytes = 256;   // flags[2][8] u32, padded

struct XgParams {
  uint8_t* bufs[kXgMaxRanks];   // exchange buffer of every rank (own one included)
  const float* in;
  float* out;
  int n, rank, world, slot;     // slot = floats per (phase, source) slot
  uint32_t epoch;
  unsigned* err;
  long long timeout_ticks;      // s_memrealtime ticks (100 MHz)
  // optional fused K8 (SSGD / full-batch GD on the [g (ldw) || count] bucket):
  // W[0..nw) is updated from the reduced sums and the bucket is left zeroed for
  // the next atomic-epilogue K1 (one launch instead of all-reduce + update)
  float* W;                     // nullptr: plain all-reduce
  int nw, cidx, upd_mode, upd_reg;   // cidx: index of the count in the vector
  float eta, lam, reg_alpha;
  double* count_acc;
};

__device__ __forceinline__ float xg_update(float w, float g, float c, const XgParams& p) {
  if (p.upd_mode == 1) return w - p.eta * g;                    // GD: sum, not mean
  const float gm = c > 0.f ? g / c : 0.f;
  float r = 0.f;
  const float sg = (w > 0.f) ? 1.f : (w < 0.f ? -1.f : 0.f);
  if (p.upd_reg == 1) r = w;
  else if (p.upd_reg == 2) r = sg;
  else if (p.upd_reg == 3) r = p.reg_alpha * sg + (1.f - p.reg_alpha) * w;
  return w - p.eta * (gm + p.lam * r);
}

__device__ __forceinline__ uint32_t* xg_flags(uint8_t* b) { return reinterpret_cast<uint32_t*>(b); }
__device__ __forceinline__ float* xg_slot(uint8_t* b, int ph, int src, int slot) {
  return reinterpret_cast<float*>(b + kXgHeaderBytes) + ((int64_t)ph * kXgMaxRanks + src) * slot;
}

__global__ void __launch_bounds__(1024) xgmi_allreduce_kernel(XgParams p) {
  const int tid = threadIdx.x;
  const int ph = (int)(p.epoch & 1u);
  // 1. push: every destination gets this rank's vector (destinations rotated so the
  //    W-1 links are loaded evenly as the threads sweep)
  for (int k = 0; k < p.world; ++k) {
    const int r = (p.rank + k) % p.world;
    float* dst = xg_slot(p.bufs[r], ph, p.rank, p.slot);
    for (int i = tid; i < p.n; i += blockDim.x) dst[i] = p.in[i];
  }
  __threadfence_system();
  __syncthreads();
  // 2. publish: one flag per destination
  if (tid < p.world)
    __hip_atomic_store(&xg_flags(p.bufs[tid])[ph * kXgMaxRanks + p.rank], p.epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every source's flag of this epoch in the local buffer
  if (tid < p.world) {
    uint32_t* f = &xg_flags(p.bufs[p.rank])[ph * kXgMaxRanks + tid];
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != p.epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > p.timeout_ticks) {
        atomicOr(p.err, 1u);
        break;
      }
    }
  }
  __syncthreads();
  // 4. reduce in rank order (identical on every rank)
  uint8_t* mine = p.bufs[p.rank];
  auto reduced = [&](int i) {
    float s = 0.f;
    for (int r = 0; r < p.world; ++r) s += __builtin_nontemporal_load(xg_slot(mine, ph, r, p.slot) + i);
    return s;
  };
  if (p.W == nullptr) {
    for (int i = tid; i < p.n; i += blockDim.x) p.out[i] = reduced(i);
    return;
  }
  const float c = reduced(p.cidx);                 // the global minibatch size
  for (int i = tid; i < p.nw; i += blockDim.x) p.W[i] = xg_update(p.W[i], reduced(i), c, p);
  for (int i = tid; i < p.n; i += blockDim.x) p.out[i] = 0.f;
  if (tid == 0 && p.count_acc) p.count_acc[0] += (double)c;
}

}  // namespace dalgo

using namespace dalgo;

extern "C" {

size_t dalgo_xgmi_buffer_bytes(int slot_floats) {
  return kXgHeaderBytes + (size_t)2 * kXgMaxRanks * slot_floats * sizeof(float);
}

hipError_t dalgo_xgmi_alloc(size_t bytes, void** ptr) {
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  return hipMemset(*ptr, 0, bytes);
}

hipError_t dalgo_xgmi_free(void* ptr) { return hipFree(ptr); }

// handle: 64 opaque bytes (hipIpcMemHandle_t)
hipError_t dalgo_xgmi_get_handle(void* ptr, void* handle) {
  return hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle), ptr);
}

hipError_t dalgo_xgmi_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

hipError_t dalgo_xgmi_close(void* ptr) { return hipIpcCloseMemHandle(ptr); }

hipError_t dalgo_xgmi_allreduce(const float* in, float* out, int n, int rank, int world,
                                void* const* bufs, int slot, uint32_t epoch, unsigned* err,
                                double timeout_s, float* W, int nw, int cidx, int upd_mode,
                                int upd_reg, float eta, float lam, float reg_alpha,
                                double* count_acc, hipStream_t st) {
  if (W != nullptr && (cidx < 0 || cidx >= n || nw > cidx)) return hipErrorInvalidValue;
  if (world < 1 || world > kXgMaxRanks || rank < 0 || rank >= world || n < 0 || n > slot ||
      epoch == 0)
    return hipErrorInvalidValue;
  XgParams p{};
  for (int r = 0; r < world; ++r) {
    if (bufs[r] == nullptr) return hipErrorInvalidValue;
    p.bufs[r] = static_cast<uint8_t*>(bufs[r]);
  }
  p.in = in; p.out = out; p.n = n; p.rank = rank; p.world = world; p.slot = slot;
  p.epoch = epoch; p.err = err;
  p.timeout_ticks = (long long)(timeout_s * 1e8);
  p.W = W; p.nw = nw; p.cidx = cidx; p.upd_mode = upd_mode; p.upd_reg = upd_reg;
  p.eta = eta; p.lam = lam; p.reg_alpha = reg_alpha; p.count_acc = count_acc;
  hipLaunchKernelGGL(xgmi_allreduce_kernel, dim3(1), dim3(1024), 0, st, p);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
