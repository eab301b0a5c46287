// Device side of the K11 one-shot xGMI exchange, shared by the stand-alone
// all-reduce (csrc/kernels/xgmi_allreduce.hip) and the tail of the LR gradient
// kernel (csrc/kernels/lr_grad.hip), so both walk the same epoch / phase
// sequence on the same IPC-mapped buffers. Protocol: see xgmi_allreduce.hip.
#pragma once
#include "dalgo/common.h"

namespace dalgo {

constexpr int kXgMaxRanks = 8;
constexpr int kXgHeaderBytes = 256;   // flags[2][8] u32, padded

struct XgLink {
  uint8_t* bufs[kXgMaxRanks];   // exchange buffer of every rank (own one included)
  int rank, world, slot;        // slot = floats per (phase, source) slot
  // Device-resident exchange epoch: the last epoch this rank used (0 before the first
  // exchange; identical on all ranks). A launch with k exchanges reads it once, uses
  // base + 1 .. base + k and stores base + k when its last exchange is done. No launch
  // argument changes from step to step, so the launches can be captured in a hipGraph
  // and replayed (the epochs advance on the device). 2^32 - 1 exchanges per run.
  uint32_t* epoch_dev;
  unsigned* err;                // set to 1 if a wait timed out
  long long timeout_ticks;      // s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ uint32_t xg_epoch_base(const XgLink& L) {
  return __hip_atomic_load(L.epoch_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void xg_epoch_store(const XgLink& L, uint32_t e) {
  __hip_atomic_store(L.epoch_dev, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// SSGD (mode 0: mean + regulariser) / full-batch GD (mode 1: sum) update rule
struct XgUpdate {
  int mode, reg;
  float eta, lam, reg_alpha;
};

__device__ __forceinline__ uint32_t* xg_flags(uint8_t* b) { return reinterpret_cast<uint32_t*>(b); }
__device__ __forceinline__ float* xg_slot(uint8_t* b, int ph, int src, int slot) {
  return reinterpret_cast<float*>(b + kXgHeaderBytes) + ((int64_t)ph * kXgMaxRanks + src) * slot;
}

__device__ __forceinline__ float xg_update(float w, float g, float c, const XgUpdate& u) {
  if (u.mode == 1) return w - u.eta * g;                       // GD: sum, not mean
  const float gm = c > 0.f ? g / c : 0.f;
  const float sg = (w > 0.f) ? 1.f : (w < 0.f ? -1.f : 0.f);
  float r = 0.f;
  if (u.reg == 1) r = w;
  else if (u.reg == 2) r = sg;
  else if (u.reg == 3) r = u.reg_alpha * sg + (1.f - u.reg_alpha) * w;
  return w - u.eta * (gm + u.lam * r);
}

// Block-wide: push get(i), i < n, into slot [phase][rank] of every rank's buffer,
// publish one flag per destination and wait (bounded) until all W sources of this
// epoch have landed in the local buffer. Every thread of the block must call it.
// `epoch` is passed separately (a persistent launch walks base + 1, base + 2, ...
// without copying the link, whose pointer array would otherwise land in scratch).
template <class Get>
__device__ __forceinline__ void xg_push_publish_wait(const XgLink& L, uint32_t epoch, int n, Get get) {
  const int tid = threadIdx.x;
  const int ph = (int)(epoch & 1u);
  for (int k = 0; k < L.world; ++k) {            // destinations rotated: links evenly loaded
    const int r = (L.rank + k) % L.world;
    float* dst = xg_slot(L.bufs[r], ph, L.rank, L.slot);
    for (int i = tid; i < n; i += blockDim.x) dst[i] = get(i);
  }
  // Ordering (HIP memory model, not a gfx9 side effect): every thread's slot stores are
  // made visible at system scope by its own fence; the barrier then orders them before
  // the flag-storing thread, whose flag store is itself a SYSTEM-scope RELEASE (fence
  // cumulativity covers the other threads' stores it synchronised with through the
  // barrier). The peer's ACQUIRE load of the flag below pairs with it.
  __threadfence_system();
  __syncthreads();
  if (tid < L.world)
    __hip_atomic_store(&xg_flags(L.bufs[tid])[ph * kXgMaxRanks + L.rank], epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < L.world) {
    uint32_t* f = &xg_flags(L.bufs[L.rank])[ph * kXgMaxRanks + tid];
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > L.timeout_ticks) {
        atomicOr(L.err, 1u);
        break;
      }
    }
  }
  __syncthreads();
}

// rank-ordered sum of element i over the W landed slots (identical on every rank)
__device__ __forceinline__ float xg_sum(const XgLink& L, uint32_t epoch, int i) {
  uint8_t* mine = L.bufs[L.rank];
  const int ph = (int)(epoch & 1u);
  float s = 0.f;
  for (int r = 0; r < L.world; ++r) s += __builtin_nontemporal_load(xg_slot(mine, ph, r, L.slot) + i);
  return s;
}

}  // namespace dalgo
