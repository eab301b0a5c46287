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
//   2. system-scope fence, then one flag word per destination (a system-scope release):
//      flags[phase][rank] = epoch (device-resident counter, see dalgo/xgmi.h),
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
#include "dalgo/xgmi.h"
#include <cstring>

namespace dalgo {

struct XgParams {
  XgLink L;
  const float* in;
  float* out;
  int n;
  // optional fused K8 (SSGD / full-batch GD on the [g (ldw) || count] bucket):
  // W[0..nw) is updated from the reduced sums and the bucket is left zeroed for
  // the next atomic-epilogue K1 (one launch instead of all-reduce + update)
  float* W;                     // nullptr: plain all-reduce
  int nw, cidx;                 // cidx: index of the count in the vector
  XgUpdate u;
  double* count_acc;
};

__global__ void __launch_bounds__(1024) xgmi_allreduce_kernel(XgParams p) {
  const int tid = threadIdx.x;
  // one exchange: epoch = device base + 1 (read by every thread before any store below:
  // the wait inside xg_push_publish_wait ends with a block barrier)
  const uint32_t e = xg_epoch_base(p.L) + 1u;
  xg_push_publish_wait(p.L, e, p.n, [&](int i) { return p.in[i]; });
  if (p.W == nullptr) {
    for (int i = tid; i < p.n; i += blockDim.x) p.out[i] = xg_sum(p.L, e, i);
  } else {
    const float c = xg_sum(p.L, e, p.cidx);             // the global minibatch size
    for (int i = tid; i < p.nw; i += blockDim.x) p.W[i] = xg_update(p.W[i], xg_sum(p.L, e, i), c, p.u);
    for (int i = tid; i < p.n; i += blockDim.x) p.out[i] = 0.f;
    if (tid == 0 && p.count_acc) p.count_acc[0] += (double)c;
  }
  if (tid == 0) xg_epoch_store(p.L, e);
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
                                void* const* bufs, int slot, uint32_t* epoch_dev, unsigned* err,
                                double timeout_s, float* W, int nw, int cidx, int upd_mode,
                                int upd_reg, float eta, float lam, float reg_alpha,
                                double* count_acc, hipStream_t st) {
  if (W != nullptr && (cidx < 0 || cidx >= n || nw > cidx)) return hipErrorInvalidValue;
  if (world < 1 || world > kXgMaxRanks || rank < 0 || rank >= world || n < 0 || n > slot ||
      epoch_dev == nullptr)
    return hipErrorInvalidValue;
  XgParams p{};
  for (int r = 0; r < world; ++r) {
    if (bufs[r] == nullptr) return hipErrorInvalidValue;
    p.L.bufs[r] = static_cast<uint8_t*>(bufs[r]);
  }
  p.L.rank = rank; p.L.world = world; p.L.slot = slot; p.L.epoch_dev = epoch_dev; p.L.err = err;
  p.L.timeout_ticks = (long long)(timeout_s * 1e8);
  p.in = in; p.out = out; p.n = n;
  p.W = W; p.nw = nw; p.cidx = cidx;
  p.u = XgUpdate{upd_mode, upd_reg, eta, lam, reg_alpha};
  p.count_acc = count_acc;
  hipLaunchKernelGGL(xgmi_allreduce_kernel, dim3(1), dim3(1024), 0, st, p);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
