// K9 sparse mode: semi-naive transitive-closure round on a device hash set.
//
// Reference: graph_computation/transitive_closure.py:31-40 — every round joins the
// path RDD with the reversed edges (`paths.join(edges)`, :35: a path y ~> z and an
// edge x -> y give x ~> z), then `union(...).distinct()` (:37) and a `count()` (:38)
// until the count stops changing. Spark shuffles both sides and sorts / hashes the
// union every round.
//
// Here one rank owns the paths whose target z satisfies z % world == rank (the edges
// are replicated), stored as 64-bit keys (x << 32 | z) in two device structures:
//   keys  : append-only array of every path found so far; the paths added by the last
//           round are the contiguous tail [d0, d1) = the semi-naive frontier (delta);
//   table : open-addressing hash set (linear probing, capacity a power of two, load
//           kept <= 1/2 by the host) holding the same keys.
// One round = tcs_degree (in-degree of each frontier path's source y -> frontier
// candidate counts, scanned on the host side) + tcs_expand over the candidates:
// candidate c of frontier path i is (in_src[in_ptr[y] + j], z); it is inserted with a
// 64-bit compare-and-swap, and only the thread whose CAS claimed an empty slot appends
// the key (wave-aggregated atomic on the key counter). Dedup, the membership test
// against all earlier paths and the merge into P are that single CAS: nothing is ever
// sorted, and the work per round is proportional to the frontier's candidates.
//
// Load balance over power-law in-degrees: each block owns a contiguous range of
// CANDIDATES (not frontier paths); the block finds the frontier paths that cover its
// range with two binary searches over the exclusive candidate prefix, stages that
// slice of the prefix in LDS and every thread binary-searches its candidate there
// (global-memory search only when a block's range spans more than kLdsSpan paths).
//
// Coherence: the table is touched only by device-scope atomics (relaxed agent-scope
// loads while probing, CAS to claim), which are coherent across the 8 XCDs' L2s; the
// appended keys are plain stores read by the NEXT launch (kernel boundary).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dalgo {
namespace {

constexpr uint64_t kEmpty = ~0ull;
constexpr int kThreads = 256;
constexpr int kPerThread = 8;                       // candidates per thread
constexpr int kBlockCands = kThreads * kPerThread;  // 2048 candidates per block
constexpr int kLdsSpan = 2048;                      // prefix entries staged per block

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// true iff this call inserted `key` (it was absent). Bounded probe sequence: the host
// keeps the load <= 1/2, so a full sweep means corruption -> error word, no hang.
__device__ __forceinline__ bool hs_insert(uint64_t* table, uint64_t mask, uint64_t key,
                                          unsigned* err) {
  uint64_t h = mix64(key) & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    uint64_t cur = __hip_atomic_load(&table[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return false;
    if (cur == kEmpty) {
      uint64_t expected = kEmpty;
      if (__hip_atomic_compare_exchange_strong(&table[h], &expected, key, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        return true;
      if (expected == key) return false;
    }
    h = (h + 1) & mask;
  }
  atomicOr(err, 1u);
  return false;
}

// Wave-aggregated append of the keys whose lanes have `take` set.
__device__ __forceinline__ void wave_append(bool take, uint64_t key, uint64_t* keys,
                                            unsigned long long* n_keys, uint64_t cap,
                                            unsigned* err) {
  const uint64_t mask = __ballot(take);
  if (mask == 0) return;
  const int lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(n_keys, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader);
  if (take) {
    const uint64_t below = mask & ((lane == 0) ? 0ull : (~0ull >> (64 - lane)));
    const uint64_t pos = base + (uint64_t)__popcll(below);
    if (pos < cap) keys[pos] = key;
    else atomicOr(err, 2u);
  }
}

// first index i in [lo, hi) with pre[i] > c (pre non-decreasing), hi if none
template <typename P>
__device__ __forceinline__ int64_t upper_bound(const P* pre, int64_t lo, int64_t hi, int64_t c) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)pre[mid] <= c) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// deg[i] = in-degree of the source y of frontier path keys[d0 + i]
__global__ void __launch_bounds__(kThreads)
tcs_degree_kernel(const uint64_t* __restrict__ keys, int64_t d0, int64_t nd,
                  const int64_t* __restrict__ in_ptr, int64_t* __restrict__ deg) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nd;
       i += (int64_t)gridDim.x * kThreads) {
    const uint64_t y = keys[d0 + i] >> 32;
    deg[i] = in_ptr[y + 1] - in_ptr[y];
  }
}

// Candidates [c_lo, c_hi) of the frontier keys[d0, d0 + nd); excl[i] = first candidate
// of frontier path i (excl[nd] = total). New keys are appended at *n_keys.
__global__ void __launch_bounds__(kThreads)
tcs_expand_kernel(const uint64_t* __restrict__ fkeys, int64_t nd, const int64_t* __restrict__ excl,
                  int64_t c_lo, int64_t c_hi, const int64_t* __restrict__ in_ptr,
                  const int32_t* __restrict__ in_src, uint64_t* table, uint64_t mask,
                  uint64_t* keys, unsigned long long* n_keys, uint64_t cap, unsigned* err) {
  __shared__ int64_t s_pre[kLdsSpan + 1];
  __shared__ int64_t s_span[2];
  const int64_t b0 = c_lo + (int64_t)blockIdx.x * kBlockCands;
  if (b0 >= c_hi) return;
  const int64_t b1 = (b0 + kBlockCands < c_hi) ? b0 + kBlockCands : c_hi;
  if (threadIdx.x == 0) {
    // frontier paths covering [b0, b1): i0 = last i with excl[i] <= b0, i1 likewise for b1-1
    s_span[0] = upper_bound(excl, 0, nd + 1, b0) - 1;
    s_span[1] = upper_bound(excl, 0, nd + 1, b1 - 1) - 1;
  }
  __syncthreads();
  const int64_t i0 = s_span[0], i1 = s_span[1];
  const int64_t span = i1 - i0 + 2;   // excl[i0 .. i1 + 1]
  const bool in_lds = span <= kLdsSpan + 1;
  if (in_lds) {
    for (int64_t t = threadIdx.x; t < span; t += kThreads) s_pre[t] = excl[i0 + t];
    __syncthreads();
  }
#pragma unroll 2
  for (int k = 0; k < kPerThread; ++k) {
    const int64_t c = b0 + (int64_t)k * kThreads + threadIdx.x;
    bool take = false;
    uint64_t nk = 0;
    if (c < b1) {
      int64_t i, first;
      if (in_lds) {
        const int64_t r = upper_bound(s_pre, 0, span, c - 0) - 1;   // s_pre[r] <= c
        i = i0 + r;
        first = s_pre[r];
      } else {
        i = upper_bound(excl, i0, i1 + 2, c) - 1;
        first = excl[i];
      }
      const uint64_t key = fkeys[i];
      const uint64_t y = key >> 32;
      const uint64_t z = key & 0xffffffffull;
      const uint64_t x = (uint64_t)(uint32_t)in_src[in_ptr[y] + (c - first)];
      nk = (x << 32) | z;
      take = hs_insert(table, mask, nk, err);
    }
    wave_append(take, nk, keys, n_keys, cap, err);
  }
}

// Insert src[0, n) (duplicates allowed); append the new ones when `append` is set
// (initial edge set: dedup + path array in one pass; rehash: append = 0).
__global__ void __launch_bounds__(kThreads)
tcs_insert_kernel(const uint64_t* __restrict__ src, int64_t n, uint64_t* table, uint64_t mask,
                  int append, uint64_t* keys, unsigned long long* n_keys, uint64_t cap,
                  unsigned* err) {
  for (int64_t base = (int64_t)blockIdx.x * kThreads; base < n;
       base += (int64_t)gridDim.x * kThreads) {
    const int64_t i = base + threadIdx.x;
    bool take = false;
    uint64_t k = 0;
    if (i < n) {
      k = src[i];
      take = hs_insert(table, mask, k, err);
    }
    if (append) wave_append(take, k, keys, n_keys, cap, err);
  }
}

}  // namespace
}  // namespace dalgo

extern "C" {

hipError_t dalgo_tcs_degree(const uint64_t* keys, int64_t d0, int64_t nd, const int64_t* in_ptr,
                            int64_t* deg, hipStream_t st) {
  if (nd <= 0) return hipSuccess;
  int64_t g = (nd + dalgo::kThreads - 1) / dalgo::kThreads;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(dalgo::tcs_degree_kernel, dim3((unsigned)g), dim3(dalgo::kThreads), 0, st,
                     keys, d0, nd, in_ptr, deg);
  return hipGetLastError();
}

hipError_t dalgo_tcs_expand(const uint64_t* fkeys, int64_t nd, const int64_t* excl, int64_t c_lo,
                            int64_t c_hi, const int64_t* in_ptr, const int32_t* in_src,
                            uint64_t* table, uint64_t mask, uint64_t* keys,
                            unsigned long long* n_keys, uint64_t cap, unsigned* err,
                            hipStream_t st) {
  if (c_hi <= c_lo || nd <= 0) return hipSuccess;
  const int64_t g = (c_hi - c_lo + dalgo::kBlockCands - 1) / dalgo::kBlockCands;
  if (g > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dalgo::tcs_expand_kernel, dim3((unsigned)g), dim3(dalgo::kThreads), 0, st,
                     fkeys, nd, excl, c_lo, c_hi, in_ptr, in_src, table, mask, keys, n_keys, cap,
                     err);
  return hipGetLastError();
}

hipError_t dalgo_tcs_insert(const uint64_t* src, int64_t n, uint64_t* table, uint64_t mask,
                            int append, uint64_t* keys, unsigned long long* n_keys, uint64_t cap,
                            unsigned* err, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t g = (n + dalgo::kThreads - 1) / dalgo::kThreads;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(dalgo::tcs_insert_kernel, dim3((unsigned)g), dim3(dalgo::kThreads), 0, st,
                     src, n, table, mask, append, keys, n_keys, cap, err);
  return hipGetLastError();
}

}  // extern "C"
