// Native adjacency build of the PageRank job (graph_computation/pagerank.py:41,44:
// ``links.distinct().groupByKey().cache()`` + ``count()``), gfx950.
//
// The K4b layout (pr_binned.hip) wants the deduplicated edges ordered by (source chunk,
// destination, source): one 64-bit key per edge = block | local destination | source
// offset in its 8192-source block, so ONE radix sort (rocPRIM onesweep over only the
// key's bits) puts the edges in layout order, and the decode pass skips the duplicates
// (a distinct edge = the last copy of its key). The passes around it are single sweeps:
//   degree   -- raw out-degree of the input edges (degree relabeling): ids partitioned
//               on their high bits by a 2-pass radix sort, one LDS histogram per bucket;
//               on one rank the (src, dst) pairs themselves are partitioned (packed u64),
//               so the key pass's source relabeling reads one 32 KB table slice per bucket;
//   keys     -- relabel, keep this rank's destinations, map sources to the [own | ghost]
//               index space and pack the key (two-phase compaction: count, write);
//   decode   -- per distinct edge the u16 source offset + entry-end bit, the entry list
//               (end edge, block, destination) and the deduplicated out-degree of every
//               source (LDS-privatised histogram per 8192-source block, no global atomic
//               per edge);
//   entries  -- run-start bits (a run = the entries of one (block, destination bin)),
//               chunk starts, bin-major destination offsets and tile starts, from the
//               (block, bin) cell matrix: row scans give each run's first entry and index,
//               column scans its bin-major position (gb_cell_* kernels).
// Everything else (per-chunk / per-run tables, a few thousand to a few million rows) is
// torch on the device (dalgo/ops/graph.py::build_blocked_native).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdint>
#include <cstdlib>

#include "dalgo/common.h"
#include "launchers.h"

namespace dalgo {
namespace {

constexpr int kSpan = 8192;          // sources per block (pr_binned.hip kPbSpan / graph.SRC_SPAN)
constexpr int kSpanBits = 13;

// ---------------------------------------------------------------------------- degree
__global__ void __launch_bounds__(256) gb_degree_kernel(const int32_t* __restrict__ ids, int64_t n,
                                                        uint32_t* __restrict__ deg) {
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      const int4 v = *reinterpret_cast<const int4*>(ids + i);
      atomicAdd(deg + v.x, 1u);
      atomicAdd(deg + v.y, 1u);
      atomicAdd(deg + v.z, 1u);
      atomicAdd(deg + v.w, 1u);
    } else {
      for (int64_t j = i; j < n; ++j) atomicAdd(deg + ids[j], 1u);
    }
  }
}

// degree by partition: the ids sorted on their HIGH bits only (2 radix passes at 2^26
// ids), so every bucket of 2^kBktBits consecutive ids is one contiguous range; one block
// per bucket counts it in an LDS histogram and adds it to deg (each entry owned by one
// block: no global atomics)
constexpr int kBktBits = 13;

// the id of an element: u32 ids as they are; u64 packed edges (src << 32 | dst): src
__device__ __forceinline__ uint32_t gb_id(uint32_t x) { return x; }
__device__ __forceinline__ uint32_t gb_id(uint64_t x) { return (uint32_t)(x >> 32); }

template <typename E>
__global__ void __launch_bounds__(256) gb_bucket_starts_kernel(const E* __restrict__ sorted, int64_t n,
                                                               int nb, int64_t* __restrict__ starts) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b > nb) return;
  if (b == nb) { starts[b] = n; return; }
  int64_t lo = 0, hi = n;   // first i with (id(sorted[i]) >> kBktBits) >= b
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)(gb_id(sorted[mid]) >> kBktBits) < b) lo = mid + 1;
    else hi = mid;
  }
  starts[b] = lo;
}

template <typename E>
__global__ void __launch_bounds__(256) gb_bucket_degree_kernel(const E* __restrict__ sorted,
                                                               const int64_t* __restrict__ starts,
                                                               int32_t* __restrict__ deg) {
  __shared__ uint32_t hist[1 << kBktBits];
  for (int j = threadIdx.x; j < (1 << kBktBits); j += 256) hist[j] = 0u;
  __syncthreads();
  const int64_t b = blockIdx.x, i0 = starts[b], i1 = starts[b + 1];
  constexpr uint32_t mask = (1u << kBktBits) - 1u;
  if constexpr (sizeof(E) == 4) {
    // 16-B loads from the first aligned position on
    const int64_t a0 = min(i1, (i0 + 3) & ~(int64_t)3);
    for (int64_t i = i0 + threadIdx.x; i < a0; i += 256) atomicAdd(&hist[gb_id(sorted[i]) & mask], 1u);
    const int64_t nv = (i1 - a0) >> 2;
    const uint4* v = reinterpret_cast<const uint4*>(sorted + a0);
    for (int64_t q = threadIdx.x; q < nv; q += 256) {
      const uint4 x = v[q];
      atomicAdd(&hist[x.x & mask], 1u);
      atomicAdd(&hist[x.y & mask], 1u);
      atomicAdd(&hist[x.z & mask], 1u);
      atomicAdd(&hist[x.w & mask], 1u);
    }
    for (int64_t i = a0 + (nv << 2) + threadIdx.x; i < i1; i += 256) atomicAdd(&hist[gb_id(sorted[i]) & mask], 1u);
  } else {
    // 4 independent loads in flight per thread before their LDS atomics
    constexpr int U = 4;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += 256 * U) {
      E w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = i + u * 256 < i1 ? sorted[i + u * 256] : E(0);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (i + u * 256 < i1) atomicAdd(&hist[gb_id(w[u]) & mask], 1u);
    }
  }
  __syncthreads();
  int32_t* d = deg + (b << kBktBits);
  for (int j = threadIdx.x; j < (1 << kBktBits); j += 256) d[j] += (int32_t)hist[j];
}

// packed edges partitioned on the source: the source relabelled in place (the gathers of
// one block stay inside a few 32 KB slices of new_id)
// 4 edges per thread per step (two 16-B loads, 4 independent gathers, two 16-B stores):
// one edge per thread serialised load -> gather -> store (7.8 ms at scale 26, r5_45)
__global__ void __launch_bounds__(256) gb_relabel_src_kernel(uint64_t* __restrict__ packed, int64_t n,
                                                             const int32_t* __restrict__ new_id) {
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      uint4* p4 = reinterpret_cast<uint4*>(packed + i);
      uint4 a = p4[0], b = p4[1];                       // (dst, src) word pairs
      a.y = (uint32_t)new_id[a.y];
      a.w = (uint32_t)new_id[a.w];
      b.y = (uint32_t)new_id[b.y];
      b.w = (uint32_t)new_id[b.w];
      p4[0] = a;
      p4[1] = b;
    } else {
      for (int64_t j = i; j < n; ++j) {
        const uint64_t w = packed[j];
        packed[j] = ((uint64_t)(uint32_t)new_id[(uint32_t)(w >> 32)] << 32) | (w & 0xffffffffull);
      }
    }
  }
}

// the same over edges partitioned on src >> kBktBits (gb_degree_packed's output): one block
// per 8192-source bucket stages its 32 KB slice of new_id in LDS and relabels the bucket's
// edges from there; the global gathers of the flat kernel made it 7.8 ms at scale 26
// (r5_42). The bucket ranges come from a SEPARATE launch (gb_bucket_starts_kernel): a
// binary search inside this kernel would read words other blocks are rewriting (the r5_60
// .. r5_64 race that changed the scale-26 edge set run to run)
__global__ void __launch_bounds__(256) gb_relabel_bucket_kernel(uint64_t* __restrict__ packed,
                                                                const int64_t* __restrict__ starts,
                                                                const int32_t* __restrict__ new_id, int64_t nv) {
  __shared__ int32_t s_id[1 << kBktBits];
  const int64_t b = blockIdx.x;
  const int64_t r0 = starts[b], r1 = starts[b + 1];
  const int64_t v0 = b << kBktBits;
  for (int j = threadIdx.x; j < (1 << kBktBits); j += 256) s_id[j] = v0 + j < nv ? new_id[v0 + j] : 0;
  __syncthreads();
  constexpr int U = 4;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += 256 * U) {
    uint64_t w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = i + u * 256 < r1 ? packed[i + u * 256] : 0ull;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < r1) {
        const uint32_t sl = (uint32_t)(w[u] >> 32) & ((1u << kBktBits) - 1u);
        packed[i + u * 256] = ((uint64_t)(uint32_t)s_id[sl] << 32) | (w[u] & 0xffffffffull);
      }
  }
}

// packed edges: out[i] = src[i] << 32 | dst[i]
__global__ void __launch_bounds__(256) gb_pack_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                                      int64_t n, uint64_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    out[i] = ((uint64_t)(uint32_t)src[i] << 32) | (uint64_t)(uint32_t)dst[i];
}

// ---------------------------------------------------------------------------- owners
// The sharded build's shuffle (graph_computation/pagerank.py:41 ``groupByKey`` over W
// ranks): every rank relabels its E/W input edges through new_id and groups them by the
// rank that owns the destination (owner = dst / sl) for one all_to_all. Phase 0 relabels
// and packs (src << 32 | dst) at the edge's own position of a scratch array (the only
// random new_id gathers) and counts the block's edges per owner; phase 2 re-reads the
// packed words and scatters them owner-major at the scanned offsets. Per-owner counting
// is wave-aggregated (one LDS atomic per distinct owner in a wave, <= W per step).
// The phase-0 gathers dominate (5.2 of the 5.9 ms at the W = 8 share, 134M edges: ~55 G
// random new_id reads/s, profiles/round6/r6_23); relabelling in 2-4 id-range passes first, so
// that each pass gathers from a 1/P slice of new_id, was slower (7.6-8.1 ms, r6_24).
// Blocks walk the edges grid-stride in 1024-edge steps (block b: steps b, b + G, ...), so the
// edges in flight at any moment are one ~G * 1024-edge window: over destination-partitioned
// input (the source-bucketed path) that window's destinations come from one or two 1 MB
// slices of new_id, which every XCD's L2 then holds (16384-edge blocks put ~32 slices in
// flight on every XCD). The scatter walks the same steps per block, so the (owner, block)
// counts of the first pass place its words.
constexpr int kOwnStep = 1024;       // edges per block step (256 threads x 4)
constexpr int kOwnMax = 64;          // largest world size

// Logical block of hardware block b of g: blocks b and b + 8 share an XCD (round-robin
// dealing, observed), so the XCD of b % 8 == x gets the consecutive logical blocks
// [x * (g / 8) + min(x, g % 8), ...): within each g-step window an XCD walks its own
// contiguous eighth, and its L2 holds one eighth of the window's new_id slices. A bijection
// for any g; placement only affects speed.
__device__ __forceinline__ int64_t gb_xcd_block(int64_t b, int64_t g) {
  const int64_t x = b & 7, i = b >> 3, per = g >> 3, rem = g & 7;
  return x * per + (x < rem ? x : rem) + i;
}

__device__ __forceinline__ int gb_owner_slot(int o, bool valid, int* s_cnt, bool want_base, int lane) {
  uint64_t act = __ballot(valid);
  int mine = 0;
  while (act) {
    const int leader = __ffsll((long long)act) - 1;
    const int ol = __shfl(o, leader);
    const uint64_t m = __ballot(valid && o == ol);
    int base = 0;
    if (lane == leader) base = atomicAdd(&s_cnt[ol], __popcll(m));
    if (want_base) {
      base = __shfl(base, leader);
      if (valid && o == ol) mine = base + __popcll(m & ((1ull << lane) - 1ull));
    }
    act &= ~m;
  }
  return mine;
}

__global__ void __launch_bounds__(256) gb_owner_count_kernel(const int32_t* __restrict__ src,
                                                             const int32_t* __restrict__ dst, int64_t n,
                                                             const int32_t* __restrict__ new_id, uint32_t sl,
                                                             int world, uint64_t* __restrict__ tmp,
                                                             int64_t* __restrict__ counts) {
  __shared__ int s_cnt[kOwnMax];
  if (threadIdx.x < kOwnMax) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t r1 = n;
  // src == nullptr: the edges are already packed in tmp with relabelled sources (the
  // source-bucketed path, gb_relabel_src + a destination-bit partition): only the
  // destinations are relabelled, from the L2-resident new_id slice of their bucket, in place
  const bool packed_in = src == nullptr;
  const int64_t lb = gb_xcd_block(blockIdx.x, gridDim.x);
  for (int64_t i = (lb * 256 + threadIdx.x) * 4; i < r1; i += (int64_t)gridDim.x * kOwnStep) {
    int32_t s4[4], d4[4];
    bool in[4];
    if (packed_in) {
      uint64_t w[4];
      if (i + 4 <= r1) {                       // 16-B aligned (binding checks the base)
        const uint4 a = *reinterpret_cast<const uint4*>(tmp + i);
        const uint4 b = *reinterpret_cast<const uint4*>(tmp + i + 2);
        w[0] = ((uint64_t)a.y << 32) | a.x; w[1] = ((uint64_t)a.w << 32) | a.z;
        w[2] = ((uint64_t)b.y << 32) | b.x; w[3] = ((uint64_t)b.w << 32) | b.z;
#pragma unroll
        for (int v = 0; v < 4; ++v) in[v] = true;
      } else {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          in[v] = i + v < r1;
          w[v] = in[v] ? tmp[i + v] : 0ull;
        }
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        s4[v] = (int32_t)(w[v] >> 32);
        d4[v] = (int32_t)(uint32_t)w[v];
      }
      if (new_id) {
#pragma unroll
        for (int v = 0; v < 4; ++v) d4[v] = in[v] ? new_id[d4[v]] : 0;
      }
    } else if (i + 4 <= r1) {
      const int4 a = *reinterpret_cast<const int4*>(src + i);
      const int4 b = *reinterpret_cast<const int4*>(dst + i);
      s4[0] = a.x; s4[1] = a.y; s4[2] = a.z; s4[3] = a.w;
      d4[0] = b.x; d4[1] = b.y; d4[2] = b.z; d4[3] = b.w;
#pragma unroll
      for (int v = 0; v < 4; ++v) in[v] = true;
    } else {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        in[v] = i + v < r1;
        s4[v] = in[v] ? src[i + v] : 0;
        d4[v] = in[v] ? dst[i + v] : 0;
      }
    }
    if (new_id && !packed_in) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        s4[v] = new_id[s4[v]];
        d4[v] = new_id[d4[v]];
      }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      if (in[v] && (new_id || !packed_in)) tmp[i + v] = ((uint64_t)(uint32_t)s4[v] << 32) | (uint32_t)d4[v];
      gb_owner_slot((int)((uint32_t)d4[v] / sl), in[v], s_cnt, false, lane);
    }
  }
  __syncthreads();
  if (threadIdx.x < world) counts[(int64_t)threadIdx.x * gridDim.x + lb] = s_cnt[threadIdx.x];
}

__global__ void __launch_bounds__(256) gb_owner_scatter_kernel(const uint64_t* __restrict__ tmp, int64_t n,
                                                               uint32_t sl, const int64_t* __restrict__ offsets,
                                                               uint64_t* __restrict__ out) {
  __shared__ int s_cur[kOwnMax];
  if (threadIdx.x < kOwnMax) s_cur[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t r1 = n;
  const int64_t lb = gb_xcd_block(blockIdx.x, gridDim.x);
  for (int64_t i = (lb * 256 + threadIdx.x) * 4; i < r1; i += (int64_t)gridDim.x * kOwnStep) {
    uint64_t w[4];
    bool in[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      in[v] = i + v < r1;
      w[v] = in[v] ? tmp[i + v] : 0ull;
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int o = (int)((uint32_t)w[v] / sl);
      const int pos = gb_owner_slot(o, in[v], s_cur, true, lane);
      if (in[v]) out[offsets[(int64_t)o * gridDim.x + lb] + pos] = w[v];
    }
  }
}

// byte map (one byte per id, 0 / 1) -> bitmap (one bit per id): 32 bytes per word
__global__ void __launch_bounds__(256) gb_bytes_to_bits_kernel(const uint4* __restrict__ marks, int64_t nw,
                                                               uint32_t* __restrict__ bits) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += stride) {
    const uint4 a = marks[2 * w], b = marks[2 * w + 1];
    const uint32_t q[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // bytes (0 / 1) of q[i] -> 4 bits: bit j of the nibble = byte j != 0
      const uint32_t v = q[i];
      const uint32_t nib = ((v & 0xffu) ? 1u : 0u) | (((v >> 8) & 0xffu) ? 2u : 0u) |
                           (((v >> 16) & 0xffu) ? 4u : 0u) | ((v >> 24) ? 8u : 0u);
      m |= nib << (4 * i);
    }
    bits[w] = m;
  }
}

// W > 1: the ghost list (sorted ids of the bitmap's set bits) at the words' exclusive
// popcount prefix, one thread per word (the torch form expanded every bit to an int64:
// ~15 ms of the W = 8 per-rank build share at scale 26)
__global__ void __launch_bounds__(256) gb_bitmap_ids_kernel(const uint32_t* __restrict__ bm, int64_t nw,
                                                            const int64_t* __restrict__ prefix,
                                                            int64_t* __restrict__ ids) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= nw) return;
  uint32_t b = bm[w];
  int64_t o = prefix[w];
  while (b) {
    const int t = __ffs((int)b) - 1;
    ids[o++] = w * 32 + t;
    b &= b - 1u;
  }
}

// deal of the ranked vertex list (pagerank_app.deal_ids, W > 1, every slice full): rank j
// goes to slice r = j % W (snake: odd rounds W - 1 .. 0), position j / W
// order[j] & id_mask = the j-th vertex (id_mask strips the sort key's degree bits)
__global__ void __launch_bounds__(256) gb_deal_kernel(const int64_t* __restrict__ order, int64_t n, int world,
                                                      int64_t sl, int64_t id_mask, int32_t* __restrict__ new_id) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += stride) {
    const int64_t p = j / world, q = j - p * world;
    const int64_t r = (p & 1) ? world - 1 - q : q;
    new_id[order[j] & id_mask] = (int32_t)(r * sl + p);
  }
}

// The degree ranking's sort keys in one pass: keys[j] = (dmax - deg[v]) << ibits | v for
// v = n - 1 - j (descending ids, so the stable sort on the degree bits breaks ties by
// descending id) -- was six torch elementwise kernels, ~1.1 ms at 2^26 vertices.
__global__ void __launch_bounds__(256) gb_rank_keys_kernel(const int32_t* __restrict__ deg, int64_t n,
                                                           int64_t dmax, int ibits, uint64_t* __restrict__ keys) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += stride) {
    const int64_t v = n - 1 - j;
    keys[j] = ((uint64_t)(dmax - (int64_t)deg[v]) << ibits) | (uint64_t)v;
  }
}

// ---------------------------------------------------------------------------- keys
// Local source index of a global (relabelled) source id and its block:
//   own slice [v_lo, v_hi): li = s - v_lo, segment 0;
//   remote (W > 1): li = sl + ghost rank of s (ghosts sorted by id = grouped by owner),
//   segment = the owner's ghost block.
// Blocks restart at every segment start; blk = seg_blk0[seg] + (li - seg_start[seg]) / 8192.
struct GbKeyCtx {
  int64_t v_lo, v_hi, sl;
  int world, rank, dbits;
  const int32_t* new_id;        // nullable: no relabeling
  const uint32_t* bitmap;       // W > 1: remote sources with an edge into this slice
  const int64_t* word_prefix;   // W > 1: exclusive popcount prefix of the bitmap words
  const int64_t* seg_start;     // [W]: local index where segment p starts (p = owner)
  const int64_t* seg_blk0;      // [W]: first block id of segment p
  int src_new;                  // the sources are already relabelled
};

__device__ __forceinline__ bool gb_edge(const GbKeyCtx& c, int32_t s0, int32_t d0, int32_t& s,
                                        int64_t& dl) {
  const int32_t d = c.new_id ? c.new_id[d0] : d0;
  dl = (int64_t)d - c.v_lo;
  const bool keep = d >= c.v_lo && d < c.v_hi;
  // (one rank: every edge is kept; several: the source is relabelled only where kept)
  s = c.new_id && !c.src_new && (c.world == 1 || keep) ? c.new_id[s0] : s0;
  return keep;
}

__device__ __forceinline__ uint64_t gb_key(const GbKeyCtx& c, int32_t s, int64_t dl) {
  int64_t rel, blk0;
  if (c.world == 1 || (s >= c.v_lo && s < c.v_hi)) {
    rel = (int64_t)s - c.v_lo;
    blk0 = 0;
  } else {
    const int p = (int)((int64_t)s / c.sl);
    const int64_t w = s >> 5;
    const uint32_t below = c.bitmap[w] & ((1u << (s & 31)) - 1u);
    const int64_t g = c.word_prefix[w] + __popc(below);          // ghost rank of s
    rel = c.sl + g - c.seg_start[p];
    blk0 = c.seg_blk0[p];
  }
  const uint64_t blk = (uint64_t)(blk0 + (rel >> kSpanBits));
  return (blk << (c.dbits + kSpanBits)) | ((uint64_t)dl << kSpanBits) | (uint64_t)(rel & (kSpan - 1));
}

constexpr int kKeyR = 16384;         // edges per block of the two key phases
constexpr int kKeyV = 4;             // edges per thread per step (int4 loads, 8 gathers in flight)

__device__ __forceinline__ void gb_load4(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                         int64_t i, int64_t r1, int32_t (&s)[kKeyV], int32_t (&d)[kKeyV],
                                         bool (&in)[kKeyV], const uint64_t* __restrict__ packed = nullptr) {
  if (packed != nullptr) {   // (src << 32 | dst) words: two 16-B loads per 4 edges
    static_assert(kKeyV == 4, "packed loads assume 4 edges per step");
    if (i + kKeyV <= r1) {
      const uint4 a = *reinterpret_cast<const uint4*>(packed + i);
      const uint4 b = *reinterpret_cast<const uint4*>(packed + i + 2);
      d[0] = (int32_t)a.x; s[0] = (int32_t)a.y; d[1] = (int32_t)a.z; s[1] = (int32_t)a.w;
      d[2] = (int32_t)b.x; s[2] = (int32_t)b.y; d[3] = (int32_t)b.z; s[3] = (int32_t)b.w;
#pragma unroll
      for (int v = 0; v < kKeyV; ++v) in[v] = true;
    } else {
#pragma unroll
      for (int v = 0; v < kKeyV; ++v) {
        in[v] = i + v < r1;
        const uint64_t w = in[v] ? packed[i + v] : 0ull;
        s[v] = (int32_t)(w >> 32);
        d[v] = (int32_t)(uint32_t)w;
      }
    }
    return;
  }
  if (i + kKeyV <= r1) {
    const int4 a = *reinterpret_cast<const int4*>(src + i);
    const int4 b = *reinterpret_cast<const int4*>(dst + i);
    s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
    d[0] = b.x; d[1] = b.y; d[2] = b.z; d[3] = b.w;
#pragma unroll
    for (int v = 0; v < kKeyV; ++v) in[v] = true;
  } else {
#pragma unroll
    for (int v = 0; v < kKeyV; ++v) {
      in[v] = i + v < r1;
      s[v] = in[v] ? src[i + v] : 0;
      d[v] = in[v] ? dst[i + v] : 0;
    }
  }
}

// phase 0: count the kept edges per block (and mark remote sources, W > 1: one plain byte
// store per remote source into a byte map -- idempotent, no read-modify-write; a u32
// atomicOr per edge into the bitmap made this phase 18.9 ms of the W = 8 per-rank build
// share at scale 26, profiles/round6/r6_5 -- packed into the bitmap by gb_bytes_to_bits)
__global__ void __launch_bounds__(256) gb_keys_count_kernel(const int32_t* __restrict__ src,
                                                            const int32_t* __restrict__ dst, int64_t n,
                                                            GbKeyCtx c, uint8_t* __restrict__ marks,
                                                            int32_t* __restrict__ counts) {
  __shared__ int s_cnt;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kKeyR;
  const int64_t r1 = r0 + kKeyR < n ? r0 + kKeyR : n;
  int mine = 0;
  for (int64_t i = r0 + (int64_t)threadIdx.x * kKeyV; i < r1; i += 256 * kKeyV) {
    int32_t s0[kKeyV], d0[kKeyV];
    bool in[kKeyV];
    gb_load4(src, dst, i, r1, s0, d0, in);
#pragma unroll
    for (int v = 0; v < kKeyV; ++v) {
      int32_t sv;
      int64_t dl;
      if (in[v] && gb_edge(c, s0[v], d0[v], sv, dl)) {
        ++mine;
        if (c.world > 1 && !(sv >= c.v_lo && sv < c.v_hi)) marks[sv] = 1;
      }
    }
  }
  atomicAdd(&s_cnt, mine);
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = s_cnt;
}

// phase 1: write the kept edges' keys at offsets[block] + (any order inside the block:
// the keys are sorted afterwards)
__global__ void __launch_bounds__(256) gb_keys_write_kernel(const int32_t* __restrict__ src,
                                                            const int32_t* __restrict__ dst, int64_t n,
                                                            GbKeyCtx c, const int64_t* __restrict__ offsets,
                                                            int64_t base_all, uint64_t* __restrict__ keys,
                                                            const uint64_t* __restrict__ packed) {
  __shared__ int s_cur;
  if (threadIdx.x == 0) s_cur = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kKeyR;
  const int64_t r1 = r0 + kKeyR < n ? r0 + kKeyR : n;
  const int64_t base = offsets ? offsets[blockIdx.x] : base_all + r0;
  const int lane = threadIdx.x & 63;
  for (int64_t i0 = r0; i0 < r1; i0 += 256 * kKeyV) {
    const int64_t i = i0 + (int64_t)threadIdx.x * kKeyV;
    int32_t s0[kKeyV], d0[kKeyV], sv[kKeyV];
    int64_t dl[kKeyV];
    bool in[kKeyV], keep[kKeyV];
    gb_load4(src, dst, i, r1, s0, d0, in, packed);
    int cnt = 0;
#pragma unroll
    for (int v = 0; v < kKeyV; ++v) {
      keep[v] = in[v] && gb_edge(c, s0[v], d0[v], sv[v], dl[v]);
      cnt += keep[v] ? 1 : 0;
    }
    // wave-inclusive scan of the counts, one LDS cursor bump per wave
    int x = cnt;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    int wbase = 0;
    if (lane == 63 && x) wbase = atomicAdd(&s_cur, x);
    wbase = __shfl(wbase, 63, 64);
    int64_t o = base + wbase + x - cnt;
#pragma unroll
    for (int v = 0; v < kKeyV; ++v)
      if (keep[v]) keys[o++] = gb_key(c, sv[v], dl[v]);
  }
}

// one rank, packed (src << 32 | dst) edges with relabelled sources: every edge is kept, so
// key i is written at i (no compaction) and the key is three fields: source block, new
// destination, source offset. 8 edges per thread per step (four 16-B loads, 8 gathers,
// four 16-B stores); the general kernel's wave scan and per-lane stores cost 12.9 ms (r5_42)
__global__ void __launch_bounds__(256) gb_keys_one_kernel(const uint64_t* __restrict__ packed, int64_t n,
                                                          const int32_t* __restrict__ new_id, int dbits,
                                                          uint64_t* __restrict__ keys) {
  constexpr int V = 8;
  const int64_t stride = (int64_t)gridDim.x * 256 * V;
  const int sh = dbits + kSpanBits;
  const int64_t lb = gb_xcd_block(blockIdx.x, gridDim.x);
  for (int64_t i = (lb * 256 + threadIdx.x) * V; i < n; i += stride) {
    if (i + V <= n) {
      uint4 q[V / 2];
#pragma unroll
      for (int u = 0; u < V / 2; ++u) q[u] = reinterpret_cast<const uint4*>(packed + i)[u];
      uint32_t d[V];
#pragma unroll
      for (int u = 0; u < V / 2; ++u) {
        d[2 * u] = (uint32_t)new_id[q[u].x];
        d[2 * u + 1] = (uint32_t)new_id[q[u].z];
      }
#pragma unroll
      for (int u = 0; u < V / 2; ++u) {
        const uint64_t k0 = ((uint64_t)(q[u].y >> kSpanBits) << sh) | ((uint64_t)d[2 * u] << kSpanBits) |
                            (q[u].y & (kSpan - 1));
        const uint64_t k1 = ((uint64_t)(q[u].w >> kSpanBits) << sh) | ((uint64_t)d[2 * u + 1] << kSpanBits) |
                            (q[u].w & (kSpan - 1));
        reinterpret_cast<uint4*>(keys + i)[u] =
            make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32));
      }
    } else {
      for (int64_t j = i; j < n; ++j) {
        const uint64_t w = packed[j];
        const uint32_t s = (uint32_t)(w >> 32), d = (uint32_t)new_id[(uint32_t)w];
        keys[j] = ((uint64_t)(s >> kSpanBits) << sh) | ((uint64_t)d << kSpanBits) | (s & (kSpan - 1));
      }
    }
  }
}

// ---------------------------------------------------------------------------- decode
// Over the SORTED keys with duplicates (the dedup is folded in: no separate unique pass).
// The last copy of every key stands for the distinct edge; an entry (block, destination)
// ends at the last copy of its last key. Blocks of kDecR keys, each thread 4 consecutive
// keys per step (coalesced), one block scan per step places the distinct edges and the
// entries in key order.
constexpr int kDecR = 16384;         // keys per block of the decode kernels: decode phase at
                                     // scale 26 7.4-7.8 ms (4096: 10.9-11.3, 8192: 8.4-8.6,
                                     // 32768: 7.6, 65536: 8.5, 131072: 9.8-10.0;
                                     // profiles/round6/r6_92)
constexpr int kDecT = 256;
constexpr int kDecV = 4;             // keys per thread per step (8: decode 11.3 -> 13.1 ms,
                                     // profiles/round5/r5_41)

// keys ib .. ib + 3 (ib % 4 == 0) and the key after them: two 16-B loads and one 8-B load;
// positions past n read as ~0 (no key's value: keys are < 2^63). Split from the flags so
// the decode loops can issue the next step's loads before they work on this one.
struct GbQuad {
  uint64_t k[kDecV];
  uint64_t kn;
};

__device__ __forceinline__ void gb_load4(const uint64_t* __restrict__ K, int64_t n, int64_t ib, GbQuad& q) {
  static_assert(kDecV == 4, "4 keys per thread per step");
  if (ib + kDecV <= n) {
    const uint4 a = *reinterpret_cast<const uint4*>(K + ib);
    const uint4 b = *reinterpret_cast<const uint4*>(K + ib + 2);
    q.k[0] = ((uint64_t)a.y << 32) | a.x;
    q.k[1] = ((uint64_t)a.w << 32) | a.z;
    q.k[2] = ((uint64_t)b.y << 32) | b.x;
    q.k[3] = ((uint64_t)b.w << 32) | b.z;
  } else {
#pragma unroll
    for (int v = 0; v < kDecV; ++v) q.k[v] = ib + v < n ? K[ib + v] : ~0ull;
  }
  q.kn = ib + kDecV < n ? K[ib + kDecV] : ~0ull;
}

// last: the key differs from the next one (the copy that stands for a distinct edge); end:
// also the last key of its (block, destination) entry. Positions >= r1 are flagged out.
__device__ __forceinline__ void gb_quad_flags(const GbQuad& q, int64_t ib, int64_t r1, bool (&last)[kDecV],
                                              bool (&end)[kDecV]) {
#pragma unroll
  for (int v = 0; v < kDecV; ++v) {
    const uint64_t nx = v + 1 < kDecV ? q.k[v + 1] : q.kn;
    last[v] = ib + v < r1 && nx != q.k[v];
    end[v] = last[v] && ((nx ^ q.k[v]) >> kSpanBits) != 0;
  }
}

// per block: distinct edges, entries, and the distinct out-degree per local source (LDS
// histogram of the block's first source block; other source blocks: global atomics)
__global__ void __launch_bounds__(kDecT) gb_decode_count_kernel(const uint64_t* __restrict__ K, int64_t n,
                                                                int64_t dr,
                                                                int shift, const int64_t* __restrict__ blk_base,
                                                                int64_t* __restrict__ counts,
                                                                uint32_t* __restrict__ outdeg) {
  __shared__ uint32_t hist[kSpan];
  __shared__ int s_d, s_e;
  for (int j = threadIdx.x; j < kSpan; j += kDecT) hist[j] = 0u;
  if (threadIdx.x == 0) { s_d = 0; s_e = 0; }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * dr;
  const int64_t r1 = r0 + dr < n ? r0 + dr : n;
  const uint64_t blk0 = K[r0] >> shift;
  int md = 0, me = 0;
  constexpr int64_t kStep = (int64_t)kDecT * kDecV;
  int64_t ib = r0 + (int64_t)threadIdx.x * kDecV;
  GbQuad cur;
  if (ib < r1) gb_load4(K, n, ib, cur);
  for (; ib < r1; ib += kStep) {
    GbQuad nxt;
    const bool more = ib + kStep < r1;
    if (more) gb_load4(K, n, ib + kStep, nxt);          // in flight while this step works
    bool last[kDecV], end[kDecV];
    gb_quad_flags(cur, ib, r1, last, end);
#pragma unroll
    for (int v = 0; v < kDecV; ++v) {
      if (last[v]) {
        ++md;
        const uint64_t blk = cur.k[v] >> shift;
        const uint32_t off = (uint32_t)(cur.k[v] & (kSpan - 1));
        if (blk == blk0) atomicAdd(hist + off, 1u);
        else atomicAdd(outdeg + blk_base[blk] + off, 1u);
      }
      me += end[v] ? 1 : 0;
    }
    if (more) cur = nxt;
  }
  atomicAdd(&s_d, md);
  atomicAdd(&s_e, me);
  __syncthreads();
  const int64_t b0 = blk_base[blk0];
  for (int j = threadIdx.x; j < kSpan; j += kDecT)
    if (hist[j]) atomicAdd(outdeg + b0 + j, hist[j]);
  if (threadIdx.x == 0) {
    counts[2 * blockIdx.x] = s_d;
    counts[2 * blockIdx.x + 1] = s_e;
  }
}

// offsets[2 b] / [2 b + 1]: distinct edges / entries before block b
__global__ void __launch_bounds__(kDecT) gb_decode_write_kernel(const uint64_t* __restrict__ K, int64_t n,
                                                                int64_t dr, int shift, int dbits,
                                                                const int64_t* __restrict__ offsets,
                                                                uint16_t* __restrict__ srcl,
                                                                int64_t* __restrict__ ent_end,
                                                                int32_t* __restrict__ ent_blk,
                                                                int32_t* __restrict__ ent_dst) {
  __shared__ int s_wd[kDecT / 64], s_we[kDecT / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * dr;
  const int64_t r1 = r0 + dr < n ? r0 + dr : n;
  int64_t dbase = offsets[2 * blockIdx.x], ebase = offsets[2 * blockIdx.x + 1];
  const uint64_t dmask = (1ull << dbits) - 1ull;
  constexpr int64_t kStep = (int64_t)kDecT * kDecV;
  GbQuad cur;
  gb_load4(K, n, r0 + (int64_t)threadIdx.x * kDecV, cur);
  for (int64_t i0 = r0; i0 < r1; i0 += kStep) {
    const int64_t ib = i0 + (int64_t)threadIdx.x * kDecV;
    GbQuad nxt;
    const bool more = i0 + kStep < r1;                   // block-uniform
    if (more) gb_load4(K, n, ib + kStep, nxt);          // in flight while this step works
    bool last[kDecV], end[kDecV];
    const uint64_t (&k)[kDecV] = cur.k;
    int cd = 0, ce = 0;
    gb_quad_flags(cur, ib, r1, last, end);
#pragma unroll
    for (int v = 0; v < kDecV; ++v) {
      cd += last[v] ? 1 : 0;
      ce += end[v] ? 1 : 0;
    }
    // block-wide exclusive scan of (cd, ce), packed (each <= 1024 per step)
    int x = cd | (ce << 16);
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) { s_wd[wid] = x & 0xffff; s_we[wid] = x >> 16; }
    __syncthreads();
    int pd = (x & 0xffff) - cd, pe = (x >> 16) - ce, td = 0, te = 0;
#pragma unroll
    for (int w = 0; w < kDecT / 64; ++w) {
      if (w < wid) { pd += s_wd[w]; pe += s_we[w]; }
      td += s_wd[w];
      te += s_we[w];
    }
    int64_t d = dbase + pd, e = ebase + pe;
#pragma unroll
    for (int v = 0; v < kDecV; ++v) {
      if (last[v]) {
        srcl[d] = (uint16_t)((k[v] & (kSpan - 1)) | (end[v] ? 0x8000u : 0u));
        if (end[v]) {
          ent_end[e] = d;
          ent_blk[e] = (int32_t)(k[v] >> shift);
          ent_dst[e] = (int32_t)((k[v] >> kSpanBits) & dmask);
          ++e;
        }
        ++d;
      }
    }
    dbase += td;
    ebase += te;
    if (more) cur = nxt;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------- entries
// run starts (new block or new destination bin), chunk starts (new block); the run-start
// bit 0x4000 goes on the entry's end edge
__global__ void __launch_bounds__(256) gb_entry_flags_kernel(const int32_t* __restrict__ ent_blk,
                                                             const int32_t* __restrict__ ent_dst,
                                                             const int64_t* __restrict__ ent_end, int64_t nent,
                                                             int bin_shift, uint8_t* __restrict__ rs,
                                                             uint8_t* __restrict__ cs,
                                                             uint16_t* __restrict__ srcl) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nent; e += stride) {
    const int32_t b = ent_blk[e];
    const int32_t bin = ent_dst[e] >> bin_shift;
    bool c = true, r = true;
    if (e > 0) {
      const int32_t pb = ent_blk[e - 1];
      c = pb != b;
      r = c || (ent_dst[e - 1] >> bin_shift) != bin;
    }
    rs[e] = r;
    cs[e] = c;
    if (r) srcl[ent_end[e]] |= (uint16_t)0x4000;
  }
}

// bin-major destination offsets: entry e of run q lives at e + run_delta[q]; and tile
// starts: within a chunk, a new work unit every wu_e edges and a new tile every tlen[chunk]
// edges of the unit, both on entry boundaries (dalgo/ops/graph.py::build_blocked)
__global__ void __launch_bounds__(256) gb_entry_place_kernel(const int32_t* __restrict__ ent_dst,
                                                             const int64_t* __restrict__ ent_end, int64_t nent,
                                                             const int32_t* __restrict__ run_of_ent,
                                                             const int32_t* __restrict__ run_delta,
                                                             const int32_t* __restrict__ run_chunk,
                                                             const uint8_t* __restrict__ cs,
                                                             const int64_t* __restrict__ ce_lo,
                                                             const int64_t* __restrict__ tlen, int64_t wu_e,
                                                             int bin_mask, int16_t* __restrict__ dloc,
                                                             uint8_t* __restrict__ ts) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nent; e += stride) {
    const int q = run_of_ent[e];
    dloc[e + run_delta[q]] = (int16_t)(ent_dst[e] & bin_mask);
    const int ch = run_chunk[q];
    bool t = cs[e] != 0;
    if (!t) {
      const int64_t tl = tlen[ch];
      const int64_t a = (e > 1 ? ent_end[e - 2] + 1 : 0) - ce_lo[ch];   // entry e - 1's first edge
      const int64_t b = ent_end[e - 1] + 1 - ce_lo[ch];                 // entry e's first edge
      t = (a / wu_e) != (b / wu_e) || ((a % wu_e) / tl) != ((b % wu_e) / tl);
    }
    ts[e] = t;
  }
}


// ---------------------------------------------------------------------------- cells
// The runs of the K4b layout are the non-empty cells of the (block, destination bin)
// matrix: entries are in chunk-major (block, destination) order, so the entries of one cell
// are contiguous, a row-major scan of the cell counts gives every run's first entry and
// its index, and a column-major scan gives its bin-major position -- no per-entry scans,
// sorts or searches (nblk x nbins cells: 33.5M at R-MAT scale 26 on one rank).

constexpr int kCellEpt = 4;          // entries per thread and step (gb_cell_count, gb_entry_cells): 4.1 ms at
                                     // scale 26 (1: 4.9, 8: 5.2; profiles/round6/r6_93)

// C[cell] += entries of the cell; one atomic per run of equal cells inside a wave
__global__ void __launch_bounds__(256) gb_cell_count_kernel(const int32_t* __restrict__ ent_blk,
                                                            const int32_t* __restrict__ ent_dst, int64_t nent,
                                                            int bshift, int nblk, int nbins,
                                                            int32_t* __restrict__ C) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * 256 * kCellEpt;
  // kCellEpt entries per thread and step, all loads issued first (as gb_entry_cells)
  for (int64_t e0 = (int64_t)blockIdx.x * 256 * kCellEpt; e0 < nent; e0 += stride) {
    int32_t bv[kCellEpt], dv[kCellEpt];
#pragma unroll
    for (int j = 0; j < kCellEpt; ++j) {
      const int64_t e = e0 + threadIdx.x + (int64_t)j * 256;
      bv[j] = e < nent ? ent_blk[e] : -1;
      dv[j] = e < nent ? ent_dst[e] : 0;
    }
#pragma unroll
    for (int j = 0; j < kCellEpt; ++j) {
      const int64_t e = e0 + threadIdx.x + (int64_t)j * 256;
      const bool in = e < nent;
      int64_t cell = -1;
      if (in) {
        const int32_t b = bv[j], bin = dv[j] >> bshift;
        if (b >= 0 && b < nblk && bin >= 0 && bin < nbins) cell = (int64_t)b * nbins + bin;
      }
      const int64_t prev = __shfl_up(cell, 1, 64);
      const bool head = cell >= 0 && (lane == 0 || prev != cell);
      const uint64_t hm = __ballot(head), vm = __ballot(in);
      if (head) {
        const uint64_t above = hm & ~((2ull << lane) - 1ull);   // heads after this lane
        const int end = above ? __ffsll((long long)above) - 1 : 64 - __clzll((long long)vm);
        atomicAdd(C + cell, end - lane);
      }
    }
  }
}

// per row (block): entries T and non-empty cells R
__global__ void __launch_bounds__(256) gb_cell_rows_kernel(const int32_t* __restrict__ C, int nbins,
                                                           int64_t* __restrict__ T, int64_t* __restrict__ R) {
  __shared__ int64_t s_t[4], s_r[4];
  const int64_t row = blockIdx.x;
  const int32_t* c = C + row * nbins;
  int64_t t = 0, r = 0;
  for (int j = threadIdx.x; j < nbins; j += 256) {
    const int32_t v = c[j];
    t += v;
    r += v > 0;
  }
  for (int off = 32; off >= 1; off >>= 1) {
    t += __shfl_xor(t, off, 64);
    r += __shfl_xor(r, off, 64);
  }
  if ((threadIdx.x & 63) == 0) { s_t[threadIdx.x >> 6] = t; s_r[threadIdx.x >> 6] = r; }
  __syncthreads();
  if (threadIdx.x == 0) {
    T[row] = s_t[0] + s_t[1] + s_t[2] + s_t[3];
    R[row] = s_r[0] + s_r[1] + s_r[2] + s_r[3];
  }
}

// per row: CM[cell] = first entry of the cell (RE[row] + exclusive count prefix), RID[cell]
// = its run index (RR[row] + exclusive non-empty prefix); 4 cells per thread per step
__global__ void __launch_bounds__(256) gb_cell_scan_kernel(const int32_t* __restrict__ C, int nbins,
                                                           const int64_t* __restrict__ RE,
                                                           const int64_t* __restrict__ RR,
                                                           int32_t* __restrict__ CM, int32_t* __restrict__ RID) {
  __shared__ int s_c[4], s_n[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t row = blockIdx.x;
  const int64_t base = row * nbins;
  int64_t ce = RE[row], cr = RR[row];
  for (int j0 = 0; j0 < nbins; j0 += 1024) {
    const int j = j0 + threadIdx.x * 4;
    int v[4];
    int sc = 0, sn = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u] = j + u < nbins ? C[base + j + u] : 0;
      sc += v[u];
      sn += v[u] > 0;
    }
    int xc = sc, xn = sn;
    for (int off = 1; off < 64; off <<= 1) {
      const int yc = __shfl_up(xc, off, 64), yn = __shfl_up(xn, off, 64);
      if (lane >= off) { xc += yc; xn += yn; }
    }
    if (lane == 63) { s_c[wid] = xc; s_n[wid] = xn; }
    __syncthreads();
    int pc = xc - sc, pn = xn - sn, tc = 0, tn = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (w < wid) { pc += s_c[w]; pn += s_n[w]; }
      tc += s_c[w];
      tn += s_n[w];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (j + u < nbins) {
        CM[base + j + u] = (int32_t)(ce + pc);
        RID[base + j + u] = (int32_t)(cr + pn);
      }
      pc += v[u];
      pn += v[u] > 0;
    }
    ce += tc;
    cr += tn;
    __syncthreads();
  }
}

// P[g][bin] = entries of column bin over rows [g G, (g + 1) G)
__global__ void __launch_bounds__(256) gb_cell_colsum_kernel(const int32_t* __restrict__ C, int nblk, int nbins,
                                                             int G, int64_t* __restrict__ P) {
  const int bin = blockIdx.x * 256 + threadIdx.x;
  const int g = blockIdx.y;
  if (bin >= nbins) return;
  const int r1 = min(nblk, (g + 1) * G);
  int64_t s = 0;
  for (int r = g * G; r < r1; ++r) s += C[(int64_t)r * nbins + bin];
  P[(int64_t)g * nbins + bin] = s;
}

// walks column bin over rows [g G, (g + 1) G) from its bin-major start Poff[g][bin]: every
// non-empty cell (= run q) gets run_delta[q] = bin-major start - chunk-major start, its
// chunk and its first entry
__global__ void __launch_bounds__(256) gb_cell_place_kernel(const int32_t* __restrict__ C,
                                                            const int32_t* __restrict__ CM,
                                                            const int32_t* __restrict__ RID, int nblk,
                                                            int nbins, int G, const int64_t* __restrict__ Poff,
                                                            const int32_t* __restrict__ CI, int64_t nruns,
                                                            int32_t* __restrict__ run_delta,
                                                            int32_t* __restrict__ run_chunk,
                                                            int64_t* __restrict__ run_first) {
  const int bin = blockIdx.x * 256 + threadIdx.x;
  const int g = blockIdx.y;
  if (bin >= nbins) return;
  const int r1 = min(nblk, (g + 1) * G);
  int64_t pos = Poff[(int64_t)g * nbins + bin];
  for (int r = g * G; r < r1; ++r) {
    const int64_t cell = (int64_t)r * nbins + bin;
    const int32_t c = C[cell];
    if (c > 0) {
      const int32_t q = RID[cell];
      if (q >= 0 && q < nruns) {
        const int32_t cm = CM[cell];
        run_delta[q] = (int32_t)(pos - cm);
        run_chunk[q] = CI[r];
        run_first[q] = cm;
      }
      pos += c;
    }
  }
}

// per entry: bin-major destination (dloc), run-start bit on the end edge of a run's first
// entry, tile starts (a new work unit every wu_e edges of a chunk and a new tile every
// tlen[chunk] edges of the unit, on entry boundaries; chunk starts always)
__global__ void __launch_bounds__(256) gb_entry_cells_kernel(
    const int32_t* __restrict__ ent_blk, const int32_t* __restrict__ ent_dst, const int64_t* __restrict__ ent_end,
    int64_t nent, int bshift, int nblk, int nbins, const int32_t* __restrict__ CM,
    const int32_t* __restrict__ RID, const int32_t* __restrict__ run_delta, int64_t nruns,
    const int64_t* __restrict__ RE, const int32_t* __restrict__ CI, const int64_t* __restrict__ ce_lo,
    const int64_t* __restrict__ tlen, int64_t nch, int64_t wu_e, int bin_mask, int16_t* __restrict__ dloc,
    int64_t ndloc, int32_t* __restrict__ tiles, unsigned long long* __restrict__ n_tiles, int64_t tile_cap,
    uint16_t* __restrict__ srcl, int64_t nsrcl) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * 256 * kCellEpt;
  // kCellEpt entries per thread and step, each level of the dependent loads (entry -> cell
  // -> run -> chunk tables) issued for all of them before the next: one entry per thread
  // and step left the pass latency-bound (4.7 ms at scale 26, profiles/round6/r6_48)
  // (block-uniform loop: every lane reaches the ballots below)
  for (int64_t e0 = (int64_t)blockIdx.x * 256 * kCellEpt; e0 < nent; e0 += stride) {
    int64_t ev[kCellEpt], ee[kCellEpt], cell[kCellEpt];
    int32_t bv[kCellEpt], dv[kCellEpt], q[kCellEpt], cm[kCellEpt];
#pragma unroll
    for (int j = 0; j < kCellEpt; ++j) {
      ev[j] = e0 + threadIdx.x + (int64_t)j * 256;
      const bool in = ev[j] < nent;
      bv[j] = in ? ent_blk[ev[j]] : -1;
      dv[j] = in ? ent_dst[ev[j]] : 0;
      ee[j] = in ? ent_end[ev[j]] : -1;
    }
#pragma unroll
    for (int j = 0; j < kCellEpt; ++j) {
      const int32_t bin = dv[j] >> bshift;
      const bool okc = bv[j] >= 0 && bv[j] < nblk && bin >= 0 && bin < nbins;
      cell[j] = okc ? (int64_t)bv[j] * nbins + bin : 0;
      q[j] = okc ? RID[cell[j]] : -1;
      cm[j] = okc ? CM[cell[j]] : -1;
    }
    bool ok[kCellEpt];
    int32_t rd[kCellEpt], ch[kCellEpt];
    int64_t re[kCellEpt];
#pragma unroll
    for (int j = 0; j < kCellEpt; ++j) {
      ok[j] = q[j] >= 0 && q[j] < nruns;
      rd[j] = ok[j] ? run_delta[q[j]] : 0;
      ch[j] = ok[j] ? CI[bv[j]] : -1;
      re[j] = ok[j] ? RE[bv[j]] : -1;
    }
    bool need[kCellEpt];
    int64_t tl[kCellEpt], cl[kCellEpt], a2[kCellEpt], a1[kCellEpt];
#pragma unroll
    for (int j = 0; j < kCellEpt; ++j) {
      const int64_t e = ev[j];
      need[j] = ok[j] && e != re[j] && e > 0 && ch[j] >= 0 && ch[j] < nch;
      tl[j] = need[j] ? tlen[ch[j]] : 1;
      cl[j] = need[j] ? ce_lo[ch[j]] : 0;
      a2[j] = need[j] && e > 1 ? ent_end[e - 2] : -1;
      a1[j] = need[j] ? ent_end[e - 1] : -1;
    }
#pragma unroll
    for (int j = 0; j < kCellEpt; ++j) {
      const int64_t e = ev[j];
      bool t = false;
      if (ok[j]) {
        const int64_t pos = e + rd[j];
        if (pos >= 0 && pos < ndloc) dloc[pos] = (int16_t)(dv[j] & bin_mask);
        if (e == cm[j] && ee[j] >= 0 && ee[j] < nsrcl) srcl[ee[j]] |= (uint16_t)0x4000;
        t = e == re[j];
        if (need[j]) {
          const int64_t a = a2[j] + 1 - cl[j];                    // entry e - 1's first edge
          const int64_t bb = a1[j] + 1 - cl[j];                   // entry e's first edge
          t = (a / wu_e) != (bb / wu_e) || ((a % wu_e) / tl[j]) != ((bb % wu_e) / tl[j]);
        }
      }
      // tile starts -> an unordered list (one global atomic per wave that has any; sorted
      // on the host side afterwards): no per-entry flag array, no compaction pass
      const uint64_t m = __ballot(t);
      if (m != 0ull) {
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(n_tiles, (unsigned long long)__popcll(m));
        base = __shfl(base, 0);
        if (t) {
          const long long slot = (long long)base + __popcll(m & ((1ull << lane) - 1ull));
          if (slot < tile_cap) tiles[slot] = (int32_t)e;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------- run sort
// The key sort runs over the bits ABOVE the source offset only (39 of 52 bits at scale 26:
// 5 radix passes instead of 7); the runs of keys equal above lo_bits (one entry's edges:
// 449M runs over 1.07B keys at scale 26, 75 % of length 1, 6.6M of 17-256 keys, 140K
// longer, profiles/round5/r5_44) are then sorted on their low lo_bits in place, which makes
// the copies of an edge adjacent again for the decode's dedup. One block stages a tile of
// keys plus a halo in LDS, sorts the runs starting in its tile there and writes the changed
// keys back coalesced: a run of <= kRankMax keys by per-key ranks (each key's thread counts
// the run's keys below it), <= kRunMid keys by one wave (bitonic network over registers
// and lane shuffles); a longer one is listed (one global atomic per block that has any) and
// counting-sorted by one block of gb_run_long_kernel over an LDS histogram of the
// 2^lo_bits offsets. No per-run global atomics: 6.6M of them on one counter took ~60 ms.
constexpr int kRankMax = 64;         // runs sorted by per-key ranks
constexpr int kRunMid = 256;          // runs sorted by one wave's network
constexpr int kRunTile = 2048;        // run starts per block of the tile kernel
constexpr int kRunT = 256;

// ascending bitonic sort of the 64 * R values of a wave, element lane * R + r in v[r]
template <int R>
__device__ __forceinline__ void gb_wave_sort(uint32_t (&v)[R], int lane) {
#pragma unroll
  for (int k = 2; k <= 64 * R; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= R) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int i = lane * R + r;
          const uint32_t o = __shfl_xor(v[r], j / R, 64);
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          v[r] = keep_min ? min(v[r], o) : max(v[r], o);
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int l = r ^ j;
          if (l > r) {
            const bool up = ((lane * R + r) & k) == 0;
            const uint32_t a = v[r], b = v[l];
            v[r] = up ? min(a, b) : max(a, b);
            v[l] = up ? max(a, b) : min(a, b);
          }
        }
      }
    }
  }
}

// one wave: the run at tile offset j (L = its length, 17..64 * R) sorted in the staged
// keys; changed positions flagged for the block's write-out
template <int R>
__device__ __forceinline__ void gb_wave_run(uint64_t* s_k, uint8_t* s_chg, int j, int L, int lane,
                                            uint64_t lmask) {
  const uint64_t hi = s_k[j] & ~lmask;
  uint32_t v[R], o[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = lane * R + r;
    o[r] = v[r] = e < L ? (uint32_t)(s_k[j + e] & lmask) : 0xffffffffu;
  }
  gb_wave_sort<R>(v, lane);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = lane * R + r;
    if (e < L && v[r] != o[r]) {
      s_k[j + e] = hi | v[r];
      s_chg[j + e] = 1;
    }
  }
}

// consecutive set bits of the bitmap from bit q on, counted up to at least `limit` (the
// bitmap ends with a zero word)
__device__ __forceinline__ int gb_ones_from(const uint64_t* eqb, int q, int limit) {
  int c = 0;
  for (;;) {
    const int b = q & 63;
    const uint64_t inv = ~(eqb[q >> 6] >> b);            // ones above the 64 - b valid bits
    const int t = inv ? __builtin_ctzll(inv) : 64;
    c += t;
    if (t < 64 - b || c > limit) return c;
    q += t;
  }
}

__global__ void __launch_bounds__(kRunT) gb_run_tile_kernel(uint64_t* __restrict__ K, int64_t n, int lo_bits,
                                                            int64_t* __restrict__ longs,
                                                            unsigned long long* __restrict__ nlong) {
  constexpr int W = kRunTile + kRunMid + 2;    // keys staged: the tile, a halo, one spare
  constexpr int kMaxMid = kRunTile / (kRankMax + 1) + 1;
  constexpr int kMaxLong = kRunTile / (kRunMid + 1) + 1;
  __shared__ __attribute__((aligned(16))) uint64_t s_k[W];
  constexpr int kEqW = (W + kRunT - 1) / kRunT * (kRunT / 64) + 1;
  // bit j: key j equal to key j - 1 above lo_bits (one ballot per 64 keys; a zero spare word)
  __shared__ uint64_t s_eqb[kEqW];
  __shared__ uint8_t s_chg[W];                 // key j rewritten
  __shared__ int s_mid[kMaxMid];
  __shared__ int s_long[kMaxLong];
  __shared__ int s_nmid, s_nlong;
  __shared__ unsigned long long s_lbase;
  const int64_t base = (int64_t)blockIdx.x * kRunTile;   // even: 16-B aligned pairs
  const uint64_t lmask = (1ull << lo_bits) - 1ull;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) { s_nmid = 0; s_nlong = 0; s_eqb[kEqW - 1] = 0ull; }
  // keys past n: ~0 (its high bits equal no key's: keys are < 2^63)
  for (int j = 2 * threadIdx.x; j < W; j += 2 * kRunT) {
    const int64_t p = base + j;
    uint64_t k0 = ~0ull, k1 = ~0ull;
    if (p + 1 < n) {
      const uint4 v = *reinterpret_cast<const uint4*>(K + p);
      k0 = ((uint64_t)v.y << 32) | v.x;
      k1 = ((uint64_t)v.w << 32) | v.z;
    } else if (p < n) {
      k0 = K[p];
    }
    s_k[j] = k0;
    s_k[j + 1] = k1;
  }
  const uint64_t kprev = base > 0 ? K[base - 1] : ~0ull;
  __syncthreads();
  for (int j = threadIdx.x; j < (kEqW - 1) * 64; j += kRunT) {
    bool eq = false;
    if (j < W) {
      const uint64_t pk = j ? s_k[j - 1] : kprev;
      eq = base + j < n && ((pk ^ s_k[j]) >> lo_bits) == 0;
      s_chg[j] = 0;
    }
    const uint64_t b = __ballot(eq);
    if (lane == 0) s_eqb[j >> 6] = b;
  }
  __syncthreads();
  // runs of 2 .. kRankMax keys: every key's place is its rank in its run (keys below it,
  // ties by position: stable), counted by the key's own thread over the run's staged low
  // bits (lanes of one run read the same LDS words: broadcasts); the run of key q starts
  // at the last zero bit of the bitmap at or below q. The ranks of a thread's keys are
  // held in registers and the keys moved after a barrier. A longer run is listed by the
  // thread at its first key for the wave tier below.
  constexpr int NQ = (kRunTile + kRankMax + kRunT - 1) / kRunT;
  const uint32_t* klo = reinterpret_cast<const uint32_t*>(s_k);   // low words (little endian)
  int tgt[NQ];
  uint64_t kv[NQ];
#pragma unroll
  for (int it = 0; it < NQ; ++it) {
    const int q = it * kRunT + threadIdx.x;
    tgt[it] = -1;
    int w = q >> 6;
    uint64_t z = ~s_eqb[w] & ((q & 63) == 63 ? ~0ull : ((2ull << (q & 63)) - 1ull));
#pragma unroll
    for (int k = 0; k < kRankMax / 64; ++k)              // a run of <= kRankMax keys: its start
      if (!z && w > 0) z = ~s_eqb[--w];                  // is <= kRankMax / 64 words back
    if (!z) continue;                                    // started in the previous tile, or longer
    const int st = w * 64 + 63 - __builtin_clzll(z);
    if (st >= kRunTile || q - st >= kRankMax) continue;  // the next block's run, or longer
    const int L = 1 + gb_ones_from(s_eqb, st + 1, kRankMax);
    if (L > kRankMax) {
      if (q == st) s_mid[atomicAdd(&s_nmid, 1)] = st;
      continue;
    }
    if (L == 1) continue;
    const uint32_t v = klo[2 * q] & (uint32_t)lmask;
    int rank = 0;
    for (int i = 0; i < L; ++i) {
      const uint32_t u = klo[2 * (st + i)] & (uint32_t)lmask;
      rank += (u < v || (u == v && st + i < q)) ? 1 : 0;
    }
    if (st + rank != q) {
      tgt[it] = st + rank;
      kv[it] = s_k[q];
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NQ; ++it)
    if (tgt[it] >= 0) {
      s_k[tgt[it]] = kv[it];
      s_chg[tgt[it]] = 1;
    }
  __syncthreads();
  // runs of kRankMax + 1 .. kRunMid keys: one wave each (bitonic network); longer: listed
  const int nmid = s_nmid;
  for (int m = wid; m < nmid; m += kRunT / 64) {
    const int j = s_mid[m];
    constexpr int R = kRunMid / 64;
    const int L = 1 + gb_ones_from(s_eqb, j + 1, kRunMid);   // kRunMid + 1: longer
    if (L > kRunMid) {
      if (lane == 0) s_long[atomicAdd(&s_nlong, 1)] = j;
      continue;
    }
    gb_wave_run<R>(s_k, s_chg, j, L, lane, lmask);   // a 128-key network for <= 128: no gain (r5_56)
  }
  __syncthreads();
  // coalesced write-out of the rewritten keys (tile and halo: a run started here may reach
  // into the next tile, whose block never rewrites it)
  for (int j = threadIdx.x; j < W; j += kRunT)
    if (s_chg[j]) K[base + j] = s_k[j];
  // longer runs: appended to the global list, one atomic per block that has any
  const int nl = s_nlong;
  if (nl) {
    if (threadIdx.x == 0) s_lbase = atomicAdd(nlong, (unsigned long long)nl);
    __syncthreads();
    if (threadIdx.x < nl) longs[s_lbase + threadIdx.x] = base + s_long[threadIdx.x];
  }
}

// one block per listed run (block-uniform loop over the device count): histogram of the
// low offsets, exclusive scan, the run rewritten in offset order (copies kept adjacent)
__global__ void __launch_bounds__(kRunT) gb_run_long_kernel(uint64_t* __restrict__ K, int64_t n, int lo_bits,
                                                            const int64_t* __restrict__ longs,
                                                            const unsigned long long* __restrict__ nlong) {
  // count of offset v at h[v + v / 32]: the scan's per-thread 32-word rows are 33 words
  // apart, so a wave's reads hit distinct banks (unpadded: 17.9 conflict cycles per LDS
  // instruction, profiles/round5/r5_49)
  constexpr int kH = kSpan + kSpan / 32;
  __shared__ __attribute__((aligned(16))) uint32_t h[kH];
  __shared__ int s_len[2][kRunT / 64];
  __shared__ uint32_t s_ws[kRunT / 64];
  constexpr int PER = kSpan / kRunT;                  // histogram words per thread
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nv = 1 << lo_bits;                        // <= kSpan (launcher checks)
  const uint64_t lmask = (uint64_t)nv - 1ull;
  const int64_t cnt = (int64_t)*nlong;
  for (int64_t r = blockIdx.x; r < cnt; r += gridDim.x) {
    const int64_t p = longs[r];
    const uint64_t hi = K[p] & ~lmask;
    for (int j = threadIdx.x; j < kH / 4; j += kRunT) reinterpret_cast<uint4*>(h)[j] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    // one pass over the run, 256 keys per step: histogram of the in-run offsets and the
    // equal-prefix count from per-wave ballots (double-buffered: one barrier per step)
    int64_t L = 0;
    for (int buf = 0;; buf ^= 1) {
      const int64_t q = p + L + threadIdx.x;
      const uint64_t k = q < n ? K[q] : ~0ull;          // ~0: no key's high bits (keys < 2^63)
      const bool in = (k & ~lmask) == hi;
      if (in) {
        const int v = (int)(k & lmask);
        atomicAdd(&h[v + (v >> 5)], 1u);
      }
      const uint64_t b = __ballot(in);
      if (lane == 0) s_len[buf][wid] = __popcll(b);
      __syncthreads();
      int step = 0;
#pragma unroll
      for (int w = 0; w < kRunT / 64; ++w) step += s_len[buf][w];
      L += step;
      if (step < kRunT) break;                         // keys equal above lo_bits are contiguous
    }
    // exclusive scan of h[0 .. nv): PER consecutive words per thread
    uint32_t c[PER], s = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int v = threadIdx.x * PER + u;
      c[u] = v < nv ? h[v + (v >> 5)] : 0u;
      s += c[u];
    }
    uint32_t x = s;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) s_ws[wid] = x;
    __syncthreads();
    uint32_t ofs = x - s;
#pragma unroll
    for (int w = 0; w < kRunT / 64; ++w) ofs += w < wid ? s_ws[w] : 0u;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const uint64_t key = hi | (uint64_t)(threadIdx.x * PER + u);
      for (uint32_t m = 0; m < c[u]; ++m) K[p + ofs + m] = key;
      ofs += c[u];
    }
    __syncthreads();                                   // h and s_ws reused by the next run
  }
}

}  // namespace
}  // namespace dalgo

using namespace dalgo;

extern "C" {

hipError_t dalgo_gb_degree(const int32_t* ids, int64_t n, uint32_t* deg, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t g = std::min<int64_t>(cdiv(n, 256 * 4), 256 * 64);
  hipLaunchKernelGGL(gb_degree_kernel, dim3((unsigned)g), dim3(256), 0, st, ids, n, deg);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_gb_sort32(void* tmp, size_t* tmp_bytes, const uint32_t* in, uint32_t* out, int64_t n,
                           int begin_bit, int end_bit, hipStream_t st) {
  if (n < 0 || n >= (int64_t)0x7fffffffLL || end_bit < 1 || end_bit > 32 || begin_bit < 0 || begin_bit >= end_bit)
    return hipErrorInvalidValue;
  return rocprim::radix_sort_keys(tmp, *tmp_bytes, in, out, (size_t)n, (unsigned)begin_bit, (unsigned)end_bit, st);
}

int dalgo_gb_bucket_bits() { return kBktBits; }

// ids sorted on bits [kBktBits, end_bit): deg[v] += occurrences of v (ids < 2^end_bit);
// starts: int64[2^(end_bit - kBktBits) + 1] workspace
hipError_t dalgo_gb_bucket_degree(const void* sorted, int packed, int64_t n, int end_bit, int64_t* starts,
                                  int32_t* deg, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (end_bit <= kBktBits || end_bit > 31 || n >= (int64_t)0x7fffffffLL) return hipErrorInvalidValue;
  const int nb = 1 << (end_bit - kBktBits);
  if (packed) {
    hipLaunchKernelGGL(gb_bucket_starts_kernel<uint64_t>, dim3((unsigned)cdiv(nb + 1, 256)), dim3(256), 0, st,
                       (const uint64_t*)sorted, n, nb, starts);
    DALGO_LAUNCH_CHECK();
    hipLaunchKernelGGL(gb_bucket_degree_kernel<uint64_t>, dim3((unsigned)nb), dim3(256), 0, st,
                       (const uint64_t*)sorted, (const int64_t*)starts, deg);
  } else {
    hipLaunchKernelGGL(gb_bucket_starts_kernel<uint32_t>, dim3((unsigned)cdiv(nb + 1, 256)), dim3(256), 0, st,
                       (const uint32_t*)sorted, n, nb, starts);
    DALGO_LAUNCH_CHECK();
    hipLaunchKernelGGL(gb_bucket_degree_kernel<uint32_t>, dim3((unsigned)nb), dim3(256), 0, st,
                       (const uint32_t*)sorted, (const int64_t*)starts, deg);
  }
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// marks: >= 32 nw bytes (16-B aligned); bits: nw words
hipError_t dalgo_gb_bytes_to_bits(const uint8_t* marks, int64_t nw, uint32_t* bits, hipStream_t st) {
  if (nw <= 0) return hipSuccess;
  if (reinterpret_cast<uintptr_t>(marks) % 16) return hipErrorInvalidValue;
  const int64_t g = std::min<int64_t>(cdiv(nw, (int64_t)256), 256 * 64);
  hipLaunchKernelGGL(gb_bytes_to_bits_kernel, dim3((unsigned)g), dim3(256), 0, st,
                     reinterpret_cast<const uint4*>(marks), nw, bits);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_gb_bitmap_ids(const uint32_t* bm, int64_t nw, const int64_t* prefix, int64_t* ids,
                               hipStream_t st) {
  if (nw <= 0) return hipSuccess;
  hipLaunchKernelGGL(gb_bitmap_ids_kernel, dim3((unsigned)cdiv(nw, (int64_t)256)), dim3(256), 0, st, bm, nw,
                     prefix, ids);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_gb_deal(const int64_t* order, int64_t n, int world, int64_t sl, int id_bits, int32_t* new_id,
                         hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (world < 1 || sl * world < n || sl > 0x7fffffffLL || id_bits < 0 || id_bits > 62) return hipErrorInvalidValue;
  const int64_t mask = id_bits ? (int64_t)((1ull << id_bits) - 1ull) : (int64_t)-1;
  const int64_t g = std::min<int64_t>(cdiv(n, (int64_t)256), 256 * 64);
  hipLaunchKernelGGL(gb_deal_kernel, dim3((unsigned)g), dim3(256), 0, st, order, n, world, sl, mask, new_id);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_gb_rank_keys(const int32_t* deg, int64_t n, int64_t dmax, int ibits, uint64_t* keys, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ibits < 1 || ibits > 40 || (n - 1) >> ibits) return hipErrorInvalidValue;
  const int64_t g = std::min<int64_t>(cdiv(n, (int64_t)256), 256 * 64);
  hipLaunchKernelGGL(gb_rank_keys_kernel, dim3((unsigned)g), dim3(256), 0, st, deg, n, dmax, ibits, keys);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// DALGO_GB_OWNER_BLOCKS overrides the grid (default 1024: at the W = 8 share the bucketed
// relabel + owner pass took 5.16 / 4.42 / 4.69 / 4.68 ms at 512 / 1024 / 2048 / 4096 blocks,
// 5.2 ms with 16384-edge blocks, profiles/round6/r6_28; with XCD-aware logical blocks 4.30 /
// 4.47 / 4.59 at 1024 / 2048 / 4096, r6_29)
int64_t dalgo_gb_owner_blocks(int64_t n) {
  static int64_t g = -1;
  if (g < 0) {
    const char* e = std::getenv("DALGO_GB_OWNER_BLOCKS");
    g = e ? std::max<int64_t>(1, std::atoll(e)) : 1024;
  }
  return std::max<int64_t>(1, std::min<int64_t>(cdiv(n, (int64_t)kOwnStep), g));
}

// phase 0 (src == dst == nullptr: tmp holds the packed edges, sources relabelled, and only the
// destinations go through new_id, in place):
// phase 0: tmp[i] = new_id[src[i]] << 32 | new_id[dst[i]] (new_id nullable), counts[o * nb + b] =
// edges of block b owned by rank o = dst' / sl; phase 2 (offsets = exclusive scan of counts):
// out[offsets[o * nb + b] + ...] = the block's words owned by o
hipError_t dalgo_gb_owner_scatter(int phase, const int32_t* src, const int32_t* dst, int64_t n,
                                  const int32_t* new_id, int64_t sl, int world, uint64_t* tmp,
                                  int64_t* counts, const int64_t* offsets, uint64_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (world < 1 || world > kOwnMax || sl < 1 || sl > 0x7fffffffLL) return hipErrorInvalidValue;
  const int64_t g = dalgo_gb_owner_blocks(n);
  if (phase == 0)
    hipLaunchKernelGGL(gb_owner_count_kernel, dim3((unsigned)g), dim3(256), 0, st, src, dst, n, new_id,
                       (uint32_t)sl, world, tmp, counts);
  else
    hipLaunchKernelGGL(gb_owner_scatter_kernel, dim3((unsigned)g), dim3(256), 0, st, (const uint64_t*)tmp, n,
                       (uint32_t)sl, offsets, out);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

int64_t dalgo_gb_key_blocks(int64_t n) { return cdiv(n, (int64_t)kKeyR); }

hipError_t dalgo_gb_keys(const int32_t* src, const int32_t* dst, int64_t n, const DalgoGbKeyArgs* a,
                         int phase, uint32_t* bitmap, int32_t* counts, const int64_t* offsets,
                         int64_t base_all, uint64_t* keys, const uint64_t* packed, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (a->dbits < 0 || a->dbits > 31 || a->world < 1) return hipErrorInvalidValue;
  GbKeyCtx c{a->v_lo, a->v_hi, a->sl, a->world, a->rank, a->dbits, a->new_id, a->bitmap,
             a->word_prefix, a->seg_start, a->seg_blk0, a->src_new};
  if (c.world > 1 && (c.sl <= 0 || (phase == 1 && (!c.bitmap || !c.word_prefix || !c.seg_start || !c.seg_blk0))))
    return hipErrorInvalidValue;
  const int64_t g = cdiv(n, (int64_t)kKeyR);
  if (g > 0x7fffffffLL) return hipErrorInvalidValue;
  if (packed != nullptr && (phase == 0 || c.world > 1)) return hipErrorInvalidValue;   // one rank only
  if (packed != nullptr && c.src_new && c.new_id && c.v_lo == 0 && c.v_hi >= c.sl) {
    // DALGO_GB_KEYS_BLOCKS: grid cap (key pass at scale 26: 11.1 / 10.8 / 10.0 / 10.0 ms at
    // 16384 / 2048 / 4096 / 8192 blocks with XCD-aware logical blocks, profiles/round6/r6_30)
    static int64_t gmax = -1;
    if (gmax < 0) {
      const char* e = std::getenv("DALGO_GB_KEYS_BLOCKS");
      gmax = e ? std::max<int64_t>(1, std::atoll(e)) : 8192;
    }
    const int64_t gw = std::min<int64_t>(cdiv(n, (int64_t)256 * 8), gmax);
    hipLaunchKernelGGL(gb_keys_one_kernel, dim3((unsigned)gw), dim3(256), 0, st, packed, n, c.new_id, c.dbits,
                       keys);
    DALGO_LAUNCH_CHECK();
    return hipSuccess;
  }
  if (phase == 0)
    hipLaunchKernelGGL(gb_keys_count_kernel, dim3((unsigned)g), dim3(256), 0, st, src, dst, n, c,
                       reinterpret_cast<uint8_t*>(bitmap), counts);
  else
    hipLaunchKernelGGL(gb_keys_write_kernel, dim3((unsigned)g), dim3(256), 0, st, src, dst, n, c, offsets,
                       base_all, keys, packed);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// rocPRIM onesweep radix sort of n u64 keys over bits [0, end_bit); tmp == nullptr: query.
// rocPRIM's gfx950 default (512 threads x 12 keys per tile, 8-bit digits) measured best
// among the configurations tried on 1.07B keys / 40 bits: 32.9 ms; 1024 x 12 / 8 bits 42.0;
// 512 x 16 / 10 bits (4 passes) 43.4; 11-bit digits do not fit the histogram kernel's LDS
// (profiles/round6/r6_19)
hipError_t dalgo_gb_sort(void* tmp, size_t* tmp_bytes, const uint64_t* in, uint64_t* out, int64_t n,
                         int begin_bit, int end_bit, hipStream_t st) {
  if (n < 0 || end_bit < 1 || end_bit > 64 || begin_bit < 0 || begin_bit >= end_bit) return hipErrorInvalidValue;
  return rocprim::radix_sort_keys(tmp, *tmp_bytes, in, out, (size_t)n, (unsigned)begin_bit, (unsigned)end_bit, st);
}

// keys sorted on bits [lo_bits, 64): every run of keys equal there sorted on its low
// lo_bits in place (lo_bits <= 13), no host synchronisation.
// ws: int64[dalgo_gb_run_ws(n)] workspace = [long-run count (zeroed here), long-run list]
int64_t dalgo_gb_run_ws(int64_t n) { return 1 + n / (kRunMid + 1) + 1; }

hipError_t dalgo_gb_run_sort(uint64_t* K, int64_t n, int lo_bits, int64_t* ws, hipStream_t st) {
  if (n <= 1) return hipSuccess;
  if (lo_bits < 1 || lo_bits > kSpanBits) return hipErrorInvalidValue;
  const int64_t g = cdiv(n, (int64_t)kRunTile);
  if (g > 0x7fffffffLL) return hipErrorInvalidValue;
  auto* nlong = reinterpret_cast<unsigned long long*>(ws);
  int64_t* longs = ws + 1;
  hipError_t e = hipMemsetAsync(ws, 0, sizeof(int64_t), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gb_run_tile_kernel, dim3((unsigned)g), dim3(kRunT), 0, st, K, n, lo_bits, longs, nlong);
  DALGO_LAUNCH_CHECK();
  // 4 blocks of 32 KB LDS per CU: one resident round
  hipLaunchKernelGGL(gb_run_long_kernel, dim3(1024), dim3(kRunT), 0, st, K, n, lo_bits,
                     (const int64_t*)longs, (const unsigned long long*)nlong);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// partitioned: starts = int64[cdiv(nv, 2^kBktBits) + 1] workspace (the bucket ranges,
// found by their own launch before any edge is rewritten)
hipError_t dalgo_gb_relabel_src(uint64_t* packed, int64_t n, const int32_t* new_id, int64_t nv, int partitioned,
                                int64_t* starts, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (partitioned) {
    const int64_t nb = cdiv(nv, (int64_t)1 << kBktBits);
    if (nv <= 0 || nb > 0x7fffffffLL || starts == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gb_bucket_starts_kernel<uint64_t>, dim3((unsigned)cdiv(nb + 1, 256)), dim3(256), 0, st,
                       (const uint64_t*)packed, n, (int)nb, starts);
    DALGO_LAUNCH_CHECK();
    hipLaunchKernelGGL(gb_relabel_bucket_kernel, dim3((unsigned)nb), dim3(256), 0, st, packed,
                       (const int64_t*)starts, new_id, nv);
    DALGO_LAUNCH_CHECK();
    return hipSuccess;
  }
  const int64_t g = std::min<int64_t>(cdiv(n, 256), 256 * 64);
  hipLaunchKernelGGL(gb_relabel_src_kernel, dim3((unsigned)g), dim3(256), 0, st, packed, n, new_id);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_gb_pack(const int32_t* src, const int32_t* dst, int64_t n, uint64_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t g = std::min<int64_t>(cdiv(n, 256), 256 * 64);
  hipLaunchKernelGGL(gb_pack_kernel, dim3((unsigned)g), dim3(256), 0, st, src, dst, n, out);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// keys per decode block: kDecR, or DALGO_GB_DEC_ROWS (a multiple of kDecT * kDecV) for A/B
static int64_t gb_dec_rows() {
  static int64_t v = [] {
    const char* e = getenv("DALGO_GB_DEC_ROWS");
    const int64_t x = e ? atoll(e) : 0;
    return (x >= kDecT * kDecV && x % (kDecT * kDecV) == 0) ? x : (int64_t)kDecR;
  }();
  return v;
}

int64_t dalgo_gb_decode_blocks(int64_t n) { return cdiv(n, gb_dec_rows()); }

// phase 0: counts[2 b], [2 b + 1] = distinct edges / entries of block b, outdeg += the
// distinct out-degrees; phase 1 (offsets = exclusive scan of counts): srcl and the entries
hipError_t dalgo_gb_decode(const uint64_t* K, int64_t n, int shift, int dbits, const int64_t* blk_base,
                           int phase, int64_t* counts, uint32_t* outdeg, const int64_t* offsets,
                           uint16_t* srcl, int64_t* ent_end, int32_t* ent_blk, int32_t* ent_dst,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (shift < kSpanBits || shift > 63 || dbits < 0 || dbits > 31) return hipErrorInvalidValue;
  const int64_t dr = gb_dec_rows();
  const int64_t g = cdiv(n, dr);
  if (phase == 0)
    hipLaunchKernelGGL(gb_decode_count_kernel, dim3((unsigned)g), dim3(kDecT), 0, st, K, n, dr, shift, blk_base,
                       counts, outdeg);
  else
    hipLaunchKernelGGL(gb_decode_write_kernel, dim3((unsigned)g), dim3(kDecT), 0, st, K, n, dr, shift, dbits,
                       offsets, srcl, ent_end, ent_blk, ent_dst);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_gb_entry_flags(const int32_t* ent_blk, const int32_t* ent_dst, const int64_t* ent_end,
                                int64_t nent, int bin_shift, uint8_t* rs, uint8_t* cs, uint16_t* srcl,
                                hipStream_t st) {
  if (nent <= 0) return hipSuccess;
  const int64_t g = std::min<int64_t>(cdiv(nent, 256), 256 * 64);
  hipLaunchKernelGGL(gb_entry_flags_kernel, dim3((unsigned)g), dim3(256), 0, st, ent_blk, ent_dst, ent_end,
                     nent, bin_shift, rs, cs, srcl);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_gb_entry_place(const int32_t* ent_dst, const int64_t* ent_end, int64_t nent,
                                const int32_t* run_of_ent, const int32_t* run_delta, const int32_t* run_chunk,
                                const uint8_t* cs, const int64_t* ce_lo, const int64_t* tlen, int64_t wu_e,
                                int bin_mask, int16_t* dloc, uint8_t* ts, hipStream_t st) {
  if (nent <= 0) return hipSuccess;
  if (wu_e < 1) return hipErrorInvalidValue;
  const int64_t g = std::min<int64_t>(cdiv(nent, 256), 256 * 64);
  hipLaunchKernelGGL(gb_entry_place_kernel, dim3((unsigned)g), dim3(256), 0, st, ent_dst, ent_end, nent,
                     run_of_ent, run_delta, run_chunk, cs, ce_lo, tlen, wu_e, bin_mask, dloc, ts);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}


hipError_t dalgo_gb_cells(int phase, const int32_t* ent_blk, const int32_t* ent_dst, int64_t nent, int bshift,
                          int nblk, int nbins, int32_t* C, int64_t* T, int64_t* R, const int64_t* RE,
                          const int64_t* RR, int32_t* CM, int32_t* RID, int G, int64_t* P, const int64_t* Poff,
                          const int32_t* CI, int64_t nruns, int32_t* run_delta, int32_t* run_chunk,
                          int64_t* run_first, hipStream_t st) {
  if (nblk < 1 || nbins < 1 || (int64_t)nblk * nbins > ((int64_t)1 << 31)) return hipErrorInvalidValue;
  const int ng = G > 0 ? (nblk + G - 1) / G : 0;
  switch (phase) {
    case 0: {   // counts
      if (nent <= 0) return hipSuccess;
      const int64_t g = std::min<int64_t>(cdiv(nent, 256 * kCellEpt), 256 * 64);
      hipLaunchKernelGGL(gb_cell_count_kernel, dim3((unsigned)g), dim3(256), 0, st, ent_blk, ent_dst, nent, bshift,
                         nblk, nbins, C);
      break;
    }
    case 1:     // row totals
      hipLaunchKernelGGL(gb_cell_rows_kernel, dim3((unsigned)nblk), dim3(256), 0, st, (const int32_t*)C, nbins, T, R);
      break;
    case 2:     // row scans
      hipLaunchKernelGGL(gb_cell_scan_kernel, dim3((unsigned)nblk), dim3(256), 0, st, (const int32_t*)C, nbins, RE,
                         RR, CM, RID);
      break;
    case 3:     // column sums per row group
      if (G < 1) return hipErrorInvalidValue;
      hipLaunchKernelGGL(gb_cell_colsum_kernel, dim3((unsigned)cdiv(nbins, 256), (unsigned)ng), dim3(256), 0, st,
                         (const int32_t*)C, nblk, nbins, G, P);
      break;
    case 4:     // run tables
      if (G < 1) return hipErrorInvalidValue;
      hipLaunchKernelGGL(gb_cell_place_kernel, dim3((unsigned)cdiv(nbins, 256), (unsigned)ng), dim3(256), 0, st,
                         (const int32_t*)C, (const int32_t*)CM, (const int32_t*)RID, nblk, nbins, G, Poff, CI, nruns,
                         run_delta, run_chunk, run_first);
      break;
    default:
      return hipErrorInvalidValue;
  }
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t dalgo_gb_entry_cells(const int32_t* ent_blk, const int32_t* ent_dst, const int64_t* ent_end, int64_t nent,
                                int bshift, int nblk, int nbins, const int32_t* CM, const int32_t* RID,
                                const int32_t* run_delta, int64_t nruns, const int64_t* RE, const int32_t* CI,
                                const int64_t* ce_lo, const int64_t* tlen, int64_t nch, int64_t wu_e, int bin_mask,
                                int16_t* dloc, int64_t ndloc, int32_t* tiles, unsigned long long* n_tiles,
                                int64_t tile_cap, uint16_t* srcl, int64_t nsrcl, hipStream_t st) {
  if (nent <= 0) return hipSuccess;
  if (wu_e < 1 || nent >= (int64_t)0x7fffffffLL) return hipErrorInvalidValue;
  const int64_t g = std::min<int64_t>(cdiv(nent, 256 * kCellEpt), 256 * 64);
  hipLaunchKernelGGL(gb_entry_cells_kernel, dim3((unsigned)g), dim3(256), 0, st, ent_blk, ent_dst, ent_end, nent,
                     bshift, nblk, nbins, CM, RID, run_delta, nruns, RE, CI, ce_lo, tlen, nch, wu_e, bin_mask, dloc,
                     ndloc, tiles, n_tiles, tile_cap, srcl, nsrcl);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
