// Native adjacency build of the PageRank job (graph_computation/pagerank.py:41,44:
// ``links.distinct().groupByKey().cache()`` + ``count()``), gfx950.
//
// The K4b layout (pr_binned.hip) wants the deduplicated edges ordered by (source chunk,
// destination, source): one 64-bit key per edge = block | local destination | source
// offset in its 8192-source block, so ONE radix sort (rocPRIM onesweep over only the
// key's bits) puts the edges in layout order, and the decode pass skips the duplicates
// (a distinct edge = the last copy of its key). The passes around it are single sweeps:
//   degree   -- raw out-degree of the input edges (degree relabeling), u32 atomics;
//   keys     -- relabel, keep this rank's destinations, map sources to the [own | ghost]
//               index space and pack the key (two-phase compaction: count, write);
//   decode   -- per distinct edge the u16 source offset + entry-end bit, the entry list
//               (end edge, block, destination) and the deduplicated out-degree of every
//               source (LDS-privatised histogram per 8192-source block, no global atomic
//               per edge);
//   entries  -- run-start bits (a run = the entries of one (block, destination bin)),
//               chunk starts, bin-major destination offsets and tile starts.
// Everything else (per-chunk / per-run tables, a few thousand to a few million rows) is
// torch on the device (dalgo/ops/graph.py::build_blocked_native).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdint>

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

// degree by sort: over the SORTED ids, every run boundary records where the run of its id
// starts and where the previous id's run ends (deg = end - start; absent ids stay 0 / 0)
__global__ void __launch_bounds__(256) gb_runs_kernel(const uint32_t* __restrict__ sorted, int64_t n,
                                                      int32_t* __restrict__ start, int32_t* __restrict__ end) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i <= n; i += stride) {
    const uint32_t cur = i < n ? sorted[i] : 0u;
    const uint32_t prev = i > 0 ? sorted[i - 1] : 0u;
    if (i == n) {
      end[prev] = (int32_t)n;
    } else if (i == 0 || cur != prev) {
      start[cur] = (int32_t)i;
      if (i > 0) end[prev] = (int32_t)i;
    }
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
};

__device__ __forceinline__ bool gb_edge(const GbKeyCtx& c, int32_t s0, int32_t d0, int32_t& s,
                                        int64_t& dl) {
  s = c.new_id ? c.new_id[s0] : s0;
  const int32_t d = c.new_id ? c.new_id[d0] : d0;
  dl = (int64_t)d - c.v_lo;
  return d >= c.v_lo && d < c.v_hi;
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
                                         bool (&in)[kKeyV]) {
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

// phase 0: count the kept edges per block (and mark remote sources, W > 1)
__global__ void __launch_bounds__(256) gb_keys_count_kernel(const int32_t* __restrict__ src,
                                                            const int32_t* __restrict__ dst, int64_t n,
                                                            GbKeyCtx c, uint32_t* __restrict__ bitmap,
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
        if (c.world > 1 && !(sv >= c.v_lo && sv < c.v_hi)) atomicOr(bitmap + (sv >> 5), 1u << (sv & 31));
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
                                                            int64_t base_all, uint64_t* __restrict__ keys) {
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
    gb_load4(src, dst, i, r1, s0, d0, in);
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

// ---------------------------------------------------------------------------- decode
// Over the SORTED keys with duplicates (the dedup is folded in: no separate unique pass).
// The last copy of every key stands for the distinct edge; an entry (block, destination)
// ends at the last copy of its last key. Blocks of kDecR keys, each thread 4 consecutive
// keys per step (coalesced), one block scan per step places the distinct edges and the
// entries in key order.
constexpr int kDecR = 65536;         // keys per block of the decode kernels
constexpr int kDecT = 256;
constexpr int kDecV = 4;             // keys per thread per step

__device__ __forceinline__ void gb_flags(const uint64_t* __restrict__ K, int64_t n, int64_t i,
                                         bool& last, bool& end, uint64_t& k) {
  k = K[i];
  const bool has_next = i + 1 < n;
  const uint64_t kn = has_next ? K[i + 1] : ~0ull;
  last = !has_next || kn != k;
  end = last && (!has_next || (kn >> kSpanBits) != (k >> kSpanBits));
}

// per block: distinct edges, entries, and the distinct out-degree per local source (LDS
// histogram of the block's first source block; other source blocks: global atomics)
__global__ void __launch_bounds__(kDecT) gb_decode_count_kernel(const uint64_t* __restrict__ K, int64_t n,
                                                                int shift, const int64_t* __restrict__ blk_base,
                                                                int64_t* __restrict__ counts,
                                                                uint32_t* __restrict__ outdeg) {
  __shared__ uint32_t hist[kSpan];
  __shared__ int s_d, s_e;
  for (int j = threadIdx.x; j < kSpan; j += kDecT) hist[j] = 0u;
  if (threadIdx.x == 0) { s_d = 0; s_e = 0; }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kDecR;
  const int64_t r1 = r0 + kDecR < n ? r0 + kDecR : n;
  const uint64_t blk0 = K[r0] >> shift;
  int md = 0, me = 0;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += kDecT) {
    bool last, end;
    uint64_t k;
    gb_flags(K, n, i, last, end, k);
    if (last) {
      ++md;
      const uint64_t blk = k >> shift;
      const uint32_t off = (uint32_t)(k & (kSpan - 1));
      if (blk == blk0) atomicAdd(hist + off, 1u);
      else atomicAdd(outdeg + blk_base[blk] + off, 1u);
    }
    me += end ? 1 : 0;
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
                                                                int shift, int dbits,
                                                                const int64_t* __restrict__ offsets,
                                                                uint16_t* __restrict__ srcl,
                                                                int64_t* __restrict__ ent_end,
                                                                int32_t* __restrict__ ent_blk,
                                                                int32_t* __restrict__ ent_dst) {
  __shared__ int s_wd[kDecT / 64], s_we[kDecT / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * kDecR;
  const int64_t r1 = r0 + kDecR < n ? r0 + kDecR : n;
  int64_t dbase = offsets[2 * blockIdx.x], ebase = offsets[2 * blockIdx.x + 1];
  const uint64_t dmask = (1ull << dbits) - 1ull;
  for (int64_t i0 = r0; i0 < r1; i0 += (int64_t)kDecT * kDecV) {
    const int64_t ib = i0 + (int64_t)threadIdx.x * kDecV;
    bool last[kDecV], end[kDecV];
    uint64_t k[kDecV];
    int cd = 0, ce = 0;
#pragma unroll
    for (int v = 0; v < kDecV; ++v) {
      last[v] = end[v] = false;
      k[v] = 0;
      if (ib + v < r1) gb_flags(K, n, ib + v, last[v], end[v], k[v]);
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
                           int end_bit, hipStream_t st) {
  if (n < 0 || n >= (int64_t)0x7fffffffLL || end_bit < 1 || end_bit > 32) return hipErrorInvalidValue;
  return rocprim::radix_sort_keys(tmp, *tmp_bytes, in, out, (size_t)n, 0u, (unsigned)end_bit, st);
}

hipError_t dalgo_gb_runs(const uint32_t* sorted, int64_t n, int32_t* start, int32_t* end, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n >= (int64_t)0x7fffffffLL) return hipErrorInvalidValue;
  const int64_t g = std::min<int64_t>(cdiv(n + 1, 256), 256 * 64);
  hipLaunchKernelGGL(gb_runs_kernel, dim3((unsigned)g), dim3(256), 0, st, sorted, n, start, end);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

int64_t dalgo_gb_key_blocks(int64_t n) { return cdiv(n, (int64_t)kKeyR); }

hipError_t dalgo_gb_keys(const int32_t* src, const int32_t* dst, int64_t n, const DalgoGbKeyArgs* a,
                         int phase, uint32_t* bitmap, int32_t* counts, const int64_t* offsets,
                         int64_t base_all, uint64_t* keys, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (a->dbits < 0 || a->dbits > 31 || a->world < 1) return hipErrorInvalidValue;
  GbKeyCtx c{a->v_lo, a->v_hi, a->sl, a->world, a->rank, a->dbits, a->new_id, a->bitmap,
             a->word_prefix, a->seg_start, a->seg_blk0};
  if (c.world > 1 && (c.sl <= 0 || (phase == 1 && (!c.bitmap || !c.word_prefix || !c.seg_start || !c.seg_blk0))))
    return hipErrorInvalidValue;
  const int64_t g = cdiv(n, (int64_t)kKeyR);
  if (g > 0x7fffffffLL) return hipErrorInvalidValue;
  if (phase == 0)
    hipLaunchKernelGGL(gb_keys_count_kernel, dim3((unsigned)g), dim3(256), 0, st, src, dst, n, c, bitmap, counts);
  else
    hipLaunchKernelGGL(gb_keys_write_kernel, dim3((unsigned)g), dim3(256), 0, st, src, dst, n, c, offsets,
                       base_all, keys);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// rocPRIM onesweep radix sort of n u64 keys over bits [0, end_bit); tmp == nullptr: query
hipError_t dalgo_gb_sort(void* tmp, size_t* tmp_bytes, const uint64_t* in, uint64_t* out, int64_t n,
                         int end_bit, hipStream_t st) {
  if (n < 0 || end_bit < 1 || end_bit > 64) return hipErrorInvalidValue;
  return rocprim::radix_sort_keys(tmp, *tmp_bytes, in, out, (size_t)n, 0u, (unsigned)end_bit, st);
}

int64_t dalgo_gb_decode_blocks(int64_t n) { return cdiv(n, (int64_t)kDecR); }

// phase 0: counts[2 b], [2 b + 1] = distinct edges / entries of block b, outdeg += the
// distinct out-degrees; phase 1 (offsets = exclusive scan of counts): srcl and the entries
hipError_t dalgo_gb_decode(const uint64_t* K, int64_t n, int shift, int dbits, const int64_t* blk_base,
                           int phase, int64_t* counts, uint32_t* outdeg, const int64_t* offsets,
                           uint16_t* srcl, int64_t* ent_end, int32_t* ent_blk, int32_t* ent_dst,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (shift < kSpanBits || shift > 63 || dbits < 0 || dbits > 31) return hipErrorInvalidValue;
  const int64_t g = cdiv(n, (int64_t)kDecR);
  if (phase == 0)
    hipLaunchKernelGGL(gb_decode_count_kernel, dim3((unsigned)g), dim3(kDecT), 0, st, K, n, shift, blk_base,
                       counts, outdeg);
  else
    hipLaunchKernelGGL(gb_decode_write_kernel, dim3((unsigned)g), dim3(kDecT), 0, st, K, n, shift, dbits,
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

}  // extern "C"
