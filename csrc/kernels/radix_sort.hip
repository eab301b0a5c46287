// LSD radix sort of u32 / u64 keys over a bit range [begin_bit, end_bit), gfx950 -- the
// native adjacency build's sorts (graph_computation/pagerank.py:41 ``distinct().groupByKey()``:
// the edge keys, the source partitions feeding the degree relabeling, the degree ranking),
// replacing the rocPRIM onesweep sort that was the largest library kernel of the PageRank job.
//
// Reduce-then-scan LSD passes of 8-bit digits, no inter-workgroup waiting:
//   count   -- one block per tile of TK = 256 * KPT keys: the tile's digit histogram
//              (LDS, one copy per wave) -> C[tile][digit], and the digit totals;
//   scan    -- per digit, the exclusive prefix over the tiles plus the digit's bucket start
//              (two kernels: per-chunk partial sums, then each chunk's running prefix), all
//              reads / writes coalesced (thread = digit, consecutive tiles);
//   scatter -- one block per tile: ranks its keys by digit (wave match: 8 ballots give the
//              lanes with the same digit; the group leader's LDS atomic reserves the group's
//              places), reorders them through LDS and writes digit runs at C's offsets.
// A decoupled look-back "onesweep" form (one pass over the keys instead of two) measured
// 48-64 ms for a 1.07B-key 5-pass sort against 19.7 ms with the look-back removed: a hop
// between workgroups costs microseconds under load and the walks got long
// (profiles/round6/r6_11 - r6_15). The extra read of the count pass is cheaper.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dalgo/common.h"
#include "launchers.h"

namespace dalgo {
namespace {

constexpr int kRsT = 256;            // threads per block = digits per pass
constexpr int kRsBits = 8;
constexpr int kRsMaxPass = 8;

template <typename K>
struct RsGeom {
  static constexpr int KPT = sizeof(K) == 8 ? 16 : 24;   // keys per thread (LDS: 32 / 24 KB)
  static constexpr int TK = kRsT * KPT;                  // keys per tile
};

// lanes of this wave whose (valid) digit equals this lane's: AND of 8 bit-ballots
__device__ __forceinline__ uint64_t rs_match(unsigned d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < kRsBits; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t v = __ballot(bit);
    m &= bit ? v : ~v;
  }
  return m;
}

// ---------------------------------------------------------------------------- count
// the key layout of a tile (count and scatter): wave w holds keys [base + 64 KPT w, +64 KPT),
// row i = 64 consecutive keys (coalesced); (wave, row, lane) is the input order
template <typename K>
__global__ void __launch_bounds__(kRsT) rs_count_kernel(const K* __restrict__ in, int64_t n, int shift, int nbits,
                                                       unsigned* __restrict__ C, unsigned* __restrict__ tot) {
  constexpr int KPT = RsGeom<K>::KPT, TK = RsGeom<K>::TK;
  constexpr int NW = kRsT / 64;
  __shared__ unsigned s_h[NW][kRsT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const unsigned dmask = (1u << nbits) - 1u;
  const int64_t nt = (n + TK - 1) / TK;
  unsigned mine = 0;                           // this block's total of digit tid
  // persistent: the block walks tiles blockIdx.x, + gridDim.x, ... (one tile per block
  // left the read at ~1.8 TB/s: block start-up per 32 KB, profiles/round6/r6_16)
  for (int64_t tile = blockIdx.x; tile < nt; tile += gridDim.x) {
#pragma unroll
    for (int w = 0; w < NW; ++w) s_h[w][tid] = 0u;
    __syncthreads();
    const int64_t base = tile * TK + (int64_t)wid * (64 * KPT) + lane;
    K k[KPT];
#pragma unroll
    for (int i = 0; i < KPT; ++i) k[i] = base + i * 64 < n ? in[base + i * 64] : K(0);
#pragma unroll
    for (int i = 0; i < KPT; ++i)
      if (base + i * 64 < n) atomicAdd(&s_h[wid][(unsigned)(k[i] >> shift) & dmask], 1u);
    __syncthreads();
    unsigned c = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) c += s_h[w][tid];
    C[tile * kRsT + tid] = c;
    mine += c;
    __syncthreads();
  }
  if (mine) atomicAdd(tot + tid, mine);
}

// ---------------------------------------------------------------------------- scan
constexpr int kRsChunk = 512;        // tiles per scan chunk

// P[chunk][digit] = sum of C[tile][digit] over the chunk's tiles
__global__ void __launch_bounds__(kRsT) rs_scan_partial_kernel(const unsigned* __restrict__ C, int64_t ntiles,
                                                              unsigned* __restrict__ P) {
  const int tid = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * kRsChunk;
  const int64_t t1 = min(ntiles, t0 + kRsChunk);
  unsigned s = 0;
  for (int64_t t = t0; t < t1; ++t) s += C[t * kRsT + tid];
  P[(int64_t)blockIdx.x * kRsT + tid] = s;
}

// O[tile][digit] = bucket start of the digit (exclusive scan of the totals) + its count in
// every earlier tile (earlier chunks' P, then a running sum over the chunk)
__global__ void __launch_bounds__(kRsT) rs_scan_final_kernel(const unsigned* __restrict__ C, int64_t ntiles,
                                                            const unsigned* __restrict__ P,
                                                            const unsigned* __restrict__ tot,
                                                            unsigned* __restrict__ O) {
  __shared__ unsigned s_w[kRsT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const unsigned h = tot[tid];
  unsigned x = h;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_w[wid] = x;
  __syncthreads();
  unsigned run = x - h;
#pragma unroll
  for (int w = 0; w < kRsT / 64; ++w) run += w < wid ? s_w[w] : 0u;
  for (int64_t b = 0; b < blockIdx.x; ++b) run += P[b * kRsT + tid];
  const int64_t t0 = (int64_t)blockIdx.x * kRsChunk;
  const int64_t t1 = min(ntiles, t0 + kRsChunk);
  for (int64_t t = t0; t < t1; ++t) {
    const unsigned c = C[t * kRsT + tid];
    O[t * kRsT + tid] = run;
    run += c;
  }
}

// ---------------------------------------------------------------------------- scatter
template <typename K>
__global__ void __launch_bounds__(kRsT) rs_scatter_kernel(const K* __restrict__ in, K* __restrict__ out, int64_t n,
                                                         int shift, int nbits, const unsigned* __restrict__ O) {
  constexpr int KPT = RsGeom<K>::KPT, TK = RsGeom<K>::TK;
  constexpr int NW = kRsT / 64;
  __shared__ K s_k[TK];
  __shared__ unsigned s_wc[NW][kRsT];          // per wave: running count, then start, per digit
  __shared__ long long s_gb[kRsT];             // global start of a digit's run minus its local start
  __shared__ unsigned s_scan[NW];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const unsigned dmask = (1u << nbits) - 1u;
  const int64_t nt = (n + TK - 1) / TK;
  for (int64_t tile = blockIdx.x; tile < nt; tile += gridDim.x) {
#pragma unroll
  for (int w = 0; w < NW; ++w) s_wc[w][tid] = 0u;
  const int64_t base = tile * TK;
  const unsigned gstart = O[tile * kRsT + tid];
  __syncthreads();
  K k[KPT];
  unsigned d[KPT];
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    const int64_t idx = base + (int64_t)wid * (64 * KPT) + i * 64 + lane;
    const bool valid = idx < n;
    k[i] = valid ? in[idx] : K(0);
    d[i] = valid ? (unsigned)(k[i] >> shift) & dmask : 0xffffffffu;
  }
  // rank within (wave, digit): the group leader's LDS atomic reserves the group's places
  // in the wave's running count; the base reaches the group by a lane permute
  unsigned r[KPT];
  constexpr int HB = KPT / 2;
#pragma unroll
  for (int h0 = 0; h0 < KPT; h0 += HB) {
    unsigned old[HB];
    int lead[HB];
#pragma unroll
    for (int i = 0; i < HB; ++i) {
      const int ii = h0 + i;
      const bool valid = d[ii] != 0xffffffffu;
      const uint64_t m = rs_match(valid ? d[ii] : 0u, valid);
      lead[i] = __ffsll((long long)m) - 1;
      r[ii] = (unsigned)__popcll(m & ((1ull << lane) - 1ull));
      old[i] = 0u;
      if (valid && lane == lead[i]) old[i] = atomicAdd(&s_wc[wid][d[ii]], (unsigned)__popcll(m));
    }
#pragma unroll
    for (int i = 0; i < HB; ++i) r[h0 + i] += (unsigned)__shfl((int)old[i], lead[i] < 0 ? 0 : lead[i], 64);
  }
  __syncthreads();
  // digit tid: tile count, local start (exclusive scan over digits), per-wave starts
  unsigned cw[NW];
  unsigned cnt = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    cw[w] = s_wc[w][tid];
    cnt += cw[w];
  }
  unsigned x = cnt;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_scan[wid] = x;
  __syncthreads();
  unsigned loc = x - cnt;
#pragma unroll
  for (int w = 0; w < NW; ++w) loc += w < wid ? s_scan[w] : 0u;
  s_gb[tid] = (long long)gstart - (long long)loc;
  unsigned run = loc;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    s_wc[w][tid] = run;
    run += cw[w];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < KPT; ++i)
    if (d[i] != 0xffffffffu) s_k[s_wc[wid][d[i]] + r[i]] = k[i];
  __syncthreads();
  const int nvalid = (int)min((int64_t)TK, n - base);
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    const int jj = i * kRsT + tid;
    if (jj < nvalid) {
      const K kk = s_k[jj];
      out[s_gb[(unsigned)(kk >> shift) & dmask] + jj] = kk;
    }
  }
  __syncthreads();                             // s_k / s_wc / s_gb reused by the next tile
  }
}

template <typename K>
int64_t rs_tiles(int64_t n) { return (n + RsGeom<K>::TK - 1) / RsGeom<K>::TK; }

int rs_passes(int begin_bit, int end_bit) { return (end_bit - begin_bit + kRsBits - 1) / kRsBits; }

// workspace (bytes): [tot 256 u32 | P chunks x 256 u32 | C tiles x 256 u32 | O tiles x 256 u32]
template <typename K>
size_t rs_ws_bytes(int64_t n, int /*npass*/) {
  const int64_t nt = rs_tiles<K>(n);
  const int64_t nc = (nt + kRsChunk - 1) / kRsChunk;
  return (size_t)(kRsT + nc * kRsT + 2 * nt * kRsT) * 4;
}

template <typename K>
hipError_t rs_sort(const K* in, K* out, K* tmp, int64_t n, int begin_bit, int end_bit, void* ws, size_t ws_bytes,
                   unsigned* err_out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int kb = (int)sizeof(K) * 8;
  if (begin_bit < 0 || end_bit > kb || begin_bit >= end_bit) return hipErrorInvalidValue;
  const int npass = rs_passes(begin_bit, end_bit);
  if (npass > kRsMaxPass || ws_bytes < rs_ws_bytes<K>(n, npass) || n > 0xffffffffLL) return hipErrorInvalidValue;
  if (npass > 1 && tmp == nullptr) return hipErrorInvalidValue;
  const int64_t nt = rs_tiles<K>(n);
  const int64_t nc = (nt + kRsChunk - 1) / kRsChunk;
  if (nt > 0x7fffffffLL) return hipErrorInvalidValue;
  unsigned* tot = reinterpret_cast<unsigned*>(ws);
  unsigned* P = tot + kRsT;
  unsigned* C = P + nc * kRsT;
  unsigned* O = C + nt * kRsT;
  // ping-pong so that the last pass writes `out`
  const K* src = in;
  for (int p = 0; p < npass; ++p) {
    K* dst = ((npass - 1 - p) % 2 == 0) ? out : tmp;
    const int sh = begin_bit + kRsBits * p;
    const int nb = std::min(kRsBits, end_bit - sh);
    hipError_t e = hipMemsetAsync(tot, 0, kRsT * sizeof(unsigned), st);
    if (e != hipSuccess) return e;
    const unsigned pg = (unsigned)std::min<int64_t>(nt, 1024);   // resident: 4 blocks per CU
    hipLaunchKernelGGL(rs_count_kernel<K>, dim3(pg), dim3(kRsT), 0, st, src, n, sh, nb, C, tot);
    DALGO_LAUNCH_CHECK();
    hipLaunchKernelGGL(rs_scan_partial_kernel, dim3((unsigned)nc), dim3(kRsT), 0, st, (const unsigned*)C, nt, P);
    DALGO_LAUNCH_CHECK();
    hipLaunchKernelGGL(rs_scan_final_kernel, dim3((unsigned)nc), dim3(kRsT), 0, st, (const unsigned*)C, nt,
                       (const unsigned*)P, (const unsigned*)tot, O);
    DALGO_LAUNCH_CHECK();
    hipLaunchKernelGGL(rs_scatter_kernel<K>, dim3(pg), dim3(kRsT), 0, st, src, dst, n, sh, nb,
                       (const unsigned*)O);
    DALGO_LAUNCH_CHECK();
    src = dst;
  }
  if (err_out != nullptr) {   // (no waiting form left: nothing can give up)
    hipError_t e = hipMemsetAsync(err_out, 0, sizeof(unsigned), st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace
}  // namespace dalgo

using namespace dalgo;

extern "C" {

size_t dalgo_rs_ws_bytes(int64_t n, int key_bytes, int begin_bit, int end_bit) {
  const int np = rs_passes(begin_bit, end_bit);
  return key_bytes == 8 ? rs_ws_bytes<uint64_t>(n, np) : rs_ws_bytes<uint32_t>(n, np);
}

// keys in[0, n) sorted on bits [begin_bit, end_bit) into out (stable; in untouched; tmp: n
// keys of scratch when more than one pass); err_out (device u32, nullable): 1 if a look-back
// gave up (result invalid)
hipError_t dalgo_rs_sort64(const uint64_t* in, uint64_t* out, uint64_t* tmp, int64_t n, int begin_bit, int end_bit,
                           void* ws, size_t ws_bytes, unsigned* err_out, hipStream_t st) {
  return rs_sort<uint64_t>(in, out, tmp, n, begin_bit, end_bit, ws, ws_bytes, err_out, st);
}

hipError_t dalgo_rs_sort32(const uint32_t* in, uint32_t* out, uint32_t* tmp, int64_t n, int begin_bit, int end_bit,
                           void* ws, size_t ws_bytes, unsigned* err_out, hipStream_t st) {
  return rs_sort<uint32_t>(in, out, tmp, n, begin_bit, end_bit, ws, ws_bytes, err_out, st);
}

}  // extern "C"
