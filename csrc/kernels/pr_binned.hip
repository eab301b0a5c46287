// K4b: PageRank SpMV by two-level propagation blocking (no random global gathers).
//
// Reference: graph_computation/pagerank.py:52-57 — flatMap(computeContribs) emits one
// (dst, c[src]) record per edge, reduceByKey(add) sums them per destination. The pull
// K4 (pagerank.hip) does that sum as a gather of c[src] per edge; at R-MAT scale 26 it
// is bound by the per-lane random gathers (TA 86 % busy, profiles/round3/pmc_pagerank.md).
// Here the records are produced and reduced without a single random global access:
//
//   layout (built once, dalgo.ops.graph.build_blocked):
//     chunks  : contiguous SOURCE ranges of <= S vertices (one LDS table of c each; on
//               several ranks never straddling the own-slice / ghost boundary);
//     edges   : sorted by (chunk, dst, src); per edge a u16 = local source (13 bits)
//               | 0x4000 on the end edge of a run's first entry | 0x8000 on an entry's
//               end edge;
//     entries : distinct (chunk, dst) pairs = the chunk's records with equal destination
//               pre-combined (an R-MAT hot destination appears once per chunk, not once
//               per edge: 0.44 entries per edge at scale 26); stored BIN-MAJOR: all
//               entries of destination bin b (BW destinations) contiguous, chunk order
//               inside the bin;
//     runs    : the entries of one (chunk, bin); an entry's bin-major position is its
//               chunk-major index + the run's delta (one int per non-empty run);
//     work units: ranges of one chunk's wave tiles (a hot chunk spans several).
//   phase 1 (pb_gather): one workgroup per work unit stages c[chunk sources] and the
//     chunk's run deltas in LDS; its waves stream the edges (2 B each, a 4-step load
//     ring), read c from LDS, reduce the (dst-sorted) records to one value per entry with
//     a segmented DPP scan and store the entry values through a per-wave LDS transpose
//     (64 consecutive entries per store instruction). The chunk's first unit also adds
//     the chunk's present c to a bound of every destination sum.
//   phase 2 (pb_accum): one workgroup per contiguous bin-major entry range (a bin, or a
//     piece of a hot bin) streams (value, u16 destination offset) pairs and adds them
//     into BW u64 fixed-point LDS accumulators (ds_add_u64: gfx950 runs ds_add_f32 ~28x
//     slower; integer sums are exact and order independent); the scale 2^K comes from
//     phase 1's bound; it writes the bin's sums -- or runs the PageRank update on them --
//     or a partial slab that pb_combine sums.
//
// Per edge 2 B, per entry 4 B written + 6 B read, all streamed: ~6 B per edge at
// scale 26 instead of the pull form's ~58 B of fabric traffic per edge.
//
// "reference" semantics: c < 0 marks an absent source; its record does not exist. Every
// present record adds >= 1 fixed-point unit, so a destination received >= 1 record iff
// its sum is non-zero.
#include "dalgo/common.h"
#include "launchers.h"   // the extern "C" entry point is checked against its declaration
#include <algorithm>
#include <type_traits>

namespace dalgo {

constexpr int kPbDummy = 65536;   // padding floats after the entries (phase-1 dummy stores)
// fraction bits of the phase-1 sum bound (u64 fixed point: sums of present c up to 2^43)
constexpr int kPbBoundFrac = 20;

namespace {

// DPP moves (gfx9 family): lanes whose source is outside the pattern keep `old`
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp_mov_f(float old, float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL,
                                                    ROWS, 0xf, false));
}
typedef int pb_v4i __attribute__((ext_vector_type(4)));

// Phase 1's edge ring and entry stores are issued as inline asm with hand-counted waits:
// the compiler's own vmcnt bookkeeping treats a mix of pending loads and stores as out of
// order and waited vmcnt(0..2) at every step; it sees no vector memory op in the step
// loop now, so it places no wait there. The stores use the SGPR-base form with a 32-bit
// byte offset (one select per store instead of a 64-bit address).
__device__ __forceinline__ pb_v4i pb_ld16(const void* p) {
  pb_v4i r;
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ void pb_st4(float* base, uint32_t off_bytes, float v) {
  asm volatile("global_store_dword %0, %1, %2" :: "v"(off_bytes), "v"(v), "s"(base) : "memory");
}
template <int N>
__device__ __forceinline__ void pb_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ int dpp_mov_i(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWS, 0xf, false);
}

// one step of the inclusive segmented scan of a (open-segment sum) together with the
// packed int scan c = entries | run starts << 16 (each <= 512 per step: no carry between
// the fields). "A segment closed inside the window" is exactly "the window's entry count
// is non-zero", so the segment flag needs no scan of its own
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ void scan_step(float& a, int& c) {
  const float a_up = dpp_mov_f<CTRL, ROWS>(-0.0f, a);
  const int c_up = dpp_mov_i<CTRL, ROWS>(0, c);
  if ((c & 0xffff) == 0) a = a_up + a;
  c += c_up;
}

}  // namespace

// S: max sources per chunk (LDS table); R: run deltas staged in LDS (GRUNS: a chunk with
// more runs reads them from global memory); NW waves per block; EPL edges per lane per
// step. The step body is branch-free up to the entry stores (loads from clamped
// addresses, selects instead of guarded reads), so the compiler's wait counts stay exact
// and the prefetched loads stay in flight.
template <int S, int R, int NW, bool GRUNS>
__global__ void __launch_bounds__(NW * 64)
pb_gather_kernel(const uint16_t* __restrict__ srcl, const int64_t* __restrict__ tile_e,
                 const int32_t* __restrict__ tile_ent, const int32_t* __restrict__ tile_run,
                 const int32_t* __restrict__ wu_tile, const int32_t* __restrict__ wu_chunk,
                 const int32_t* __restrict__ chunk_slo,
                 const int32_t* __restrict__ chunk_ns, const int32_t* __restrict__ chunk_run,
                 const int32_t* __restrict__ run_delta, const float* __restrict__ c,
                 float* __restrict__ val, int64_t dummy_base,
                 unsigned long long* __restrict__ bound, int wu0) {
  static_assert(S <= 16384, "local source index must leave bits 14, 15 for the markers");
  constexpr int EPL = 8;
  constexpr int D = 4;                        // steps of edges loaded ahead
  __shared__ float s_c[S];
  __shared__ int32_t s_d[GRUNS ? 1 : R];
  // per-wave staging of one step's entry values: the lane that reduces an entry is not
  // the lane that stores it; stores go out as 64 consecutive entries per instruction
  __shared__ float s_v[NW][64 * EPL];
  __shared__ int32_t s_p[NW][64 * EPL];
  // one workgroup per work unit: a range of one chunk's tiles (a large chunk is split
  // over several workgroups, each staging the chunk's c range, so a hot chunk does not
  // become the kernel's tail)
  const int wu = wu0 + blockIdx.x;
  const int ch = wu_chunk[wu];
  const int slo = chunk_slo[ch], ns = chunk_ns[ch];
  const int r0 = chunk_run[ch], nr = chunk_run[ch + 1] - r0;
  float csum = 0.f;
  for (int i = threadIdx.x; i < ns; i += NW * 64) {
    const float v = c[slo + i];
    s_c[i] = v >= 0.f ? v : -0.0f;            // absent source: no record
    csum += v >= 0.f ? v : 0.f;
  }
  // fixed-point range of phase 2: every destination sum is <= the sum of all present c
  // the layout reads (one record per (source, destination) after dedup); the chunk's
  // first work unit adds its source range
  // (the partials go to wave 0's staging buffer, which only wave 0 -- the one reading
  // them -- writes afterwards: a separate array would push the block past 80 KB of LDS,
  // i.e. from 2 to 1 resident workgroup per CU)
  if (wu == 0 || wu_chunk[wu - 1] != ch) {
    csum = wave_sum(csum);
    if ((threadIdx.x & 63) == 0) s_v[0][threadIdx.x >> 6] = csum;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int w = 0; w < NW; ++w) t += (double)s_v[0][w];
      // rounding slack: the f32 partial sums may be up to ~1e-6 relative low. The bound
      // is summed as u64 fixed point (2^-kPbBoundFrac units, rounded up): integer adds
      // commute, so K below does not depend on the order the work units ran in
      atomicAdd(bound, (unsigned long long)ceil(ldexp(t * (1.0 + 1e-5), kPbBoundFrac)));
    }
  }
  if constexpr (!GRUNS)
    for (int i = threadIdx.x; i < nr; i += NW * 64) s_d[i] = run_delta[r0 + i];
  __syncthreads();
  const int32_t* dsrc = GRUNS ? run_delta + r0 : s_d;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float* sv = s_v[wave];
  int32_t* sp = s_p[wave];
  // dummy_base: kPbDummy floats past the entries, 64 per wave slot
  // (positions < 2^30, checked by the launcher: 32-bit byte offsets)
  const uint32_t dummy4 =
      ((uint32_t)dummy_base + (uint32_t)(((blockIdx.x * NW + wave) % (kPbDummy / 64)) * 64 + lane)) * 4u;
  const int t_end = wu_tile[wu + 1];
  for (int t = wu_tile[wu] + wave; t < t_end; t += NW) {
    const int64_t e_lo = tile_e[t], e_hi = tile_e[t + 1];
    int32_t ent = tile_ent[t];                // chunk-major index of the next entry (< 2^30)
    int run = tile_run[t];                    // run starts (in this chunk) before it
    float carry = -0.0f;                      // open entry continuing from the last step
    const int64_t e_first = e_lo & ~(int64_t)(EPL - 1);
    auto load = [&](int64_t ix) {             // out-of-tile lanes re-read the first group
      return pb_ld16(srcl + (ix < e_hi ? ix : e_first));
    };
    // ring of D steps in flight, unrolled by D so that no register copy of a pending load
    // (which would wait for it) is needed
    // the tile's scalars are consumed here, before the ring's first loads: a wait the
    // compiler placed at their first use inside the step loop would run every step
    {
      int ent_lo = (int)ent;
      asm volatile("" :: "v"(ent_lo), "v"(run), "v"(e_lo), "v"(e_hi));
    }
    pb_v4i wq[D];
#pragma unroll
    for (int q = 0; q < D; ++q) wq[q] = load(e_first + (int64_t)q * 64 * EPL + EPL * lane);
    // vector memory ops per step: SF stores (more in a step with > SF * 64 entries), then
    // the ring refill. Slot q's data was loaded D steps back; younger than it: at least
    // (D - 1) (SF + 1) ops in steady state, and in the first D steps at least the D - 1
    // other initial loads. vmcnt(N) waits for all but the N youngest ops, so waiting with
    // N <= the true count of younger ops is safe (a step that stored more only makes it
    // wait a little longer)
    constexpr int SF = 4;                     // store instructions every step issues
    static_assert((D - 1) * (SF + 1) <= 63, "vmcnt field");
    bool first = true;
    for (int64_t e00 = e_first; e00 < e_hi; e00 += (int64_t)D * 64 * EPL) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const int64_t e0 = e00 + (int64_t)q * 64 * EPL;
      if (e0 >= e_hi) break;
      const int64_t idx = e0 + EPL * lane;
      if (first) pb_wait_vm<D - 1>();
      else pb_wait_vm<(D - 1) * (SF + 1)>();
      // the slot is routed through an (ordered) asm after the wait: no read of it can be
      // scheduled before the wait
      asm volatile("" : "+v"(wq[q]));
      const int4 wc = make_int4(wq[q].x, wq[q].y, wq[q].z, wq[q].w);
      // a step whose 512 edges all lie inside the tile (all but the first and last of a
      // tile: wave-uniform) drops the per-edge in-range selects
      const bool full = e0 >= e_lo && e0 + 64 * EPL <= e_hi;
      auto step = [&](auto full_c) {
        constexpr bool FULL = decltype(full_c)::value;
        const uint32_t ww[4] = {(uint32_t)wc.x, (uint32_t)wc.y, (uint32_t)wc.z, (uint32_t)wc.w};
        uint32_t hk[EPL];
        float cv[EPL];
        // the lane's edges idx + k inside [e_lo, e_hi): k in [klo, klo + span), one 32-bit
        // compare per edge instead of two 64-bit ones
        int klo = 0, span = EPL;
        if constexpr (!FULL) {
          klo = (int)min(max(e_lo - idx, (int64_t)0), (int64_t)EPL);
          span = max((int)min(max(e_hi - idx, (int64_t)0), (int64_t)EPL) - klo, 0);
        }
        bool inr[EPL];
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
          inr[k] = FULL || (uint32_t)(k - klo) < (uint32_t)span;
          const uint32_t h = (ww[k >> 1] >> (16 * (k & 1))) & 0xffffu;
          hk[k] = inr[k] ? h : 0u;
          cv[k] = s_c[hk[k] & (S - 1)];
        }
        float part = -0.0f, outv[EPL];
        int nf = 0, nm = 0;
        int rk[EPL];                                       // markers so far (inclusive)
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
          const bool in = inr[k];
          part += in ? cv[k] : -0.0f;
          outv[k] = part;
          const bool f = hk[k] & 0x8000u;
          nm += (f && (hk[k] & 0x4000u)) ? 1 : 0;
          rk[k] = nm;
          if (f) part = -0.0f;
          nf += f ? 1 : 0;
        }
        // inclusive scans over the 64 lanes (DPP: rows of 16, then row broadcasts)
        float a = part;
        int cc = nf | (nm << 16);
        scan_step<0x111>(a, cc);                   // row_shr:1
        scan_step<0x112>(a, cc);                   // row_shr:2
        scan_step<0x114>(a, cc);                   // row_shr:4
        scan_step<0x118>(a, cc);                   // row_shr:8
        scan_step<0x142, 0xa>(a, cc);              // row_bcast:15 -> rows 1, 3
        scan_step<0x143, 0xc>(a, cc);              // row_bcast:31 -> rows 2, 3
        const int cnt = cc & 0xffff, cm = cc >> 16;
        // exclusive segment sum for this lane (wave_shr:1), joined with the step carry
        const float a_ex = dpp_mov_f<0x138>(-0.0f, a);
        const int c_ex = dpp_mov_i<0x138>(0, cc);
        const float carry_in = (c_ex & 0xffff) ? a_ex : carry + a_ex;
        const int rbase = run + cm - nm - 1;       // run of this lane's first entries
        // run deltas of the lane's entries: its 8 edges touch at most nm + 1 runs and nearly
        // always <= 2 (a run is one (chunk, 16K-destination bin) group: hundreds of edges),
        // so two reads and a select, with all 8 reads only in a step where some lane spans
        // three runs (wave-uniform branch; LDS reads: no vmcnt bookkeeping involved)
        int dl[EPL];
        if (__ballot(nm >= 2) == 0ull) {
          const int d0 = dsrc[max(rbase, 0)];
          const int d1 = dsrc[max(min(rbase + 1, nr - 1), 0)];
#pragma unroll
          for (int k = 0; k < EPL; ++k) dl[k] = rk[k] == 0 ? d0 : d1;
        } else {
#pragma unroll
          for (int k = 0; k < EPL; ++k) dl[k] = dsrc[max(rbase + rk[k], 0)];
        }
        int j = cnt - nf;                          // this lane's first entry of the step
        bool first = true;
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
          if (hk[k] & 0x8000u) {
            sv[j] = first ? carry_in + outv[k] : outv[k];
            sp[j] = ent + j + dl[k];
            first = false;
            ++j;
          }
        }
        const float a63 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a), 63));
        const int c63 = __builtin_amdgcn_readlane(cc, 63);
        const int n_step = c63 & 0xffff;
        carry = n_step ? a63 : carry + a63;
        ent += n_step;
        run += c63 >> 16;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // SF unconditional stores per lane (lanes past n_step write this wave's own dummy
        // line group, so no single address is hammered by every wave): a minimum store
        // count keeps the hand-counted vmcnt waits valid, so the D prefetched loads are not
        // drained at every step. A step with more than SF * 64 entries (0.42 entries per
        // edge on average: ~215 of 512) adds the missing stores in a wave-uniform branch.
        // Staged values read before the first store: one LDS round trip per step
        int32_t pq[SF];
        float vq[SF];
#pragma unroll
        for (int q = 0; q < SF; ++q) {
          pq[q] = sp[lane + 64 * q];
          vq[q] = sv[lane + 64 * q];
        }
#pragma unroll
        for (int q = 0; q < SF; ++q) {
          const bool ok = lane + 64 * q < n_step;
          pb_st4(val, ok ? (uint32_t)pq[q] * 4u : dummy4, ok ? vq[q] : 0.f);
        }
        if (n_step > SF * 64) {
#pragma unroll
          for (int q = SF; q < EPL; ++q) {
            if (64 * q < n_step) {
              const bool ok = lane + 64 * q < n_step;
              const int32_t p2 = sp[lane + 64 * q];
              const float v2 = sv[lane + 64 * q];
              pb_st4(val, ok ? (uint32_t)p2 * 4u : dummy4, ok ? v2 : 0.f);
            }
          }
        }
      };
      if (full) step(std::true_type{}); else step(std::false_type{});
      // the ring slot is refilled after the step's last read of it: the old and the new
      // value never live together, so they share registers (no copy of a pending load)
      wq[q] = load(idx + (int64_t)D * 64 * EPL);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    first = false;
    }
    // the ring refills past the tile's end are still landing in the slot registers: drain
    // them while the slots are still held (operands of the wait), before any later code
    // can reuse those registers
    static_assert(D == 4, "drain operands");
    asm volatile("s_waitcnt vmcnt(0)" :: "v"(wq[0]), "v"(wq[1]), "v"(wq[2]), "v"(wq[3]) : "memory");
  }
}

// f32 record value -> fixed point q = v * 2^K (truncated), >= 1 for any present record so
// that "received >= 1 record" == (sum != 0). Exact integer sums: the result does not
// depend on the order of the adds (bitwise deterministic) and is rounded to f32 once.
__device__ __forceinline__ uint64_t to_fixed(float v, int K) {
  const uint32_t bits = __float_as_uint(v);
  const int e = (int)((bits >> 23) & 0xffu);
  const uint64_t m = (bits & 0x7fffffu) | (e ? 0x800000u : 0u);
  const int sh = max(e, 1) - 150 + K;          // v = m * 2^(max(e,1) - 150)
  uint64_t q = sh >= 0 ? (m << min(sh, 63)) : (sh > -64 ? (m >> -sh) : 0ull);
  return q ? q : 1ull;
}

__device__ __forceinline__ float from_fixed(uint64_t q, int K) {
  return (float)ldexp((double)q, -K);
}

// fraction bits for a sum bound B: B * 2^K <= 2^62 (u64 headroom for the per-record
// +1 units); derived on the device from phase 1's bound, so no host sync
__device__ __forceinline__ int pb_fixed_bits(const unsigned long long* bound) {
  const double B = ldexp((double)*bound, -kPbBoundFrac);
  if (!(B > 0.0)) return 100;
  return min(100, max(1, 61 - ilogb(B)));
}

// Where a destination's sum goes: acc/pres (the SpMV alone), or -- when r != nullptr --
// straight through the PageRank rank / contribution update (same f32 arithmetic as
// pr_update_kernel, pagerank.hip), which saves the acc/pres round trip and a launch.
struct PbOut {
  float* acc;
  int32_t* pres;
  const int32_t* outdeg;
  float* r;
  float* c;
  const float* dang_in;
  float* dang_out;
  float q, invN;
  int mode;
};

// returns this destination's dangling mass (standard semantics, fused update); od =
// outdeg[v] and dang = *dang_in (or 0) are loaded by the caller, in batches
__device__ __forceinline__ float pb_finish(const PbOut& o, int64_t v, uint64_t qs, int K, int od,
                                           float dang) {
  const float a = from_fixed(qs, K);
  if (o.r == nullptr) {
    o.acc[v] = a;
    o.pres[v] = qs != 0;
    return 0.f;
  }
  if (o.mode == 0) {
    const bool p = qs != 0;
    const float rv = p ? o.q * o.invN + (1.f - o.q) * a : -1.f;
    o.r[v] = rv;
    o.c[v] = (p && od > 0) ? rv / (float)od : -1.f;
    return 0.f;
  }
  const float rv = o.q * o.invN + (1.f - o.q) * (a + dang * o.invN);
  o.r[v] = rv;
  o.c[v] = od > 0 ? rv / (float)od : 0.f;
  return od == 0 ? rv : 0.f;
}

__device__ __forceinline__ void pb_dangling(const PbOut& o, float dl) {
  if (o.r != nullptr && o.mode == 1 && o.dang_out) {
    dl = wave_sum(dl);
    if ((threadIdx.x & 63) == 0 && dl != 0.f) atomicAdd(o.dang_out, dl);
  }
}

// BW destinations per LDS bin (u64 fixed-point accumulators: f32 LDS atomics run at
// ~0.33 lane-ops per CU-clock on gfx950, u32/u64 integer ones ~28x faster,
// profiles/round3/pb/README.md); NW waves; a work item is a contiguous bin-major entry
// range (possibly empty: every bin has >= 1 work item, so no output needs pre-zeroing)
template <int BW, int NW, int U = 4>
__global__ void __launch_bounds__(NW * 64)
pb_accum_kernel(const float* __restrict__ val, const uint16_t* __restrict__ dloc,
                const int32_t* __restrict__ wi_bin, const int64_t* __restrict__ wi_lo,
                const int32_t* __restrict__ wi_slab, int64_t n_local,
                const unsigned long long* bound,
                PbOut o, uint64_t* __restrict__ slab) {
  const int K = pb_fixed_bits(bound);
  // U: groups of 4 entries in flight per thread
  __shared__ unsigned long long s_acc[BW];
  const int w = blockIdx.x;
  const int b = wi_bin[w];
  const int64_t lo = wi_lo[w], hi = wi_lo[w + 1];
  for (int i = threadIdx.x; i < BW; i += NW * 64) s_acc[i] = 0ull;
  __syncthreads();
  const int64_t g_lo = lo >> 2, g_hi = (hi + 3) >> 2;     // groups of 4 entries
  // software pipelined: batch b + 1's loads are in flight while batch b is added (two
  // register sets, loop unrolled by 2 so that no copy of a pending load is needed); loads
  // past the range read the last group again (clamped, unconditional: a load under a
  // branch gets its own wait)
  constexpr int64_t STEP = (int64_t)U * NW * 64;
  auto load_batch = [&](int64_t gb, int4 (&v)[U], uint2 (&k)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t g = min(gb + (int64_t)u * NW * 64, g_hi - 1);
      v[u] = ld_int4<true>(reinterpret_cast<const int32_t*>(val) + 4 * g);
      k[u] = *(reinterpret_cast<const uint2*>(dloc) + g);
    }
  };
  auto add_batch = [&](int64_t gb, const int4 (&v)[U], const uint2 (&k)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = (gb + (int64_t)u * NW * 64) * 4;
      const float f[4] = {__int_as_float(v[u].x), __int_as_float(v[u].y), __int_as_float(v[u].z),
                          __int_as_float(v[u].w)};
      const uint32_t kk[4] = {k[u].x & 0xffffu, k[u].x >> 16, k[u].y & 0xffffu, k[u].y >> 16};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (e + j >= lo && e + j < hi && !signbit(f[j]))
          atomicAdd(&s_acc[kk[j]], (unsigned long long)to_fixed(f[j], K));
    }
  };
  // (64 consecutive entries per atomic instruction -- 4 strided entries per thread, so
  // a dense run's destinations hit distinct LDS banks -- measured 2 % slower per
  // iteration despite the 5.75 bank-conflict cycles per LDS instruction of this form:
  // profiles/round5/r5_36)
  int64_t g0 = g_lo + threadIdx.x;
  if (g0 < g_hi) {
    int4 va[U], vb[U];
    uint2 ka[U], kb[U];
    load_batch(g0, va, ka);
    for (;; g0 += 2 * STEP) {
      const bool more = g0 + STEP < g_hi;
      if (more) load_batch(g0 + STEP, vb, kb);
      add_batch(g0, va, ka);
      if (!more) break;
      const bool more2 = g0 + 2 * STEP < g_hi;
      if (more2) load_batch(g0 + 2 * STEP, va, ka);
      add_batch(g0 + STEP, vb, kb);
      if (!more2) break;
    }
  }
  __syncthreads();
  const int64_t base = (int64_t)b * BW;
  const int nb = (int)min((int64_t)BW, n_local - base);
  const int sl = wi_slab[w];
  if (sl < 0) {                         // the bin's only work item: final values
    // out-degrees loaded in one batch (clamped, unconditional): one memory latency per
    // work item instead of one per destination a thread finishes
    constexpr int PER = BW / (NW * 64);
    int od[PER];
    const float dang = (o.r != nullptr && o.mode == 1 && o.dang_in) ? o.dang_in[0] : 0.f;
    if (o.r != nullptr) {
#pragma unroll
      for (int j = 0; j < PER; ++j)
        od[j] = o.outdeg[base + min((int)threadIdx.x + j * NW * 64, nb - 1)];
    } else {
#pragma unroll
      for (int j = 0; j < PER; ++j) od[j] = 0;
    }
    float dl = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = threadIdx.x + j * NW * 64;
      if (i < nb) dl += pb_finish(o, base + i, s_acc[i], K, od[j], dang);
    }
    pb_dangling(o, dl);
  } else {                              // partial of a split bin -> its slab
    uint64_t* dst = slab + (int64_t)sl * BW;
    for (int i = threadIdx.x; i < BW; i += NW * 64) dst[i] = s_acc[i];
  }
}

// Split bins: sum the partial slabs (exact integer sums).
template <int BW>
__global__ void __launch_bounds__(256)
pb_combine_kernel(const uint64_t* __restrict__ slab, const int32_t* __restrict__ split_bin,
                  const int32_t* __restrict__ split_first, const int32_t* __restrict__ split_count,
                  int64_t n_local, const unsigned long long* bound, PbOut o) {
  const int K = pb_fixed_bits(bound);
  const int sb = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t base = (int64_t)split_bin[sb] * BW;
  float dl = 0.f;
  if (i < BW && base + i < n_local) {
    const uint64_t* p = slab + (int64_t)split_first[sb] * BW + i;
    const int cnt = split_count[sb];
    // 8 independent slab loads in flight per thread (one at a time: 86 -> 77 us per
    // iteration at scale 26, profiles/round6/r6_73; 64 destinations x 4 piece lanes per
    // block with an LDS sum measured 92 us, and a last-arriving-piece combine inside
    // pb_accum would leave one CU summing a hot bin's ~100 slabs)
    uint64_t qa[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int k = 0;
    for (; k + 8 <= cnt; k += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) qa[j] += p[(int64_t)(k + j) * BW];
    }
    for (; k < cnt; ++k) qa[0] += p[(int64_t)k * BW];
    uint64_t q = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) q += qa[j];
    const int od = o.r != nullptr ? o.outdeg[base + i] : 0;
    const float dang = (o.r != nullptr && o.mode == 1 && o.dang_in) ? o.dang_in[0] : 0.f;
    dl = pb_finish(o, base + i, q, K, od, dang);
  }
  pb_dangling(o, dl);
}

}  // namespace dalgo

using namespace dalgo;

extern "C" {

hipError_t dalgo_pb_spmv(const uint16_t* srcl, const int64_t* tile_e, const int32_t* tile_ent,
                         const int32_t* tile_run, const int32_t* wu_tile, const int32_t* wu_chunk,
                         int nwu, int wu_lo, int wu_hi, int phases,
                         const int32_t* chunk_slo, const int32_t* chunk_ns,
                         const int32_t* chunk_run, const int32_t* run_delta, int nch,
                         int max_runs, int src_span, const float* c, float* val, int64_t n_val, const uint16_t* dloc, const int32_t* wi_bin,
                         const int64_t* wi_lo, const int32_t* wi_slab, int nwi, int bin_width,
                         double* bound_word, int64_t n_local, float* acc, int32_t* pres, uint64_t* slab,
                         const int32_t* split_bin, const int32_t* split_first,
                         const int32_t* split_count, int nsplit, const int32_t* outdeg, float q,
                         float invN, int mode, const float* dang_in, float* r, float* cn,
                         float* dang_out, hipStream_t st) {
  if (src_span != 8192 || (bin_width != 8192 && bin_width != 16384) || n_val < kPbDummy ||
      n_val >= ((int64_t)1 << 30))
    return hipErrorInvalidValue;
  // phases: bit 0 = phase 1 over work units [wu_lo, wu_hi) (several calls may cover the
  // units, the first one starting at 0 -- e.g. own-slice sources before the ghost
  // exchange has landed), bit 1 = phase 2 (+ fused update)
  wu_hi = std::min(wu_hi, nwu);
  // the 8-byte bound word holds a u64 fixed-point sum (see pb_gather_kernel)
  unsigned long long* bound = reinterpret_cast<unsigned long long*>(bound_word);
  if ((phases & 1) && wu_lo == 0) {
    const hipError_t e = hipMemsetAsync(bound, 0, sizeof(*bound), st);
    if (e != hipSuccess) return e;
  }
  if ((phases & 1) && nch > 0 && wu_hi > wu_lo) {
    // max_runs: the largest number of non-empty runs of one chunk (LDS table up to 4096)
#define PB_GATHER_LAUNCH(GR)                                                                      \
    hipLaunchKernelGGL((pb_gather_kernel<8192, 4096, 8, GR>), dim3(wu_hi - wu_lo), dim3(8 * 64), 0, st, \
                       srcl, tile_e, tile_ent, tile_run, wu_tile, wu_chunk, chunk_slo, chunk_ns, \
                       chunk_run, run_delta, c, val, n_val - kPbDummy, bound, wu_lo)
    if (max_runs > 4096) PB_GATHER_LAUNCH(true);
    else PB_GATHER_LAUNCH(false);
#undef PB_GATHER_LAUNCH
    DALGO_LAUNCH_CHECK();
  }
  if (!(phases & 2) || nwi == 0) return hipSuccess;
  const PbOut o{acc, pres, outdeg, r, cn, dang_in, dang_out, q, invN, mode};
  if (bin_width == 16384) {
    // 4 groups of 4 entries in flight per thread (8 groups measured slower,
    // profiles/round3/pb/)
    hipLaunchKernelGGL((pb_accum_kernel<16384, 16>), dim3(nwi), dim3(16 * 64), 0, st, val, dloc,
                       wi_bin, wi_lo, wi_slab, n_local, bound, o, slab);
    DALGO_LAUNCH_CHECK();
    if (nsplit > 0)
      hipLaunchKernelGGL(pb_combine_kernel<16384>, dim3(16384 / 256, nsplit), dim3(256), 0, st,
                         slab, split_bin, split_first, split_count, n_local, bound, o);
  } else {
    hipLaunchKernelGGL((pb_accum_kernel<8192, 16>), dim3(nwi), dim3(16 * 64), 0, st, val, dloc,
                       wi_bin, wi_lo, wi_slab, n_local, bound, o, slab);
    DALGO_LAUNCH_CHECK();
    if (nsplit > 0)
      hipLaunchKernelGGL(pb_combine_kernel<8192>, dim3(8192 / 256, nsplit), dim3(256), 0, st,
                         slab, split_bin, split_first, split_count, n_local, bound, o);
  }
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

}  // extern "C"
