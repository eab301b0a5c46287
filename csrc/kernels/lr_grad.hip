// K1 + K7 + K10: fused Bernoulli-sampled logistic-regression gradient and eval.
//
// Replaces the reference's per-record Python hot loop
//   points.sample(False, f, 42+t).map(gradient).treeAggregate(...)
// (optimization/ssgd.py:97-103, gradient at ssgd.py:27-33, logistic_f at
// ssgd.py:23-24; per-partition mean at optimization/ma.py:39-43) with ONE pass over
// the sampled rows of X held in HBM:
//   sel(row)  = philox(seed, step, global_row) < frac * 2^32        (K7, in-register)
//   z         = x . w (+ bias)                                      (row GEMV)
//   r         = sigma(z) - y,  sigma = 1/(exp(-z) + 1 + eps)
//   g        += r * x,  g_bias += r,  cnt += 1                      (rank-1 accumulate)
// The gradient is GEMV-shaped (about 1 FLOP/B) so the roofline is HBM bandwidth:
// each selected row is read exactly once with 16-byte vector loads, four rows per
// wave in flight, the per-row dot product reduced across the 64 lanes with 7
// cross-lane ops (permlane32/permlane16 swaps + DPP row rotations, no LDS), and
// the gradient accumulated in VGPRs (each lane owns a fixed set of columns, so
// g never crosses lanes). Per-block partials go to a slab and are combined by a
// deterministic two-level last-arriver reduction (agent-scope release/acquire,
// fixed summation order) — no float atomics, bitwise reproducible.
//
// Segments: rows [seg_lo[s], seg_lo[s+1]) use model s (MA/BMUF/EASGD keep one
// local model per logical worker, ma.py:86-87); SSGD uses a single segment.
#include <cstdlib>

#include "dalgo/common.h"
#include "dalgo/xgmi.h"
#include "launchers.h"

namespace dalgo {

struct LrParams {
  const void* X;        // [n_local, ld] row-major, T = bf16 or f32
  const float* y;       // [n_local] labels in {0,1}
  const float* W;       // [n_seg, ldw]  (w[0..D) features, w[D] bias if has_bias)
  const int64_t* seg;   // [n_seg + 1] local row bounds (device)
  int64_t ld;           // row stride of X in elements (multiple of the 16-B vector)
  int64_t row_offset;   // global index of local row 0 (sampling is keyed by global row)
  int D;                // feature count (columns [D, ld) are ignored: zero weights, no writes)
  int ldw;              // row stride of W / G
  int has_bias;
  float eps;            // 0 (ssgd.py:24) or 1e-6 (ma.py:26)
  uint64_t seed, step;  // sampling stream
  // graph replay (hipGraph): the stream index is step + step_mul * (*step_dev), read
  // from device memory so one captured graph serves every training step
  const int64_t* step_dev;
  int64_t step_mul;
  uint32_t thr;         // Bernoulli threshold: select iff u32 < thr
  int full;             // 1: every row selected (full-batch GD)
  int rows_per_block;   // multiple of 4 (the Philox row quad)
  // grad outputs
  float* slab;          // [n_seg * gx, S]
  float* gslab;         // [n_seg * ngroups, S]
  unsigned* cnt1;       // [n_seg * ngroups]   arrival counters (zeroed)
  unsigned* cnt2;       // [n_seg]
  float* G;             // [n_seg, ldw] gradient sum
  float* C;             // [n_seg] selected-row count
  int S;                // slab row stride (>= ldw + 1)
  // eval outputs
  unsigned long long* correct;  // [n_seg] (eval mode)
  float* loss;                  // [n_seg] sum of log-loss (eval mode)
  double* count_acc;    // optional: += local selected-row count of THIS step
  int atomic_out;       // 1: blocks add their partials to G/C with float atomics
                        //    (G/C zeroed by the caller; summation order not fixed)
  int fine_q;             // work claims switch from 256-row groups to 64-row quarters once
                          // fewer than fine_q quarters of the block are unclaimed (0 = never)
  int unit_shift;         // sampling: work units of 2^unit_shift rows (2..8; fine claims take one)
  // diagnostics only (dalgo_lr_set_trace): per-wave timeline, 8 u64 per wave at
  // [(block * NW + wave) * 8]: start, first row batch issued, sweep done, epilogue
  // done (s_memrealtime, 100 MHz), selected rows, hardware CU/SE id
  unsigned long long* trace;
  // fused tail (SSGD / GD, one segment, atomic epilogue): the last block to finish
  // (ticket) exchanges [g || count] with the other ranks over xGMI (xg.world > 1)
  // and applies the update to W, leaving G / C zeroed: one launch per training step.
  unsigned* ticket;     // nullptr: no tail; zero on entry, re-armed by the last block
  XgLink xg;
  XgUpdate tu;
  double* tail_count_acc;  // += the GLOBAL minibatch size
  // persistent multi-step mode (fused tail only): nsteps > 1 runs steps step ..
  // step + nsteps - 1 in ONE cooperative launch (every block resident). The tail block
  // of step i writes W / G / C / ticket through to the coherence point, then publishes
  // epoch_base + i + 1 in *epoch; every block waits for it (bounded by spin_ticks of
  // s_memrealtime; a timeout sets *perr and ends the launch) before it reads W for step
  // i + 1 - by then its first row batch of step i + 1 is already in flight.
  int nsteps;
  unsigned* epoch;
  uint32_t epoch_base;
  unsigned* perr;
  uint64_t spin_ticks;
  // persistent mode, cross-block balance: local rows [pool_lo, seg_hi) belong to no block's
  // static range; a wave whose block has no unit left claims 2^pool_shift-row units of them
  // from pool[step & 1] (agent-scope atomic; the step's tail block re-arms it)
  int* pool;
  int64_t pool_lo;
  int pool_shift;
};

__device__ __forceinline__ void wt_store(float* a, float v) {
  __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The last block of a fused-tail launch: every other block's atomics are performed
// (each waited vmcnt(0) before taking its ticket), so agent-scope loads see the
// complete local sums.
__device__ __forceinline__ void lr_tail(const LrParams& p, uint32_t xg_epoch) {
  const int n = p.ldw;                 // G row; index n carries the count
  float* G = p.G;
  float* W = const_cast<float*>(p.W);
  auto get = [&](int i) -> float {
    return __hip_atomic_load(i < n ? &G[i] : &p.C[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // W is read with agent-scope loads too: in the persistent mode an earlier step's tail
  // block (another CU / XCD) wrote it, and a plain load could hit a stale L2 line
  auto getw = [&](int i) -> float {
    return __hip_atomic_load(&W[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  float c;
  if (p.xg.world > 1) {
    // persistent mode: one exchange epoch per step (xg_epoch = device base + step + 1)
    xg_push_publish_wait(p.xg, xg_epoch, n + 1, get);
    c = xg_sum(p.xg, xg_epoch, n);
    for (int i = threadIdx.x; i < n; i += blockDim.x)
      wt_store(&W[i], xg_update(getw(i), xg_sum(p.xg, xg_epoch, i), c, p.tu));
  } else {
    c = get(n);
    for (int i = threadIdx.x; i < n; i += blockDim.x) wt_store(&W[i], xg_update(getw(i), get(i), c, p.tu));
  }
  // write-through (agent-scope) stores: in the persistent mode other XCDs' blocks read
  // W and add into G / C right after the epoch release, without a kernel boundary
  for (int i = threadIdx.x; i < n; i += blockDim.x) wt_store(&G[i], 0.f);
  __syncthreads();                     // every thread has read the count
  if (threadIdx.x == 0) {
    wt_store(&p.C[0], 0.f);
    if (p.tail_count_acc)
      __hip_atomic_fetch_add(p.tail_count_acc, (double)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

constexpr int kGroup = 16;   // blocks per first-level reduction group

template <typename T> struct VecTraits;
template <> struct VecTraits<uint16_t> { static constexpr int VEC = 8; };
template <> struct VecTraits<float>    { static constexpr int VEC = 4; };

template <typename T>
__device__ __forceinline__ void unpack(const uint4& v, float (&o)[VecTraits<T>::VEC]);
template <>
__device__ __forceinline__ void unpack<uint16_t>(const uint4& v, float (&o)[8]) {
  o[0] = bf16lo(v.x); o[1] = bf16hi(v.x); o[2] = bf16lo(v.y); o[3] = bf16hi(v.y);
  o[4] = bf16lo(v.z); o[5] = bf16hi(v.z); o[6] = bf16lo(v.w); o[7] = bf16hi(v.w);
}
template <>
__device__ __forceinline__ void unpack<float>(const uint4& v, float (&o)[4]) {
  o[0] = __uint_as_float(v.x); o[1] = __uint_as_float(v.y);
  o[2] = __uint_as_float(v.z); o[3] = __uint_as_float(v.w);
}

// Cross-workgroup hand-off without L2 writeback/invalidate (guide §6 G16, sc1
// form): slab words are stored write-through (agent-scope relaxed atomic store =
// global_store ... sc1), every storing wave drains vmcnt before the block's
// ticket add, and the reducer reads every handed-off word with sc1 loads. An
// agent-scope release/acquire fence here costs a full L2 writeback/invalidate
// per block, which dominated small launches.
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// sum of column `col` over nrows slab rows (stride S): 16 loads issued back to
// back per round (indices clamped, not branched, so hipcc keeps them in flight)
__device__ __forceinline__ float sum_slab_col(const float* src, int nrows, int S, int col) {
  float s = 0.f;
  for (int k0 = 0; k0 < nrows; k0 += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = ld_wt(&src[(int64_t)min(k0 + u, nrows - 1) * S + col]);
#pragma unroll
    for (int u = 0; u < 16; ++u) s += (k0 + u < nrows) ? v[u] : 0.f;
  }
  return s;
}

// A batch of (up to) U selected rows held in VGPRs (U = 4 or 8). With PIPE the
// row loads of batch i+1 are issued before batch i is computed (two named
// register sets, manual unroll); with U = 8 a single set keeps 16 KB per wave
// in flight. Bytes in flight per wave are bounded by VGPRs (4 B per VGPR-lane),
// which is what the variants trade against occupancy.
template <int NC, int U>
struct Batch {
  uint4 x[U][NC];
  float yq[U / 4];  // label of row 4j + (lane >> 4)
  float v[U];       // 1 = valid row, 0 = padding
  int n;            // valid rows (0 = no more work)
};

constexpr int kRing = 512;   // per-wave ring of selected local row indices
constexpr int kPoolSlots = 64;   // pool chunks one block can take per step
constexpr int kPoolPre = 3;      // units before a chunk's end at which the next is claimed

// EVAL=false: gradient; EVAL=true: accuracy + log-loss over every row.
// PIPE: software-pipelined (two register sets) vs. single-buffered sweep.
// LEAN compiles out the fixed-order (deterministic) epilogue and claim map, which the
// default (atomic-epilogue) launch never takes. Each launch starts from a cold
// instruction cache, and inlined paths that sit between the executed instructions of the
// start-up path and the refill loop cost time: variant 8 without a cross-block work pool
// measured 56.5 -> 53.5 us per 1.25M-row step (profiles/round2/README.md). The launcher
// picks the full build only for deterministic launches.
// Measured and removed (profiles/round2, profiles/round3): a cross-block work pool, a
// fused previous-step update prologue (1.5-8 % slower than the separate 2-us update),
// balanced slices of a precomputed compacted selection (2.7 us faster in K1, more lost
// in the side-stream hand-off) and 11 other launch shapes.
template <typename T, int NC, bool EVAL, int NW, bool PIPE, int U, bool PERSIST, int AUX = 0,
          bool LEAN = false>
__global__ void __launch_bounds__(NW * 64)
lr_rows_kernel(const LrParams p) {
  // the persistent form (fused tail, atomic epilogue: host checks) is lean as well
  constexpr bool kLean = LEAN || PERSIST;
  constexpr int VEC = VecTraits<T>::VEC;
  constexpr int COLS = NC * 64 * VEC;  // columns covered per lane-set
  constexpr int RED_FLOATS = NW * (COLS + 4);
  constexpr int RING_INTS = NW * kRing;
  constexpr int ARENA = (RED_FLOATS > RING_INTS) ? RED_FLOATS : RING_INTS;
  // one LDS arena: per-wave selection rings during the sweep, then the
  // cross-wave reduction buffer
  __shared__ __attribute__((aligned(16))) float s_arena[ARENA];
  __shared__ int s_flag;
  __shared__ int s_next;   // next unclaimed work unit of this block (dynamic balancing)
  __shared__ int s_ok;     // persistent mode: the epoch wait succeeded
  // persistent mode with a cross-block pool: the block's claimed pool chunks (by claim
  // order) and the next unit of them
  __shared__ int s_chunk[kLean ? kPoolSlots : 1];
  __shared__ int s_pnext;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned long long* const tr =
      p.trace ? p.trace + ((int64_t)(blockIdx.y * gridDim.x + blockIdx.x) * NW + wid) * 8 : nullptr;
  const unsigned long long t_start = tr ? (unsigned long long)__builtin_amdgcn_s_memrealtime() : 0ull;
  const int seg = blockIdx.y;
  const int bx = blockIdx.x;
  const int gx = gridDim.x;
  const int64_t seg_lo = p.seg[seg], seg_hi = p.seg[seg + 1];
  const bool use_pool = kLean && p.pool != nullptr;   // fused-tail launches only (the tail re-arms)
  const int64_t static_hi = use_pool ? min(seg_hi, p.pool_lo) : seg_hi;
  const int64_t lo = seg_lo + (int64_t)bx * p.rows_per_block;
  const int64_t hi = max(lo, min(static_hi, lo + (int64_t)p.rows_per_block));
  // ---- step loop (one iteration unless persistent: p.nsteps > 1)
  // (a separate instantiation: the step loop costs registers the one-step kernel keeps)
  const int nst = PERSIST && p.nsteps > 1 ? p.nsteps : 1;
  // persistent mode: wait until the tail block of the previous step released W
  auto wait_epoch = [&](int it) -> bool {
    if (threadIdx.x == 0) {
      const uint32_t want = p.epoch_base + (uint32_t)it;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int ok = 1;
      while ((int32_t)(__hip_atomic_load(p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
        if (__hip_atomic_load(p.perr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
            __builtin_amdgcn_s_memrealtime() - t0 > p.spin_ticks) {
          __hip_atomic_store(p.perr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
  };
  const uint64_t step_base =
      p.step + (p.step_dev != nullptr ? (uint64_t)(p.step_mul * p.step_dev[0]) : 0ull);
  for (int it = 0; it < nst; ++it) {
  // the kernel argument block is never written (a modified copy would live in scratch)
  const uint64_t step_cur = step_base + (uint64_t)it;
  // model fragment in registers. Fetched AFTER the first row batch is issued (see the
  // sweep): the W reads then overlap the first rows' HBM latency instead of preceding
  // them, and the work-claim barrier below does not wait for them.
  float wr[NC][VEC];
  float wb = 0.f;
  // persistent mode: W was written by another CU in this launch -> agent-scope loads
  auto ldw_ = [&](const float* a) -> float {
    if constexpr (PERSIST)
      return __hip_atomic_load(const_cast<float*>(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      return *a;
  };
  auto load_w = [&]() {
    {
      const float* w = p.W + (int64_t)seg * p.ldw;
      // 16-B aligned model row (SSGD: one model): each lane's VEC contiguous weights
      // with VEC / 4 vector loads instead of VEC bounds-checked scalar ones (fewer
      // instructions on the cold start-up path)
      const bool vec_ok = !PERSIST && (reinterpret_cast<uintptr_t>(w) & 15) == 0;
      if (vec_ok) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int col0 = (c * 64 + lane) * VEC;
          if (col0 + VEC <= p.D) {
#pragma unroll
            for (int v = 0; v < VEC / 4; ++v) {
              const float4 f = *reinterpret_cast<const float4*>(w + col0 + 4 * v);
              wr[c][4 * v] = f.x; wr[c][4 * v + 1] = f.y; wr[c][4 * v + 2] = f.z; wr[c][4 * v + 3] = f.w;
            }
          } else {
#pragma unroll
            for (int e = 0; e < VEC; ++e) wr[c][e] = (col0 + e < p.D) ? w[col0 + e] : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            int col = (c * 64 + lane) * VEC + e;
            wr[c][e] = (col < p.D) ? ldw_(w + col) : 0.f;
          }
      }
      wb = p.has_bias ? ldw_(w + p.D) : 0.f;
    }
  };

  float g[NC][VEC];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < VEC; ++e) g[c][e] = 0.f;
  float gb = 0.f;      // bias gradient (sum r), identical in every lane
  float cntf = 0.f;    // selected rows
  float lossf = 0.f;   // eval: log-loss sum
  unsigned correct = 0;

  const T* X = reinterpret_cast<const T*>(p.X);
  // group walk in global-row space, 256 rows per group, 4 rows per lane
  const int64_t glo = p.row_offset + lo, ghi = p.row_offset + hi;
  const int64_t gstart = glo & ~(int64_t)3;
  int* ring = reinterpret_cast<int*>(s_arena) + wid * kRing;
  const int q = lane >> 4;
  uint32_t head = 0, tail = 0;
  // work units are counted in 2^qs-row units (64 rows when sampling, 8 when every row is
  // taken: a unit then holds 8x the selected rows); a claim takes a whole 256-row group
  // (upg units) until fewer than the fine threshold's groups of the block are unclaimed,
  // then single units, so the block's waves finish within ~1.5 row batches of each other
  const int qs = (EVAL || p.full) ? 3 : p.unit_shift;
  const int upg = 256 >> qs;
  const int fine_u = (p.fine_q * upg) >> 2;   // fine_q counts 64-row quarters
  const int nq = (int)((ghi - gstart + (1 << qs) - 1) >> qs);
  // a block with few rows pre-assigns and claims single units (whole groups would leave
  // most of its waves idle)
  const bool small = nq < upg * NW + fine_u;
  const int w0 = small ? 1 : upg;
  if (threadIdx.x == 0) s_next = w0 * NW;   // units 0..w0 * NW - 1 are pre-assigned
  if (use_pool) {
    if (threadIdx.x < kPoolSlots) s_chunk[threadIdx.x] = -2;
    if (threadIdx.x == 0) s_pnext = 0;
  }
  __syncthreads();
  const unsigned long long t_bar = tr ? (unsigned long long)__builtin_amdgcn_s_memrealtime() : 0ull;

  int64_t gnext = gstart + ((int64_t)(wid * w0) << qs);
  int64_t ulo = glo;                       // current work unit: rows [max(gnext, ulo), uhi)
  int64_t uhi = min(ghi, gnext + ((int64_t)w0 << qs));
  bool more = gnext < ghi;
  int sclaim = w0 * (NW + wid);            // next unit of this wave in the fixed map

  // ---- K7: Bernoulli selection of the next work unit, compacted into the ring
  auto refill = [&]() {
    while ((tail - head) < (uint32_t)(2 * U) && more) {
      const int64_t r0 = gnext + 4 * lane;
      u32x4 h{0u, 0u, 0u, 0u};
      if (!p.full && !EVAL && r0 < uhi) h = philox_block(p.seed, step_cur, (uint64_t)r0 >> 2);
      const uint32_t hv[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t gr = r0 + j;
        const bool sel = (gr >= ulo) && (gr < uhi) && (EVAL || p.full || hv[j] < p.thr);
        const uint64_t m = __ballot(sel);
        const uint32_t pos = tail + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (sel) ring[pos & (kRing - 1)] = (int)(gr - p.row_offset - lo);
        tail += (uint32_t)__popcll(m);
      }
      // claim the next unit dynamically: waves that drew few selected rows
      // take more units, so the block's waves finish together
      {
        int gi = 0, w = w0;
        if (!kLean && !p.atomic_out) {
          // fixed-order epilogue: a fixed group -> wave map (wave w takes groups
          // w, w + NW, ...), so every partial sum is bitwise repeatable
          gi = sclaim;
          sclaim += w0 * NW;
        } else {
          if (lane == 0) {
            if (small || (fine_u > 0 && nq - *(volatile int*)&s_next <= fine_u)) w = 1;
            gi = atomicAdd(&s_next, w);
          }
          gi = __builtin_amdgcn_readfirstlane(gi);
          w = __builtin_amdgcn_readfirstlane(w);
        }
        if (gi < nq) {
          gnext = gstart + ((int64_t)gi << qs);
          uhi = min(ghi, gnext + ((int64_t)w << qs));
        } else if (use_pool) {
          // the block's own units are gone: units of pool chunks. The BLOCK claims chunks
          // of 2^pool_shift rows (one agent-scope atomic each: a per-wave claim of single
          // units serialised ~2000 atomics on one address, 51 -> 82 us per step, r6_35);
          // its waves draw the chunk's 2^qs-row units from an LDS counter. The drawer of
          // unit upc - kPoolPre of chunk m claims chunk m + 1 ahead; chunk 0 is claimed by
          // the first drawer. Slot states: -2 pending, -1 pool exhausted, else the chunk.
          const int upc = 1 << (p.pool_shift - qs);
          int k = 0;
          if (lane == 0) k = atomicAdd(&s_pnext, 1);
          k = __builtin_amdgcn_readfirstlane(k);
          const int m = k >> (p.pool_shift - qs), j = k & (upc - 1);
          if (m >= kPoolSlots) {
            more = false;
          } else {
            const int64_t nchunk = (seg_hi - p.pool_lo + ((int64_t)1 << p.pool_shift) - 1) >> p.pool_shift;
            auto claim = [&](int mm) {
              if (lane == 0) {
                const int c = __hip_atomic_fetch_add(p.pool + (step_cur & 1), 1, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                *(volatile int*)&s_chunk[mm] = c < nchunk ? c : -1;
              }
            };
            if (m == 0 && j == 0) claim(0);
            if (j == max(0, upc - kPoolPre) && m + 1 < kPoolSlots) claim(m + 1);
            int c = 0;
            if (lane == 0) {
              // bounded like the step-release wait: a slot never written would be a bug;
              // it then ends this wave's sweep and raises the persistent error word
              const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
              while ((c = *(volatile int*)&s_chunk[m]) == -2) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > p.spin_ticks) {
                  __hip_atomic_store(p.perr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                  c = -1;
                  break;
                }
                __builtin_amdgcn_s_sleep(1);
              }
            }
            c = __builtin_amdgcn_readfirstlane(c);
            const int64_t g0 = p.row_offset + p.pool_lo + ((int64_t)c << p.pool_shift) + ((int64_t)j << qs);
            const int64_t gend = p.row_offset + seg_hi;
            if (c >= 0 && g0 < gend) {
              // (the Philox quad stays aligned: the walk starts at the unit's quad)
              gnext = g0 & ~(int64_t)3;
              ulo = g0;
              uhi = min(gend, g0 + ((int64_t)1 << qs));
            } else {
              more = false;
            }
          }
        } else {
          more = false;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  };

  auto take_and_load = [&](Batch<NC, U>& b) {
    int64_t r[U];
    {
    const uint32_t avail = tail - head;
    b.n = (int)min(avail, (uint32_t)U);
    if (b.n == 0) return;
    const uint32_t last = b.n - 1;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      r[k] = lo + __builtin_amdgcn_readfirstlane(ring[(head + min((uint32_t)k, last)) & (kRing - 1)]);
      b.v[k] = (k < b.n) ? 1.f : 0.f;
    }
    head += b.n;
    }
    // one buffer descriptor per row (wave-uniform SGPRs, base = row start,
    // num_records = row bytes): lanes past the row read 0 via the range check
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(X + r[k] * p.ld), (short)0, (int)(p.ld * (int64_t)sizeof(T)), 0x00020000);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (c * 64 + lane) * 16, 0, AUX);
        b.x[k][c] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
#pragma unroll
    for (int j = 0; j < U / 4; ++j) {
      const int64_t rq = q == 0 ? r[4 * j] : (q == 1 ? r[4 * j + 1] : (q == 2 ? r[4 * j + 2] : r[4 * j + 3]));
      b.yq[j] = p.y[rq];
    }
  };

  auto compute = [&](Batch<NC, U>& b) {
    float d[U];
#pragma unroll
    for (int k = 0; k < U; ++k) d[k] = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        float f[VEC];
        unpack<T>(b.x[k][c], f);
#pragma unroll
        for (int e = 0; e < VEC; ++e) d[k] = fmaf(f[e], wr[c][e], d[k]);
      }
    }
    float z[U / 4];
#pragma unroll
    for (int j = 0; j < U / 4; ++j)
      z[j] = wave_sum4(d[4 * j], d[4 * j + 1], d[4 * j + 2], d[4 * j + 3]) + wb;
    // Opaque re-definition of the raw rows: forces the bf16->f32 unpack to be
    // recomputed in the rank-1 update instead of keeping U*NC*VEC unpacked
    // floats live across the reduction (saves ~64 VGPRs -> 2x occupancy).
#pragma unroll
    for (int k = 0; k < U; ++k)
#pragma unroll
      for (int c = 0; c < NC; ++c)
        asm volatile("" : "+v"(b.x[k][c].x), "+v"(b.x[k][c].y), "+v"(b.x[k][c].z), "+v"(b.x[k][c].w));
    float rs[U];
#pragma unroll
    for (int j = 0; j < U / 4; ++j) {
      const float sig = 1.f / (__expf(-z[j]) + 1.f + p.eps);
      const float vq = q == 0 ? b.v[4 * j] : (q == 1 ? b.v[4 * j + 1] : (q == 2 ? b.v[4 * j + 2] : b.v[4 * j + 3]));
      const float yq = b.yq[j];
      if constexpr (EVAL) {
        // pred = sigma < 0.5 ? 0 : 1  (ssgd.py:108-109)
        const float pred = sig < 0.5f ? 0.f : 1.f;
        const float ok = (pred == yq) ? vq : 0.f;
        const float sc = fminf(fmaxf(sig, 1e-7f), 1.f - 1e-7f);
        const float l = -(yq * __logf(sc) + (1.f - yq) * __logf(1.f - sc)) * vq;
        correct += (unsigned)(readlane_f(ok, 0) + readlane_f(ok, 16) + readlane_f(ok, 32) +
                              readlane_f(ok, 48));
        lossf += readlane_f(l, 0) + readlane_f(l, 16) + readlane_f(l, 32) + readlane_f(l, 48);
      } else {
        const float r = (sig - yq) * vq;
#pragma unroll
        for (int k = 0; k < 4; ++k) rs[4 * j + k] = readlane_f(r, 16 * k);
      }
    }
    if constexpr (!EVAL) {
#pragma unroll
      for (int k = 0; k < U; ++k) gb += rs[k];
      cntf += (float)b.n;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
#pragma unroll
        for (int k0 = 0; k0 < U; k0 += 4) {
          float f[4][VEC];
#pragma unroll
          for (int k = 0; k < 4; ++k) unpack<T>(b.x[k0 + k][c], f[k]);
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            float acc = g[c][e];
#pragma unroll
            for (int k = 0; k < 4; ++k) acc = fmaf(rs[k0 + k], f[k][e], acc);
            g[c][e] = acc;
          }
        }
      }
    }
  };

  // ---- software-pipelined sweep: load(i+1) || compute(i)
  Batch<NC, U> A;
  unsigned long long t_first = 0ull, t_refill = 0ull;
  if constexpr (PIPE && PERSIST) {
    // persistent steps: TWO row batches are issued before the wait for the previous
    // step's model release (the selection does not depend on W), so the release chain
    // (last block's epilogue -> tail update -> epoch -> W reads) overlaps two batches'
    // HBM traffic instead of one; then the same one-ahead pipeline
    Batch<NC, U> B;
    refill();
    if (tr) t_refill = __builtin_amdgcn_s_memrealtime();
    take_and_load(A);
    refill();
    take_and_load(B);
    if (it > 0 && !wait_epoch(it)) return;
    load_w();
    if (tr) t_first = __builtin_amdgcn_s_memrealtime();
    while (true) {
      if (A.n == 0) break;
      compute(A);
      if (B.n == 0) break;
      refill();
      take_and_load(A);
      compute(B);
      if (A.n == 0) break;
      refill();
      take_and_load(B);
    }
  } else if constexpr (PIPE) {
    Batch<NC, U> B;
    refill();
    if (tr) t_refill = __builtin_amdgcn_s_memrealtime();
    take_and_load(A);
    if (PERSIST && it > 0 && !wait_epoch(it)) return;
    load_w();
    if (tr) t_first = __builtin_amdgcn_s_memrealtime();
    while (true) {
      if (A.n == 0) break;
      refill();
      take_and_load(B);
      compute(A);
      if (B.n == 0) break;
      refill();
      take_and_load(A);
      compute(B);
    }
  } else {
    if (PERSIST && it > 0 && !wait_epoch(it)) return;
    load_w();
    while (true) {
      refill();
      take_and_load(A);
      if (A.n == 0) break;
      compute(A);
    }
  }
  if (tr && lane == 0) {
    tr[0] = t_start;
    tr[1] = t_first;
    tr[2] = __builtin_amdgcn_s_memrealtime();
    tr[4] = (unsigned long long)cntf;
    tr[5] = __smid();
    tr[6] = t_bar;
    tr[7] = t_refill;
  }
  __syncthreads();   // rings are dead: the arena becomes the reduction buffer

  if constexpr (EVAL) {
    __shared__ float s_ev[NW][2];
    if (lane == 0) { s_ev[wid][0] = (float)correct; s_ev[wid][1] = lossf; }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long c = 0; float l = 0.f;
      for (int k = 0; k < NW; ++k) { c += (unsigned long long)s_ev[k][0]; l += s_ev[k][1]; }
      atomicAdd(&p.correct[seg], c);
      atomicAdd(&p.loss[seg], l);
    }
    continue;
  } else {
    // ---- block reduction across waves (fixed order)
    auto red_row = [&](int k) { return s_arena + k * (COLS + 4); };
    float* red = red_row(wid);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int e = 0; e < VEC; ++e) red[(c * 64 + lane) * VEC + e] = g[c][e];
    if (lane == 0) { red[COLS] = gb; red[COLS + 1] = cntf; }
    __syncthreads();
    const int S = p.S;
    const int D = p.D;
    if (kLean || p.atomic_out) {
      float* Gs = p.G + (int64_t)seg * p.ldw;
      for (int col = threadIdx.x; col < D; col += NW * 64) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) s += red_row(k)[col];
        __hip_atomic_fetch_add(&Gs[col], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (threadIdx.x == 0) {
        float sb = 0.f, sc = 0.f;
        for (int k = 0; k < NW; ++k) { sb += red_row(k)[COLS]; sc += red_row(k)[COLS + 1]; }
        if (p.has_bias) __hip_atomic_fetch_add(&Gs[D], sb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&p.C[seg], sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p.count_acc)
          __hip_atomic_fetch_add(p.count_acc, (double)sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (tr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) tr[3] = __builtin_amdgcn_s_memrealtime();
      }
      if (p.ticket == nullptr) continue;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this block's adds are performed
      __syncthreads();
      if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(p.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_flag = (t == gridDim.x * gridDim.y - 1u);
      }
      __syncthreads();
      if (s_flag) {
        if (p.tu.mode == 2) {
          // no fused update (a plain gradient launch with the row pool): the last block
          // only re-arms the ticket and the pool
          if (threadIdx.x == 0) __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          // exchange epoch of step it: device base (unchanged until this launch's last
          // exchange is done) + it + 1; the last step's tail stores the new base
          const uint32_t xbase = p.xg.world > 1 ? xg_epoch_base(p.xg) : 0u;
          lr_tail(p, xbase + (uint32_t)it + 1u);
          if (p.xg.world > 1 && it == nst - 1 && threadIdx.x == 0)
            xg_epoch_store(p.xg, xbase + (uint32_t)nst);
        }
        if (use_pool && threadIdx.x == 0)   // every block is past this step's pool claims
          __hip_atomic_store(p.pool + (step_cur & 1), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (PERSIST && nst > 1) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // W / G / C / ticket written through
          __syncthreads();
          if (threadIdx.x == 0)
            __hip_atomic_store(p.epoch, p.epoch_base + (uint32_t)it + 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      continue;
    }
    float* my = p.slab + ((int64_t)seg * gx + bx) * S;
    for (int col = threadIdx.x; col < D; col += NW * 64) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < NW; ++k) s += red_row(k)[col];
      st_wt(&my[col], s);
    }
    if (threadIdx.x == 0) {
      float sb = 0.f, sc = 0.f;
      for (int k = 0; k < NW; ++k) { sb += red_row(k)[COLS]; sc += red_row(k)[COLS + 1]; }
      st_wt(&my[D], sb);       // bias grad slot
      st_wt(&my[D + 1], sc);   // count slot
    }
    // ---- level 1: last arriver of each 16-block group sums the group's slabs
    const int ngroups = (gx + kGroup - 1) / kGroup;
    const int grp = bx / kGroup;
    const int gsize = min(kGroup, gx - grp * kGroup);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned t = __hip_atomic_fetch_add(&p.cnt1[seg * ngroups + grp], 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
      s_flag = (t == (unsigned)(gsize - 1));
    }
    __syncthreads();
    if (!s_flag) continue;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: keep loads below
    const int nv = D + 2;
    {
      const float* src = p.slab + ((int64_t)seg * gx + grp * kGroup) * S;
      float* dst = p.gslab + ((int64_t)seg * ngroups + grp) * S;
      for (int col = threadIdx.x; col < nv; col += NW * 64) {
        st_wt(&dst[col], sum_slab_col(src, gsize, S, col));
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      p.cnt1[seg * ngroups + grp] = 0u;   // re-arm for the next launch
      unsigned t = __hip_atomic_fetch_add(&p.cnt2[seg], 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
      s_flag = (t == (unsigned)(ngroups - 1));
    }
    __syncthreads();
    if (!s_flag) continue;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- level 2: sum group slabs in order -> G[seg], C[seg]
    {
      const float* src = p.gslab + (int64_t)seg * ngroups * S;
      float* Gs = p.G + (int64_t)seg * p.ldw;
      for (int col = threadIdx.x; col < nv; col += NW * 64) {
        const float s = sum_slab_col(src, ngroups, S, col);
        if (col < D) Gs[col] = s;
        else if (col == D) { if (p.has_bias) Gs[D] = s; }
        else {
          p.C[seg] = s;
          if (p.count_acc) p.count_acc[0] += (double)s;
        }
      }
    }
    if (threadIdx.x == 0) p.cnt2[seg] = 0u;
  }
  }  // step loop
}

}  // namespace dalgo

using namespace dalgo;

template <typename T, int NC, bool EVAL, int NW, bool PIPE, int U, int AUX = 0, bool LEAN = false>
static hipError_t launch_lr(const LrParams& p, int gx, int nseg, hipStream_t st) {
  dim3 grid(gx, nseg), block(NW * 64);
  if (p.nsteps > 1) {
    if constexpr (!EVAL) {
      // persistent mode: every block must be resident (blocks wait on each other);
      // the cooperative launch refuses a grid that cannot be. DALGO_PERSIST_COOP=0: a plain
      // launch instead (experiment: the cooperative path's fixed cost per launch)
      static int coop = -1;
      if (coop < 0) {
        const char* e = std::getenv("DALGO_PERSIST_COOP");
        coop = (e != nullptr && e[0] == '0') ? 0 : 1;
      }
      if (!coop) {
        hipLaunchKernelGGL((lr_rows_kernel<T, NC, EVAL, NW, PIPE, U, true, AUX>), grid, block, 0, st, p);
        DALGO_LAUNCH_CHECK();
        return hipSuccess;
      }
      void* args[] = {const_cast<LrParams*>(&p)};
      return hipLaunchCooperativeKernel((const void*)lr_rows_kernel<T, NC, EVAL, NW, PIPE, U, true, AUX>,
                                        grid, block, args, 0, st);
    }
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL((lr_rows_kernel<T, NC, EVAL, NW, PIPE, U, false, AUX, LEAN>), grid, block, 0, st, p);
  DALGO_LAUNCH_CHECK();
  return hipSuccess;
}

// Launch shape (A/B-tested in bench/lr_kernel_sweep.py, profiles/round1-2): 8 waves per
// block, 4-row batches, non-temporal row loads (buffer-load aux bit 2); two register sets
// (row loads of batch i+1 in flight while batch i is computed) while the model fragment
// fits (<= 2 column chunks per lane), one set at 4 chunks. The atomic epilogue runs the
// LEAN build, the deterministic fixed-order epilogue the full one.
template <typename T, int NC, bool EVAL>
static hipError_t launch_shape(const LrParams& p, int gx, int nseg, hipStream_t st) {
  constexpr bool kPipe = NC < 4;   // register budget: one 4-row set at 4 chunks/lane
  if constexpr (!EVAL) {
    if (p.atomic_out) return launch_lr<T, NC, EVAL, 8, kPipe, 4, 2, true>(p, gx, nseg, st);
  }
  return launch_lr<T, NC, EVAL, 8, kPipe, 4, 2, false>(p, gx, nseg, st);
}

template <bool EVAL>
static hipError_t dispatch_lr(const LrParams& p, int is_bf16, int gx, int nseg, hipStream_t st) {
  const int vec = is_bf16 ? 8 : 4;
  const int64_t nchunks = p.ld / vec;
  const int nc = (int)cdiv(nchunks, 64);
  if (is_bf16) {
    switch (nc) {
      case 1: return launch_shape<uint16_t, 1, EVAL>(p, gx, nseg, st);
      case 2: return launch_shape<uint16_t, 2, EVAL>(p, gx, nseg, st);
      case 3: case 4: return launch_shape<uint16_t, 4, EVAL>(p, gx, nseg, st);
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (nc) {
      case 1: return launch_shape<float, 1, EVAL>(p, gx, nseg, st);
      case 2: return launch_shape<float, 2, EVAL>(p, gx, nseg, st);
      case 3: case 4: return launch_shape<float, 4, EVAL>(p, gx, nseg, st);
      default: return hipErrorInvalidValue;
    }
  }
}

static unsigned long long* g_lr_trace = nullptr;

extern "C" {

// diagnostics: route the per-wave timeline of later dalgo_lr_grad launches to `buf`
// (nullptr: off). Sized by the caller: 8 u64 per wave of the launch.
void dalgo_lr_set_trace(void* buf) { g_lr_trace = static_cast<unsigned long long*>(buf); }

// Maximum supported row stride: 4 chunks/lane -> 2048 bf16 or 1024 f32 columns.
int dalgo_lr_max_cols(int is_bf16) { return is_bf16 ? 2048 : 1024; }

// flags: bit 8 = atomic epilogue; bits 16..23 = fine-claim threshold (64-row quarters of
// the block's groups); bits 24..27 = log2 rows per sampled work unit (0 = 6)
hipError_t dalgo_lr_grad(const void* X, const float* y, const float* W, const int64_t* seg,
                         int64_t ld, int64_t row_offset, int D, int ldw, int has_bias, float eps,
                         uint64_t seed, uint64_t step, uint32_t thr, int full, int is_bf16,
                         int gx, int nseg, int rows_per_block, float* slab, float* gslab,
                         unsigned* cnt1, unsigned* cnt2, float* G, float* C, int S, int flags,
                         double* count_acc, const DalgoLrTail* tail, const int64_t* step_dev,
                         int64_t step_mul, hipStream_t st) {
  LrParams p{};
  p.step_dev = step_dev;
  p.step_mul = step_mul;
  if (tail != nullptr) {
    if (tail->mode == 2 && (tail->world != 1 || tail->nsteps > 1 || tail->pool == nullptr))
      return hipErrorInvalidValue;   // mode 2: a pooled gradient launch without the update
    if (nseg != 1 || !((flags >> 8) & 1) || tail->ticket == nullptr ||
        tail->world < 1 || tail->world > kXgMaxRanks || tail->rank < 0 || tail->rank >= tail->world ||
        (tail->world > 1 && (tail->epoch_dev == nullptr || tail->slot < ldw + 1)))
      return hipErrorInvalidValue;
    p.ticket = tail->ticket;
    for (int r = 0; r < tail->world; ++r) {
      if (tail->world > 1 && tail->bufs[r] == nullptr) return hipErrorInvalidValue;
      p.xg.bufs[r] = static_cast<uint8_t*>(tail->bufs[r]);
    }
    p.xg.rank = tail->rank; p.xg.world = tail->world; p.xg.slot = tail->slot;
    p.xg.epoch_dev = tail->epoch_dev; p.xg.err = tail->err;
    p.xg.timeout_ticks = (long long)(tail->timeout_s * 1e8);
    p.tu = XgUpdate{tail->mode, tail->reg, tail->eta, tail->lam, tail->reg_alpha};
    p.tail_count_acc = tail->count_acc;
    if (tail->nsteps > 1) {
      if (tail->epoch_ctr == nullptr || tail->perr == nullptr) return hipErrorInvalidValue;
      p.nsteps = tail->nsteps;
      p.epoch = tail->epoch_ctr;
      p.epoch_base = tail->epoch_base;
      p.perr = tail->perr;
      p.spin_ticks = (uint64_t)(tail->spin_s * 1e8);
    }
    if (tail->pool != nullptr) {
      if (tail->pool_lo < 0 || tail->pool_shift < 6 || tail->pool_shift > 16) return hipErrorInvalidValue;
      p.pool = tail->pool;
      p.pool_lo = tail->pool_lo;
      p.pool_shift = tail->pool_shift;
      if (p.spin_ticks == 0) p.spin_ticks = (uint64_t)(2.0 * 1e8);   // the chunk-slot wait bound
      p.perr = tail->perr;
      if (p.perr == nullptr) return hipErrorInvalidValue;
    }
  }
  p.count_acc = count_acc;
  p.X = X; p.y = y; p.W = W; p.seg = seg; p.ld = ld; p.row_offset = row_offset; p.D = D;
  p.ldw = ldw; p.has_bias = has_bias; p.eps = eps; p.seed = seed; p.step = step; p.thr = thr;
  p.full = full; p.rows_per_block = rows_per_block; p.slab = slab; p.gslab = gslab;
  p.cnt1 = cnt1; p.cnt2 = cnt2; p.G = G; p.C = C; p.S = S;
  p.atomic_out = (flags >> 8) & 1;
  p.fine_q = 4 * ((flags >> 16) & 0xff);
  p.unit_shift = ((flags >> 24) & 0xf) ? ((flags >> 24) & 0xf) : 6;
  if (p.unit_shift < 2 || p.unit_shift > 8) return hipErrorInvalidValue;
  p.trace = g_lr_trace;
  return dispatch_lr<false>(p, is_bf16, gx, nseg, st);
}

hipError_t dalgo_lr_eval(const void* X, const float* y, const float* W, const int64_t* seg,
                         int64_t ld, int D, int ldw, int has_bias, float eps, int is_bf16, int gx,
                         int nseg, int rows_per_block, unsigned long long* correct, float* loss,
                         hipStream_t st) {
  LrParams p{};
  p.X = X; p.y = y; p.W = W; p.seg = seg; p.ld = ld; p.row_offset = 0; p.D = D; p.ldw = ldw;
  p.has_bias = has_bias; p.eps = eps; p.full = 1; p.rows_per_block = rows_per_block;
  p.correct = correct; p.loss = loss;
  return dispatch_lr<true>(p, is_bf16, gx, nseg, st);
}

}  // extern "C"
