// dalgo torch-op registrations (TORCH_LIBRARY "dalgo").
//
// Every op validates shapes/dtypes/devices on the host (a kernel is never
// launched on operands whose shape disagrees with what its grid assumes), then
// calls the extern "C" launcher of the gfx950 kernel on the caller's current HIP
// stream, so ops compose with torch streams and hipGraph capture. Launch
// failures surface as c10::Error with the op name.
#include <map>
#include <string>
#include <cstdlib>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "launchers.h"

namespace {

using at::Tensor;

// ROCm torch exposes HIP devices as DeviceType::CUDA ("masquerading"), so the
// guard/stream helpers are the masquerading variants.
inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
using DeviceGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

// a failed launch leaves its error in the runtime's last-error slot, which the next torch
// call on the stream would report again: cleared here, reported once
#define DALGO_CHECK_HIP(expr, name)                                                   \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) (void)hipGetLastError();                                    \
    TORCH_CHECK(_e == hipSuccess, "dalgo::" name " launch failed: ", hipGetErrorString(_e)); \
  } while (0)

inline void check_dev(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), "dalgo: ", what, " must be a GPU (HIP) tensor");
}
inline void check_f32(const Tensor& t, const char* what) {
  check_dev(t, what);
  TORCH_CHECK(t.scalar_type() == at::kFloat, "dalgo: ", what, " must be float32");
  TORCH_CHECK(t.is_contiguous(), "dalgo: ", what, " must be contiguous");
}

inline uint32_t frac_threshold(double frac) {
  if (frac <= 0.0) return 0u;
  if (frac >= 1.0) return 0xffffffffu;
  double t = std::floor(frac * 4294967296.0);
  return t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
}

void check_lr_inputs(const Tensor& X, const Tensor& y, const Tensor& W, const Tensor& seg,
                     int64_t D, bool has_bias) {
  check_dev(X, "X");
  TORCH_CHECK(X.dim() == 2, "X must be 2-D");
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 || X.scalar_type() == at::kFloat,
              "X must be bf16 or f32");
  TORCH_CHECK(X.stride(1) == 1, "X rows must be contiguous");
  const int vec = X.scalar_type() == at::kBFloat16 ? 8 : 4;
  const int64_t ld = X.stride(0);
  TORCH_CHECK(ld % vec == 0, "X row stride must be a multiple of ", vec, " elements (16 B)");
  TORCH_CHECK(X.size(1) >= D && ld >= X.size(1), "X has fewer columns than D");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0, "X must be 16-B aligned");
  TORCH_CHECK(ld <= dalgo_lr_max_cols(vec == 8), "row stride too large for lr kernels");
  check_f32(y, "y");
  TORCH_CHECK(y.numel() >= X.size(0), "y shorter than X");
  check_f32(W, "W");
  TORCH_CHECK(W.dim() == 2 && W.size(1) >= D + (has_bias ? 1 : 0), "W shape");
  check_dev(seg, "seg");
  TORCH_CHECK(seg.scalar_type() == at::kLong && seg.dim() == 1 && seg.numel() == W.size(0) + 1,
              "seg must be int64 [n_seg+1]");
  TORCH_CHECK(X.get_device() == W.get_device() && X.get_device() == y.get_device(),
              "device mismatch");
}

// ---------------------------------------------------------------------------
void lr_grad(const Tensor& X, const Tensor& y, const Tensor& W, const Tensor& seg,
             int64_t row_offset, int64_t D, bool has_bias, double eps, int64_t seed, int64_t step,
             double frac, int64_t gx, int64_t rows_per_block, Tensor slab, Tensor gslab,
             Tensor cnt1, Tensor cnt2, Tensor G, Tensor C, int64_t flags,
             const std::optional<Tensor>& count_acc,
             const std::optional<Tensor>& ticket, at::OptionalIntArrayRef xg_bufs, int64_t xg_rank,
             int64_t xg_slot, const std::optional<Tensor>& xg_epoch, const std::optional<Tensor>& xg_err,
             double xg_timeout, int64_t tail_mode, int64_t tail_reg, double tail_eta,
             double tail_lam, double tail_reg_alpha, const std::optional<Tensor>& tail_count_acc,
             int64_t nsteps, const std::optional<Tensor>& epoch, int64_t epoch_base,
             const std::optional<Tensor>& perr, double spin_s,
             const std::optional<Tensor>& step_dev, int64_t step_mul, const std::optional<Tensor>& pool,
             int64_t pool_lo, int64_t pool_shift) {
  check_lr_inputs(X, y, W, seg, D, has_bias);
  const int64_t* stepp = nullptr;
  if (step_dev.has_value()) {
    check_dev(*step_dev, "step_dev");
    TORCH_CHECK(step_dev->scalar_type() == at::kLong && step_dev->numel() >= 1,
                "step_dev: int64[1] device step counter");
    TORCH_CHECK(step_mul >= 0, "step_mul >= 0");
    stepp = step_dev->data_ptr<int64_t>();
  }
  DalgoLrTail tail{};
  const DalgoLrTail* tailp = nullptr;
  TORCH_CHECK(nsteps <= 1 || ticket.has_value(), "persistent launch needs the fused tail");
  if (ticket.has_value()) {
    check_dev(*ticket, "ticket");
    TORCH_CHECK(ticket->scalar_type() == at::kInt && ticket->numel() >= 1, "ticket int32[1]");
    TORCH_CHECK(W.size(0) == 1 && (flags & 256), "fused tail: one model, atomic epilogue");
    TORCH_CHECK(tail_mode == 0 || tail_mode == 1 || (tail_mode == 2 && nsteps <= 1 && pool.has_value()),
                "fused tail mode: 0 SSGD, 1 GD, 2 none (pooled gradient launch)");
    tail.ticket = reinterpret_cast<unsigned*>(ticket->data_ptr<int>());
    tail.world = 1;
    if (xg_bufs.has_value() && xg_bufs->size() > 1) {
      TORCH_CHECK(xg_bufs->size() <= 8 && xg_rank >= 0 && xg_rank < (int64_t)xg_bufs->size(),
                  "fused tail: 2..8 ranks");
      TORCH_CHECK(xg_epoch.has_value() && xg_epoch->scalar_type() == at::kInt && xg_epoch->numel() >= 1,
                  "fused tail: device epoch int32[1]");
      check_dev(*xg_epoch, "xg_epoch");
      TORCH_CHECK(xg_slot >= W.size(1) + 1, "fused tail: bucket larger than the slot");
      TORCH_CHECK(xg_err.has_value() && xg_err->scalar_type() == at::kInt, "fused tail: err int32");
      check_dev(*xg_err, "xg_err");
      tail.world = (int)xg_bufs->size();
      for (int r = 0; r < tail.world; ++r) tail.bufs[r] = reinterpret_cast<void*>((*xg_bufs)[r]);
      tail.rank = (int)xg_rank;
      tail.slot = (int)xg_slot;
      tail.epoch_dev = reinterpret_cast<uint32_t*>(xg_epoch->data_ptr<int32_t>());
      tail.err = reinterpret_cast<unsigned*>(xg_err->data_ptr<int>());
      tail.timeout_s = xg_timeout;
    }
    tail.mode = (int)tail_mode; tail.reg = (int)tail_reg; tail.eta = (float)tail_eta;
    tail.lam = (float)tail_lam; tail.reg_alpha = (float)tail_reg_alpha;
    if (tail_count_acc.has_value()) {
      check_dev(*tail_count_acc, "tail_count_acc");
      TORCH_CHECK(tail_count_acc->scalar_type() == at::kDouble, "tail_count_acc f64");
      tail.count_acc = tail_count_acc->data_ptr<double>();
    }
    if (nsteps > 1) {
      TORCH_CHECK(epoch.has_value() && perr.has_value(), "persistent launch: epoch + perr counters");
      check_dev(*epoch, "epoch");
      check_dev(*perr, "perr");
      TORCH_CHECK(epoch->scalar_type() == at::kInt && perr->scalar_type() == at::kInt,
                  "persistent launch: int32 epoch / perr");
      TORCH_CHECK(nsteps < (1LL << 30) && epoch_base >= 0 && epoch_base <= 0xffffffffLL && spin_s > 0,
                  "persistent launch: bad nsteps / epoch_base / spin_s");
      tail.nsteps = (int)nsteps;
      tail.epoch_ctr = reinterpret_cast<unsigned*>(epoch->data_ptr<int>());
      tail.epoch_base = (uint32_t)epoch_base;
      tail.perr = reinterpret_cast<unsigned*>(perr->data_ptr<int>());
      tail.spin_s = spin_s;
    }
    if (pool.has_value()) {
      check_dev(*pool, "pool");
      TORCH_CHECK(pool->scalar_type() == at::kInt && pool->numel() >= 2, "pool: int32[2] counters");
      TORCH_CHECK(pool_lo >= 0 && pool_lo <= X.size(0) && pool_shift >= 6 && pool_shift <= 16,
                  "pool: 0 <= pool_lo <= rows, 6 <= pool_shift <= 16");
      TORCH_CHECK(perr.has_value() && perr->scalar_type() == at::kInt, "pool: needs the perr error word");
      check_dev(*perr, "perr");
      tail.pool = pool->data_ptr<int>();
      tail.pool_lo = pool_lo;
      tail.pool_shift = (int)pool_shift;
      tail.perr = reinterpret_cast<unsigned*>(perr->data_ptr<int>());
    }
    tailp = &tail;
  }
  double* cacc = nullptr;
  if (count_acc.has_value()) {
    check_dev(*count_acc, "count_acc");
    TORCH_CHECK(count_acc->scalar_type() == at::kDouble, "count_acc f64");
    cacc = count_acc->data_ptr<double>();
  }
  const int64_t nseg = W.size(0);
  TORCH_CHECK(gx >= 1 && gx <= 65535, "gx");
  TORCH_CHECK(rows_per_block > 0 && rows_per_block % 4 == 0, "rows_per_block % 4");
  const int64_t ngroups = (gx + 15) / 16;
  check_f32(slab, "slab"); check_f32(gslab, "gslab"); check_f32(G, "G"); check_f32(C, "C");
  const int64_t S = slab.size(1);
  TORCH_CHECK(S >= D + 2, "slab stride");
  TORCH_CHECK(slab.size(0) >= nseg * gx && gslab.size(0) >= nseg * ngroups &&
              gslab.size(1) == S, "slab/gslab shape");
  TORCH_CHECK(cnt1.scalar_type() == at::kInt && cnt1.numel() >= nseg * ngroups, "cnt1");
  TORCH_CHECK(cnt2.scalar_type() == at::kInt && cnt2.numel() >= nseg, "cnt2");
  TORCH_CHECK(G.dim() == 2 && G.size(0) == nseg && G.size(1) == W.size(1), "G shape");
  TORCH_CHECK(C.numel() >= nseg, "C shape");
  DeviceGuard guard(X.device());
  const bool full = frac >= 1.0;
  DALGO_CHECK_HIP(
      dalgo_lr_grad(X.data_ptr(), y.data_ptr<float>(), W.data_ptr<float>(), seg.data_ptr<int64_t>(),
                    X.stride(0), row_offset, (int)D, (int)W.size(1), has_bias ? 1 : 0, (float)eps,
                    (uint64_t)seed, (uint64_t)step, frac_threshold(frac), full ? 1 : 0,
                    X.scalar_type() == at::kBFloat16 ? 1 : 0, (int)gx, (int)nseg,
                    (int)rows_per_block, slab.data_ptr<float>(), gslab.data_ptr<float>(),
                    reinterpret_cast<unsigned*>(cnt1.data_ptr<int>()),
                    reinterpret_cast<unsigned*>(cnt2.data_ptr<int>()), G.data_ptr<float>(),
                    C.data_ptr<float>(), (int)S, (int)flags, cacc, tailp, stepp, step_mul,
                    cur_stream()),
      "lr_grad");
}

void lr_eval(const Tensor& X, const Tensor& y, const Tensor& W, const Tensor& seg, int64_t D,
             bool has_bias, double eps, int64_t gx, int64_t rows_per_block, Tensor correct,
             Tensor loss) {
  check_lr_inputs(X, y, W, seg, D, has_bias);
  const int64_t nseg = W.size(0);
  TORCH_CHECK(rows_per_block > 0 && rows_per_block % 4 == 0, "rows_per_block % 4");
  TORCH_CHECK(correct.scalar_type() == at::kLong && correct.numel() >= nseg, "correct");
  check_f32(loss, "loss");
  TORCH_CHECK(loss.numel() >= nseg, "loss");
  DeviceGuard guard(X.device());
  DALGO_CHECK_HIP(
      dalgo_lr_eval(X.data_ptr(), y.data_ptr<float>(), W.data_ptr<float>(), seg.data_ptr<int64_t>(),
                    X.stride(0), (int)D, (int)W.size(1), has_bias ? 1 : 0, (float)eps,
                    X.scalar_type() == at::kBFloat16 ? 1 : 0, (int)gx, (int)nseg,
                    (int)rows_per_block,
                    reinterpret_cast<unsigned long long*>(correct.data_ptr<int64_t>()),
                    loss.data_ptr<float>(), cur_stream()),
      "lr_eval");
}

// ---------------------------------------------------------------------------
void sync_update(Tensor W, const std::optional<Tensor>& G, const std::optional<Tensor>& C,
                 const std::optional<Tensor>& center, const std::optional<Tensor>& S,
                 const std::optional<Tensor>& Dl, const std::optional<Tensor>& count_acc, int64_t n,
                 int64_t mode, int64_t reg, double eta, double lam, double alpha, double reg_alpha,
                 double mu, double zeta, double beta, double inv_p, bool zero_grad) {
  check_f32(W, "W");
  TORCH_CHECK(W.dim() == 2 && n <= W.size(1), "W must be [rows, ld] with n <= ld");
  const int64_t nrow = W.size(0), ld = W.size(1);
  auto ptr = [&](const std::optional<Tensor>& t, const char* nm, int64_t need) -> float* {
    if (!t.has_value()) return nullptr;
    check_f32(*t, nm);
    TORCH_CHECK(t->numel() >= need, "dalgo::sync_update: ", nm, " too small");
    return t->data_ptr<float>();
  };
  float* g = ptr(G, "G", nrow * ld);
  float* c = ptr(C, "C", nrow);
  float* ce = ptr(center, "center", n);
  float* s = ptr(S, "S", n);
  float* dl = ptr(Dl, "Dl", n);
  double* cacc = nullptr;
  if (count_acc.has_value()) {
    check_dev(*count_acc, "count_acc");
    TORCH_CHECK(count_acc->scalar_type() == at::kDouble && count_acc->numel() >= 1, "count_acc f64");
    TORCH_CHECK(c, "count_acc needs C");
    cacc = count_acc->data_ptr<double>();
  }
  switch (mode) {
    case 0: TORCH_CHECK(g && c, "SSGD needs G, C"); break;
    case 1: TORCH_CHECK(g, "GD needs G"); break;
    case 2: TORCH_CHECK(g && c, "local needs G, C"); break;
    case 3: TORCH_CHECK(g && c && ce, "elastic local needs G, C, center"); break;
    case 4: case 6: TORCH_CHECK(s && nrow == 1, "sync needs S and one row"); break;
    case 5: TORCH_CHECK(s && dl && nrow == 1, "BMUF needs S, Dl and one row"); break;
    default: TORCH_CHECK(false, "unknown update mode ", mode);
  }
  DeviceGuard guard(W.device());
  DALGO_CHECK_HIP(dalgo_sync_update(W.data_ptr<float>(), g, c, ce, s, dl, cacc, (int)n, (int)ld,
                                    (int)nrow, (int)mode, (int)reg, (float)eta, (float)lam,
                                    (float)alpha, (float)reg_alpha, (float)mu, (float)zeta,
                                    (float)beta, (float)inv_p, zero_grad ? 1 : 0, cur_stream()),
                  "sync_update");
}

void rows_sum(const Tensor& W, int64_t n, Tensor out) {
  check_f32(W, "W");
  check_f32(out, "out");
  TORCH_CHECK(W.dim() == 2 && n <= W.size(1) && out.numel() >= n, "rows_sum shapes");
  DeviceGuard guard(W.device());
  DALGO_CHECK_HIP(dalgo_rows_sum(W.data_ptr<float>(), (int)W.size(0), (int)W.size(1), (int)n,
                                 out.data_ptr<float>(), cur_stream()),
                  "rows_sum");
}

void rows_broadcast(Tensor W, int64_t n, const Tensor& src) {
  check_f32(W, "W");
  check_f32(src, "src");
  TORCH_CHECK(W.dim() == 2 && n <= W.size(1) && src.numel() >= n, "rows_broadcast shapes");
  DeviceGuard guard(W.device());
  DALGO_CHECK_HIP(dalgo_rows_broadcast(W.data_ptr<float>(), (int)W.size(0), (int)W.size(1),
                                       (int)n, src.data_ptr<float>(), cur_stream()),
                  "rows_broadcast");
}

// ---------------------------------------------------------------------------
void philox_fill(Tensor out, int64_t D, int64_t row_offset, int64_t seed, int64_t stream,
                 int64_t dist, double a, double b) {
  check_dev(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1, "philox_fill: out must be 2-D, row-contiguous");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat,
              "philox_fill: bf16 or f32");
  TORCH_CHECK(out.stride(0) == out.size(1), "philox_fill: out must be contiguous");
  TORCH_CHECK(D <= out.size(1), "philox_fill: D > columns");
  TORCH_CHECK(dist == 0 || dist == 1, "philox_fill: dist");
  DeviceGuard guard(out.device());
  DALGO_CHECK_HIP(dalgo_philox_fill(out.data_ptr(), out.scalar_type() == at::kBFloat16 ? 1 : 0,
                                    out.size(0), D, out.size(1), row_offset, (uint64_t)seed,
                                    (uint64_t)stream, (int)dist, (float)a, (float)b, cur_stream()),
                  "philox_fill");
}

void mc_pi(int64_t seed, int64_t stream, int64_t offset, int64_t n, Tensor count) {
  check_dev(count, "count");
  TORCH_CHECK(count.scalar_type() == at::kLong && count.numel() >= 1, "mc_pi: count int64[1]");
  TORCH_CHECK(offset % 2 == 0 && n >= 0, "mc_pi: offset must be even");
  DeviceGuard guard(count.device());
  DALGO_CHECK_HIP(dalgo_mc_pi((uint64_t)seed, (uint64_t)stream, (uint64_t)offset, (uint64_t)n,
                              reinterpret_cast<unsigned long long*>(count.data_ptr<int64_t>()),
                              cur_stream()),
                  "mc_pi");
}


// diagnostics: per-wave K1 timeline (u64, 8 per wave) for the following lr_grad launches

void lr_set_trace(const c10::optional<Tensor>& buf) {
  if (buf.has_value()) {
    check_dev(*buf, "trace");
    TORCH_CHECK(buf->scalar_type() == at::kLong && buf->is_contiguous(), "trace must be contiguous int64");
    dalgo_lr_set_trace(buf->data_ptr());
  } else {
    dalgo_lr_set_trace(nullptr);
  }
}


// ---------------------------------------------------------------------------
// k-means
void check_i32(const Tensor& t, const char* what);
inline int kmeans_dp(int64_t d) {
  for (int dp : {16, 32, 64, 128})
    if (d <= dp) return dp;
  return -1;
}

void check_points(const Tensor& X, int DP) {
  check_dev(X, "X");
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "X must be 2-D with contiguous rows");
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 || X.scalar_type() == at::kFloat, "X bf16/f32");
  TORCH_CHECK(X.stride(0) >= DP, "X row stride must cover the padded dim ", DP);
  TORCH_CHECK((X.stride(0) * X.element_size()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0,
              "X rows must be 16-B aligned");
}

void kmeans_assign(const Tensor& X, const Tensor& Cq, const Tensor& hn, Tensor assign,
                   const std::optional<Tensor>& mind, const std::optional<Tensor>& sse) {
  TORCH_CHECK(Cq.dim() == 2, "Cq [kpad, DP]");
  const int DP = (int)Cq.size(1);
  TORCH_CHECK(kmeans_dp(DP) == DP, "Cq columns must be 16/32/64/128");
  check_points(X, DP);
  check_dev(Cq, "Cq");
  TORCH_CHECK(Cq.scalar_type() == X.scalar_type() && Cq.is_contiguous(), "Cq dtype/layout");
  const int64_t kpad = Cq.size(0);
  TORCH_CHECK(kpad % 32 == 0 && kpad > 0, "kpad % 32");
  check_f32(hn, "hn");
  TORCH_CHECK(hn.numel() >= kpad, "hn");
  check_dev(assign, "assign");
  TORCH_CHECK(assign.scalar_type() == at::kInt && assign.numel() >= X.size(0), "assign int32[n]");
  float* md = nullptr;
  if (mind.has_value()) {
    check_f32(*mind, "mind");
    TORCH_CHECK(mind->numel() >= X.size(0), "mind");
    md = mind->data_ptr<float>();
  }
  double* ss = nullptr;
  int sse_mask = 0;   // blocks add their SSE to slot (block & mask): a power-of-two
                      // prefix of `sse` (one slot = every block on one address)
  if (sse.has_value()) {
    check_dev(*sse, "sse");
    TORCH_CHECK(sse->scalar_type() == at::kDouble && sse->numel() >= 1 && sse->is_contiguous(),
                "sse f64[>=1]");
    ss = sse->data_ptr<double>();
    while (sse_mask < 1023 && 2 * (sse_mask + 1) <= sse->numel()) sse_mask = 2 * sse_mask + 1;
  }
  DeviceGuard guard(X.device());
  DALGO_CHECK_HIP(dalgo_kmeans_assign(X.data_ptr(), X.scalar_type() == at::kBFloat16, X.size(0),
                                      X.stride(0), DP, Cq.data_ptr(), hn.data_ptr<float>(),
                                      (int)kpad, assign.data_ptr<int>(), md, ss, sse_mask, cur_stream()),
                  "kmeans_assign");
}

void kmeans_accumulate_sorted(const Tensor& X, const Tensor& assign, int64_t k, int64_t DP,
                              int64_t seg, Tensor block_counts, Tensor cluster_start,
                              Tensor seg_start, Tensor perm, Tensor S, Tensor cnt) {
  TORCH_CHECK(kmeans_dp(DP) == DP, "DP must be 16/32/64/128");
  check_points(X, (int)DP);
  const int64_t n = X.size(0);
  TORCH_CHECK(n < 0x7fffffffLL, "kmeans_accumulate_sorted: n must fit int32 (shard larger inputs)");
  TORCH_CHECK(assign.scalar_type() == at::kInt && assign.numel() >= n, "assign");
  check_i32(block_counts, "block_counts");
  TORCH_CHECK(block_counts.numel() % k == 0 && block_counts.numel() >= k, "block_counts [B*k]");
  const int64_t B = block_counts.numel() / k;
  TORCH_CHECK(cluster_start.scalar_type() == at::kLong && cluster_start.numel() >= k + 1, "cluster_start");
  TORCH_CHECK(seg_start.scalar_type() == at::kLong && seg_start.numel() >= k + 1, "seg_start");
  check_i32(perm, "perm");
  TORCH_CHECK(perm.numel() >= n, "perm");
  check_f32(S, "S");
  TORCH_CHECK(S.numel() >= k * DP, "S");
  TORCH_CHECK(cnt.scalar_type() == at::kLong && cnt.numel() >= k, "cnt");
  DeviceGuard guard(X.device());
  DALGO_CHECK_HIP(dalgo_kmeans_accumulate_sorted(
                      X.data_ptr(), X.scalar_type() == at::kBFloat16, n, X.stride(0), (int)DP,
                      assign.data_ptr<int>(), (int)k, (int)B, (int)seg, block_counts.data_ptr<int>(),
                      cluster_start.data_ptr<int64_t>(), seg_start.data_ptr<int64_t>(),
                      perm.data_ptr<int>(), S.data_ptr<float>(),
                      reinterpret_cast<unsigned long long*>(cnt.data_ptr<int64_t>()), cur_stream()),
                  "kmeans_accumulate_sorted");
}

// K3 incremental: changed rows of (a_new vs a_old), then move them between the f64 sums
void kmeans_diff(const Tensor& a_new, const Tensor& a_old, Tensor changed, Tensor n_changed) {
  check_dev(a_new, "a_new");
  check_dev(a_old, "a_old");
  check_dev(changed, "changed");
  check_dev(n_changed, "n_changed");
  TORCH_CHECK(a_new.scalar_type() == at::kInt && a_old.scalar_type() == at::kInt &&
                  changed.scalar_type() == at::kInt && a_new.is_contiguous() &&
                  a_old.is_contiguous() && changed.is_contiguous(), "kmeans_diff: int32 vectors");
  TORCH_CHECK(a_old.numel() == a_new.numel() && a_new.numel() < 0x7fffffffLL, "kmeans_diff: sizes");
  TORCH_CHECK(n_changed.scalar_type() == at::kLong && n_changed.numel() >= 1, "n_changed int64[1]");
  DeviceGuard guard(a_new.device());
  DALGO_CHECK_HIP(dalgo_km_diff(a_new.data_ptr<int32_t>(), a_old.data_ptr<int32_t>(), a_new.numel(),
                                changed.data_ptr<int32_t>(),
                                reinterpret_cast<unsigned long long*>(n_changed.data_ptr<int64_t>()),
                                changed.numel(), cur_stream()),
                  "kmeans_diff");
}

// sort-based incremental K3 (workspace from the caller, see dalgo_kmeans_move_sorted)
void kmeans_move_sorted(const Tensor& X, int64_t DP, const Tensor& changed, int64_t m,
                        const Tensor& a_new, const Tensor& a_old, Tensor S64, Tensor cnt,
                        const std::optional<Tensor>& xh, const std::optional<Tensor>& Q, int64_t seg,
                        Tensor block_counts, Tensor cluster_start, Tensor seg_start, Tensor perm,
                        Tensor ec, Tensor er, const std::optional<Tensor>& m_dev, int64_t chunk,
                        const std::optional<Tensor>& cnew, const std::optional<Tensor>& cold) {
  TORCH_CHECK(kmeans_dp(DP) == DP, "DP must be 16/32/64/128");
  TORCH_CHECK(cnew.has_value() == cold.has_value(), "kmeans_move_sorted: cnew and cold together");
  const int32_t* cnp = nullptr;
  const int32_t* cop = nullptr;
  if (cnew.has_value()) {     // clusters aligned with `changed` (the K2 epilogue's)
    check_i32(*cnew, "cnew");
    check_i32(*cold, "cold");
    TORCH_CHECK(cnew->numel() >= m && cold->numel() >= m, "cnew / cold [m]");
    cnp = cnew->data_ptr<int32_t>();
    cop = cold->data_ptr<int32_t>();
  }
  check_points(X, (int)DP);
  check_dev(changed, "changed");
  TORCH_CHECK(changed.scalar_type() == at::kInt && m >= 0 && m <= changed.numel(), "changed");
  TORCH_CHECK(a_new.scalar_type() == at::kInt && a_old.scalar_type() == at::kInt &&
                  a_new.numel() >= X.size(0) && a_old.numel() >= X.size(0), "assignments");
  check_dev(S64, "S64");
  TORCH_CHECK(S64.scalar_type() == at::kDouble && S64.is_contiguous(), "S64 f64");
  TORCH_CHECK(cnt.scalar_type() == at::kLong && cnt.is_contiguous(), "cnt int64");
  const int64_t k = S64.numel() / DP;
  TORCH_CHECK(S64.numel() % DP == 0 && cnt.numel() >= k, "S64 [k, DP] / cnt [k]");
  TORCH_CHECK(xh.has_value() == Q.has_value(), "kmeans_move_sorted: xh and Q together");
  const float* xp = nullptr;
  double* qp = nullptr;
  if (Q.has_value()) {
    check_f32(*xh, "xh");
    TORCH_CHECK(xh->numel() >= X.size(0), "xh [n]");
    check_dev(*Q, "Q");
    TORCH_CHECK(Q->scalar_type() == at::kDouble && Q->numel() >= k && Q->is_contiguous(), "Q f64 [k]");
    xp = xh->data_ptr<float>();
    qp = Q->data_ptr<double>();
  }
  for (const Tensor* t : {&block_counts, &perm, &ec, &er}) {
    check_dev(*t, "workspace");
    TORCH_CHECK(t->scalar_type() == at::kInt && t->is_contiguous(), "int32 workspace");
  }
  check_dev(cluster_start, "cluster_start");
  check_dev(seg_start, "seg_start");
  TORCH_CHECK(cluster_start.scalar_type() == at::kLong && seg_start.scalar_type() == at::kLong &&
                  cluster_start.numel() >= k + 1 && seg_start.numel() >= k + 1, "starts int64 [k+1]");
  TORCH_CHECK(perm.numel() >= 2 * m && ec.numel() >= 2 * m && er.numel() >= 2 * m, "[2m] workspace");
  const int64_t B = block_counts.numel() / std::max<int64_t>(k, 1);
  TORCH_CHECK(B >= 1 && seg >= 1 && chunk >= 1, "block_counts [B * k], seg >= 1, chunk >= 1");
  const unsigned long long* mdp = nullptr;
  if (m_dev.has_value()) {   // device-resident count (<= m, the workspace capacity)
    check_dev(*m_dev, "m_dev");
    TORCH_CHECK(m_dev->scalar_type() == at::kLong && m_dev->numel() >= 1, "m_dev int64[1]");
    mdp = reinterpret_cast<const unsigned long long*>(m_dev->data_ptr<int64_t>());
    TORCH_CHECK(m <= X.size(0), "m_dev capacity: m <= n");
  }
  DeviceGuard guard(X.device());
  DALGO_CHECK_HIP(dalgo_kmeans_move_sorted(
                      X.data_ptr(), X.scalar_type() == at::kBFloat16, X.stride(0), (int)DP,
                      changed.data_ptr<int32_t>(), m, a_new.data_ptr<int32_t>(), a_old.data_ptr<int32_t>(),
                      (int)k, (int)std::min<int64_t>(B, 1 << 20), (int)seg, ec.data_ptr<int>(), er.data_ptr<int>(),
                      block_counts.data_ptr<int>(), cluster_start.data_ptr<int64_t>(),
                      seg_start.data_ptr<int64_t>(), perm.data_ptr<int>(), S64.data_ptr<double>(),
                      reinterpret_cast<unsigned long long*>(cnt.data_ptr<int64_t>()), xp, qp, mdp, chunk,
                      cnp, cop, cur_stream()),
                  "kmeans_move_sorted");
}

// bound-filtered Lloyd: active rows (u + delta[a] >= s[a]) -> idx, their assignment -> a_prev
// ul [n][2] f32: the Hamerly bounds (u, l) of a row, stored as one 8-byte pair
static void check_ul(const Tensor& ul, int64_t n, const char* what) {
  check_f32(ul, what);
  TORCH_CHECK(ul.dim() == 2 && ul.size(1) == 2 && ul.is_contiguous() && ul.size(0) >= n,
              what, ": ul must be a contiguous [n, 2] float32 tensor");
}

void kmeans_filter(const Tensor& assign, Tensor ul, const Tensor& delta, const Tensor& s,
                   const std::optional<Tensor>& a_prev, Tensor idx, Tensor n_active,
                   const std::optional<Tensor>& acl) {
  const int64_t n = assign.numel();
  check_i32(assign, "assign");
  check_ul(ul, n, "kmeans_filter");
  check_f32(delta, "delta");
  check_f32(s, "s");
  int32_t* app = nullptr;
  if (a_prev.has_value()) {   // the Hamerly-only K2 reads the previous clusters per row
    check_i32(*a_prev, "a_prev");
    TORCH_CHECK(a_prev->numel() >= n, "kmeans_filter: a_prev [n]");
    app = a_prev->data_ptr<int32_t>();
  }
  check_i32(idx, "idx");
  TORCH_CHECK(idx.numel() >= n, "kmeans_filter sizes");
  TORCH_CHECK(delta.numel() == s.numel(), "delta / s [k]");
  TORCH_CHECK(n_active.scalar_type() == at::kLong && n_active.numel() >= 1, "n_active int64[1]");
  int32_t* aclp = nullptr;
  if (acl.has_value()) {
    check_i32(*acl, "acl");
    TORCH_CHECK(acl->numel() >= idx.numel(), "kmeans_filter: acl [cap]");
    aclp = acl->data_ptr<int32_t>();
  }
  DeviceGuard guard(assign.device());
  DALGO_CHECK_HIP(dalgo_km_filter(assign.data_ptr<int32_t>(), ul.data_ptr<float>(),
                                  delta.data_ptr<float>(), s.data_ptr<float>(), (int)delta.numel(), n,
                                  app, idx.data_ptr<int32_t>(),
                                  reinterpret_cast<unsigned long long*>(n_active.data_ptr<int64_t>()),
                                  idx.numel(), aclp, cur_stream()),
                  "kmeans_filter");
}

// bounds after the full first pass (u, l from the K2 distances; tol from the K2 max)
void kmeans_bounds_init(const Tensor& mind, const Tensor& mind2, const Tensor& xmax, int64_t n,
                        Tensor ul, Tensor tol) {
  for (const Tensor* t : std::initializer_list<const Tensor*>{&mind, &mind2}) {
    check_f32(*t, "bounds");
    TORCH_CHECK(t->numel() >= n, "bounds [n]");
  }
  check_ul(ul, n, "kmeans_bounds_init");
  check_f32(tol, "tol");
  check_dev(xmax, "xmax");
  TORCH_CHECK(xmax.scalar_type() == at::kInt && xmax.numel() >= 1, "xmax int32[1]");
  DeviceGuard guard(mind.device());
  DALGO_CHECK_HIP(dalgo_km_bounds_init(mind.data_ptr<float>(), mind2.data_ptr<float>(),
                                       reinterpret_cast<const unsigned*>(xmax.data_ptr<int32_t>()), n,
                                       ul.data_ptr<float>(), tol.data_ptr<float>(),
                                       cur_stream()),
                  "kmeans_bounds_init");
}

// bound-filter geometry of new vs previous (rounded) centres: delta [k], s [k] (f32)
void kmeans_centre_bounds(const Tensor& cnow, const Tensor& cprev, int64_t k, int64_t d,
                          Tensor delta, Tensor s) {
  check_dev(cnow, "cnow");
  check_dev(cprev, "cprev");
  TORCH_CHECK(cnow.dim() == 2 && cprev.dim() == 2 && cnow.is_contiguous() && cprev.is_contiguous() &&
                  cnow.size(1) == cprev.size(1) && cnow.scalar_type() == cprev.scalar_type() &&
                  cnow.size(0) >= k && cprev.size(0) >= k, "centres [>=k, DP], same dtype");
  TORCH_CHECK(cnow.scalar_type() == at::kBFloat16 || cnow.scalar_type() == at::kFloat, "centres bf16/f32");
  TORCH_CHECK(d >= 1 && d <= 128 && d <= cnow.size(1), "d <= 128");
  check_f32(delta, "delta");
  check_f32(s, "s");
  TORCH_CHECK(delta.numel() >= k && s.numel() >= k, "delta / s [k]");
  DeviceGuard guard(cnow.device());
  DALGO_CHECK_HIP(dalgo_km_centre_bounds(cnow.data_ptr(), cprev.data_ptr(),
                                         cnow.scalar_type() == at::kBFloat16, (int)k, (int)d,
                                         (int)cnow.size(1), delta.data_ptr<float>(), s.data_ptr<float>(),
                                         cur_stream()),
                  "kmeans_centre_bounds");
}

void kmeans_qsum(const Tensor& assign, const Tensor& xh, int64_t k, Tensor Q) {
  check_i32(assign, "assign");
  check_f32(xh, "xh");
  check_dev(Q, "Q");
  TORCH_CHECK(Q.scalar_type() == at::kDouble && Q.numel() >= k && Q.is_contiguous(), "Q f64 [k]");
  TORCH_CHECK(xh.numel() >= assign.numel() && k <= 2048, "kmeans_qsum sizes");
  DeviceGuard guard(assign.device());
  DALGO_CHECK_HIP(dalgo_km_qsum(assign.data_ptr<int32_t>(), xh.data_ptr<float>(), assign.numel(),
                                (int)k, Q.data_ptr<double>(), cur_stream()),
                  "kmeans_qsum");
}

// K2 (variant 52) over the rows idx[0, m) only
void kmeans_assign_idx(const Tensor& X, const Tensor& Cq, const Tensor& hn,
                       const std::optional<Tensor>& idx, int64_t m, Tensor assign,
                       at::TensorList cand,
                       const std::optional<Tensor>& mind, const std::optional<Tensor>& mind2,
                       const std::optional<Tensor>& xh, const std::optional<Tensor>& xmax,
                       const std::optional<Tensor>& m_dev, const std::optional<Tensor>& a_prev,
                       const std::optional<Tensor>& tol, const std::optional<Tensor>& ul,
                       const std::optional<Tensor>& changed,
                       const std::optional<Tensor>& n_changed, const std::optional<Tensor>& chg_new,
                       const std::optional<Tensor>& chg_old, int64_t cand_extend,
                       const std::optional<Tensor>& acl) {
  TORCH_CHECK(Cq.dim() == 2 && Cq.is_contiguous() && Cq.scalar_type() == at::kBFloat16, "Cq bf16");
  const int DP = (int)Cq.size(1);
  TORCH_CHECK(DP == 64 || DP == 128, "kmeans_assign_idx: DP 64 or 128");
  check_points(X, DP);
  TORCH_CHECK(X.scalar_type() == at::kBFloat16, "kmeans_assign_idx: bf16 points");
  const int64_t kpad = Cq.size(0);
  TORCH_CHECK(kpad % 128 == 0, "kmeans_assign_idx: kpad % 128");
  check_f32(hn, "hn");
  const int32_t* ip = nullptr;
  if (idx.has_value()) {
    check_i32(*idx, "idx");
    TORCH_CHECK(m >= 0 && m <= idx->numel(), "kmeans_assign_idx: m");
    ip = idx->data_ptr<int32_t>();
  } else {
    TORCH_CHECK(m >= 0 && m <= X.size(0), "kmeans_assign_idx: m <= n");
  }
  check_i32(assign, "assign");
  TORCH_CHECK(assign.numel() >= X.size(0), "assign [n]");
  auto f32n = [&](const std::optional<Tensor>& t, const char* nm) -> float* {
    if (!t.has_value()) return nullptr;
    check_f32(*t, nm);
    TORCH_CHECK(t->numel() >= X.size(0), nm, " [n]");
    return t->data_ptr<float>();
  };
  float* md = f32n(mind, "mind");
  float* m2 = f32n(mind2, "mind2");
  float* xhp = f32n(xh, "xh");
  unsigned* xmp = nullptr;
  if (xmax.has_value()) {
    check_dev(*xmax, "xmax");
    TORCH_CHECK(xmax->scalar_type() == at::kInt && xmax->numel() >= 1, "xmax int32[1] (float bits)");
    xmp = reinterpret_cast<unsigned*>(xmax->data_ptr<int32_t>());
  }
  DalgoKmPost post{};
  const DalgoKmPost* pp = nullptr;
  if (m_dev.has_value()) {   // filtered iteration: rows = *m_dev (device), m = its upper bound
    // previous clusters: a_prev[row], acl[p] (the filter's list order), the candidate
    // form's tiles, or (none given, dense form) assign itself
    TORCH_CHECK(tol.has_value() && ul.has_value() &&
                    changed.has_value() && n_changed.has_value(),
                "kmeans_assign_idx: the device-count form needs a_prev, tol, ul, changed, n_changed");
    check_dev(*m_dev, "m_dev");
    TORCH_CHECK(m_dev->scalar_type() == at::kLong && m_dev->numel() >= 1, "m_dev int64[1]");
    if (a_prev.has_value()) {
      check_i32(*a_prev, "a_prev");
      TORCH_CHECK(a_prev->numel() >= X.size(0), "a_prev [n]");
      post.a_prev = a_prev->data_ptr<int32_t>();
    }
    if (acl.has_value()) {
      check_i32(*acl, "acl");
      TORCH_CHECK(ip != nullptr && acl->numel() >= m, "kmeans_assign_idx: acl [m] with idx");
      post.acl = acl->data_ptr<int32_t>();
    }
    check_i32(*changed, "changed");
    TORCH_CHECK(chg_new.has_value() == chg_old.has_value(), "chg_new and chg_old together");
    if (chg_new.has_value()) {
      check_i32(*chg_new, "chg_new");
      check_i32(*chg_old, "chg_old");
      TORCH_CHECK(chg_new->numel() >= changed->numel() && chg_old->numel() >= changed->numel(),
                  "chg_new / chg_old [cap]");
      post.chg_new = chg_new->data_ptr<int32_t>();
      post.chg_old = chg_old->data_ptr<int32_t>();
    }
    check_f32(*tol, "tol");
    TORCH_CHECK(n_changed->scalar_type() == at::kLong && n_changed->numel() >= 1, "n_changed int64[1]");
    check_dev(*n_changed, "n_changed");
    post.mcount = reinterpret_cast<const unsigned long long*>(m_dev->data_ptr<int64_t>());
    post.tol = tol->data_ptr<float>();
    check_ul(*ul, X.size(0), "kmeans_assign_idx");
    post.ul = ul->data_ptr<float>();
    post.changed = changed->data_ptr<int32_t>();
    post.n_changed = reinterpret_cast<unsigned long long*>(n_changed->data_ptr<int64_t>());
    post.cap = changed->numel();
    pp = &post;
  } else {
    TORCH_CHECK(md != nullptr, "kmeans_assign_idx: mind");
  }
  // candidate-pruned form: [tiles int32 [T, 4], n_tiles, hnb, nb, nd] (+ [ndb, dnb]: drift-aware)
  DalgoKmCand cd{};
  const DalgoKmCand* cp = nullptr;
  if (!cand.empty()) {
    TORCH_CHECK((cand.size() == 5 || cand.size() == 7 || cand.size() == 8) && pp != nullptr && ip != nullptr,
                "kmeans_assign_idx: cand = 5 (7, 8) tensors, with the device-count form and idx");
    for (const Tensor& t : cand) check_dev(t, "cand");
    TORCH_CHECK(cand[0].scalar_type() == at::kInt && cand[1].scalar_type() == at::kLong &&
                    cand[2].scalar_type() == at::kFloat && cand[3].scalar_type() == at::kInt &&
                    cand[4].scalar_type() == at::kFloat,
                "kmeans_assign_idx: cand dtypes");
    const int64_t k = cand[2].numel() / kpad;
    TORCH_CHECK(kpad <= 1024 && k >= 1 && k <= kpad && cand[3].numel() >= k * kpad &&
                    cand[4].numel() >= k * kpad && cand[0].numel() % 4 == 0,
                "kmeans_assign_idx: cand sizes (kpad <= 1024)");
    cd.tiles = cand[0].data_ptr<int32_t>();
    cd.n_tiles = reinterpret_cast<const unsigned long long*>(cand[1].data_ptr<int64_t>());
    cd.hnb = cand[2].data_ptr<float>();
    cd.nb = cand[3].data_ptr<int32_t>();
    cd.nd = cand[4].data_ptr<float>();
    cd.extend = (cand_extend & 1) != 0;
    cd.tile16 = (cand_extend & 2) != 0;   // bit 1: tiles of <= 384 rows, 16x16x32 form
    cd.max_tiles = cand[0].numel() / 4;
    if (cand.size() >= 7) {
      TORCH_CHECK(cand[5].scalar_type() == at::kFloat && cand[6].scalar_type() == at::kFloat &&
                      cand[5].numel() >= k * kpad && cand[6].numel() >= k * kpad,
                  "kmeans_assign_idx: ndb / dnb f32 [k * kpad]");
      cd.ndb = cand[5].data_ptr<float>();
      cd.dnb = cand[6].data_ptr<float>();
    }
    if (cand.size() == 8) {
      TORCH_CHECK(cand[7].scalar_type() == at::kFloat && cand[7].numel() >= 1, "kmeans_assign_idx: tau_cap f32[1]");
      cd.tau_cap = cand[7].data_ptr<float>();
    }
    cp = &cd;
  }
  DeviceGuard guard(X.device());
  DALGO_CHECK_HIP(dalgo_kmeans_assign_idx(X.data_ptr(), m, X.stride(0), DP, Cq.data_ptr(),
                                          hn.data_ptr<float>(), (int)kpad, ip,
                                          assign.data_ptr<int>(), md, m2, nullptr, 0, xhp, xmp, pp,
                                          cp, cur_stream()),
                  "kmeans_assign_idx");
}

// candidate-pruned K2 preparation: active rows sorted by cluster + tile table
void kmeans_sort_active(const Tensor& acl, const Tensor& idx, const Tensor& n_active, int64_t k,
                        int64_t chunk, Tensor block_counts, Tensor cstart, Tensor seg_start,
                        Tensor rows_sorted, int64_t tile, Tensor tiles, Tensor n_tiles) {
  check_i32(acl, "acl");
  check_i32(idx, "idx");
  check_i32(rows_sorted, "rows_sorted");
  check_i32(block_counts, "block_counts");
  check_i32(tiles, "tiles");
  for (const Tensor* t : std::initializer_list<const Tensor*>{&n_active, &cstart, &seg_start, &n_tiles}) {
    check_dev(*t, "sort_active");
    TORCH_CHECK(t->scalar_type() == at::kLong && t->is_contiguous(), "sort_active: int64 tensors");
  }
  const int64_t cap = idx.numel();
  TORCH_CHECK(acl.numel() >= cap && rows_sorted.numel() >= cap && k >= 1 && k <= 2048 &&
                  cstart.numel() >= k + 1 && seg_start.numel() >= k + 1 && tile >= 1 && chunk >= 1,
              "kmeans_sort_active sizes");
  const int64_t B = std::max<int64_t>(1, std::min<int64_t>((cap + chunk - 1) / chunk,
                                                           block_counts.numel() / k));
  TORCH_CHECK(B * chunk >= cap, "kmeans_sort_active: block_counts too small for cap / chunk");
  TORCH_CHECK(tiles.numel() % 4 == 0 && tiles.numel() / 4 >= (cap + tile - 1) / tile + k,
              "kmeans_sort_active: tile table [cap / tile + k, 4]");
  DeviceGuard guard(idx.device());
  DALGO_CHECK_HIP(dalgo_kmeans_sort_active(
                      acl.data_ptr<int32_t>(), idx.data_ptr<int32_t>(), cap,
                      reinterpret_cast<const unsigned long long*>(n_active.data_ptr<int64_t>()), (int)k,
                      (int)B, chunk, block_counts.data_ptr<int>(), cstart.data_ptr<int64_t>(),
                      seg_start.data_ptr<int64_t>(), rows_sorted.data_ptr<int32_t>(), (int)tile,
                      tiles.data_ptr<int32_t>(),
                      reinterpret_cast<unsigned long long*>(n_tiles.data_ptr<int64_t>()),
                      tiles.numel() / 4, cur_stream()),
                  "kmeans_sort_active");
}

// centre geometry of the candidate-pruned iteration: delta, s and the neighbour lists
void kmeans_centre_nbrs(const Tensor& cq, const Tensor& cprev, const Tensor& hn, int64_t k,
                        int64_t d, Tensor delta, Tensor s, Tensor nd, Tensor nb, Tensor hnb,
                        const std::optional<Tensor>& ndb, const std::optional<Tensor>& dnb) {
  check_dev(cq, "cq");
  check_dev(cprev, "cprev");
  TORCH_CHECK(cq.dim() == 2 && cq.is_contiguous() && cq.scalar_type() == at::kBFloat16 &&
                  cprev.is_contiguous() && cprev.scalar_type() == at::kBFloat16 &&
                  cprev.size(1) == cq.size(1) && cprev.size(0) >= k,
              "kmeans_centre_nbrs: bf16 centres [kpad, DP]");
  const int64_t kpad = cq.size(0), DP = cq.size(1);
  TORCH_CHECK(k >= 1 && k <= kpad && kpad <= 2048 && d >= 1 && d <= 128 && d <= DP, "kmeans_centre_nbrs: k, d");
  check_f32(hn, "hn");
  check_f32(delta, "delta");
  check_f32(s, "s");
  check_f32(nd, "nd");
  check_f32(hnb, "hnb");
  check_i32(nb, "nb");
  TORCH_CHECK(hn.numel() >= kpad && delta.numel() >= k && s.numel() >= k && nd.numel() >= k * kpad &&
                  nb.numel() >= k * kpad && hnb.numel() >= k * kpad,
              "kmeans_centre_nbrs sizes");
  TORCH_CHECK(ndb.has_value() == dnb.has_value(), "kmeans_centre_nbrs: ndb and dnb together");
  float* ndbp = nullptr;
  float* dnbp = nullptr;
  if (ndb.has_value()) {
    check_f32(*ndb, "ndb");
    check_f32(*dnb, "dnb");
    TORCH_CHECK(ndb->numel() >= k * kpad && dnb->numel() >= k * kpad, "ndb / dnb [k * kpad]");
    ndbp = ndb->data_ptr<float>();
    dnbp = dnb->data_ptr<float>();
  }
  DeviceGuard guard(cq.device());
  DALGO_CHECK_HIP(dalgo_km_centre_nbrs(cq.data_ptr(), cprev.data_ptr(), hn.data_ptr<float>(), (int)k,
                                       (int)kpad, (int)d, (int)DP, delta.data_ptr<float>(),
                                       s.data_ptr<float>(), nd.data_ptr<float>(), nb.data_ptr<int32_t>(),
                                       hnb.data_ptr<float>(), ndbp, dnbp, cur_stream()),
                  "kmeans_centre_nbrs");
}

void kmeans_update(Tensor C, const Tensor& S, const Tensor& cnt, Tensor Cq, Tensor hn,
                   const std::optional<Tensor>& shift2) {
  check_f32(C, "C");
  TORCH_CHECK(C.dim() == 2, "C [k, d]");
  const int64_t k = C.size(0), d = C.size(1);
  check_dev(Cq, "Cq");
  TORCH_CHECK(Cq.dim() == 2 && Cq.is_contiguous() && Cq.size(0) >= k && Cq.size(0) % 32 == 0 &&
                  Cq.size(1) >= d, "Cq [kpad, DP]");
  TORCH_CHECK(Cq.scalar_type() == at::kBFloat16 || Cq.scalar_type() == at::kFloat, "Cq dtype");
  const int64_t DP = Cq.size(1), kpad = Cq.size(0);
  check_f32(S, "S");
  TORCH_CHECK(S.numel() >= k * DP, "S");
  TORCH_CHECK(cnt.scalar_type() == at::kLong && cnt.numel() >= k, "cnt");
  check_f32(hn, "hn");
  TORCH_CHECK(hn.numel() >= kpad, "hn");
  float* sh = nullptr;
  if (shift2.has_value()) { check_f32(*shift2, "shift2"); sh = shift2->data_ptr<float>(); }
  DeviceGuard guard(C.device());
  DALGO_CHECK_HIP(dalgo_kmeans_update(C.data_ptr<float>(), S.data_ptr<float>(),
                                      reinterpret_cast<const unsigned long long*>(cnt.data_ptr<int64_t>()),
                                      (int)k, (int)d, (int)DP, Cq.data_ptr(),
                                      Cq.scalar_type() == at::kBFloat16, hn.data_ptr<float>(),
                                      (int)kpad, sh, cur_stream()),
                  "kmeans_update");
}

// ---------------------------------------------------------------------------
// PageRank
void check_i32(const Tensor& t, const char* what) {
  check_dev(t, what);
  TORCH_CHECK(t.scalar_type() == at::kInt && t.is_contiguous(), "dalgo: ", what, " must be int32");
}

void rmat_edges(int64_t seed, int64_t scale, int64_t e_off, double a, double b, double c,
                bool scramble, Tensor src, Tensor dst) {
  check_i32(src, "src");
  check_i32(dst, "dst");
  TORCH_CHECK(src.numel() == dst.numel(), "src/dst size");
  TORCH_CHECK(scale >= 1 && scale <= 31, "scale in [1, 31]");
  DeviceGuard guard(src.device());
  DALGO_CHECK_HIP(dalgo_rmat((uint64_t)seed, (int)scale, e_off, src.numel(), (float)a, (float)b,
                             (float)c, scramble ? 1 : 0, src.data_ptr<int32_t>(),
                             dst.data_ptr<int32_t>(), cur_stream()),
                  "rmat_edges");
}

// ---- native PageRank adjacency build (graph_build.hip)
inline void check_t(const Tensor& t, at::ScalarType st, const char* what) {
  check_dev(t, what);
  TORCH_CHECK(t.scalar_type() == st && t.is_contiguous(), "dalgo: ", what, " has the wrong dtype / layout");
}
template <typename T>
inline T* opt_ptr(const std::optional<Tensor>& t) {
  return t.has_value() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

void gb_degree(const Tensor& ids, Tensor deg) {
  check_i32(ids, "ids");
  check_i32(deg, "deg");
  DeviceGuard guard(ids.device());
  DALGO_CHECK_HIP(dalgo_gb_degree(ids.data_ptr<int32_t>(), ids.numel(),
                                  reinterpret_cast<uint32_t*>(deg.data_ptr<int32_t>()), cur_stream()),
                  "gb_degree");
}

// phase 0: counts[block] = kept edges, remote sources marked in bitmap; phase 1: keys
void gb_keys(const Tensor& src, const Tensor& dst, const std::optional<Tensor>& new_id, int64_t v_lo,
             int64_t v_hi, int64_t sl, int64_t world, int64_t rank, int64_t dbits, int64_t phase,
             const std::optional<Tensor>& bitmap, const std::optional<Tensor>& counts,
             const std::optional<Tensor>& offsets, int64_t base_all, const std::optional<Tensor>& keys,
             const std::optional<Tensor>& word_prefix, const std::optional<Tensor>& seg_start,
             const std::optional<Tensor>& seg_blk0) {
  check_i32(src, "src");
  check_i32(dst, "dst");
  TORCH_CHECK(src.numel() == dst.numel(), "gb_keys: src / dst size");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0, "gb_keys: src / dst 16-B aligned");
  const int64_t n = src.numel();
  const int64_t nb = dalgo_gb_key_blocks(n);
  if (new_id) check_i32(*new_id, "new_id");
  if (world > 1) {
    // phase 0: a byte map (uint8, one byte per vertex id) of the remote sources; phase 1:
    // the bitmap packed from it (gb_bytes_to_bits)
    TORCH_CHECK(bitmap.has_value(), "gb_keys: bitmap needed at world > 1");
    if (phase == 0) {
      check_t(*bitmap, at::kByte, "marks");
      TORCH_CHECK(bitmap->numel() >= sl * world, "gb_keys: marks [>= n_vertices] bytes");
    } else {
      check_i32(*bitmap, "bitmap");
    }
  }
  if (phase == 0) {
    TORCH_CHECK(counts.has_value() && counts->numel() >= nb, "gb_keys: counts [blocks]");
    check_i32(*counts, "counts");
  } else {
    TORCH_CHECK(keys.has_value(), "gb_keys: keys");
    check_t(*keys, at::kLong, "keys");
    if (offsets) {
      check_t(*offsets, at::kLong, "offsets");
      TORCH_CHECK(offsets->numel() >= nb, "gb_keys: offsets [blocks]");
    } else {
      TORCH_CHECK(base_all >= 0 && base_all + n <= keys->numel(), "gb_keys: keys too short");
    }
    if (world > 1) {
      TORCH_CHECK(word_prefix && seg_start && seg_blk0, "gb_keys: ghost tables needed at world > 1");
      check_t(*word_prefix, at::kLong, "word_prefix");
      check_t(*seg_start, at::kLong, "seg_start");
      check_t(*seg_blk0, at::kLong, "seg_blk0");
      TORCH_CHECK(seg_start->numel() >= world && seg_blk0->numel() >= world, "gb_keys: segment tables");
    }
  }
  DalgoGbKeyArgs a{v_lo, v_hi, sl, (int)world, (int)rank, (int)dbits, opt_ptr<const int32_t>(new_id),
                   opt_ptr<const uint32_t>(bitmap), opt_ptr<const int64_t>(word_prefix),
                   opt_ptr<const int64_t>(seg_start), opt_ptr<const int64_t>(seg_blk0)};
  DeviceGuard guard(src.device());
  DALGO_CHECK_HIP(dalgo_gb_keys(src.data_ptr<int32_t>(), dst.data_ptr<int32_t>(), n, &a, (int)phase,
                                opt_ptr<uint32_t>(bitmap), opt_ptr<int32_t>(counts),
                                opt_ptr<const int64_t>(offsets), base_all, opt_ptr<uint64_t>(keys), nullptr,
                                cur_stream()),
                  "gb_keys");
}

// one rank: keys of the packed (src << 32 | dst) edges (every destination is kept)
void gb_keys_packed(const Tensor& packed, const std::optional<Tensor>& new_id, int64_t n_vertices, int64_t dbits,
                    Tensor keys, int64_t src_new) {
  check_t(packed, at::kLong, "packed");
  check_t(keys, at::kLong, "keys");
  const int64_t n = packed.numel();
  TORCH_CHECK(keys.numel() >= n, "gb_keys_packed: keys too short");
  if (new_id) {
    check_i32(*new_id, "new_id");
    TORCH_CHECK(new_id->numel() >= n_vertices, "gb_keys_packed: new_id [n_vertices]");
  }
  DalgoGbKeyArgs a{0, n_vertices, n_vertices, 1, 0, (int)dbits, opt_ptr<const int32_t>(new_id), nullptr, nullptr,
                   nullptr, nullptr, (int)(src_new != 0)};
  DeviceGuard guard(packed.device());
  DALGO_CHECK_HIP(dalgo_gb_keys(nullptr, nullptr, n, &a, 1, nullptr, nullptr, nullptr, 0, reinterpret_cast<uint64_t*>(keys.data_ptr<int64_t>()),
                                reinterpret_cast<const uint64_t*>(packed.data_ptr<int64_t>()), cur_stream()),
                  "gb_keys_packed");
}

// packed (src << 32 | dst) words: src := new_id[src], in place
// partitioned: packed is sorted on src >> 13 (gb_degree_packed's output), every src <
// new_id.numel(): one block per 8192-source bucket with its id slice in LDS
void gb_relabel_src(Tensor packed, const Tensor& new_id, int64_t partitioned) {
  check_t(packed, at::kLong, "packed");
  check_i32(new_id, "new_id");
  DeviceGuard guard(packed.device());
  const int64_t nb = (new_id.numel() + ((int64_t)1 << dalgo_gb_bucket_bits()) - 1) >> dalgo_gb_bucket_bits();
  Tensor starts = at::empty({partitioned ? nb + 1 : 1}, packed.options());
  DALGO_CHECK_HIP(dalgo_gb_relabel_src(reinterpret_cast<uint64_t*>(packed.data_ptr<int64_t>()), packed.numel(),
                                       new_id.data_ptr<int32_t>(), new_id.numel(), (int)partitioned,
                                       starts.data_ptr<int64_t>(), cur_stream()),
                  "gb_relabel_src");
}

// sharded build shuffle: the edges relabelled through new_id (optional) and grouped by the
// owner rank of their destination (dst' / sl) into out (packed src << 32 | dst); returns
// the per-owner counts [world] (int64, device)
Tensor gb_owner_partition(const Tensor& src, const Tensor& dst, const std::optional<Tensor>& new_id, int64_t sl,
                          int64_t world, Tensor out) {
  check_i32(src, "src");
  check_i32(dst, "dst");
  check_t(out, at::kLong, "out");
  const int64_t n = src.numel();
  TORCH_CHECK(dst.numel() == n && out.numel() >= n, "gb_owner_partition: sizes");
  TORCH_CHECK(world >= 1 && world <= 64 && sl >= 1, "gb_owner_partition: 1..64 ranks");
  TORCH_CHECK(src.is_contiguous() && dst.is_contiguous() && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
              "gb_owner_partition: src / dst must be contiguous and 16-B aligned (int4 loads)");
  if (new_id) check_i32(*new_id, "new_id");
  DeviceGuard guard(src.device());
  const int64_t nb = std::max<int64_t>(dalgo_gb_owner_blocks(n), 1);
  Tensor counts = at::zeros({world, nb}, src.options().dtype(at::kLong));
  if (n == 0) return counts.sum(1);
  Tensor tmp = at::empty({n}, src.options().dtype(at::kLong));
  auto* tp = reinterpret_cast<uint64_t*>(tmp.data_ptr<int64_t>());
  DALGO_CHECK_HIP(dalgo_gb_owner_scatter(0, src.data_ptr<int32_t>(), dst.data_ptr<int32_t>(), n,
                                         opt_ptr<const int32_t>(new_id), sl, (int)world, tp,
                                         counts.data_ptr<int64_t>(), nullptr, nullptr, cur_stream()),
                  "gb_owner_scatter(count)");
  Tensor flat = counts.view({-1});
  Tensor offs = flat.cumsum(0) - flat;
  DALGO_CHECK_HIP(dalgo_gb_owner_scatter(2, nullptr, nullptr, n, nullptr, sl, (int)world, tp, nullptr,
                                         offs.data_ptr<int64_t>(),
                                         reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>()), cur_stream()),
                  "gb_owner_scatter(scatter)");
  return counts.sum(1);
}

// the same over edges already packed (src << 32 | dst) with RELABELLED sources, partitioned
// on their destination bits (dalgo.ops.graph.relabel_partition_dst): the destinations are
// relabelled in place in `packed` (new_id optional), then the owner-major scatter into out
Tensor gb_owner_partition_packed(Tensor packed, const std::optional<Tensor>& new_id, int64_t sl, int64_t world,
                                 Tensor out) {
  check_t(packed, at::kLong, "packed");
  check_t(out, at::kLong, "out");
  const int64_t n = packed.numel();
  TORCH_CHECK(out.numel() >= n && packed.is_contiguous() && reinterpret_cast<uintptr_t>(packed.data_ptr()) % 16 == 0,
              "gb_owner_partition_packed: packed must be contiguous and 16-B aligned");
  TORCH_CHECK(world >= 1 && world <= 64 && sl >= 1, "gb_owner_partition_packed: 1..64 ranks");
  if (new_id) check_i32(*new_id, "new_id");
  DeviceGuard guard(packed.device());
  const int64_t nb = std::max<int64_t>(dalgo_gb_owner_blocks(n), 1);
  Tensor counts = at::zeros({world, nb}, packed.options());
  if (n == 0) return counts.sum(1);
  auto* tp = reinterpret_cast<uint64_t*>(packed.data_ptr<int64_t>());
  DALGO_CHECK_HIP(dalgo_gb_owner_scatter(0, nullptr, nullptr, n, opt_ptr<const int32_t>(new_id), sl, (int)world, tp,
                                         counts.data_ptr<int64_t>(), nullptr, nullptr, cur_stream()),
                  "gb_owner_scatter(count, packed)");
  Tensor flat = counts.view({-1});
  Tensor offs = flat.cumsum(0) - flat;
  DALGO_CHECK_HIP(dalgo_gb_owner_scatter(2, nullptr, nullptr, n, nullptr, sl, (int)world, tp, nullptr,
                                         offs.data_ptr<int64_t>(),
                                         reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>()), cur_stream()),
                  "gb_owner_scatter(scatter, packed)");
  return counts.sum(1);
}

// bits[w] = bit j set iff marks[32 w + j] != 0
void gb_bytes_to_bits(const Tensor& marks, Tensor bits) {
  check_t(marks, at::kByte, "marks");
  check_i32(bits, "bits");
  TORCH_CHECK(marks.numel() >= 32 * bits.numel(), "gb_bytes_to_bits: 32 bytes per word");
  DeviceGuard guard(marks.device());
  DALGO_CHECK_HIP(dalgo_gb_bytes_to_bits(marks.data_ptr<uint8_t>(), bits.numel(),
                                         reinterpret_cast<uint32_t*>(bits.data_ptr<int32_t>()), cur_stream()),
                  "gb_bytes_to_bits");
}

// ids of the set bits of a u32 bitmap, ascending, at the words' exclusive popcount prefix
void gb_bitmap_ids(const Tensor& bitmap, const Tensor& prefix, Tensor ids) {
  check_i32(bitmap, "bitmap");
  check_t(prefix, at::kLong, "prefix");
  check_t(ids, at::kLong, "ids");
  TORCH_CHECK(prefix.numel() >= bitmap.numel(), "gb_bitmap_ids: prefix per word");
  DeviceGuard guard(bitmap.device());
  DALGO_CHECK_HIP(dalgo_gb_bitmap_ids(reinterpret_cast<const uint32_t*>(bitmap.data_ptr<int32_t>()), bitmap.numel(),
                                      prefix.data_ptr<int64_t>(), ids.data_ptr<int64_t>(), cur_stream()),
                  "gb_bitmap_ids");
}

// new_id[order[j]] = snake-dealt position of rank j over `world` full slices of size sl
// id_bits > 0: order holds sort keys whose low id_bits bits are the vertex (gb_rank_keys)
void gb_deal(const Tensor& order, int64_t world, int64_t sl, int64_t id_bits, Tensor new_id) {
  check_t(order, at::kLong, "order");
  check_i32(new_id, "new_id");
  TORCH_CHECK(new_id.numel() >= order.numel() && sl * world >= order.numel(), "gb_deal: sizes");
  TORCH_CHECK(id_bits == 0 || (order.numel() - 1) >> id_bits == 0, "gb_deal: ids must fit id_bits");
  DeviceGuard guard(order.device());
  DALGO_CHECK_HIP(dalgo_gb_deal(order.data_ptr<int64_t>(), order.numel(), (int)world, sl, (int)id_bits,
                                new_id.data_ptr<int32_t>(), cur_stream()),
                  "gb_deal");
}

// keys[j] = (dmax - deg[n-1-j]) << ibits | (n-1-j): the degree ranking's sort keys
void gb_rank_keys(const Tensor& deg, int64_t dmax, int64_t ibits, Tensor keys) {
  check_i32(deg, "deg");
  check_t(keys, at::kLong, "keys");
  const int64_t n = deg.numel();
  TORCH_CHECK(keys.numel() >= n && ibits >= 1 && ibits <= 40 && ((n - 1) >> ibits) == 0 && dmax >= 0 &&
                  ibits + (int64_t)(64 - __builtin_clzll((unsigned long long)dmax | 1ull)) <= 63,
              "gb_rank_keys: sizes");
  DeviceGuard guard(deg.device());
  DALGO_CHECK_HIP(dalgo_gb_rank_keys(deg.data_ptr<int32_t>(), n, dmax, (int)ibits,
                                     reinterpret_cast<uint64_t*>(keys.data_ptr<int64_t>()), cur_stream()),
                  "gb_rank_keys");
}

// packed[i] = src[i] << 32 | dst[i]
void gb_pack(const Tensor& src, const Tensor& dst, Tensor out) {
  check_i32(src, "src");
  check_i32(dst, "dst");
  check_t(out, at::kLong, "out");
  TORCH_CHECK(src.numel() == dst.numel() && out.numel() >= src.numel(), "gb_pack: sizes");
  DeviceGuard guard(src.device());
  DALGO_CHECK_HIP(dalgo_gb_pack(src.data_ptr<int32_t>(), dst.data_ptr<int32_t>(), src.numel(),
                                reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>()), cur_stream()),
                  "gb_pack");
}

// ---- the adjacency build's sorts: rocPRIM's onesweep radix sort by default, the native
// reduce-then-scan LSD sort (radix_sort.hip) with DALGO_SORT=native. Measured on one MI355X
// (bench/probes/sort_bench.py, profiles/round6/r6_16): 1.07B u64 keys over 40 bits, native
// 51.2 ms (count passes 1.6 ms each at 5.4 TB/s, scatter passes 7.4 ms: 128-B digit runs
// written at scattered places) against rocPRIM 33.3 ms -- rocPRIM stays the default.
// rs_sort_error() keeps the (always clear: nothing in the native sort waits) error word.
static bool use_rocprim_sort() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("DALGO_SORT");
    v = (e != nullptr && std::string(e) == "native") ? 0 : 1;
  }
  return v == 1;
}
static Tensor rs_err_word(const at::Device& dev) {
  static std::map<int, Tensor> words;
  auto it = words.find(dev.index());
  if (it != words.end()) return it->second;
  Tensor t = at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(dev));
  words[dev.index()] = t;
  return t;
}
static void native_sort(const void* in, void* out, int key_bytes, int64_t n, int begin_bit, int end_bit,
                        const at::TensorOptions& opts, const char* what) {
  const size_t wsb = dalgo_rs_ws_bytes(n, key_bytes, begin_bit, end_bit);
  Tensor ws = at::empty({(int64_t)wsb}, opts.dtype(at::kByte));
  const int np = (end_bit - begin_bit + 7) / 8;
  Tensor tmp = np > 1 ? at::empty({n * key_bytes}, opts.dtype(at::kByte)) : Tensor();
  Tensor errw = at::empty({1}, opts.dtype(at::kInt));
  hipError_t e = key_bytes == 8
      ? dalgo_rs_sort64(reinterpret_cast<const uint64_t*>(in), reinterpret_cast<uint64_t*>(out),
                        np > 1 ? reinterpret_cast<uint64_t*>(tmp.data_ptr()) : nullptr, n, begin_bit, end_bit,
                        ws.data_ptr(), wsb, reinterpret_cast<unsigned*>(errw.data_ptr<int>()), cur_stream())
      : dalgo_rs_sort32(reinterpret_cast<const uint32_t*>(in), reinterpret_cast<uint32_t*>(out),
                        np > 1 ? reinterpret_cast<uint32_t*>(tmp.data_ptr()) : nullptr, n, begin_bit, end_bit,
                        ws.data_ptr(), wsb, reinterpret_cast<unsigned*>(errw.data_ptr<int>()), cur_stream());
  TORCH_CHECK(e == hipSuccess, "dalgo::", what, " launch failed: ", hipGetErrorString(e));
  Tensor acc = rs_err_word(opts.device());
  acc.bitwise_or_(errw);
}

Tensor rs_sort_error(const Tensor& like) { return rs_err_word(like.device()); }

// packed edges partitioned on the HIGH bits of their source (bits [kb, end_bit) of src,
// 2 radix passes at 2^26) into out, and deg[src] += the raw out-degree (one LDS histogram
// per bucket of 2^kb sources)
void gb_degree_packed(const Tensor& packed, int64_t end_bit, Tensor deg, Tensor out) {
  check_t(packed, at::kLong, "packed");
  check_t(out, at::kLong, "out");
  check_i32(deg, "deg");
  const int64_t n = packed.numel();
  const int kb = dalgo_gb_bucket_bits();
  TORCH_CHECK(end_bit > kb && end_bit <= 31 && deg.numel() >= ((int64_t)1 << end_bit) && out.numel() >= n,
              "gb_degree_packed: sizes");
  if (n == 0) return;
  DeviceGuard guard(packed.device());
  auto* in = reinterpret_cast<const uint64_t*>(packed.data_ptr<int64_t>());
  auto* o = reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>());
  if (!use_rocprim_sort()) {
    native_sort(in, o, 8, n, 32 + kb, 32 + (int)end_bit, packed.options(), "rs_sort64(degree partition)");
  } else {
    size_t bytes = 0;
    DALGO_CHECK_HIP(dalgo_gb_sort(nullptr, &bytes, in, o, n, 32 + kb, 32 + (int)end_bit, cur_stream()),
                    "gb_sort(size)");
    Tensor tmp = at::empty({(int64_t)bytes + 256}, packed.options().dtype(at::kByte));
    DALGO_CHECK_HIP(dalgo_gb_sort(tmp.data_ptr(), &bytes, in, o, n, 32 + kb, 32 + (int)end_bit, cur_stream()),
                    "gb_sort");
  }
  Tensor starts = at::empty({((int64_t)1 << (end_bit - kb)) + 1}, packed.options());
  DALGO_CHECK_HIP(dalgo_gb_bucket_degree(o, 1, n, (int)end_bit, starts.data_ptr<int64_t>(), deg.data_ptr<int32_t>(),
                                         cur_stream()),
                  "gb_bucket_degree");
}

// deg[v] = occurrences of v in ids (int32, ids < 2^end_bit): one rocPRIM radix sort of the
// ids over end_bit bits + one pass over the run boundaries (no per-id atomics)
void gb_degree_sorted(const Tensor& ids, int64_t end_bit, Tensor deg) {
  check_i32(ids, "ids");
  check_i32(deg, "deg");
  const int64_t n = ids.numel();
  TORCH_CHECK(end_bit >= 1 && end_bit <= 31 && deg.numel() >= ((int64_t)1 << end_bit),
              "gb_degree_sorted: deg must cover 2^end_bit ids");
  if (n == 0) return;
  DeviceGuard guard(ids.device());
  auto* in = reinterpret_cast<const uint32_t*>(ids.data_ptr<int32_t>());
  const int kb = dalgo_gb_bucket_bits();
  if (end_bit <= kb + 2) {   // small id space: one atomic per id
    DALGO_CHECK_HIP(dalgo_gb_degree(ids.data_ptr<int32_t>(), n,
                                    reinterpret_cast<uint32_t*>(deg.data_ptr<int32_t>()), cur_stream()),
                    "gb_degree");
    return;
  }
  // partition on the high bits only, then one LDS histogram per bucket
  Tensor sorted = at::empty_like(ids);
  auto* out = reinterpret_cast<uint32_t*>(sorted.data_ptr<int32_t>());
  if (!use_rocprim_sort()) {
    native_sort(in, out, 4, n, kb, (int)end_bit, ids.options(), "rs_sort32(degree partition)");
  } else {
    size_t bytes = 0;
    DALGO_CHECK_HIP(dalgo_gb_sort32(nullptr, &bytes, in, out, n, kb, (int)end_bit, cur_stream()), "gb_sort32(size)");
    Tensor tmp = at::empty({(int64_t)bytes + 256}, ids.options().dtype(at::kByte));
    DALGO_CHECK_HIP(dalgo_gb_sort32(tmp.data_ptr(), &bytes, in, out, n, kb, (int)end_bit, cur_stream()), "gb_sort32");
  }
  Tensor starts = at::empty({((int64_t)1 << (end_bit - kb)) + 1}, ids.options().dtype(at::kLong));
  DALGO_CHECK_HIP(dalgo_gb_bucket_degree(out, 0, n, (int)end_bit, starts.data_ptr<int64_t>(), deg.data_ptr<int32_t>(),
                                         cur_stream()),
                  "gb_bucket_degree");
}

// sort keys[:n] over bits [begin_bit, end_bit) into out[:n] (native LSD radix sort, stable:
// keys equal on those bits keep their input order)
void gb_sort(const Tensor& keys, int64_t n, int64_t end_bit, Tensor out, int64_t begin_bit) {
  check_t(keys, at::kLong, "keys");
  check_t(out, at::kLong, "out");
  TORCH_CHECK(n >= 0 && n <= keys.numel() && n <= out.numel(), "gb_sort: sizes");
  TORCH_CHECK(end_bit >= 1 && end_bit <= 64 && begin_bit >= 0 && begin_bit < end_bit, "gb_sort: bits");
  if (n == 0) return;
  DeviceGuard guard(keys.device());
  auto* k = reinterpret_cast<const uint64_t*>(keys.data_ptr<int64_t>());
  auto* o = reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>());
  TORCH_CHECK(keys.data_ptr() != out.data_ptr(), "gb_sort: keys and out must differ");
  if (!use_rocprim_sort()) {
    native_sort(k, o, 8, n, (int)begin_bit, (int)end_bit, keys.options(), "rs_sort64");
    return;
  }
  size_t bytes = 0;
  DALGO_CHECK_HIP(dalgo_gb_sort(nullptr, &bytes, k, o, n, (int)begin_bit, (int)end_bit, cur_stream()),
                  "gb_sort(size)");
  Tensor tmp = at::empty({(int64_t)bytes + 256}, keys.options().dtype(at::kByte));
  DALGO_CHECK_HIP(dalgo_gb_sort(tmp.data_ptr(), &bytes, k, o, n, (int)begin_bit, (int)end_bit, cur_stream()),
                  "gb_sort");
}

// keys[:n] sorted on bits [lo_bits, 64) only: each run of keys equal there sorted on its
// low lo_bits in place (graph_build.hip gb_run_*), so the whole range ends up sorted;
// returns the device count of the runs (> 256 keys) handed to the block kernel
Tensor gb_run_sort(Tensor keys, int64_t n, int64_t lo_bits) {
  check_t(keys, at::kLong, "keys");
  TORCH_CHECK(n >= 0 && n <= keys.numel(), "gb_run_sort: sizes");
  TORCH_CHECK(lo_bits >= 1 && lo_bits <= 13, "gb_run_sort: lo_bits");
  if (n <= 1) return at::zeros({1}, keys.options());
  DeviceGuard guard(keys.device());
  Tensor ws = at::empty({dalgo_gb_run_ws(n)}, keys.options());
  DALGO_CHECK_HIP(dalgo_gb_run_sort(reinterpret_cast<uint64_t*>(keys.data_ptr<int64_t>()), n, (int)lo_bits,
                                    ws.data_ptr<int64_t>(), cur_stream()),
                  "gb_run_sort");
  return ws.slice(0, 0, 1).clone();
}

// blocks of the decode kernels over n sorted keys (size of their counts / offsets tables)
int64_t gb_decode_blocks(int64_t n) { return dalgo_gb_decode_blocks(n); }

void gb_decode(const Tensor& K, int64_t n, int64_t shift, int64_t dbits, const Tensor& blk_base,
               int64_t phase, const std::optional<Tensor>& counts, const std::optional<Tensor>& outdeg,
               const std::optional<Tensor>& offsets, const std::optional<Tensor>& srcl,
               const std::optional<Tensor>& ent_end, const std::optional<Tensor>& ent_blk,
               const std::optional<Tensor>& ent_dst) {
  check_t(K, at::kLong, "K");
  TORCH_CHECK(n >= 0 && n <= K.numel(), "gb_decode: n");
  check_t(blk_base, at::kLong, "blk_base");
  const int64_t nb = dalgo_gb_decode_blocks(n);
  if (phase == 0) {
    TORCH_CHECK(counts && outdeg, "gb_decode: counts / outdeg");
    check_t(*counts, at::kLong, "counts");
    check_i32(*outdeg, "outdeg");
    TORCH_CHECK(counts->numel() >= 2 * nb, "gb_decode: counts [2 blocks]");
  } else {
    TORCH_CHECK(offsets && srcl && ent_end && ent_blk && ent_dst, "gb_decode: outputs");
    check_t(*offsets, at::kLong, "offsets");
    TORCH_CHECK(offsets->numel() >= 2 * nb, "gb_decode: offsets [2 blocks]");
    check_t(*srcl, at::kShort, "srcl");
    check_t(*ent_end, at::kLong, "ent_end");
    check_i32(*ent_blk, "ent_blk");
    check_i32(*ent_dst, "ent_dst");
  }
  DeviceGuard guard(K.device());
  DALGO_CHECK_HIP(dalgo_gb_decode(reinterpret_cast<const uint64_t*>(K.data_ptr<int64_t>()), n, (int)shift,
                                  (int)dbits, blk_base.data_ptr<int64_t>(), (int)phase,
                                  opt_ptr<int64_t>(counts), opt_ptr<uint32_t>(outdeg),
                                  opt_ptr<const int64_t>(offsets), opt_ptr<uint16_t>(srcl),
                                  opt_ptr<int64_t>(ent_end), opt_ptr<int32_t>(ent_blk),
                                  opt_ptr<int32_t>(ent_dst), cur_stream()),
                  "gb_decode");
}

void gb_entry_flags(const Tensor& ent_blk, const Tensor& ent_dst, const Tensor& ent_end, int64_t bin_shift,
                    Tensor rs, Tensor cs, Tensor srcl) {
  check_i32(ent_blk, "ent_blk");
  check_i32(ent_dst, "ent_dst");
  check_t(ent_end, at::kLong, "ent_end");
  check_t(rs, at::kByte, "rs");
  check_t(cs, at::kByte, "cs");
  check_t(srcl, at::kShort, "srcl");
  const int64_t ne = ent_blk.numel();
  TORCH_CHECK(ent_dst.numel() == ne && ent_end.numel() == ne && rs.numel() >= ne && cs.numel() >= ne,
              "gb_entry_flags: sizes");
  DeviceGuard guard(ent_blk.device());
  DALGO_CHECK_HIP(dalgo_gb_entry_flags(ent_blk.data_ptr<int32_t>(), ent_dst.data_ptr<int32_t>(),
                                       ent_end.data_ptr<int64_t>(), ne, (int)bin_shift, rs.data_ptr<uint8_t>(),
                                       cs.data_ptr<uint8_t>(), reinterpret_cast<uint16_t*>(srcl.data_ptr<int16_t>()),
                                       cur_stream()),
                  "gb_entry_flags");
}

void gb_entry_place(const Tensor& ent_dst, const Tensor& ent_end, const Tensor& run_of_ent,
                    const Tensor& run_delta, const Tensor& run_chunk, const Tensor& cs, const Tensor& ce_lo,
                    const Tensor& tlen, int64_t wu_e, int64_t bin_mask, Tensor dloc, Tensor ts) {
  check_i32(ent_dst, "ent_dst");
  check_t(ent_end, at::kLong, "ent_end");
  check_i32(run_of_ent, "run_of_ent");
  check_i32(run_delta, "run_delta");
  check_i32(run_chunk, "run_chunk");
  check_t(cs, at::kByte, "cs");
  check_t(ce_lo, at::kLong, "ce_lo");
  check_t(tlen, at::kLong, "tlen");
  check_t(dloc, at::kShort, "dloc");
  check_t(ts, at::kByte, "ts");
  const int64_t ne = ent_dst.numel();
  TORCH_CHECK(ent_end.numel() == ne && run_of_ent.numel() == ne && cs.numel() >= ne && ts.numel() >= ne,
              "gb_entry_place: sizes");
  TORCH_CHECK(run_delta.numel() == run_chunk.numel() && ce_lo.numel() == tlen.numel(), "gb_entry_place: tables");
  DeviceGuard guard(ent_dst.device());
  DALGO_CHECK_HIP(dalgo_gb_entry_place(ent_dst.data_ptr<int32_t>(), ent_end.data_ptr<int64_t>(), ne,
                                       run_of_ent.data_ptr<int32_t>(), run_delta.data_ptr<int32_t>(),
                                       run_chunk.data_ptr<int32_t>(), cs.data_ptr<uint8_t>(),
                                       ce_lo.data_ptr<int64_t>(), tlen.data_ptr<int64_t>(), wu_e, (int)bin_mask,
                                       dloc.data_ptr<int16_t>(), ts.data_ptr<uint8_t>(), cur_stream()),
                  "gb_entry_place");
}

// ---- (block, bin) cell matrix of the K4b runs (graph_build.hip gb_cell_*)
static void check_cells(const Tensor& C, int64_t nblk, int64_t nbins) {
  check_i32(C, "C");
  TORCH_CHECK(nblk >= 1 && nbins >= 1 && nblk * nbins <= ((int64_t)1 << 31) && C.numel() >= nblk * nbins,
              "gb_cells: C [nblk * nbins]");
}

void gb_cell_count(const Tensor& ent_blk, const Tensor& ent_dst, int64_t bshift, int64_t nblk, int64_t nbins,
                   Tensor C) {
  check_i32(ent_blk, "ent_blk");
  check_i32(ent_dst, "ent_dst");
  check_cells(C, nblk, nbins);
  TORCH_CHECK(ent_blk.numel() == ent_dst.numel(), "gb_cell_count: entry arrays");
  DeviceGuard guard(C.device());
  DALGO_CHECK_HIP(dalgo_gb_cells(0, ent_blk.data_ptr<int32_t>(), ent_dst.data_ptr<int32_t>(), ent_blk.numel(),
                                 (int)bshift, (int)nblk, (int)nbins, C.data_ptr<int32_t>(), nullptr, nullptr, nullptr,
                                 nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                                 cur_stream()),
                  "gb_cell_count");
}

void gb_cell_rows(const Tensor& C, int64_t nblk, int64_t nbins, Tensor T, Tensor R) {
  check_cells(C, nblk, nbins);
  check_t(T, at::kLong, "T");
  check_t(R, at::kLong, "R");
  TORCH_CHECK(T.numel() >= nblk && R.numel() >= nblk, "gb_cell_rows: T / R [nblk]");
  DeviceGuard guard(C.device());
  DALGO_CHECK_HIP(dalgo_gb_cells(1, nullptr, nullptr, 0, 0, (int)nblk, (int)nbins, C.data_ptr<int32_t>(),
                                 T.data_ptr<int64_t>(), R.data_ptr<int64_t>(), nullptr, nullptr, nullptr, nullptr, 0,
                                 nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, cur_stream()),
                  "gb_cell_rows");
}

void gb_cell_scan(const Tensor& C, int64_t nblk, int64_t nbins, const Tensor& RE, const Tensor& RR, Tensor CM,
                  Tensor RID) {
  check_cells(C, nblk, nbins);
  check_t(RE, at::kLong, "RE");
  check_t(RR, at::kLong, "RR");
  check_i32(CM, "CM");
  check_i32(RID, "RID");
  TORCH_CHECK(RE.numel() >= nblk && RR.numel() >= nblk && CM.numel() >= nblk * nbins && RID.numel() >= nblk * nbins,
              "gb_cell_scan: sizes");
  DeviceGuard guard(C.device());
  DALGO_CHECK_HIP(dalgo_gb_cells(2, nullptr, nullptr, 0, 0, (int)nblk, (int)nbins, C.data_ptr<int32_t>(), nullptr,
                                 nullptr, RE.data_ptr<int64_t>(), RR.data_ptr<int64_t>(), CM.data_ptr<int32_t>(),
                                 RID.data_ptr<int32_t>(), 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                                 cur_stream()),
                  "gb_cell_scan");
}

void gb_cell_colsum(const Tensor& C, int64_t nblk, int64_t nbins, int64_t G, Tensor P) {
  check_cells(C, nblk, nbins);
  check_t(P, at::kLong, "P");
  TORCH_CHECK(G >= 1 && P.numel() >= ((nblk + G - 1) / G) * nbins, "gb_cell_colsum: P [groups * nbins]");
  DeviceGuard guard(C.device());
  DALGO_CHECK_HIP(dalgo_gb_cells(3, nullptr, nullptr, 0, 0, (int)nblk, (int)nbins, C.data_ptr<int32_t>(), nullptr,
                                 nullptr, nullptr, nullptr, nullptr, nullptr, (int)G, P.data_ptr<int64_t>(), nullptr,
                                 nullptr, 0, nullptr, nullptr, nullptr, cur_stream()),
                  "gb_cell_colsum");
}

void gb_cell_place(const Tensor& C, const Tensor& CM, const Tensor& RID, int64_t nblk, int64_t nbins, int64_t G,
                   const Tensor& Poff, const Tensor& CI, Tensor run_delta, Tensor run_chunk, Tensor run_first) {
  check_cells(C, nblk, nbins);
  check_i32(CM, "CM");
  check_i32(RID, "RID");
  check_t(Poff, at::kLong, "Poff");
  check_i32(CI, "CI");
  check_i32(run_delta, "run_delta");
  check_i32(run_chunk, "run_chunk");
  check_t(run_first, at::kLong, "run_first");
  const int64_t nruns = run_delta.numel();
  TORCH_CHECK(G >= 1 && Poff.numel() >= ((nblk + G - 1) / G) * nbins && CI.numel() >= nblk &&
                  CM.numel() >= nblk * nbins && RID.numel() >= nblk * nbins && run_chunk.numel() == nruns &&
                  run_first.numel() == nruns,
              "gb_cell_place: sizes");
  DeviceGuard guard(C.device());
  DALGO_CHECK_HIP(dalgo_gb_cells(4, nullptr, nullptr, 0, 0, (int)nblk, (int)nbins, C.data_ptr<int32_t>(), nullptr,
                                 nullptr, nullptr, nullptr, CM.data_ptr<int32_t>(), RID.data_ptr<int32_t>(), (int)G,
                                 nullptr, Poff.data_ptr<int64_t>(), CI.data_ptr<int32_t>(), nruns,
                                 run_delta.data_ptr<int32_t>(), run_chunk.data_ptr<int32_t>(),
                                 run_first.data_ptr<int64_t>(), cur_stream()),
                  "gb_cell_place");
}

void gb_entry_cells(const Tensor& ent_blk, const Tensor& ent_dst, const Tensor& ent_end, int64_t bshift,
                    int64_t nblk, int64_t nbins, const Tensor& CM, const Tensor& RID, const Tensor& run_delta,
                    const Tensor& RE, const Tensor& CI, const Tensor& ce_lo, const Tensor& tlen, int64_t wu_e,
                    int64_t bin_mask, Tensor dloc, Tensor tiles, Tensor n_tiles, Tensor srcl) {
  check_i32(ent_blk, "ent_blk");
  check_i32(ent_dst, "ent_dst");
  check_t(ent_end, at::kLong, "ent_end");
  check_i32(CM, "CM");
  check_i32(RID, "RID");
  check_i32(run_delta, "run_delta");
  check_t(RE, at::kLong, "RE");
  check_i32(CI, "CI");
  check_t(ce_lo, at::kLong, "ce_lo");
  check_t(tlen, at::kLong, "tlen");
  check_t(dloc, at::kShort, "dloc");
  check_i32(tiles, "tiles");
  check_t(n_tiles, at::kLong, "n_tiles");
  check_t(srcl, at::kShort, "srcl");
  const int64_t ne = ent_blk.numel();
  TORCH_CHECK(ent_dst.numel() == ne && ent_end.numel() == ne && dloc.numel() >= ne && n_tiles.numel() >= 1,
              "gb_entry_cells: entry arrays");
  TORCH_CHECK(nblk >= 1 && nbins >= 1 && CM.numel() >= nblk * nbins && RID.numel() >= nblk * nbins &&
                  RE.numel() >= nblk && CI.numel() >= nblk && ce_lo.numel() == tlen.numel(),
              "gb_entry_cells: tables");
  DeviceGuard guard(ent_blk.device());
  DALGO_CHECK_HIP(dalgo_gb_entry_cells(ent_blk.data_ptr<int32_t>(), ent_dst.data_ptr<int32_t>(),
                                       ent_end.data_ptr<int64_t>(), ne, (int)bshift, (int)nblk, (int)nbins,
                                       CM.data_ptr<int32_t>(), RID.data_ptr<int32_t>(), run_delta.data_ptr<int32_t>(),
                                       run_delta.numel(), RE.data_ptr<int64_t>(), CI.data_ptr<int32_t>(),
                                       ce_lo.data_ptr<int64_t>(), tlen.data_ptr<int64_t>(), ce_lo.numel(), wu_e,
                                       (int)bin_mask, dloc.data_ptr<int16_t>(), dloc.numel(),
                                       tiles.data_ptr<int32_t>(),
                                       reinterpret_cast<unsigned long long*>(n_tiles.data_ptr<int64_t>()),
                                       tiles.numel(), reinterpret_cast<uint16_t*>(srcl.data_ptr<int16_t>()),
                                       srcl.numel(), cur_stream()),
                  "gb_entry_cells");
}

void pr_spmv(const Tensor& src, const Tensor& dstl, const Tensor& c, Tensor acc, Tensor pres,
             bool accumulate) {
  check_i32(src, "src");
  check_i32(dstl, "dstl");
  TORCH_CHECK(src.numel() == dstl.numel() && src.numel() % 4 == 0, "edge arrays: equal, % 4");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(dstl.data_ptr()) % 16 == 0, "edge arrays 16-B aligned");
  check_f32(c, "c");
  check_f32(acc, "acc");
  check_i32(pres, "pres");
  TORCH_CHECK(pres.numel() >= acc.numel(), "pres size");
  DeviceGuard guard(src.device());
  DALGO_CHECK_HIP(dalgo_pr_spmv(src.data_ptr<int32_t>(), dstl.data_ptr<int32_t>(), src.numel(),
                                c.data_ptr<float>(), c.numel(), acc.data_ptr<float>(),
                                pres.data_ptr<int32_t>(),
                                accumulate ? 1 : 0, cur_stream()),
                  "pr_spmv");
}

// K4b two-level propagation-blocked SpMV. The layout invariants (tile / entry / run
// offsets inside the arrays, chunk source ranges inside c, dloc < bin_width) are
// established and asserted once by dalgo.ops.graph.build_blocked(); here the shapes,
// dtypes and the bounds a kernel could overrun are checked.
void pb_spmv(const Tensor& srcl, const Tensor& tile_e, const Tensor& tile_ent,
             const Tensor& tile_run, const Tensor& wu_tile, const Tensor& wu_chunk,
             const Tensor& chunk_slo,
             const Tensor& chunk_ns, const Tensor& chunk_run, const Tensor& run_delta,
             const Tensor& c, Tensor val, const Tensor& dloc, const Tensor& wi_bin,
             const Tensor& wi_lo, const Tensor& wi_slab, int64_t bin_width, int64_t max_runs,
             Tensor bound,
             Tensor acc, Tensor pres, Tensor slab, const Tensor& split_bin, const Tensor& split_first,
             const Tensor& split_count, const std::optional<Tensor>& outdeg, double q, double invN,
             int64_t mode, const std::optional<Tensor>& dangling_in, const std::optional<Tensor>& r,
             const std::optional<Tensor>& c_out, const std::optional<Tensor>& dangling_out,
             int64_t wu_lo, int64_t wu_hi, int64_t phases) {
  check_dev(srcl, "srcl");
  TORCH_CHECK(wu_lo >= 0 && wu_hi >= wu_lo && phases >= 1 && phases <= 3, "pb: work-unit range / phases");
  // fused PageRank update: all of outdeg / r / c_out or none
  const bool fused = r.has_value();
  TORCH_CHECK(fused == outdeg.has_value() && fused == c_out.has_value(), "pb: fused update args");
  const int32_t* od = nullptr;
  float *rp = nullptr, *cp = nullptr, *dout = nullptr;
  const float* di = nullptr;
  if (fused) {
    check_i32(*outdeg, "outdeg");
    check_f32(*r, "r");
    check_f32(*c_out, "c_out");
    TORCH_CHECK(outdeg->numel() >= acc.numel() && r->numel() >= acc.numel() && c_out->numel() >= acc.numel(),
                "pb: update sizes");
    od = outdeg->data_ptr<int32_t>();
    rp = r->data_ptr<float>();
    cp = c_out->data_ptr<float>();
    if (dangling_in.has_value()) { check_f32(*dangling_in, "dangling_in"); di = dangling_in->data_ptr<float>(); }
    if (dangling_out.has_value()) { check_f32(*dangling_out, "dangling_out"); dout = dangling_out->data_ptr<float>(); }
  }
  TORCH_CHECK(srcl.scalar_type() == at::kShort && srcl.is_contiguous() && srcl.numel() % 16 == 0,
              "pb: srcl int16, len % 16 == 0");
  check_dev(tile_e, "tile_e");
  TORCH_CHECK(tile_e.scalar_type() == at::kLong && tile_e.is_contiguous(), "tile_e int64");
  for (const Tensor* t : {&tile_ent, &tile_run, &wu_tile, &wu_chunk, &chunk_slo, &chunk_ns, &chunk_run,
                          &run_delta})
    check_i32(*t, "pb index arrays");
  const int64_t nch = chunk_slo.numel();
  const int64_t nt = tile_ent.numel();
  const int64_t nwu = wu_chunk.numel();
  TORCH_CHECK(chunk_ns.numel() == nch && wu_tile.numel() == nwu + 1 && chunk_run.numel() == nch + 1 &&
                  tile_e.numel() == nt + 1 && tile_run.numel() == nt,
              "pb: chunk / tile arrays");
  check_f32(c, "c");
  check_f32(val, "val");
  check_dev(dloc, "dloc");
  TORCH_CHECK(dloc.scalar_type() == at::kShort && dloc.is_contiguous() && dloc.numel() == val.numel() &&
                  val.numel() % 4 == 0,
              "pb: dloc int16[len(val)], len % 4 == 0");
  check_i32(wi_bin, "wi_bin");
  check_i32(wi_slab, "wi_slab");
  check_dev(wi_lo, "wi_lo");
  TORCH_CHECK(wi_lo.scalar_type() == at::kLong && wi_lo.is_contiguous(), "wi_lo int64");
  const int64_t nwi = wi_bin.numel();
  TORCH_CHECK(wi_lo.numel() == nwi + 1 && wi_slab.numel() == nwi, "pb: work items");
  check_f32(acc, "acc");
  check_i32(pres, "pres");
  TORCH_CHECK(pres.numel() >= acc.numel(), "pres size");
  check_dev(bound, "bound");
  TORCH_CHECK(bound.scalar_type() == at::kDouble && bound.numel() >= 1, "pb: bound f64[1]");
  check_dev(slab, "slab");
  TORCH_CHECK(slab.scalar_type() == at::kLong && slab.is_contiguous(), "pb: slab int64 (u64 fixed point)");
  check_i32(split_bin, "split_bin");
  check_i32(split_first, "split_first");
  check_i32(split_count, "split_count");
  const int64_t nsp = split_bin.numel();
  TORCH_CHECK(split_first.numel() == nsp && split_count.numel() == nsp, "pb: split arrays");
  for (const Tensor* t : {&srcl, static_cast<const Tensor*>(&val), &dloc})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "pb arrays 16-B aligned");
  DeviceGuard guard(srcl.device());
  DALGO_CHECK_HIP(
      dalgo_pb_spmv(reinterpret_cast<const uint16_t*>(srcl.data_ptr<int16_t>()),
                    tile_e.data_ptr<int64_t>(), tile_ent.data_ptr<int32_t>(), tile_run.data_ptr<int32_t>(),
                    wu_tile.data_ptr<int32_t>(), wu_chunk.data_ptr<int32_t>(), (int)nwu,
                    (int)std::min<int64_t>(wu_lo, nwu), (int)std::min<int64_t>(wu_hi, nwu), (int)phases,
                    chunk_slo.data_ptr<int32_t>(),
                    chunk_ns.data_ptr<int32_t>(), chunk_run.data_ptr<int32_t>(),
                    run_delta.data_ptr<int32_t>(), (int)nch, (int)max_runs, 8192, c.data_ptr<float>(),
                    val.data_ptr<float>(), val.numel(), reinterpret_cast<const uint16_t*>(dloc.data_ptr<int16_t>()),
                    wi_bin.data_ptr<int32_t>(), wi_lo.data_ptr<int64_t>(), wi_slab.data_ptr<int32_t>(),
                    (int)nwi, (int)bin_width, bound.data_ptr<double>(), acc.numel(), acc.data_ptr<float>(),
                    pres.data_ptr<int32_t>(), reinterpret_cast<uint64_t*>(slab.data_ptr<int64_t>()),
                    split_bin.data_ptr<int32_t>(),
                    split_first.data_ptr<int32_t>(), split_count.data_ptr<int32_t>(), (int)nsp, od,
                    (float)q, (float)invN, (int)mode, di, rp, cp, dout, cur_stream()),
      "pb_spmv");
}

void pr_update(const Tensor& acc, const Tensor& pres, const Tensor& outdeg, double q, double invN,
               int64_t mode, const std::optional<Tensor>& dangling_in, Tensor r, Tensor c,
               const std::optional<Tensor>& dangling_out) {
  check_f32(acc, "acc");
  check_i32(pres, "pres");
  check_i32(outdeg, "outdeg");
  check_f32(r, "r");
  check_f32(c, "c");
  const int64_t n = acc.numel();
  TORCH_CHECK(pres.numel() >= n && outdeg.numel() >= n && r.numel() >= n && c.numel() >= n,
              "pr_update sizes");
  const float* di = nullptr;
  float* dout = nullptr;
  if (dangling_in.has_value()) { check_f32(*dangling_in, "dangling_in"); di = dangling_in->data_ptr<float>(); }
  if (dangling_out.has_value()) { check_f32(*dangling_out, "dangling_out"); dout = dangling_out->data_ptr<float>(); }
  DeviceGuard guard(acc.device());
  DALGO_CHECK_HIP(dalgo_pr_update(acc.data_ptr<float>(), pres.data_ptr<int32_t>(),
                                  outdeg.data_ptr<int32_t>(), n, (float)q, (float)invN, (int)mode,
                                  di, r.data_ptr<float>(), c.data_ptr<float>(), dout, cur_stream()),
                  "pr_update");
}

// ---------------------------------------------------------------------------
// K11 xGMI one-shot all-reduce: buffers are raw device addresses (int64) owned by
// dalgo.parallel.xgmi (allocated / IPC-opened through these ops)
int64_t xgmi_buffer_bytes(int64_t slot) { return (int64_t)dalgo_xgmi_buffer_bytes((int)slot); }

int64_t xgmi_alloc(int64_t bytes, int64_t device) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, (int)device));
  void* p = nullptr;
  DALGO_CHECK_HIP(dalgo_xgmi_alloc((size_t)bytes, &p), "xgmi_alloc");
  return reinterpret_cast<int64_t>(p);
}

void xgmi_free(int64_t ptr) {
  DALGO_CHECK_HIP(dalgo_xgmi_free(reinterpret_cast<void*>(ptr)), "xgmi_free");
}

Tensor xgmi_get_handle(int64_t ptr) {
  Tensor h = at::zeros({64}, at::TensorOptions().dtype(at::kByte));
  DALGO_CHECK_HIP(dalgo_xgmi_get_handle(reinterpret_cast<void*>(ptr), h.data_ptr()), "xgmi_get_handle");
  return h;
}

int64_t xgmi_open(const Tensor& handle, int64_t device) {
  TORCH_CHECK(!handle.is_cuda() && handle.scalar_type() == at::kByte && handle.numel() == 64 &&
                  handle.is_contiguous(), "xgmi_open: handle must be a CPU uint8[64]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, (int)device));
  void* p = nullptr;
  DALGO_CHECK_HIP(dalgo_xgmi_open(handle.data_ptr(), &p), "xgmi_open");
  return reinterpret_cast<int64_t>(p);
}

void xgmi_close(int64_t ptr) {
  DALGO_CHECK_HIP(dalgo_xgmi_close(reinterpret_cast<void*>(ptr)), "xgmi_close");
}

void xgmi_allreduce(Tensor x, at::IntArrayRef bufs, int64_t rank, int64_t slot, Tensor epoch,
                    Tensor err, double timeout_s, const std::optional<Tensor>& W, int64_t upd_mode,
                    int64_t upd_reg, double eta, double lam, double reg_alpha, int64_t count_index,
                    const std::optional<Tensor>& count_acc) {
  check_f32(x, "x");
  TORCH_CHECK(x.numel() <= slot, "xgmi_allreduce: vector larger than the slot");
  TORCH_CHECK(bufs.size() >= 1 && bufs.size() <= 8 && rank >= 0 && rank < (int64_t)bufs.size(),
              "xgmi_allreduce: 1..8 ranks");
  check_dev(epoch, "epoch");
  TORCH_CHECK(epoch.scalar_type() == at::kInt && epoch.numel() >= 1, "epoch: device int32[1]");
  check_dev(err, "err");
  TORCH_CHECK(err.scalar_type() == at::kInt && err.numel() >= 1, "err int32[1]");
  void* b[8] = {};
  for (size_t r = 0; r < bufs.size(); ++r) b[r] = reinterpret_cast<void*>(bufs[r]);
  float* w = nullptr;
  int nw = 0;
  if (W.has_value()) {
    check_f32(*W, "W");
    nw = (int)W->numel();
    TORCH_CHECK(count_index >= nw && count_index < x.numel(),
                "xgmi_allreduce: the count must follow the model-sized gradient in x");
    w = W->data_ptr<float>();
  }
  double* cacc = nullptr;
  if (count_acc.has_value()) {
    check_dev(*count_acc, "count_acc");
    TORCH_CHECK(count_acc->scalar_type() == at::kDouble && count_acc->numel() >= 1, "count_acc f64");
    cacc = count_acc->data_ptr<double>();
  }
  DeviceGuard guard(x.device());
  DALGO_CHECK_HIP(dalgo_xgmi_allreduce(x.data_ptr<float>(), x.data_ptr<float>(), (int)x.numel(),
                                       (int)rank, (int)bufs.size(), b, (int)slot,
                                       reinterpret_cast<uint32_t*>(epoch.data_ptr<int32_t>()),
                                       reinterpret_cast<unsigned*>(err.data_ptr<int>()), timeout_s,
                                       w, nw, (int)count_index, (int)upd_mode, (int)upd_reg,
                                       (float)eta, (float)lam, (float)reg_alpha, cacc, cur_stream()),
                  "xgmi_allreduce");
}

// ---------------------------------------------------------------------------
// transitive closure, sparse mode (K9 sparse: frontier join + hash-set dedup/merge)
namespace {
void check_i64_1d(const Tensor& t, const char* what) {
  check_dev(t, what);
  TORCH_CHECK(t.scalar_type() == at::kLong && t.dim() == 1 && t.is_contiguous(),
              what, ": contiguous 1-D int64");
}
uint64_t* u64(const Tensor& t) { return reinterpret_cast<uint64_t*>(t.data_ptr<int64_t>()); }
uint64_t pow2_mask(const Tensor& table) {
  const uint64_t n = (uint64_t)table.numel();
  TORCH_CHECK(n >= 2 && (n & (n - 1)) == 0, "tcs: table size must be a power of two");
  return n - 1;
}
}  // namespace

void tcs_degree(const Tensor& keys, int64_t d0, int64_t nd, const Tensor& in_ptr, Tensor deg) {
  check_i64_1d(keys, "keys");
  check_i64_1d(in_ptr, "in_ptr");
  check_i64_1d(deg, "deg");
  TORCH_CHECK(d0 >= 0 && nd >= 0 && d0 + nd <= keys.numel() && deg.numel() >= nd, "tcs_degree ranges");
  DeviceGuard guard(keys.device());
  DALGO_CHECK_HIP(dalgo_tcs_degree(u64(keys), d0, nd, in_ptr.data_ptr<int64_t>(),
                                   deg.data_ptr<int64_t>(), cur_stream()),
                  "tcs_degree");
}

void tcs_expand(Tensor keys, int64_t d0, int64_t nd, const Tensor& excl, int64_t c_lo,
                int64_t c_hi, const Tensor& in_ptr, const Tensor& in_src, Tensor table,
                Tensor n_keys, Tensor err) {
  check_i64_1d(keys, "keys");
  check_i64_1d(excl, "excl");
  check_i64_1d(in_ptr, "in_ptr");
  check_i64_1d(table, "table");
  check_i64_1d(n_keys, "n_keys");
  check_dev(in_src, "in_src");
  TORCH_CHECK(in_src.scalar_type() == at::kInt && in_src.is_contiguous(), "in_src int32");
  check_dev(err, "err");
  TORCH_CHECK(err.scalar_type() == at::kInt, "err int32");
  TORCH_CHECK(d0 >= 0 && nd >= 0 && d0 + nd <= keys.numel() && excl.numel() >= nd + 1,
              "tcs_expand: frontier range");
  TORCH_CHECK(0 <= c_lo && c_lo <= c_hi, "tcs_expand: candidate range");
  DeviceGuard guard(keys.device());
  DALGO_CHECK_HIP(dalgo_tcs_expand(u64(keys) + d0, nd, excl.data_ptr<int64_t>(), c_lo, c_hi,
                                   in_ptr.data_ptr<int64_t>(), in_src.data_ptr<int32_t>(),
                                   u64(table), pow2_mask(table), u64(keys),
                                   reinterpret_cast<unsigned long long*>(n_keys.data_ptr<int64_t>()),
                                   (uint64_t)keys.numel(),
                                   reinterpret_cast<unsigned*>(err.data_ptr<int>()), cur_stream()),
                  "tcs_expand");
}

void tcs_insert(const Tensor& src, Tensor table, bool append, Tensor keys, Tensor n_keys,
                Tensor err) {
  check_i64_1d(src, "src");
  check_i64_1d(table, "table");
  check_i64_1d(keys, "keys");
  check_i64_1d(n_keys, "n_keys");
  check_dev(err, "err");
  TORCH_CHECK(err.scalar_type() == at::kInt, "err int32");
  DeviceGuard guard(table.device());
  DALGO_CHECK_HIP(dalgo_tcs_insert(u64(src), src.numel(), u64(table), pow2_mask(table),
                                   append ? 1 : 0, u64(keys),
                                   reinterpret_cast<unsigned long long*>(n_keys.data_ptr<int64_t>()),
                                   (uint64_t)keys.numel(),
                                   reinterpret_cast<unsigned*>(err.data_ptr<int>()), cur_stream()),
                  "tcs_insert");
}

// ---------------------------------------------------------------------------
// transitive closure
void tc_step(const Tensor& A, const Tensor& Told, Tensor Tnew, Tensor count, int64_t variant) {
  for (const Tensor* t : {&A, &Told, static_cast<const Tensor*>(&Tnew)}) {
    check_dev(*t, "tc operand");
    TORCH_CHECK(t->scalar_type() == at::kByte && t->dim() == 2 && t->stride(1) == 1,
                "tc operands: 2-D uint8 (0/1) with contiguous rows");
    TORCH_CHECK(t->stride(0) % 16 == 0, "tc: row strides must be multiples of 16 bytes");
  }
  const int64_t npad = A.size(0);
  TORCH_CHECK(A.size(1) >= npad && Told.size(1) >= npad && Tnew.sizes() == Told.sizes(),
              "tc shapes");
  TORCH_CHECK(npad % 128 == 0 && Told.size(0) % 128 == 0, "tc: dims must be multiples of 128");
  TORCH_CHECK(Told.stride(0) == Tnew.stride(0), "tc: T strides");
  TORCH_CHECK(count.scalar_type() == at::kLong && count.numel() >= 1, "count int64[1]");
  DeviceGuard guard(A.device());
  DALGO_CHECK_HIP(dalgo_tc_step(A.data_ptr(), A.stride(0), Told.data_ptr(), Tnew.data_ptr(),
                                Told.stride(0), (int)npad, (int)Told.size(0), (int)variant,
                                reinterpret_cast<unsigned long long*>(count.data_ptr<int64_t>()),
                                cur_stream()),
                  "tc_step");
}

// ---------------------------------------------------------------------------
// ALS
void spd_inverse(const Tensor& G, double ridge, Tensor out, const std::optional<Tensor>& status) {
  check_f32(G, "G");
  check_f32(out, "out");
  TORCH_CHECK(G.dim() == 2 && G.size(0) == G.size(1) && out.sizes() == G.sizes(), "square k x k");
  TORCH_CHECK(G.size(0) >= 1 && G.size(0) <= 128, "spd_inverse: k <= 128");
  int* st = nullptr;
  if (status.has_value()) { check_i32(*status, "status"); st = status->data_ptr<int32_t>(); }
  DeviceGuard guard(G.device());
  DALGO_CHECK_HIP(dalgo_spd_inverse(G.data_ptr<float>(), (int)G.size(0), (int)G.stride(0),
                                    (float)ridge, out.data_ptr<float>(), (int)out.stride(0), st,
                                    cur_stream()),
                  "spd_inverse");
}

// out = (R . F) . Ginv for all rows of R at once (K5 half-sweep). Workspaces (the
// packed F^T fragments and the K-split partials) come from the torch caching allocator
// on the current stream.
void als_solve(const Tensor& R, const Tensor& F, const Tensor& Ginv, Tensor out) {
  check_dev(R, "R");
  TORCH_CHECK(R.scalar_type() == at::kFloat && R.dim() == 2 && R.stride(1) == 1,
              "als_solve: R must be 2-D float32 with contiguous rows");
  TORCH_CHECK(R.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(R.data_ptr()) % 16 == 0,
              "als_solve: R rows must be 16-B aligned (row stride a multiple of 4)");
  check_dev(F, "F");
  TORCH_CHECK(F.scalar_type() == at::kFloat && F.dim() == 2 && F.stride(1) == 1,
              "als_solve: F must be 2-D float32 with contiguous rows");
  check_f32(Ginv, "Ginv");
  check_f32(out, "out");
  const int64_t m = R.size(0), n = R.size(1), k = F.size(1);
  TORCH_CHECK(F.size(0) == n, "als_solve: F must have R.size(1) rows");
  TORCH_CHECK(k >= 1 && k <= 128, "als_solve: k <= 128");
  TORCH_CHECK(Ginv.dim() == 2 && Ginv.size(0) == k && Ginv.size(1) == k, "als_solve: Ginv k x k");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == m && out.size(1) == k, "als_solve: out m x k");
  TORCH_CHECK(m >= 1 && n >= 1, "als_solve: empty R");
  TORCH_CHECK(R.device() == F.device() && R.device() == Ginv.device() && R.device() == out.device(),
              "als_solve: operands on different devices");
  DeviceGuard guard(R.device());
  const int nsplit = dalgo_als_nsplit(m, n, (int)k);
  const int64_t kpad = dalgo_als_kpad((int)k);
  auto opts = R.options();
  Tensor Fq = at::empty({dalgo_als_fq_bytes(n, (int)k) / 4}, opts);
  Tensor P = at::empty({(int64_t)nsplit * m * kpad}, opts);
  DALGO_CHECK_HIP(dalgo_als_solve(R.data_ptr<float>(), m, n, R.stride(0), F.data_ptr<float>(),
                                  F.stride(0), (int)k, Ginv.data_ptr<float>(), (int)Ginv.stride(0),
                                  out.data_ptr<float>(), out.stride(0), Fq.data_ptr(),
                                  P.data_ptr<float>(), nsplit, cur_stream()),
                  "als_solve");
}

// G = F^T F (k x k) of an n x k f32 factor, split-n partials summed in block order
void als_gram(const Tensor& F, Tensor G) {
  check_dev(F, "F");
  TORCH_CHECK(F.scalar_type() == at::kFloat && F.dim() == 2 && F.stride(1) == 1,
              "als_gram: F must be 2-D float32 with contiguous rows");
  check_f32(G, "G");
  const int64_t n = F.size(0), k = F.size(1);
  TORCH_CHECK(k >= 1 && k <= 128, "als_gram: k <= 128");
  TORCH_CHECK(G.dim() == 2 && G.size(0) == k && G.size(1) == k, "als_gram: G k x k");
  TORCH_CHECK(F.device() == G.device(), "als_gram: operands on different devices");
  DeviceGuard guard(F.device());
  Tensor part = at::empty({(int64_t)dalgo_als_gram_blocks(n) * k * k}, F.options());
  DALGO_CHECK_HIP(dalgo_als_gram(F.data_ptr<float>(), n, (int)k, F.stride(0), G.data_ptr<float>(),
                                 (int)G.stride(0), part.data_ptr<float>(), cur_stream()),
                  "als_gram");
}

// sum_ij (R_ij - U_i . V_j)^2 -> out (f64 [1]); R rows 16-B aligned
void als_residual(const Tensor& R, const Tensor& U, const Tensor& V, Tensor out) {
  check_dev(R, "R");
  TORCH_CHECK(R.scalar_type() == at::kFloat && R.dim() == 2 && R.stride(1) == 1,
              "als_residual: R must be 2-D float32 with contiguous rows");
  TORCH_CHECK(R.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(R.data_ptr()) % 16 == 0,
              "als_residual: R rows must be 16-B aligned");
  for (const Tensor* t : {&U, &V}) {
    check_dev(*t, "factor");
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->dim() == 2 && t->stride(1) == 1,
                "als_residual: factors must be 2-D float32 with contiguous rows");
  }
  TORCH_CHECK(out.scalar_type() == at::kDouble && out.numel() >= 1 && out.is_cuda(), "out f64[1]");
  const int64_t m = R.size(0), n = R.size(1), k = U.size(1);
  TORCH_CHECK(U.size(0) == m && V.size(0) == n && V.size(1) == k, "als_residual: shapes");
  TORCH_CHECK(k >= 1 && k <= 128 && m >= 1 && n >= 1, "als_residual: k <= 128, non-empty R");
  DeviceGuard guard(R.device());
  Tensor Vq = at::empty({dalgo_als_residual_vq_bytes(n, (int)k) / 4}, R.options());
  Tensor part = at::empty({(int64_t)dalgo_als_residual_blocks(m, n)}, R.options().dtype(at::kDouble));
  DALGO_CHECK_HIP(dalgo_als_residual(R.data_ptr<float>(), m, n, R.stride(0), U.data_ptr<float>(),
                                     U.stride(0), V.data_ptr<float>(), V.stride(0), (int)k, Vq.data_ptr(),
                                     part.data_ptr<double>(), cur_stream()),
                  "als_residual");
  out.reshape(-1).narrow(0, 0, 1).copy_(part.sum().reshape(1));
}

}  // namespace

TORCH_LIBRARY(dalgo, m) {
  m.def("lr_grad(Tensor X, Tensor y, Tensor(z!) W, Tensor seg, int row_offset, int D, bool has_bias, "
        "float eps, int seed, int step, float frac, int gx, int rows_per_block, Tensor(a!) slab, "
        "Tensor(b!) gslab, Tensor(c!) cnt1, Tensor(d!) cnt2, Tensor(e!) G, Tensor(f!) C, "
        "int flags=0, Tensor(g!)? count_acc=None, "
        "Tensor(h!)? ticket=None, int[]? xg_bufs=None, int xg_rank=0, int xg_slot=0, Tensor(k!)? xg_epoch=None, "
        "Tensor(i!)? xg_err=None, float xg_timeout=0., int tail_mode=0, int tail_reg=0, "
        "float tail_eta=0., float tail_lam=0., float tail_reg_alpha=0., "
        "Tensor(j!)? tail_count_acc=None, int nsteps=1, "
        "Tensor(l!)? epoch=None, int epoch_base=0, Tensor(m!)? perr=None, float spin_s=2., "
        "Tensor? step_dev=None, int step_mul=1, Tensor(n!)? pool=None, int pool_lo=0, int pool_shift=6) -> ()");
  m.def("lr_eval(Tensor X, Tensor y, Tensor W, Tensor seg, int D, bool has_bias, float eps, "
        "int gx, int rows_per_block, Tensor(a!) correct, Tensor(b!) loss) -> ()");
  m.def("sync_update(Tensor(a!) W, Tensor(d!)? G, Tensor(e!)? C, Tensor? center, Tensor? S, "
        "Tensor(b!)? Dl, Tensor(c!)? count_acc, int n, int mode, int reg, float eta, float lam, float alpha, "
        "float reg_alpha, float mu, float zeta, float beta, float inv_p, bool zero_grad=False) -> ()");
  m.def("rows_sum(Tensor W, int n, Tensor(a!) out) -> ()");
  m.def("rows_broadcast(Tensor(a!) W, int n, Tensor src) -> ()");
  m.def("philox_fill(Tensor(a!) out, int D, int row_offset, int seed, int stream, int dist, "
        "float a, float b) -> ()");
  m.def("kmeans_assign(Tensor X, Tensor Cq, Tensor hn, Tensor(a!) assign, Tensor(b!)? mind, "
        "Tensor(c!)? sse) -> ()");
  m.def("kmeans_accumulate_sorted(Tensor X, Tensor assign, int k, int DP, int seg, "
        "Tensor(a!) block_counts, Tensor(b!) cluster_start, Tensor(c!) seg_start, Tensor(d!) perm, "
        "Tensor(e!) S, Tensor(f!) cnt) -> ()");
  m.def("kmeans_diff(Tensor a_new, Tensor a_old, Tensor(a!) changed, Tensor(b!) n_changed) -> ()");
  m.def("kmeans_move_sorted(Tensor X, int DP, Tensor changed, int m, Tensor a_new, Tensor a_old, "
        "Tensor(a!) S64, Tensor(b!) cnt, Tensor? xh, Tensor(c!)? Q, int seg, Tensor(d!) block_counts, "
        "Tensor(e!) cluster_start, Tensor(f!) seg_start, Tensor(g!) perm, Tensor(h!) ec, "
        "Tensor(i!) er, Tensor? m_dev=None, int chunk=65536, Tensor? cnew=None, "
        "Tensor? cold=None) -> ()");
  m.def("kmeans_filter(Tensor assign, Tensor(a!) ul, Tensor delta, Tensor s, "
        "Tensor(b!)? a_prev, Tensor(c!) idx, Tensor(d!) n_active, Tensor(f!)? acl=None) -> ()");
  m.def("kmeans_sort_active(Tensor acl, Tensor idx, Tensor n_active, int k, int chunk, "
        "Tensor(a!) block_counts, Tensor(b!) cstart, Tensor(c!) seg_start, Tensor(d!) rows_sorted, "
        "int tile, Tensor(e!) tiles, Tensor(g!) n_tiles) -> ()");
  m.def("kmeans_centre_nbrs(Tensor cq, Tensor cprev, Tensor hn, int k, int d, Tensor(a!) delta, "
        "Tensor(b!) s, Tensor(c!) nd, Tensor(d!) nb, Tensor(e!) hnb, Tensor(f!)? ndb=None, "
        "Tensor(g!)? dnb=None) -> ()");
  m.def("kmeans_centre_bounds(Tensor cnow, Tensor cprev, int k, int d, Tensor(a!) delta, "
        "Tensor(b!) s) -> ()");
  m.def("kmeans_qsum(Tensor assign, Tensor xh, int k, Tensor(a!) Q) -> ()");
  m.def("kmeans_assign_idx(Tensor X, Tensor Cq, Tensor hn, Tensor? idx, int m, Tensor(a!) assign, "
        "Tensor[] cand, "
        "Tensor(b!)? mind=None, Tensor(c!)? mind2=None, Tensor(d!)? xh=None, Tensor(e!)? xmax=None, "
        "Tensor? m_dev=None, Tensor? a_prev=None, Tensor? tol=None, Tensor(f!)? ul=None, "
        "Tensor(h!)? changed=None, Tensor(i!)? n_changed=None, "
        "Tensor(j!)? chg_new=None, Tensor(l!)? chg_old=None, int cand_extend=1, Tensor? acl=None) -> ()");
  m.def("kmeans_bounds_init(Tensor mind, Tensor mind2, Tensor xmax, int n, Tensor(a!) ul, "
        "Tensor(c!) tol) -> ()");
  m.def("kmeans_update(Tensor(a!) C, Tensor S, Tensor cnt, Tensor(b!) Cq, Tensor(c!) hn, "
        "Tensor(d!)? shift2) -> ()");
  m.def("rmat_edges(int seed, int scale, int e_off, float a, float b, float c, bool scramble, "
        "Tensor(a!) src, Tensor(b!) dst) -> ()");
  m.def("gb_degree(Tensor ids, Tensor(a!) deg) -> ()");
  m.def("gb_keys(Tensor src, Tensor dst, Tensor? new_id, int v_lo, int v_hi, int sl, int world, int rank, "
        "int dbits, int phase, Tensor(a!)? bitmap, Tensor(b!)? counts, Tensor? offsets, int base_all, "
        "Tensor(c!)? keys, Tensor? word_prefix, Tensor? seg_start, Tensor? seg_blk0) -> ()");
  m.def("gb_sort(Tensor keys, int n, int end_bit, Tensor(a!) out, int begin_bit=0) -> ()");
  m.def("gb_run_sort(Tensor(a!) keys, int n, int lo_bits) -> Tensor");
  m.def("gb_keys_packed(Tensor packed, Tensor? new_id, int n_vertices, int dbits, Tensor(a!) keys, int src_new=0) -> ()");
  m.def("gb_relabel_src(Tensor(a!) packed, Tensor new_id, int partitioned=0) -> ()");
  m.def("gb_pack(Tensor src, Tensor dst, Tensor(a!) out) -> ()");
  m.def("gb_owner_partition(Tensor src, Tensor dst, Tensor? new_id, int sl, int world, Tensor(a!) out) -> Tensor");
  m.def("gb_owner_partition_packed(Tensor(a!) packed, Tensor? new_id, int sl, int world, Tensor(b!) out) -> Tensor");
  m.def("gb_bitmap_ids(Tensor bitmap, Tensor prefix, Tensor(a!) ids) -> ()");
  m.def("gb_bytes_to_bits(Tensor marks, Tensor(a!) bits) -> ()");
  m.def("rs_sort_error(Tensor like) -> Tensor");
  m.def("gb_deal(Tensor order, int world, int sl, int id_bits, Tensor(a!) new_id) -> ()");
  m.def("gb_rank_keys(Tensor deg, int dmax, int ibits, Tensor(a!) keys) -> ()");
  m.def("gb_degree_packed(Tensor packed, int end_bit, Tensor(a!) deg, Tensor(b!) out) -> ()");
  m.def("gb_degree_sorted(Tensor ids, int end_bit, Tensor(a!) deg) -> ()");
  m.def("gb_decode_blocks(int n) -> int", &gb_decode_blocks);   // no tensors: catch-all kernel
  m.def("gb_decode(Tensor K, int n, int shift, int dbits, Tensor blk_base, int phase, "
        "Tensor(a!)? counts, Tensor(b!)? outdeg, Tensor? offsets, Tensor(c!)? srcl, "
        "Tensor(d!)? ent_end, Tensor(e!)? ent_blk, Tensor(f!)? ent_dst) -> ()");
  m.def("gb_cell_count(Tensor ent_blk, Tensor ent_dst, int bshift, int nblk, int nbins, Tensor(a!) C) -> ()");
  m.def("gb_cell_rows(Tensor C, int nblk, int nbins, Tensor(a!) T, Tensor(b!) R) -> ()");
  m.def("gb_cell_scan(Tensor C, int nblk, int nbins, Tensor RE, Tensor RR, Tensor(a!) CM, Tensor(b!) RID) -> ()");
  m.def("gb_cell_colsum(Tensor C, int nblk, int nbins, int G, Tensor(a!) P) -> ()");
  m.def("gb_cell_place(Tensor C, Tensor CM, Tensor RID, int nblk, int nbins, int G, Tensor Poff, Tensor CI, "
        "Tensor(a!) run_delta, Tensor(b!) run_chunk, Tensor(c!) run_first) -> ()");
  m.def("gb_entry_cells(Tensor ent_blk, Tensor ent_dst, Tensor ent_end, int bshift, int nblk, int nbins, "
        "Tensor CM, Tensor RID, Tensor run_delta, Tensor RE, Tensor CI, Tensor ce_lo, Tensor tlen, int wu_e, "
        "int bin_mask, Tensor(a!) dloc, Tensor(b!) tiles, Tensor(c!) n_tiles, Tensor(d!) srcl) -> ()");
  m.def("gb_entry_flags(Tensor ent_blk, Tensor ent_dst, Tensor ent_end, int bin_shift, Tensor(a!) rs, "
        "Tensor(b!) cs, Tensor(c!) srcl) -> ()");
  m.def("gb_entry_place(Tensor ent_dst, Tensor ent_end, Tensor run_of_ent, Tensor run_delta, "
        "Tensor run_chunk, Tensor cs, Tensor ce_lo, Tensor tlen, int wu_e, int bin_mask, Tensor(a!) dloc, "
        "Tensor(b!) ts) -> ()");
  m.def("pb_spmv(Tensor srcl, Tensor tile_e, Tensor tile_ent, Tensor tile_run, Tensor wu_tile, "
        "Tensor wu_chunk, "
        "Tensor chunk_slo, Tensor chunk_ns, Tensor chunk_run, Tensor run_delta, Tensor c, "
        "Tensor(a!) val, Tensor dloc, Tensor wi_bin, Tensor wi_lo, Tensor wi_slab, int bin_width, "
        "int max_runs, Tensor(h!) bound, Tensor(b!) acc, Tensor(c!) pres, Tensor(d!) slab, "
        "Tensor split_bin, Tensor split_first, Tensor split_count, Tensor? outdeg=None, "
        "float q=0., float invN=0., int mode=0, Tensor? dangling_in=None, Tensor(e!)? r=None, "
        "Tensor(f!)? c_out=None, Tensor(g!)? dangling_out=None, int wu_lo=0, "
        "int wu_hi=2147483647, int phases=3) -> ()");
  m.def("pr_spmv(Tensor src, Tensor dstl, Tensor c, Tensor(a!) acc, Tensor(b!) pres, "
        "bool accumulate=False) -> ()");
  m.def("pr_update(Tensor acc, Tensor pres, Tensor outdeg, float q, float invN, int mode, "
        "Tensor? dangling_in, Tensor(a!) r, Tensor(b!) c, Tensor(c!)? dangling_out) -> ()");
  m.def("xgmi_buffer_bytes(int slot) -> int", &xgmi_buffer_bytes);
  m.def("xgmi_alloc(int bytes, int device) -> int", &xgmi_alloc);
  m.def("xgmi_free(int ptr) -> ()", &xgmi_free);
  m.def("xgmi_get_handle(int ptr) -> Tensor", &xgmi_get_handle);
  m.def("xgmi_open(Tensor handle, int device) -> int", &xgmi_open);
  m.def("xgmi_close(int ptr) -> ()", &xgmi_close);
  m.def("xgmi_allreduce(Tensor(a!) x, int[] bufs, int rank, int slot, Tensor(e!) epoch, Tensor(b!) err, "
        "float timeout_s, Tensor(c!)? W=None, int upd_mode=0, int upd_reg=0, float eta=0., "
        "float lam=0., float reg_alpha=0., int count_index=-1, Tensor(d!)? count_acc=None) -> ()");
  m.def("tc_step(Tensor A, Tensor Told, Tensor(a!) Tnew, Tensor(b!) count, int variant=0) -> ()");
  m.def("tcs_degree(Tensor keys, int d0, int nd, Tensor in_ptr, Tensor(a!) deg) -> ()");
  m.def("tcs_expand(Tensor(a!) keys, int d0, int nd, Tensor excl, int c_lo, int c_hi, "
        "Tensor in_ptr, Tensor in_src, Tensor(b!) table, Tensor(c!) n_keys, Tensor(d!) err) -> ()");
  m.def("tcs_insert(Tensor src, Tensor(a!) table, bool append, Tensor(b!) keys, "
        "Tensor(c!) n_keys, Tensor(d!) err) -> ()");
  m.def("spd_inverse(Tensor G, float ridge, Tensor(a!) out, Tensor(b!)? status) -> ()");
  m.def("als_solve(Tensor R, Tensor F, Tensor Ginv, Tensor(a!) out) -> ()");
  m.def("als_gram(Tensor F, Tensor(a!) G) -> ()");
  m.def("als_residual(Tensor R, Tensor U, Tensor V, Tensor(a!) out) -> ()");
  m.def("lr_set_trace(Tensor? buf) -> ()", &lr_set_trace);
  m.def("mc_pi(int seed, int stream, int offset, int n, Tensor(a!) count) -> ()");
}

TORCH_LIBRARY_IMPL(dalgo, CUDA, m) {
  m.impl("lr_grad", &lr_grad);
  m.impl("lr_eval", &lr_eval);
  m.impl("sync_update", &sync_update);
  m.impl("rows_sum", &rows_sum);
  m.impl("rows_broadcast", &rows_broadcast);
  m.impl("philox_fill", &philox_fill);
  m.impl("mc_pi", &mc_pi);
  m.impl("spd_inverse", &spd_inverse);
  m.impl("als_solve", &als_solve);
  m.impl("als_gram", &als_gram);
  m.impl("als_residual", &als_residual);
  m.impl("tc_step", &tc_step);
  m.impl("tcs_degree", &tcs_degree);
  m.impl("tcs_expand", &tcs_expand);
  m.impl("tcs_insert", &tcs_insert);
  m.impl("xgmi_allreduce", &xgmi_allreduce);
  m.impl("rmat_edges", &rmat_edges);
  m.impl("gb_degree", &gb_degree);
  m.impl("gb_keys", &gb_keys);
  m.impl("gb_sort", &gb_sort);
  m.impl("gb_run_sort", &gb_run_sort);
  m.impl("gb_keys_packed", &gb_keys_packed);
  m.impl("gb_relabel_src", &gb_relabel_src);
  m.impl("gb_pack", &gb_pack);
  m.impl("gb_owner_partition", &gb_owner_partition);
  m.impl("gb_owner_partition_packed", &gb_owner_partition_packed);
  m.impl("gb_bitmap_ids", &gb_bitmap_ids);
  m.impl("gb_bytes_to_bits", &gb_bytes_to_bits);
  m.impl("rs_sort_error", &rs_sort_error);
  m.impl("gb_deal", &gb_deal);
  m.impl("gb_rank_keys", &gb_rank_keys);
  m.impl("gb_degree_packed", &gb_degree_packed);
  m.impl("gb_degree_sorted", &gb_degree_sorted);
  m.impl("gb_decode", &gb_decode);
  m.impl("gb_cell_count", &gb_cell_count);
  m.impl("gb_cell_rows", &gb_cell_rows);
  m.impl("gb_cell_scan", &gb_cell_scan);
  m.impl("gb_cell_colsum", &gb_cell_colsum);
  m.impl("gb_cell_place", &gb_cell_place);
  m.impl("gb_entry_cells", &gb_entry_cells);
  m.impl("gb_entry_flags", &gb_entry_flags);
  m.impl("gb_entry_place", &gb_entry_place);
  m.impl("pr_spmv", &pr_spmv);
  m.impl("pb_spmv", &pb_spmv);
  m.impl("pr_update", &pr_update);
  m.impl("kmeans_assign", &kmeans_assign);
  m.impl("kmeans_update", &kmeans_update);
  m.impl("kmeans_diff", &kmeans_diff);
  m.impl("kmeans_move_sorted", &kmeans_move_sorted);
  m.impl("kmeans_filter", &kmeans_filter);
  m.impl("kmeans_sort_active", &kmeans_sort_active);
  m.impl("kmeans_centre_nbrs", &kmeans_centre_nbrs);
  m.impl("kmeans_centre_bounds", &kmeans_centre_bounds);
  m.impl("kmeans_bounds_init", &kmeans_bounds_init);
  m.impl("kmeans_qsum", &kmeans_qsum);
  m.impl("kmeans_assign_idx", &kmeans_assign_idx);
  m.impl("kmeans_accumulate_sorted", &kmeans_accumulate_sorted);   // dispatches on its output counter
}
