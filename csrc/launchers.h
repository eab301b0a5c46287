// extern "C" entry points of the gfx950 kernels (csrc/kernels/*.hip).
// Host-only header: the torch binding layer (bindings.cpp) and the native
// C++ tests include it; no torch or device code here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Fused tail of the LR gradient launch (SSGD / full-batch GD): see lr_grad.hip.
struct DalgoLrTail {
  unsigned* ticket;             // device counter, zero
  void* bufs[8];                // K11 exchange buffers (world > 1)
  int world, rank, slot;
  uint32_t* epoch_dev;          // device-resident exchange epoch (dalgo/xgmi.h)
  unsigned* err;
  double timeout_s;
  int mode, reg;                // 0 SSGD (mean + reg), 1 GD (sum)
  float eta, lam, reg_alpha;
  double* count_acc;            // += global minibatch size (optional)
  // persistent multi-step launch (nsteps > 1): device epoch counter (holds epoch_base
  // on entry, epoch_base + nsteps on exit), error word, per-wait time limit
  int nsteps;
  unsigned* epoch_ctr;
  uint32_t epoch_base;
  unsigned* perr;
  double spin_s;
  // persistent launches (optional): local rows [pool_lo, end of the segment) are not in any
  // block's static range but claimed in 2^pool_shift-row units from a device counter
  // (int32[2], one per step parity, zero on entry; each step's tail block re-arms its own)
  int* pool;
  int64_t pool_lo;
  int pool_shift;
};

// Filtered k-means iteration (kmeans.hip dalgo_kmeans_assign_idx): the K2 epilogue
// updates the Hamerly bounds and collects the rows whose cluster changed
struct DalgoKmPost {
  const unsigned long long* mcount;   // active rows (device, written by km_filter)
  const int* a_prev;                  // their cluster before this iteration
  const float* tol;                   // distance slack (device)
  float* ul;                          // [n][2]: (u, l) per row
  int* changed;
  unsigned long long* n_changed;      // zeroed by the caller
  long long cap;
  int* chg_new;                       // optional: clusters of the changed rows (aligned)
  int* chg_old;
  const int* acl;                     // optional: previous cluster of active row p (idx order)
};

// candidate-pruned K2 (dalgo_kmeans_sort_active + dalgo_km_centre_nbrs outputs)
struct DalgoKmCand {
  const int32_t* tiles;               // [T][4]: cluster, first, end position, -
  const unsigned long long* n_tiles;
  const float* hnb;
  const int32_t* nb;
  const float* nd;
  int extend;                         // stream extra chunks for tight lower bounds
  const float* ndb;                   // nullable: drift-aware lists (nd aligned with nb)
  const float* dnb;                   //           and each entry's centre shift
  const float* tau_cap;               // nullable (device): cap of the drift threshold
  int tile16;                         // tiles of <= 384 rows for the 16x16x32 form (CND)
  int64_t max_tiles;                  // capacity of the tile table (its launch grid)
};

extern "C" {

// ---- K1/K7/K10 logistic regression (lr_grad.hip)
int dalgo_lr_max_cols(int is_bf16);
void dalgo_lr_set_trace(void* buf);
hipError_t dalgo_lr_grad(const void* X, const float* y, const float* W, const int64_t* seg,
                         int64_t ld, int64_t row_offset, int D, int ldw, int has_bias, float eps,
                         uint64_t seed, uint64_t step, uint32_t thr, int full, int is_bf16,
                         int gx, int nseg, int rows_per_block, float* slab, float* gslab,
                         unsigned* cnt1, unsigned* cnt2, float* G, float* C, int S, int flags,
                         double* count_acc, const DalgoLrTail* tail, const int64_t* step_dev,
                         int64_t step_mul, hipStream_t st);
hipError_t dalgo_lr_eval(const void* X, const float* y, const float* W, const int64_t* seg,
                         int64_t ld, int D, int ldw, int has_bias, float eps, int is_bf16, int gx,
                         int nseg, int rows_per_block, unsigned long long* correct, float* loss,
                         hipStream_t st);

// ---- K8 sync/update rules (sync_update.hip)
hipError_t dalgo_sync_update(float* W, float* G, float* C, const float* center,
                             const float* S, float* Dl, double* count_acc, int n, int ld, int nrow,
                             int mode, int reg, float eta, float lam, float alpha, float reg_alpha,
                             float mu, float zeta, float beta, float inv_p, int zero_grad,
                             hipStream_t st);
hipError_t dalgo_rows_sum(const float* W, int nrow, int ld, int n, float* out, hipStream_t st);
hipError_t dalgo_rows_broadcast(float* W, int nrow, int ld, int n, const float* src,
                                hipStream_t st);

// ---- random generation + K6 Monte-Carlo pi (random.hip)
hipError_t dalgo_philox_fill(void* out, int is_bf16, int64_t nrows, int64_t D, int64_t ld,
                             int64_t row_offset, uint64_t seed, uint64_t stream, int dist, float a,
                             float b, hipStream_t st);
hipError_t dalgo_mc_pi(uint64_t seed, uint64_t stream, uint64_t offset, uint64_t n,
                       unsigned long long* count, hipStream_t st);

// ---- K2/K3 k-means (kmeans.hip)
hipError_t dalgo_kmeans_assign(const void* X, int is_bf16, int64_t n, int64_t ldx, int DP,
                               const void* Cq, const float* hn, int kpad, int* assign, float* mind,
                               double* sse, int sse_mask, hipStream_t st);
hipError_t dalgo_kmeans_move_sorted(const void* X, int is_bf16, int64_t ldx, int DP,
                                    const int32_t* changed, int64_t m, const int32_t* a_new,
                                    const int32_t* a_old, int k, int B, int seg, int* ec, int* er,
                                    int* block_counts, int64_t* cluster_start, int64_t* seg_start,
                                    int* perm, double* S, unsigned long long* cnt, const float* xh,
                                    double* Q, const unsigned long long* mdev, int64_t chunk,
                                    const int32_t* cnew, const int32_t* cold, hipStream_t st);
hipError_t dalgo_kmeans_accumulate_sorted(const void* X, int is_bf16, int64_t n, int64_t ldx, int DP,
                                          const int* assign, int k, int B, int seg, int* block_counts,
                                          int64_t* cluster_start, int64_t* seg_start, int* perm,
                                          float* S, unsigned long long* cnt, hipStream_t st);
hipError_t dalgo_kmeans_update(float* C, const float* S, const unsigned long long* cnt, int k,
                               int d, int DP, void* Cq, int is_bf16, float* hn, int kpad,
                               float* shift2, hipStream_t st);

// ---- K4 PageRank + R-MAT generator (pagerank.hip)
hipError_t dalgo_rmat(uint64_t seed, int scale, int64_t e_off, int64_t n, float a, float b, float c,
                      int do_scramble, int32_t* src, int32_t* dst, hipStream_t st);
hipError_t dalgo_pr_spmv(const int32_t* src, const int32_t* dstl, int64_t E, const float* c,
                         int64_t n_c,
                         float* acc, int32_t* pres, int accumulate, hipStream_t st);
// ---- K4b two-level propagation-blocked SpMV (pr_binned.hip)
// r == nullptr: write acc / pres; otherwise fuse the PageRank update (pr_update semantics)
hipError_t dalgo_pb_spmv(const uint16_t* srcl, const int64_t* tile_e, const int32_t* tile_ent,
                         const int32_t* tile_run, const int32_t* wu_tile, const int32_t* wu_chunk,
                         int nwu, int wu_lo, int wu_hi, int phases,
                         const int32_t* chunk_slo, const int32_t* chunk_ns,
                         const int32_t* chunk_run, const int32_t* run_delta, int nch,
                         int max_runs, int src_span, const float* c, float* val, int64_t n_val,
                         const uint16_t* dloc, const int32_t* wi_bin, const int64_t* wi_lo,
                         const int32_t* wi_slab, int nwi, int bin_width, double* bound,
                         int64_t n_local, float* acc, int32_t* pres, uint64_t* slab,
                         const int32_t* split_bin, const int32_t* split_first,
                         const int32_t* split_count, int nsplit, const int32_t* outdeg, float q,
                         float invN, int mode, const float* dang_in, float* r, float* cn,
                         float* dang_out, hipStream_t st);
hipError_t dalgo_pr_update(const float* acc, const int32_t* pres, const int32_t* outdeg, int64_t n,
                           float q, float invN, int mode, const float* dangling_in, float* r,
                           float* c, float* dangling_out, hipStream_t st);

// ---- K9 transitive closure (closure.hip)
// ---- K3 incremental form (kmeans_inc.hip)
hipError_t dalgo_km_diff(const int32_t* a_new, const int32_t* a_old, int64_t n, int32_t* changed,
                         unsigned long long* n_changed, int64_t cap, hipStream_t st);
hipError_t dalgo_km_filter(const int32_t* assign, float* ul, const float* delta,
                           const float* s, int k, int64_t n, int32_t* a_prev, int32_t* idx,
                           unsigned long long* n_active, int64_t cap, int32_t* acl,
                           hipStream_t st);
hipError_t dalgo_km_centre_bounds(const void* cnow, const void* cprev, int is_bf16, int k, int d,
                                  int DP, float* delta, float* s, hipStream_t st);
hipError_t dalgo_km_qsum(const int32_t* assign, const float* xh, int64_t n, int k, double* Q,
                         hipStream_t st);
hipError_t dalgo_kmeans_assign_idx(const void* X, int64_t m, int64_t ldx, int DP, const void* Cq,
                                   const float* hn, int kpad, const int32_t* idx, int* assign,
                                   float* mind, float* mind2, double* sse, int sse_mask, float* xh,
                                   unsigned* xmax, const DalgoKmPost* post,
                                   const DalgoKmCand* cand, hipStream_t st);
hipError_t dalgo_kmeans_sort_active(const int32_t* acl, const int32_t* idx, int64_t cap,
                                    const unsigned long long* n_active, int k, int B, int64_t chunk,
                                    int* block_counts, int64_t* cstart, int64_t* seg_start,
                                    int32_t* rows_sorted, int tile, int32_t* tiles,
                                    unsigned long long* n_tiles,
                                    int64_t max_tiles, hipStream_t st);
hipError_t dalgo_km_centre_nbrs(const void* cq, const void* cprev, const float* hn, int k, int kpad,
                                int d, int DP, float* delta, float* s, float* nd, int32_t* nb,
                                float* hnb, float* ndb, float* dnb, hipStream_t st);
hipError_t dalgo_km_bounds_init(const float* mind, const float* mind2, const unsigned* xmax,
                                int64_t n, float* ul, float* tol, hipStream_t st);

// ---- K9 sparse closure round on a device hash set (tc_sparse.hip)
hipError_t dalgo_tcs_degree(const uint64_t* keys, int64_t d0, int64_t nd, const int64_t* in_ptr,
                            int64_t* deg, hipStream_t st);
hipError_t dalgo_tcs_expand(const uint64_t* fkeys, int64_t nd, const int64_t* excl, int64_t c_lo,
                            int64_t c_hi, const int64_t* in_ptr, const int32_t* in_src,
                            uint64_t* table, uint64_t mask, uint64_t* keys,
                            unsigned long long* n_keys, uint64_t cap, unsigned* err,
                            hipStream_t st);
hipError_t dalgo_tcs_insert(const uint64_t* src, int64_t n, uint64_t* table, uint64_t mask,
                            int append, uint64_t* keys, unsigned long long* n_keys, uint64_t cap,
                            unsigned* err, hipStream_t st);
hipError_t dalgo_tc_step(const void* A, int64_t lda, const void* Told, void* Tnew, int64_t ldt,
                         int npad, int nz, int variant, unsigned long long* count, hipStream_t st);

// ---- K5 ALS ridge SPD inverse (als.hip)
hipError_t dalgo_spd_inverse(const float* G, int k, int ldg, float ridge, float* out, int ldo,
                             int* status, hipStream_t st);
int64_t dalgo_als_fq_bytes(int64_t n, int k);
int dalgo_als_nsplit(int64_t m, int64_t n, int k);
int dalgo_als_kpad(int k);
int dalgo_als_gram_blocks(int64_t n);
int64_t dalgo_als_residual_vq_bytes(int64_t n, int k);
int dalgo_als_residual_blocks(int64_t m, int64_t n);
hipError_t dalgo_als_residual(const float* R, int64_t m, int64_t n, int64_t ldr, const float* U,
                              int64_t ldu, const float* V, int64_t ldv, int k, void* Vq, double* part,
                              hipStream_t st);
hipError_t dalgo_als_gram(const float* F, int64_t n, int k, int64_t ldf, float* G, int ldg, float* part,
                          hipStream_t st);
hipError_t dalgo_als_solve(const float* R, int64_t m, int64_t n, int64_t ldr, const float* F,
                           int64_t ldf, int k, const float* Ginv, int ldg, float* out, int64_t ldo,
                           void* Fq, float* P, int nsplit, hipStream_t st);

// ---- K11 one-shot xGMI all-reduce (xgmi_allreduce.hip)
size_t dalgo_xgmi_buffer_bytes(int slot_floats);
hipError_t dalgo_xgmi_alloc(size_t bytes, void** ptr);
hipError_t dalgo_xgmi_free(void* ptr);
hipError_t dalgo_xgmi_get_handle(void* ptr, void* handle);
hipError_t dalgo_xgmi_open(const void* handle, void** ptr);
hipError_t dalgo_xgmi_close(void* ptr);
hipError_t dalgo_xgmi_allreduce(const float* in, float* out, int n, int rank, int world,
                                void* const* bufs, int slot, uint32_t* epoch_dev, unsigned* err,
                                double timeout_s, float* W, int nw, int cidx, int upd_mode,
                                int upd_reg, float eta, float lam, float reg_alpha,
                                double* count_acc, hipStream_t st);

}  // extern "C"

// ---- native PageRank adjacency build (graph_build.hip)
struct DalgoGbKeyArgs {
  int64_t v_lo, v_hi, sl;       // this rank's destination slice, slice size (owner = id / sl)
  int world, rank, dbits;       // dbits: bits of a local destination index
  const int32_t* new_id;        // nullable: degree relabeling old -> new id
  const uint32_t* bitmap;       // W > 1: remote sources with an edge into this slice
  const int64_t* word_prefix;   // W > 1: exclusive popcount prefix per bitmap word
  const int64_t* seg_start;     // [W]: local source index where owner p's segment starts
  const int64_t* seg_blk0;      // [W]: first block id of owner p's segment
  int src_new;                  // 1: the sources are already relabelled (only dst via new_id)
};
extern "C" {
hipError_t dalgo_gb_degree(const int32_t* ids, int64_t n, uint32_t* deg, hipStream_t st);
hipError_t dalgo_gb_sort32(void* tmp, size_t* tmp_bytes, const uint32_t* in, uint32_t* out, int64_t n,
                           int begin_bit, int end_bit, hipStream_t st);
int dalgo_gb_bucket_bits();
hipError_t dalgo_gb_bucket_degree(const void* sorted, int packed, int64_t n, int end_bit, int64_t* starts,
                                  int32_t* deg, hipStream_t st);
hipError_t dalgo_gb_relabel_src(uint64_t* packed, int64_t n, const int32_t* new_id, int64_t nv, int partitioned,
                                int64_t* starts, hipStream_t st);
hipError_t dalgo_gb_pack(const int32_t* src, const int32_t* dst, int64_t n, uint64_t* out, hipStream_t st);
int64_t dalgo_gb_key_blocks(int64_t n);
int64_t dalgo_gb_owner_blocks(int64_t n);
size_t dalgo_rs_ws_bytes(int64_t n, int key_bytes, int begin_bit, int end_bit);
hipError_t dalgo_rs_sort64(const uint64_t* in, uint64_t* out, uint64_t* tmp, int64_t n, int begin_bit, int end_bit,
                           void* ws, size_t ws_bytes, unsigned* err_out, hipStream_t st);
hipError_t dalgo_rs_sort32(const uint32_t* in, uint32_t* out, uint32_t* tmp, int64_t n, int begin_bit, int end_bit,
                           void* ws, size_t ws_bytes, unsigned* err_out, hipStream_t st);
hipError_t dalgo_gb_bytes_to_bits(const uint8_t* marks, int64_t nw, uint32_t* bits, hipStream_t st);
hipError_t dalgo_gb_bitmap_ids(const uint32_t* bm, int64_t nw, const int64_t* prefix, int64_t* ids,
                               hipStream_t st);
hipError_t dalgo_gb_deal(const int64_t* order, int64_t n, int world, int64_t sl, int id_bits, int32_t* new_id,
                         hipStream_t st);
hipError_t dalgo_gb_rank_keys(const int32_t* deg, int64_t n, int64_t dmax, int ibits, uint64_t* keys, hipStream_t st);
hipError_t dalgo_gb_owner_scatter(int phase, const int32_t* src, const int32_t* dst, int64_t n,
                                  const int32_t* new_id, int64_t sl, int world, uint64_t* tmp,
                                  int64_t* counts, const int64_t* offsets, uint64_t* out, hipStream_t st);
hipError_t dalgo_gb_keys(const int32_t* src, const int32_t* dst, int64_t n, const DalgoGbKeyArgs* a,
                         int phase, uint32_t* bitmap, int32_t* counts, const int64_t* offsets,
                         int64_t base_all, uint64_t* keys, const uint64_t* packed, hipStream_t st);
hipError_t dalgo_gb_sort(void* tmp, size_t* tmp_bytes, const uint64_t* in, uint64_t* out, int64_t n,
                         int begin_bit, int end_bit, hipStream_t st);
int64_t dalgo_gb_run_ws(int64_t n);
hipError_t dalgo_gb_run_sort(uint64_t* K, int64_t n, int lo_bits, int64_t* ws, hipStream_t st);
int64_t dalgo_gb_decode_blocks(int64_t n);
hipError_t dalgo_gb_decode(const uint64_t* K, int64_t n, int shift, int dbits, const int64_t* blk_base,
                           int phase, int64_t* counts, uint32_t* outdeg, const int64_t* offsets,
                           uint16_t* srcl, int64_t* ent_end, int32_t* ent_blk, int32_t* ent_dst,
                           hipStream_t st);
hipError_t dalgo_gb_entry_flags(const int32_t* ent_blk, const int32_t* ent_dst, const int64_t* ent_end,
                                int64_t nent, int bin_shift, uint8_t* rs, uint8_t* cs, uint16_t* srcl,
                                hipStream_t st);
hipError_t dalgo_gb_cells(int phase, const int32_t* ent_blk, const int32_t* ent_dst, int64_t nent, int bshift,
                          int nblk, int nbins, int32_t* C, int64_t* T, int64_t* R, const int64_t* RE,
                          const int64_t* RR, int32_t* CM, int32_t* RID, int G, int64_t* P, const int64_t* Poff,
                          const int32_t* CI, int64_t nruns, int32_t* run_delta, int32_t* run_chunk,
                          int64_t* run_first, hipStream_t st);
hipError_t dalgo_gb_entry_cells(const int32_t* ent_blk, const int32_t* ent_dst, const int64_t* ent_end, int64_t nent,
                                int bshift, int nblk, int nbins, const int32_t* CM, const int32_t* RID,
                                const int32_t* run_delta, int64_t nruns, const int64_t* RE, const int32_t* CI,
                                const int64_t* ce_lo, const int64_t* tlen, int64_t nch, int64_t wu_e, int bin_mask,
                                int16_t* dloc, int64_t ndloc, int32_t* tiles, unsigned long long* n_tiles,
                                int64_t tile_cap, uint16_t* srcl, int64_t nsrcl, hipStream_t st);
hipError_t dalgo_gb_entry_place(const int32_t* ent_dst, const int64_t* ent_end, int64_t nent,
                                const int32_t* run_of_ent, const int32_t* run_delta, const int32_t* run_chunk,
                                const uint8_t* cs, const int64_t* ce_lo, const int64_t* tlen, int64_t wu_e,
                                int bin_mask, int16_t* dloc, uint8_t* ts, hipStream_t st);
}
