// Kernel argument structs and host launchers shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace qmfx {

// Per-slot row descriptor of a side's processing order (built once with the buckets):
// the CSR range of the row and the row itself, so a persistent row kernel reaches a row's
// signals in one dependent load instead of order → rowptr → signals.
struct RowDesc {
  int64_t beg;
  int32_t n;
  int32_t row;
};

template <typename T>
struct SolveArgs {
  const int64_t* rowptr;  // CSR of the side being solved
  const int32_t* col;     // column = row index on the fixed side
  const T* val;           // raw interaction value v
  const T* Y;             // fixed-side factors [nY][KP]
  const T* G;             // YᵀY, KP×KP
  T* X;                   // solved-side factors [nX][KP]
  double* rowloss;        // [nX]
  int32_t* status;        // [nX] non-zero: non-positive pivot (system not SPD)
  const int64_t* order;   // optional processing order (nullptr = identity)
  int64_t row_begin;      // first slot of the order handled by this launch
  int64_t nrows;          // number of rows (blocks)
  T alpha;
  T lambda;
  int k;                  // real number of factors (≤ KP)
  const RowDesc* desc;    // per-slot descriptors (persistent row kernels; indexed like order)
  const T* Gimg;          // direct kernel: G + λI as per-lane accumulator tiles (gimg_kernel)
  uint64_t* trace;        // diagnostics only (QMFX_TRACE): per-slot phase timestamps
  int32_t zrow;           // whitened kernel: index of an all-zero row of Y (padding signals)
  // Heavy rows (split-K, direct kernel only): rows with more than `heavy_min` signals are cut
  // into segments; seg_mode 1 accumulates one segment's Gram (slot = segment) into
  // part/partb/partc, heavy_reduce_kernel sums a row's segments in fp64 (fixed order) into
  // its first segment's slot, and seg_mode 2 solves the row from there (desc.beg = that
  // slot, desc.n = 0).  seg_mode 0 is the ordinary row solve.
  int seg_mode;
  T* part;                // [segments][NTT·256] accumulator-tile images
  T* partb;               // [segments][KP] right-hand sides
  double* partc;          // [segments][2]: Σc, negative-weight flag
};

// Heavy-row partial reduction: for heavy rows h0 .. h0+nh, segments hseg[h] .. hseg[h+1] are
// summed (fp64, fixed order) with G + λI into segment hseg[h]'s slot.
hipError_t launch_heavy_reduce(float* part, float* partb, double* partc, const int64_t* hseg,
                               int64_t h0, int64_t nh, const float* Gimg, int nt, hipStream_t s);
hipError_t launch_heavy_reduce(double* part, double* partb, double* partc, const int64_t* hseg,
                               int64_t h0, int64_t nh, const double* Gimg, int nt, hipStream_t s);

// The same for the multi-wave k > 128 tilings (wals_big.hip): builds G + λI's tile image in
// Gimg first (runtime tile count, no column permutation).
hipError_t launch_heavy_reduce_big(float* part, float* partb, double* partc, const int64_t* hseg,
                                   int64_t h0, int64_t nh, const float* G, float* Gimg, int nt,
                                   int k, double lambda, hipStream_t s);
hipError_t launch_heavy_reduce_big(double* part, double* partb, double* partc, const int64_t* hseg,
                                   int64_t h0, int64_t nh, const double* G, double* Gimg, int nt,
                                   int k, double lambda, hipStream_t s);

// Per-row kernels take one workgroup per row (slot = row_begin + blockIdx.x).  A launch's
// total thread count must fit 32 bits (10M rows × 512 threads does not), so rows go out in
// chunks of at most 2^31 / threads workgroups.
// (QMFX_ROW_CHUNK lowers the chunk for the tests.)
template <typename T, typename F>
hipError_t launch_row_chunks(const SolveArgs<T>& a, int threads, F launch) {
  int64_t cap = ((int64_t)1 << 31) / threads;
  if (const char* e = std::getenv("QMFX_ROW_CHUNK"))
    if (std::atoll(e) > 0 && std::atoll(e) < cap) cap = std::atoll(e);
  for (int64_t done = 0; done < a.nrows; done += cap) {
    SolveArgs<T> c = a;
    c.row_begin = a.row_begin + done;
    c.nrows = a.nrows - done < cap ? a.nrows - done : cap;
    launch(c);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// G + λI (padding diagonal 1) → the direct row kernel's accumulator-tile image
hipError_t launch_gimg(const float* G, int nt, int k, double lambda, float* img, hipStream_t s);
hipError_t launch_gimg(const double* G, int nt, int k, double lambda, double* img, hipStream_t s);

hipError_t launch_wals_direct(const SolveArgs<float>& a, int nt, hipStream_t s);
hipError_t launch_wals_direct(const SolveArgs<double>& a, int nt, hipStream_t s);
// seg_mode 1 / 2 of the direct kernel (wals_heavy.hip; launch_wals_direct forwards there)
hipError_t launch_wals_heavy(const SolveArgs<float>& a, int nt, hipStream_t s);
hipError_t launch_wals_heavy(const SolveArgs<double>& a, int nt, hipStream_t s);
// multi-wave row solve and tiled YᵀY for large factor counts (wals_big.hip; nt 5..16)
hipError_t launch_wals_big(const SolveArgs<float>& a, int nt, hipStream_t s);
hipError_t launch_wals_big(const SolveArgs<double>& a, int nt, hipStream_t s);
hipError_t launch_gram_big(const float* Y, int64_t n, int nt, float* G, double* partial,
                           int max_blocks, hipStream_t s);
hipError_t launch_gram_big(const double* Y, int64_t n, int nt, double* G, double* partial,
                           int max_blocks, hipStream_t s);
// whitened-row buckets: n ≤ 16·NTN, NTN = 1..kMaxNTN (NTN > 4 only for fp32 k = 256)
constexpr int kMaxNTN = 8;
hipError_t launch_wals_woodbury(const SolveArgs<float>& a, int nt, int ntn, hipStream_t s);
hipError_t launch_wals_woodbury(const SolveArgs<double>& a, int nt, int ntn, hipStream_t s);
hipError_t launch_whiten(const float* in, float* out, const int64_t* order, int64_t nrows,
                         int nt, const float* Linv, double* rowloss, double lambda,
                         bool unwhiten, hipStream_t s);
hipError_t launch_whiten(const double* in, double* out, const int64_t* order, int64_t nrows,
                         int nt, const double* Linv, double* rowloss, double lambda,
                         bool unwhiten, hipStream_t s);
// scratch: KP·(KP+1) doubles, used when KP > 128 (the fp64 matrix does not fit LDS)
hipError_t launch_chol_inv(const float* G, int nt, int k, double lambda, float* Linv,
                           int32_t* status, double* scratch, hipStream_t s);
hipError_t launch_chol_inv(const double* G, int nt, int k, double lambda, double* Linv,
                           int32_t* status, double* scratch, hipStream_t s);
hipError_t launch_gram(const float* Y, int64_t n, int nt, float* G, double* partial,
                       int max_blocks, hipStream_t s);
hipError_t launch_gram(const double* Y, int64_t n, int nt, double* G, double* partial,
                       int max_blocks, hipStream_t s);
hipError_t launch_sum_f64(const double* x, int64_t n, double* out, hipStream_t s);
hipError_t launch_mfma_selftest_f32(const float* A, const float* B, float* C, hipStream_t s);
hipError_t launch_mfma_selftest_f64(const double* A, const double* B, double* C,
                                    hipStream_t s);

// Pivoted fp64 re-solve of the rows flagged in `status` (fallback.hip)
template <typename T>
struct FallbackArgs {
  const int64_t* rowptr;
  const int32_t* col;
  const T* val;
  const T* Y;             // fixed side [nY][kp]
  const T* G;             // YᵀY of the fixed side, kp×kp
  T* X;                   // solved side [nX][kp]
  double* rowloss;
  int32_t* status;        // in: non-zero = flagged; out: 1 re-solved, 2 singular
  const RowDesc* desc;    // slot → row
  int64_t slot_begin, nslots;
  double alpha, lambda;
  int k, kp;
  double* scratch;        // FB_MAX_GRID × (kp + 3) × kp doubles
  unsigned long long* counters;  // [0] rows re-solved, [1] singular rows
};
constexpr int FB_MAX_GRID = 64;
hipError_t launch_wals_fallback(const FallbackArgs<float>& a, hipStream_t s);
hipError_t launch_wals_fallback(const FallbackArgs<double>& a, hipStream_t s);
// out: A (k×k row-major, λ included), then b (k), then Σc — one row's system
hipError_t launch_wals_system(const FallbackArgs<float>& a, int64_t beg, int64_t end, double* out,
                              hipStream_t s);
hipError_t launch_wals_system(const FallbackArgs<double>& a, int64_t beg, int64_t end,
                              double* out, hipStream_t s);

// out[0] = *loss, out[1..2] = fb[0..1], out[3] = *chol (0 when chol is null)
hipError_t launch_half_status(const double* loss, const unsigned long long* fb,
                              const int32_t* chol, double* out, hipStream_t s);

// BPR (bpr.hip)
template <typename T>
struct BprArgs {
  T* U;                    // [nu][KP]
  T* I;                    // [ni][KP]
  T* bias;                 // [ni] or nullptr
  const int64_t* pos_user; // positives in data order
  const int32_t* pos_item;
  int64_t npos;
  const int64_t* urowptr;  // user -> sorted positive items (rejection set)
  const int32_t* uitems;
  int64_t nitems;
  int num_neg;
  uint64_t seed;
  uint64_t perm_a, perm_b; // epoch permutation of positives: idx = (a*i + b) mod npos
  T lr, bias_lambda, user_lambda, item_lambda;
  int use_biases;
  int kp;                  // row stride (padded factors)
  int32_t* bad;            // set to 1 if a derivative was not finite
  int waves;               // concurrent waves of the epoch kernel (Hogwild width)
  int atomic_user;         // 1: add the user row's net change atomically (heavy users)
};

hipError_t launch_bpr_epoch_f32(const BprArgs<float>& a, int kp, hipStream_t s);
hipError_t launch_bpr_epoch_f64(const BprArgs<double>& a, int kp, hipStream_t s);
hipError_t launch_bpr_apply_f32(const BprArgs<float>& a, const int64_t* trip, int64_t n,
                                int kp, hipStream_t s);
hipError_t launch_bpr_apply_f64(const BprArgs<double>& a, const int64_t* trip, int64_t n,
                                int kp, hipStream_t s);
hipError_t launch_bpr_eval_f32(const float* U, const float* I, const float* bias,
                               const int64_t* trip, int64_t n, int kp, int use_biases,
                               double* partial, double* out, hipStream_t s);
hipError_t launch_bpr_eval_f64(const double* U, const double* I, const double* bias,
                               const int64_t* trip, int64_t n, int kp, int use_biases,
                               double* partial, double* out, hipStream_t s);

// Synthetic data + CSR build (data.hip)
hipError_t launch_synth_keys(uint64_t* keys, int64_t n, uint64_t space, uint64_t seed,
                             hipStream_t s);
// uniform user, Zipf(zipf_s) item popularity (keys u·nitems + i, duplicates possible)
hipError_t launch_synth_keys_zipf(uint64_t* keys, int64_t n, uint64_t nusers, uint64_t nitems,
                                  double zipf_s, uint64_t seed, hipStream_t s);
hipError_t build_csr_from_sorted_keys(const uint64_t* keys, int64_t nnz, int64_t nrows,
                                      uint64_t ncols, int64_t* rowptr, int32_t* col,
                                      hipStream_t s);
hipError_t launch_transpose_keys(const uint64_t* keys, int64_t nnz, uint64_t ncols,
                                 uint64_t nrows, uint64_t* out, hipStream_t s);
hipError_t launch_synth_values_any(const uint64_t* keys, int64_t n, uint64_t div,
                                   uint64_t nitems, int user_major, uint64_t seed, void* val,
                                   int prec, hipStream_t s);
hipError_t sort_unique_keys(uint64_t* keys, uint64_t* scratch, int64_t n, int64_t* n_out,
                            int end_bit, hipStream_t s);
hipError_t sort_keys(uint64_t* keys, uint64_t* scratch, int64_t n, int end_bit, hipStream_t s);
// Device ingest (ingest.hip): packed 24-byte (user id, item id, value) records already on
// the device → ascending id tables and both CSR orientations (buffers allocated by the
// callee, owned by the caller; val in the context precision).
struct IngestOut {
  int64_t n[2] = {0, 0};                 // distinct users, items
  int64_t* ids[2] = {nullptr, nullptr};  // ascending ids
  int64_t* rowptr[2] = {nullptr, nullptr};
  int32_t* col[2] = {nullptr, nullptr};
  void* val[2] = {nullptr, nullptr};
};
hipError_t group_records(const void* d_records, int64_t n, int prec, IngestOut& out,
                         hipStream_t s);

hipError_t launch_fill_uniform_f32(float* X, int64_t n, int kp, int k, double bound,
                                   uint64_t seed, hipStream_t s);
hipError_t launch_fill_uniform_f64(double* X, int64_t n, int kp, int k, double bound,
                                   uint64_t seed, hipStream_t s);

// Test-set ranking statistics (eval.hip)
template <typename T>
struct EvalArgs {
  const T* U;               // [nu][kp]
  const T* I;               // [ni][kp]
  const T* bias;            // [ni] item biases or nullptr
  const int64_t* users;     // [ntest] test user rows
  int64_t ntest;
  int64_t nitems;
  int k, kp;
  // labelled (user, item) pairs, grouped by test slot
  const int32_t* lab_slot;  // [nlab]
  const int64_t* lab_item;  // [nlab]
  const int64_t* lab_pidx;  // [nlab] index into the positives, or -1 (label <= 0)
  int64_t nlab;
  double* lab_score;        // [nlab] out
  // positives (label > 0), grouped by test slot: pptr[t]..pptr[t+1]
  const int64_t* pptr;      // [ntest + 1]
  double* pscore;           // [npos] scores (written by the label pass)
  unsigned long long* above;  // [npos] items scored strictly higher (zeroed by the caller)
  double* sq_part;          // [eval_chunks(ntest, nitems)][ntest] Σ score² per item chunk
  double* udbl;             // [eval_user_rows(ntest)][k] scratch: one batch's test users' rows
  int64_t chunk;            // set by the launcher
  int64_t t_base;           // set by the launcher: first test user of the current batch
};
int64_t eval_chunks(int64_t ntest, int64_t nitems);
int64_t eval_user_rows(int64_t ntest);
int64_t eval_batch_groups();
hipError_t launch_eval_ranks(const EvalArgs<float>& a, hipStream_t s);
hipError_t launch_eval_ranks(const EvalArgs<double>& a, hipStream_t s);

}  // namespace qmfx
