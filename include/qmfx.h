/*
 * qmfx.h: C ABI of the MI355X (gfx950) implicit-feedback MF engine.
 *
 * This is the device layer under the drop-in qmf::Engine API (qmf_amd/host/qmf/).  It
 * replaces the reference's in-process CPU hot path (taozhijiang/qmf, paths relative to the
 * reference root):
 *
 *   qmf/wals/WALSEngine.cpp:165-218  WALSEngine::iterate           -> qmfx_wals_half
 *   qmf/wals/WALSEngine.cpp:246-264  WALSEngine::computeXtX        -> inside qmfx_wals_half
 *   qmf/wals/WALSEngine.cpp:266-310  WALSEngine::updateFactorsForOne -> inside qmfx_wals_half
 *   qmf/Matrix.cpp:81-96             linearSymmetricSolve (dsysv_) -> inside qmfx_wals_half
 *   qmf/wals/WALSEngine.cpp:130-163  groupSignals / sortDataset    -> qmfx_group_signals (device
 *   qmf/utils/IdIndex.cpp:21-31      IdIndex (id -> idx)              sort + CSR build), qmfx_get_ids;
 *                                                                     qmfx_upload_csr / qmfx_gen_synthetic
 *   qmf/FactorData.h:55-100          FactorData::setFactors        -> qmfx_set_factors / qmfx_fill_uniform
 *   qmf/bpr/BPREngine.cpp:146-220    BPREngine::optimize / update  -> qmfx_bpr_epoch / qmfx_bpr_apply
 *   qmf/bpr/BPREngine.cpp:246-274    BPREngine::evaluate (loss)    -> qmfx_bpr_eval
 *   distributed/ (TCP broadcast + bucket gather)                   -> qmfx_dist_init + qmfx_wals_half
 *                                                                     (RCCL all-gather over xGMI)
 *
 * Conventions: plain pointers and sizes, no C++ or torch types.  Host buffers are copied;
 * device buffers are owned by the context.  Every call returns 0 on success or a negative
 * code, with a message from qmfx_last_error() (thread-local).  The reference aborts on
 * errors (glog CHECK); the C++ wrapper converts a non-zero status into that abort.  One
 * caller thread per context.  Sides: 0 = users, 1 = items.  Factors cross the ABI as
 * row-major float64 n×k (the reference's Double = double, qmf/Types.h:24); on the device
 * they are stored in the context precision (32 or 64) with rows padded to a multiple of 16.
 */
#ifndef QMFX_H_
#define QMFX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qmfx_ctx qmfx_ctx;

#define QMFX_USERS 0
#define QMFX_ITEMS 1

/* ---- library / context ---------------------------------------------------------------- */
const char* qmfx_last_error(void);
int qmfx_version(void);
int qmfx_device_count(int* count);

/* precision: 32 or 64.  nfactors: the reference's --nfactors (WALSConfig/BPRConfig). */
int qmfx_create(qmfx_ctx** out, int device, int precision, int nfactors);
int qmfx_destroy(qmfx_ctx* ctx);
int qmfx_sync(qmfx_ctx* ctx);
int qmfx_set_shape(qmfx_ctx* ctx, int64_t nusers, int64_t nitems);
int qmfx_get_shape(qmfx_ctx* ctx, int64_t* nusers, int64_t* nitems, int64_t* nnz);

/* ---- interactions (WALSEngine.cpp:130-163) --------------------------------------------- */
/* CSR of `side`: rowptr[n_side+1], colidx[nnz] = row index on the other side, values[nnz]. */
int qmfx_upload_csr(qmfx_ctx* ctx, int side, const int64_t* rowptr, const int32_t* colidx,
                    const double* values, int64_t nnz);
/* Device ingest of raw interactions (WALSEngine::init / groupSignals / sortDataset,
 * WALSEngine.cpp:37-69, 130-163; IdIndex.cpp:21-31).  `records` holds nnz packed 24-byte
 * records in the reference's DatasetElem layout (DatasetReader.h:29-33: int64 userId,
 * int64 itemId, double value), in file order.  Sets the shape (distinct users, items) and
 * builds both CSR orientations on the device: rows in ascending-id order, entries by
 * ascending column id, duplicate (u, i) pairs kept in input order.  nnz < 2^31. */
int qmfx_group_signals(qmfx_ctx* ctx, const void* records, int64_t nnz, int64_t* nusers,
                       int64_t* nitems);
/* Ascending distinct ids of `side` (n_side values; idx = position), after
 * qmfx_group_signals. */
int qmfx_get_ids(qmfx_ctx* ctx, int side, int64_t* ids);
/* Device-generated synthetic matrix: ~nnz uniform unique (u, i) pairs,
 * w in 1..5, both orientations built on the device.  *nnz_out = unique pairs kept. */
int qmfx_gen_synthetic(qmfx_ctx* ctx, int64_t nusers, int64_t nitems, int64_t nnz,
                       uint64_t seed, int64_t* nnz_out);
/* Skewed variant (SURVEY.md §8(d) "Zipf(s=1.0) item popularity", power-law rows): `ndraws`
 * (user uniform, item rank ~ continuous Zipf(zipf_s)) draws, duplicates dropped; zipf_s = 0
 * is qmfx_gen_synthetic.  *nnz_out = unique pairs kept. */
int qmfx_gen_synthetic_zipf(qmfx_ctx* ctx, int64_t nusers, int64_t nitems, int64_t ndraws,
                            uint64_t seed, double zipf_s, int64_t* nnz_out);
/* dst takes src's interactions (shape, id tables and both CSR orientations, copied device to
 * device: over xGMI between GPUs) instead of building them again: one qmfx_group_signals for
 * an n-GPU engine, then an import per peer before qmfx_dist_init_all shards them.  Both
 * contexts must have the same precision; src must not be sharded and dst must not have been
 * through qmfx_dist_init[_all].  src's stream is synchronised before the copies. */
int qmfx_import_signals(qmfx_ctx* dst, qmfx_ctx* src);
/* Copies a side's CSR back to the host (e.g. for CPU baselines on the same data).  values are
 * returned in double, exactly as the device holds them (an fp32 context's values widened). */
int qmfx_download_csr(qmfx_ctx* ctx, int side, int64_t* rowptr, int32_t* colidx,
                      double* values);

/* ---- factors (FactorData.h) ------------------------------------------------------------- */
int qmfx_set_factors(qmfx_ctx* ctx, int side, const double* rowmajor);
int qmfx_get_factors(qmfx_ctx* ctx, int side, double* rowmajor);
int qmfx_fill_uniform(qmfx_ctx* ctx, int side, double bound, uint64_t seed);

/* ---- WALS (WALSEngine.cpp:165-218) -------------------------------------------------------
 * Solves every row of `side` with the other side fixed: X ← 0, G = YᵀY, per row
 * A = G + Σ αv yyᵀ + λI, b = Σ (1+αv) y, x = A⁻¹b.  *loss_sum receives Σ over solved rows of
 * Σ(1+αv) + xᵀ(A−λI)x − 2xᵀb (divide by nusers·nitems for the reference's printed loss).
 * With a distributed context the local row range is solved and the factor matrix is
 * all-gathered over RCCL before returning; the loss is then the global sum. */
int qmfx_wals_half(qmfx_ctx* ctx, int side, double alpha, double lambda, double* loss_sum);
/* Number of rows whose system the Cholesky kernels could not factor in the last half (a
 * non-positive pivot: some 1 + α·v < 0, λ ≤ 0, or fp32 rounding on a nearly singular
 * system); their indices go to rows[] (up to cap).  qmfx_wals_half has already re-solved
 * them on the device in fp64 with partial pivoting (dsysv_'s role, Matrix.cpp:81-96) before
 * the half's all-gather, and failed with -6 if one was exactly singular (CHECK(info == 0),
 * Matrix.cpp:94). */
int qmfx_wals_failed_rows(qmfx_ctx* ctx, int64_t* rows, int64_t cap, int64_t* count);
/* The row plan of `side` on this rank (11 counts): [0..7] whitened rows in the n×n buckets
 * n ≤ 16·(i+1) (used when λ > 0), [8] direct k×k rows, [9] split-K heavy rows (more than
 * QMFX_HEAVY_MIN signals, default 16384; every k: the one-wave direct tilings and the multi-wave
 * k > 128 kernel), [10] their
 * segments (QMFX_SEG_LEN signals each, default 8192). */
int qmfx_row_classes(qmfx_ctx* ctx, int side, int64_t* counts);
/* Per-row loss terms of the last half (n_side values; the sum is *loss_sum). */
int qmfx_wals_row_losses(qmfx_ctx* ctx, double* out);
/* One row's system as the reference forms it (updateFactorsForOne, WALSEngine.cpp:266-299),
 * built on the device in fp64 from the current fixed side: A (k×k row-major, λ included),
 * b and Σ(1 + αv). */
int qmfx_wals_row_system(qmfx_ctx* ctx, int side, int64_t row, double alpha, double lambda,
                         double* A, double* b, double* csum);
int qmfx_wals_set_row(qmfx_ctx* ctx, int side, int64_t row, const double* x);

/* ---- BPR (BPREngine.cpp:146-274) ---------------------------------------------------------
 * Positives in data order as (user idx, item idx) (BPREngine::init :65-82).  Builds the
 * per-user sorted positive lists used for negative rejection. */
int qmfx_bpr_set_positives(qmfx_ctx* ctx, const int64_t* users, const int64_t* items,
                           int64_t npos);
int qmfx_bpr_set_biases(qmfx_ctx* ctx, const double* bias);  /* nitems values */
int qmfx_bpr_get_biases(qmfx_ctx* ctx, double* bias);
/* One Hogwild epoch over all positives × num_neg sampled negatives, visiting positives in
 * a seed-dependent permuted order when shuffle != 0. */
int qmfx_bpr_epoch(qmfx_ctx* ctx, uint64_t seed, int num_neg, double lr, double bias_lambda,
                   double user_lambda, double item_lambda, int use_biases, int shuffle);
/* Applies the given (u, p, n) triplets in order with one wave (exact update order). */
int qmfx_bpr_apply(qmfx_ctx* ctx, const int64_t* triplets, int64_t n, double lr,
                   double bias_lambda, double user_lambda, double item_lambda, int use_biases);
/* Σ log(1+exp(−x̂)) over triplets (host array, uploaded and cached per `slot` 0/1). */
int qmfx_bpr_eval(qmfx_ctx* ctx, int slot, const int64_t* triplets, int64_t n, int use_biases,
                  double* loss_sum);

/* ---- test-set evaluation (Engine::computeTestScores Engine.cpp:73-96 + Metrics.cpp:27-164)
 * The device replaces the dense n_test × n_items score matrix by the statistics every
 * reference metric (mse, auc, ap, p@k, r@k) is a function of.
 * qmfx_eval_set_labels: test users (user idx, ntest of them) and their labelled items as a
 * CSR over the test slots (rowptr[ntest+1], item idx, label value; zero labels may be left
 * out).  Labels > 0 are the positives.  Cached on the context until the next call. */
int qmfx_eval_set_labels(qmfx_ctx* ctx, int64_t ntest, const int64_t* users,
                         const int64_t* rowptr, const int64_t* items, const double* values);
/* Scores the current factors (score = [bias_i +] <u, q_i>, the reference's double, bit for
 * bit; use_biases adds the context's item biases) and returns
 *   label_scores[rowptr[ntest]]  the score of every labelled pair, in CSR order;
 *   above[npos]                  per positive (labelled pair with value > 0, in CSR order):
 *                                the number of items scored strictly higher;
 *   sq_sum[ntest]                Σ over all items of score². */
int qmfx_eval_ranks(qmfx_ctx* ctx, int use_biases, double* label_scores, int64_t* above,
                    double* sq_sum);

/* ---- multi-GPU (one process per GPU; RCCL over xGMI) -------------------------------------- */
int qmfx_rccl_unique_id(uint8_t* id128);
/* Joins the RCCL communicator (id128 from rank 0's qmfx_rccl_unique_id), takes this rank's
 * nnz-balanced row range of both sides, rebuilds the row buckets and keeps only this rank's
 * signals on the device.  id128 = NULL sets up the partition without a communicator: each
 * half then solves only this rank's rows and exchanges nothing (tests of the partition). */
int qmfx_dist_init(qmfx_ctx* ctx, int rank, int world, const uint8_t* id128);
/* One process driving n GPUs (the drop-in C++ engine's --ngpus): ctxs[i] (each on its own
 * device, all with the same data and factors) become ranks 0..n-1 of one RCCL clique
 * (ncclCommInitAll), partitioned and sharded as qmfx_dist_init does.  Fails when two
 * contexts share a device or a device is not visible. */
int qmfx_dist_init_all(qmfx_ctx* const* ctxs, int n);
/* qmfx_wals_half over the n contexts of one qmfx_dist_init_all, from one thread: every
 * context's solves are enqueued piece by piece and each piece's all-gather of all ranks is
 * one RCCL group, overlapping the next piece's solves.  *loss_sum: the global sum. */
int qmfx_wals_half_multi(qmfx_ctx* const* ctxs, int n, int side, double alpha, double lambda,
                         double* loss_sum);
/* nnz-balanced contiguous row range owned by `rank` (host-only helper, no GPU needed). */
int qmfx_partition_rows(const int64_t* rowptr, int64_t nrows, int world, int rank,
                        int64_t* begin, int64_t* end);
/* The all-gather schedule of a half-epoch over `world` ranks with `npieces` solve pieces
 * per rank (host only, no device): pbounds[r·(npieces+1) + j] .. [.. + j + 1] is the row
 * range rank r solves as its piece j and then broadcasts to every rank (an empty range is
 * skipped).  Ranks own contiguous nnz-balanced ranges in ascending row order (the
 * reference's bucket split, distributed/scheduler/RunOneTask.cpp:160-243). */
int qmfx_dist_plan(const int64_t* rowptr, int64_t nrows, int world, int npieces,
                   int64_t* pbounds);

/* ---- measurement -------------------------------------------------------------------------- */
/* HIP-event time of the row-solve kernel launches (on the context stream) since reset. */
int qmfx_solve_kernel_stats(qmfx_ctx* ctx, double* total_ms, int64_t* launches,
                            double* flops, double* bytes);
/* Per kernel class since reset: 0 = direct row kernel, 1 = whitened row kernels (row solve
 * + unwhitening GEMM), 2 = whole half-epoch (all kernels, collectives included).  flops /
 * bytes are the algorithmic work of that class (SURVEY.md §8(d) accounting). */
int qmfx_kernel_stats(qmfx_ctx* ctx, int cls, double* total_ms, int64_t* launches,
                      double* flops, double* bytes);
/* qmfx_kernel_stats restricted to the halves that solved `side` (0 users, 1 items): a class's
 * launches differ by side, so the per-launch time of the class's large launch is read here. */
int qmfx_kernel_stats_side(qmfx_ctx* ctx, int cls, int side, double* total_ms, int64_t* launches,
                           double* flops, double* bytes);
int qmfx_reset_stats(qmfx_ctx* ctx);
/* Multi-rank halves (qmfx_dist_init with a communicator) that solved `side`, since reset:
 * exchange_ms = Σ time of the per-piece broadcast groups on the collective stream (HIP events
 * there; a piece's group starts when its solves are done and the previous group finished);
 * exposed_ms = Σ from the last piece's solves done to its broadcasts done (the exchange not
 * hidden behind solves); solve_ms = Σ row-solve time of the pieces.  Zero on one rank. */
int qmfx_exchange_stats(qmfx_ctx* ctx, int side, double* exchange_ms, double* exposed_ms,
                        double* solve_ms, int64_t* halves);
/* The last qmfx_bpr_epoch's launch plan: concurrent waves (Hogwild width) and whether the user
 * row's change was added atomically (1: a heavy user makes concurrent holders likely) or
 * stored (0). */
int qmfx_bpr_plan(qmfx_ctx* ctx, int* waves, int* atomic_user);
/* "" for the product library; a timing-variant build (tools/build_variant.sh) returns its
 * compile flags, so a variant loaded through QMFX_LIB is never taken for the product. */
const char* qmfx_build_variant(void);

/* ---- self tests ------------------------------------------------------------------------------ */
/* C(16×16) = A(16×4)·B(4×16) through the kernels' MFMA operand/accumulator maps. */
int qmfx_selftest_mfma(int device, int precision, const double* A, const double* B, double* C);

#ifdef __cplusplus
}
#endif
#endif /* QMFX_H_ */
