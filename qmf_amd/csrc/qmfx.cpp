// Host side of the qmfx C ABI (include/qmfx.h): context, device buffers, orchestration of
// the WALS half-epoch and BPR epoch kernels, RCCL data path for multi-GPU.
#include "../../include/qmfx.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"

using namespace qmfx;

namespace {

thread_local std::string g_err;

int fail(const std::string& m, int code = -1) {
  g_err = m;
  return code;
}

#define HIPCHK(x)                                                                     \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_), -2); \
  } while (0)

#define NCCLCHK(x)                                                                      \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) return fail(std::string(#x) + ": " + ncclGetErrorString(r_), -3); \
  } while (0)

#define QMFX_MAX_PIECES 16
constexpr int kHalfStatus = 1024;  // dsum offset of the end-of-half status block

struct SideBuf {
  int64_t n = 0;
  int64_t nnz = 0;
  int64_t* rowptr = nullptr;
  int32_t* col = nullptr;
  void* val = nullptr;
  void* F = nullptr;
  std::vector<int64_t> h_rowptr;
  std::vector<int64_t> h_ids;           // ascending ids (only when built by qmfx_group_signals)
  int64_t rbeg = 0, rend = 0;           // rows solved by this rank
  // With several ranks the CSR keeps only this rank's rows (signals rowptr[rbeg] ..
  // rowptr[rend]); col/val point at that shard and shard_off = rowptr[rbeg], so kernels
  // index them with the global rowptr through colp()/valp().
  int64_t shard_off = 0;
  bool sharded = false;
  std::vector<int64_t> bounds;          // per-rank row boundaries (world+1)
  // Row buckets of this rank (device list `order`): [whitened n≤16 | ≤32 | … | ≤16·kMaxNTN |
  // direct rows, heaviest first].  wb[i]..wb[i+1] = whitened bucket NTN = i+1;
  // wb[kMaxNTN]..n_ord = direct.  nnz per bucket class for the roofline accounting.
  int64_t* d_order = nullptr;
  RowDesc* d_desc = nullptr;  // per slot of d_order: CSR range and row
  int64_t wb[kMaxNTN + 1] = {};
  int64_t n_ord = 0;
  double nnz_w = 0, nnz_d = 0;
  double flops_w = 0;  // algorithmic flops of the whitened rows per half (see qmfx_wals_half)
  bool buckets_valid = false;
  // Solve pieces: this rank's rows split into nnz-balanced contiguous sub-ranges, each with
  // its own section of the order list laid out as above (ord + wb[i] relative).  With
  // several ranks, piece j of every rank is all-gathered while piece j+1 is solved.
  struct Piece {
    int64_t rb = 0, re = 0, ord = 0, n_ord = 0;
    int64_t wb[kMaxNTN + 1] = {};
    // split-K heavy rows (the first nh direct slots): heavy indices h0 .. h0+nh, segments
    // s0 .. s0+ns (of the side's d_seg / d_heavy / d_hseg lists)
    int64_t nh = 0, h0 = 0, s0 = 0, ns = 0;
  };
  std::vector<Piece> pieces;
  std::vector<int64_t> pbounds;  // world × (npieces + 1): piece boundaries of every rank
  // split-K heavy rows of this rank: per segment {CSR begin, signals, heavy index}; per heavy
  // row {first segment, 0, row} (the seg_mode 2 solve) and the segment prefix hseg[nh+1]
  RowDesc* d_seg = nullptr;
  RowDesc* d_heavy = nullptr;
  int64_t* d_hseg = nullptr;
  int64_t nseg = 0, nheavy = 0;
};

int32_t* colp(const SideBuf& sb) { return sb.col - sb.shard_off; }
template <typename T>
const T* valp(const SideBuf& sb) {
  return (const T*)sb.val - sb.shard_off;
}
// frees the CSR arrays of a side (all of them, or only col/val)
void drop_csr(SideBuf& sb, bool rowptr_too) {
  if (rowptr_too && sb.rowptr) (void)hipFree(sb.rowptr), sb.rowptr = nullptr;
  if (sb.col) (void)hipFree(sb.col), sb.col = nullptr;
  if (sb.val) (void)hipFree(sb.val), sb.val = nullptr;
  sb.shard_off = 0;
  sb.sharded = false;
}

}  // namespace

struct qmfx_ctx {
  int device = 0;
  int prec = 32;
  int k = 0, kp = 0, nt = 0;
  size_t esz = 4;
  hipStream_t stream = nullptr;
  SideBuf s[2];
  int64_t nnz = 0;
  void* G = nullptr;
  double* gpart = nullptr;
  int gpart_blocks = 1024;
  double* rowloss = nullptr;
  int64_t rowloss_cap = 0;
  int32_t* status = nullptr;
  // pivoted re-solve of flagged rows (fallback.hip): scratch and [re-solved, singular] counts
  double* fb_scratch = nullptr;
  unsigned long long* fb_cnt = nullptr;
  int64_t fb_rows = 0;  // rows re-solved by the last half
  double* dsum = nullptr;
  double* hsum = nullptr;  // pinned
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double solve_ms = 0, solve_flops = 0, solve_bytes = 0;
  int64_t solve_launches = 0;
  int last_side = 0;
  // distributed
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  // BPR
  int64_t* pos_user = nullptr;
  int32_t* pos_item = nullptr;
  int64_t npos = 0;
  int64_t max_user_pos = 0;  // largest positive count of one user (Hogwild collision estimate)
  int64_t* urowptr = nullptr;
  int32_t* uitems = nullptr;
  void* bias = nullptr;
  int32_t* bad = nullptr;
  int64_t* trip[2] = {nullptr, nullptr};
  int64_t trip_n[2] = {0, 0};
  const void* trip_src[2] = {nullptr, nullptr};
  double* eval_partial = nullptr;
  // test-set evaluation (qmfx_eval_set_labels / qmfx_eval_ranks)
  int64_t ev_ntest = 0, ev_nlab = 0, ev_npos = 0, ev_chunks = 0;
  int64_t* ev_users = nullptr;
  int32_t* ev_slot = nullptr;
  int64_t* ev_item = nullptr;
  int64_t* ev_pidx = nullptr;
  int64_t* ev_pptr = nullptr;
  double* ev_lscore = nullptr;
  double* ev_pscore = nullptr;
  unsigned long long* ev_above = nullptr;
  double* ev_sq = nullptr;
  double* ev_udbl = nullptr;
  uint64_t bpr_epochs = 0;
  // QMFX_FAULT_COMM_RANK=<rank>[:<after>] (tests), read once at create: that rank's piece
  // broadcasts fail as if RCCL had failed once <after> of them have succeeded (-1: none)
  int fault_comm_rank = -1;
  int64_t fault_comm_after = 0, comm_pieces_done = 0;
  bool whitened_enabled = true;  // QMFX_NO_WHITEN=1 forces the direct kernel for every row
  int wb_k64_ntn = 0;            // QMFX_WB_K64_NTN: largest whitened bucket at k = 64 (0: default)
  // the half-epoch in progress (qmfx_wals_half's phases)
  struct HalfStateT {
    int side = 0;
    double alpha = 0, lambda = 0;
    bool use_w = false;
    int64_t nD = 0;
    const char* trace_path = nullptr;
  } hs;
  // split-K heavy rows (direct and multi-wave tilings): rows with more than heavy_min signals are
  // cut into segments of seg_len (QMFX_HEAVY_MIN / QMFX_SEG_LEN, read once at create;
  // heavy_min 0 = off); partials [segments][NTT·256 + KP] in the context precision + Σc/flag
  int64_t heavy_min = 16384;
  int64_t seg_len = 8192;
  void* part = nullptr;
  void* partb = nullptr;
  double* partc = nullptr;
  int64_t part_cap = 0;  // segments
  // whitened path buffers
  void* Z = nullptr;  // whitened fixed side [max(nu, ni)][kp]
  int64_t z_cap = 0;
  void* Linv = nullptr;  // kp × kp
  int32_t* chol_status = nullptr;
  double* chol_scratch = nullptr;  // KP > 128: the fp64 factorization of G + λI (global)
  void* Gimg = nullptr;  // G + λI as the direct kernel's accumulator-tile image
  uint64_t* trace = nullptr;  // QMFX_TRACE diagnostics: whitened-row phase timestamps
  int64_t trace_cap = 0;
  // per-class timing: 0 direct kernel, 1 whitened kernels (row solve + unwhiten), 2 whole half
  hipEvent_t evh[4] = {nullptr, nullptr, nullptr, nullptr};
  // solve pieces per half (QMFX_PIECES; default 1 on one rank, 8 with several: the last
  // piece's all-gather is the exposed part) and their
  // events: [piece][start, direct done, whitened done]; collectives run on comm_stream
  int npieces = 0;
  hipEvent_t evp[QMFX_MAX_PIECES][3] = {};
  hipEvent_t ev_sum = nullptr, ev_comm = nullptr;
  hipStream_t comm_stream = nullptr;
  // multi-rank halves: per piece, the collective stream's [start, end] of its broadcasts
  // (start = when the stream reached them: the piece's solves done and the previous piece's
  // broadcasts finished); per solved side since reset: Σ broadcast time, the exposed tail
  // (last piece's solves done → its broadcasts done) and Σ solve time of the pieces
  hipEvent_t evx[QMFX_MAX_PIECES][2] = {};
  double xch_ms[2] = {0, 0}, xch_tail_ms[2] = {0, 0}, xch_solve_ms[2] = {0, 0};
  int64_t xch_halves[2] = {0, 0};
  // BPR launch plan of the last epoch (qmfx_bpr_plan)
  int bpr_waves = 0, bpr_atomic_user = 0;
  double cls_ms[3] = {0, 0, 0}, cls_flops[3] = {0, 0, 0}, cls_bytes[3] = {0, 0, 0};
  int64_t cls_launches[3] = {0, 0, 0};
  // the same per solved side (a class's launches differ by side: at C3 the direct kernel
  // takes 187 ms in the item half and 69 µs in the user half)
  double side_ms[2][3] = {}, side_flops[2][3] = {}, side_bytes[2][3] = {};
  // set when qmfx_wals_half_multi aborted the clique after a failed collective
  bool comm_aborted = false;
  int64_t side_launches[2][3] = {};
};

namespace {

int set_dev(qmfx_ctx* c) {
  HIPCHK(hipSetDevice(c->device));
  return 0;
}

void dfree(void*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}
template <typename P>
void dfree_t(P*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

int ensure_side_factors(qmfx_ctx* c, int side) {
  SideBuf& sb = c->s[side];
  if (sb.F) return 0;
  if (sb.n <= 0) return fail("shape not set (qmfx_set_shape)");
  // one extra all-zero row (index n): padding signals of the row kernels gather it
  HIPCHK(hipMalloc(&sb.F, (size_t)(sb.n + 1) * c->kp * c->esz));
  HIPCHK(hipMemsetAsync(sb.F, 0, (size_t)(sb.n + 1) * c->kp * c->esz, c->stream));
  return 0;
}

void set_default_bounds(SideBuf& sb, int world, int rank) {
  sb.bounds.assign(world + 1, 0);
  const int64_t total = sb.h_rowptr.empty() ? 0 : sb.h_rowptr.back();
  for (int r = 0; r <= world; ++r) {
    if (r == world) {
      sb.bounds[r] = sb.n;
    } else if (r == 0) {
      sb.bounds[r] = 0;
    } else {
      const int64_t target = (int64_t)((__int128)total * r / world);
      sb.bounds[r] = std::lower_bound(sb.h_rowptr.begin(), sb.h_rowptr.end(), target) -
                     sb.h_rowptr.begin();
      if (sb.bounds[r] > sb.n) sb.bounds[r] = sb.n;
    }
  }
  for (int r = 1; r <= world; ++r) sb.bounds[r] = std::max(sb.bounds[r], sb.bounds[r - 1]);
  sb.rbeg = sb.bounds[rank];
  sb.rend = sb.bounds[rank + 1];
}

int ensure_rowloss(qmfx_ctx* c, int64_t n) {
  if (c->rowloss_cap >= n) return 0;
  dfree_t(c->rowloss);
  dfree_t(c->status);
  HIPCHK(hipMalloc(&c->rowloss, (size_t)std::max<int64_t>(n, 1) * sizeof(double)));
  HIPCHK(hipMalloc(&c->status, (size_t)std::max<int64_t>(n, 1) * sizeof(int32_t)));
  c->rowloss_cap = n;
  return 0;
}

template <typename T>
std::vector<T> convert(const double* src, size_t n) {
  std::vector<T> v(n);
  for (size_t i = 0; i < n; ++i) v[i] = (T)src[i];
  return v;
}

ncclDataType_t nccl_type(int prec) { return prec == 32 ? ncclFloat32 : ncclFloat64; }

// Every transfer goes through the context's (non-blocking) stream so it is ordered with the
// kernels and async memsets issued there; the call returns when the copy has completed.
hipError_t scopy(qmfx_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  if (bytes == 0) return hipSuccess;
  hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, c->stream);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(c->stream);
}

// Largest whitened-row bucket (NTN) usable for this factor tiling: n padded to 16 at most
// KP/2 and 64, except fp32 k = 128 / 256 on the streamed kernel (two signals per lane): n ≤
// 128 (the n×n system stays the smaller one up to n ≈ k; measured at C3 and C5).
// Factor counts beyond one wave's registers (fp32 k > 128, fp64 k > 64) use the multi-wave
// row kernel and the tiled YᵀY (wals_big.hip).
// YᵀY on the tiled multi-wave kernel (fp32 k > 128, fp64 k > 64)
bool use_big(const qmfx_ctx* c) { return c->prec == 32 ? c->nt > 8 : c->nt > 4; }
// direct rows on the multi-wave row kernel: k > 128 (fp64 k = 80..128 runs the one-wave
// direct kernel with its accumulators across the VGPR + AGPR file; the
// multi-wave kernel at fp64 k = 128 measured 213.7 ms per C3 item half at four waves per row
// and 206.5 ms at two, against 179.2 / 175.6 ms here: round 6, profiles/r06/ab_big128_c3_f64.txt)
bool use_big_rows(const qmfx_ctx* c) { return c->nt > 8; }

// Largest whitened-row bucket (NTN: n ≤ 16·NTN) for this factor tiling: n ≤ KP/2
// and ≤ 64, except on the streamed kernels' two-signals-per-lane buckets: fp32 k = 128 / 256
// up to n = 128, fp64 k = 128 / 256 up to n = 80 (n = 81..96 spilled 64 VGPRs; those rows stay
// direct).
int max_whitened_ntn(const qmfx_ctx* c) {
  if (!c->whitened_enabled) return 0;
  if (c->nt == 4 && c->wb_k64_ntn > 0) return std::min(c->wb_k64_ntn, 4);
  if (c->prec == 32) {
    if (c->nt == 8 || c->nt == 16) return 8;
    if (c->nt > 8) return 0;  // fp32 k = 144..240: every row on the big k×k kernel
    // k = 64: n ≤ 64 (C2 same-box A/Bs, round 5: n ≤ 32 → n ≤ 48 10.0 → 9.1 ms/epoch, → n ≤ 64
    // 8.7 → 8.2)
    if (c->nt == 4) return 4;
    return std::min(c->nt / 2, 4);
  }
  if (c->nt == 8 || c->nt == 16) return 5;
  if (c->nt > 8) return 0;
  // k = 64: n ≤ 48 on the streamed fp64 kernel (C2 fp64 same-box A/B, round 5: 18.5 → 17.6
  // ms/epoch; n ≤ 64 measured no better)
  if (c->nt == 4) return 3;
  return std::min(c->nt / 2, c->nt <= 4 ? 2 : 4);
}

// Splits this rank's rows of `side` into whitened buckets (by padded signal count) and the
// direct bucket (heaviest rows first, for load balance), and uploads the order list.
int npieces(const qmfx_ctx* c) {
  if (c->npieces > 0) return c->npieces;
  return c->world > 1 ? 8 : 1;
}

// nnz-balanced split of rows [b, e) into p contiguous pieces → out[0..p]
void split_rows(const std::vector<int64_t>& rp, int64_t b, int64_t e, int p, int64_t* out) {
  out[0] = b;
  out[p] = e;
  for (int j = 1; j < p; ++j) {
    const int64_t target = rp[b] + (int64_t)((__int128)(rp[e] - rp[b]) * j / p);
    int64_t r = std::lower_bound(rp.begin() + b, rp.begin() + e + 1, target) - rp.begin();
    out[j] = std::min(std::max(r, out[j - 1]), e);
  }
}

// The all-gather schedule of a half: rank r owns rows [bounds[r], bounds[r+1]) and splits
// them into P nnz-balanced pieces; pb[r·(P+1) + j] .. pb[r·(P+1) + j + 1] is the row range
// rank r broadcasts after solving its piece j (qmfx_wals_half), skipped when empty.
void plan_pieces(const std::vector<int64_t>& rp, const std::vector<int64_t>& bounds, int world,
                 int P, std::vector<int64_t>& pb) {
  pb.assign((size_t)world * (P + 1), 0);
  for (int r = 0; r < world; ++r) split_rows(rp, bounds[r], bounds[r + 1], P, &pb[(size_t)r * (P + 1)]);
}

// Keeps only this rank's signals of a side on the device (col/val of rows rbeg..rend).
int shard_csr(qmfx_ctx* c, SideBuf& sb);

// Splits this rank's rows of `side` into pieces, and each piece into whitened buckets (by
// padded signal count) and the direct bucket (heaviest rows first, for load balance);
// uploads the order list (piece sections back to back) and the per-slot descriptors.
int build_buckets(qmfx_ctx* c, int side) {
  SideBuf& sb = c->s[side];
  sb.buckets_valid = false;
  if (sb.h_rowptr.empty()) return 0;
  if (sb.n > INT32_MAX) return fail("more than 2^31 rows on one side are not supported");
  const int mx = max_whitened_ntn(c);
  const int P = npieces(c);
  plan_pieces(sb.h_rowptr, sb.bounds, c->world, P, sb.pbounds);
  double nnz_w = 0, nnz_d = 0, flops_w = 0;
  const double k = c->k;
  std::vector<int64_t> order;
  order.reserve(sb.rend - sb.rbeg);
  sb.pieces.assign(P, SideBuf::Piece{});
  int64_t nw_total = 0;
  // split-K heavy rows at every k (the multi-wave k > 128 kernel has segment modes too)
  const int64_t hmin = c->heavy_min;
  std::vector<RowDesc> segs, heavy;
  std::vector<int64_t> hseg;
  for (int j = 0; j < P; ++j) {
    SideBuf::Piece& pc = sb.pieces[j];
    pc.rb = sb.pbounds[(size_t)c->rank * (P + 1) + j];
    pc.re = sb.pbounds[(size_t)c->rank * (P + 1) + j + 1];
    pc.ord = (int64_t)order.size();
    std::vector<int64_t> wlist[kMaxNTN];
    std::vector<std::pair<int64_t, int64_t>> direct;
    for (int64_t r = pc.rb; r < pc.re; ++r) {
      const int64_t n = sb.h_rowptr[r + 1] - sb.h_rowptr[r];
      // RowDesc::n is int32 (segments too: seg_len is clamped at create)
      if (n > INT32_MAX) return fail("a row with more than 2^31-1 signals is not supported");
      const int64_t ntn = (std::max<int64_t>(n, 1) + 15) / 16;
      if (ntn <= mx) {
        wlist[ntn - 1].push_back(r);
        nnz_w += (double)n;
        // K (n(n+1)k), n×n Cholesky + solves (n³/3 + 2n²), Zᵀu and Zᵀc (4nk), unwhitening (2k²)
        const double dn = (double)n;
        flops_w += dn * (dn + 1) * k + dn * dn * dn / 3.0 + 2 * dn * dn + 4 * dn * k + 2 * k * k;
      } else {
        direct.emplace_back(n, r);
        nnz_d += (double)n;
      }
    }
    std::stable_sort(direct.begin(), direct.end(),
                     [](const auto& x, const auto& y) { return x.first > y.first; });
    // the heaviest direct rows (n > hmin) lead the direct section; each is cut into
    // segments of seg_len signals
    pc.h0 = (int64_t)heavy.size();
    pc.s0 = (int64_t)segs.size();
    for (const auto& d : direct) {
      if (hmin <= 0 || d.first <= hmin) break;
      const int64_t r = d.second, beg = sb.h_rowptr[r], n = d.first;
      hseg.push_back((int64_t)segs.size());
      heavy.push_back(RowDesc{(int64_t)segs.size(), 0, (int32_t)r});
      for (int64_t o = 0; o < n; o += c->seg_len)
        segs.push_back(RowDesc{beg + o, (int32_t)std::min(c->seg_len, n - o),
                               (int32_t)(heavy.size() - 1)});
    }
    pc.nh = (int64_t)heavy.size() - pc.h0;
    pc.ns = (int64_t)segs.size() - pc.s0;
    for (int i = 0; i < kMaxNTN; ++i) {
      pc.wb[i] = (int64_t)order.size() - pc.ord;
      order.insert(order.end(), wlist[i].begin(), wlist[i].end());
    }
    pc.wb[kMaxNTN] = (int64_t)order.size() - pc.ord;
    nw_total += pc.wb[kMaxNTN];
    for (const auto& d : direct) order.push_back(d.second);
    pc.n_ord = (int64_t)order.size() - pc.ord;
  }
  for (int i = 0; i < kMaxNTN; ++i) sb.wb[i] = 0;
  sb.wb[kMaxNTN] = nw_total;  // whitened rows of this rank (all pieces)
  sb.n_ord = (int64_t)order.size();
  sb.nnz_w = nnz_w;
  sb.nnz_d = nnz_d;
  sb.flops_w = flops_w;
  if (sb.d_order) (void)hipFree(sb.d_order);
  sb.d_order = nullptr;
  HIPCHK(hipMalloc(&sb.d_order, (size_t)std::max<int64_t>(sb.n_ord, 1) * 8));
  HIPCHK(scopy(c, sb.d_order, order.data(), (size_t)sb.n_ord * 8, hipMemcpyHostToDevice));
  std::vector<RowDesc> desc((size_t)sb.n_ord);
  for (size_t i = 0; i < desc.size(); ++i) {
    const int64_t r = order[i];
    desc[i] = RowDesc{sb.h_rowptr[r], (int32_t)(sb.h_rowptr[r + 1] - sb.h_rowptr[r]), (int32_t)r};
  }
  if (sb.d_desc) (void)hipFree(sb.d_desc);
  sb.d_desc = nullptr;
  HIPCHK(hipMalloc(&sb.d_desc, (size_t)std::max<int64_t>(sb.n_ord, 1) * sizeof(RowDesc)));
  HIPCHK(scopy(c, sb.d_desc, desc.data(), desc.size() * sizeof(RowDesc), hipMemcpyHostToDevice));
  hseg.push_back((int64_t)segs.size());
  dfree_t(sb.d_seg);
  dfree_t(sb.d_heavy);
  dfree_t(sb.d_hseg);
  sb.nseg = (int64_t)segs.size();
  sb.nheavy = (int64_t)heavy.size();
  if (sb.nheavy > 0) {
    HIPCHK(hipMalloc(&sb.d_seg, segs.size() * sizeof(RowDesc)));
    HIPCHK(hipMalloc(&sb.d_heavy, heavy.size() * sizeof(RowDesc)));
    HIPCHK(hipMalloc(&sb.d_hseg, hseg.size() * sizeof(int64_t)));
    HIPCHK(scopy(c, sb.d_seg, segs.data(), segs.size() * sizeof(RowDesc), hipMemcpyHostToDevice));
    HIPCHK(scopy(c, sb.d_heavy, heavy.data(), heavy.size() * sizeof(RowDesc), hipMemcpyHostToDevice));
    HIPCHK(scopy(c, sb.d_hseg, hseg.data(), hseg.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    if (c->part_cap < sb.nseg) {
      dfree(c->part);
      dfree(c->partb);
      dfree_t(c->partc);
      const size_t ntt = (size_t)c->nt * (c->nt + 1) / 2;
      HIPCHK(hipMalloc(&c->part, (size_t)sb.nseg * ntt * 256 * c->esz));
      HIPCHK(hipMalloc(&c->partb, (size_t)sb.nseg * c->kp * c->esz));
      HIPCHK(hipMalloc(&c->partc, (size_t)sb.nseg * 2 * sizeof(double)));
      c->part_cap = sb.nseg;
    }
  }
  sb.buckets_valid = true;
  return 0;
}

int shard_csr(qmfx_ctx* c, SideBuf& sb) {
  if (sb.sharded || !sb.col) return 0;
  const int64_t e0 = sb.h_rowptr[sb.rbeg], e1 = sb.h_rowptr[sb.rend];
  const size_t m = (size_t)std::max<int64_t>(e1 - e0, 1);
  int32_t* col = nullptr;
  void* val = nullptr;
  HIPCHK(hipMalloc(&col, m * sizeof(int32_t)));
  HIPCHK(hipMalloc(&val, m * c->esz));
  if (e1 > e0) {
    HIPCHK(hipMemcpyAsync(col, sb.col + e0, (size_t)(e1 - e0) * sizeof(int32_t),
                          hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(val, (char*)sb.val + (size_t)e0 * c->esz, (size_t)(e1 - e0) * c->esz,
                          hipMemcpyDeviceToDevice, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  (void)hipFree(sb.col);
  (void)hipFree(sb.val);
  sb.col = col;
  sb.val = val;
  sb.shard_off = e0;
  sb.sharded = true;
  return 0;
}

template <typename T>
FallbackArgs<T> fallback_args(qmfx_ctx* c, const SideBuf& L, const SideBuf& R, int64_t slot_begin,
                              int64_t nslots, double alpha, double lambda) {
  FallbackArgs<T> a{};
  a.rowptr = L.rowptr;
  a.col = colp(L);
  a.val = valp<T>(L);
  a.Y = (const T*)R.F;
  a.G = (const T*)c->G;
  a.X = (T*)L.F;
  a.rowloss = c->rowloss;
  a.status = c->status;
  a.desc = L.d_desc;
  a.slot_begin = slot_begin;
  a.nslots = nslots;
  a.alpha = alpha;
  a.lambda = lambda;
  a.k = c->k;
  a.kp = c->kp;
  a.scratch = c->fb_scratch;
  a.counters = c->fb_cnt;
  return a;
}

// One launch of the direct-row kernels over `n` slots from `b`: seg_mode 0 = slots of the
// side's order (rows), 1 = split-K segments (d_seg), 2 = split-K heavy-row solves (d_heavy).
template <typename T>
hipError_t launch_direct_t(qmfx_ctx* c, const SideBuf& L, const SideBuf& R, int64_t b, int64_t n,
                           double alpha, double lambda, const char* trace_path, int mode) {
  SolveArgs<T> a{L.rowptr, colp(L), valp<T>(L), (const T*)R.F, (const T*)c->G, (T*)L.F,
                 c->rowloss, c->status, L.d_order, b, n, (T)alpha, (T)lambda, c->k,
                 mode == 1 ? L.d_seg : mode == 2 ? L.d_heavy : L.d_desc, (const T*)c->Gimg,
                 (trace_path && mode == 0) ? c->trace : nullptr, (int32_t)R.n};
  a.seg_mode = mode;
  a.part = (T*)c->part;
  a.partb = (T*)c->partb;
  a.partc = c->partc;
  return use_big_rows(c) ? launch_wals_big(a, c->nt, c->stream)
                         : launch_wals_direct(a, c->nt, c->stream);
}

int launch_direct_range(qmfx_ctx* c, const SideBuf& L, const SideBuf& R, int64_t b, int64_t n,
                        double alpha, double lambda, const char* trace_path, int mode) {
  if (n <= 0) return 0;
  const hipError_t e = c->prec == 32
                           ? launch_direct_t<float>(c, L, R, b, n, alpha, lambda, trace_path, mode)
                           : launch_direct_t<double>(c, L, R, b, n, alpha, lambda, trace_path, mode);
  if (e != hipSuccess) return fail(std::string("row kernel launch: ") + hipGetErrorString(e), -2);
  return 0;
}

}  // namespace

extern "C" {

const char* qmfx_last_error(void) { return g_err.c_str(); }
int qmfx_version(void) { return 1; }

int qmfx_device_count(int* count) {
  HIPCHK(hipGetDeviceCount(count));
  return 0;
}

int qmfx_create(qmfx_ctx** out, int device, int precision, int nfactors) {
  if (!out) return fail("out is null");
  if (precision != 32 && precision != 64) return fail("precision must be 32 or 64");
  if (nfactors <= 0) return fail("nfactors must be positive");
  const int nt = (nfactors + 15) / 16;
  if (nt > 16) return fail("nfactors > 256 not supported yet");
  auto* c = new qmfx_ctx();
  if (nt > 8) c->gpart_blocks = 256;  // YᵀY partials: NTT·256 doubles per block
  c->device = device;
  c->prec = precision;
  c->k = nfactors;
  c->nt = nt;
  c->kp = 16 * nt;
  c->esz = precision == 32 ? 4 : 8;
  if (const char* nw = std::getenv("QMFX_NO_WHITEN")) c->whitened_enabled = std::atoi(nw) == 0;
  if (const char* w = std::getenv("QMFX_WB_K64_NTN")) c->wb_k64_ntn = std::min(std::max(std::atoi(w), 1), 4);
  if (const char* f = std::getenv("QMFX_FAULT_COMM_RANK")) {
    c->fault_comm_rank = std::atoi(f);
    if (const char* a = std::strchr(f, ':')) c->fault_comm_after = std::atoll(a + 1);
  }
  if (const char* hm = std::getenv("QMFX_HEAVY_MIN")) c->heavy_min = std::max<int64_t>(std::atoll(hm), 0);
  if (const char* sl = std::getenv("QMFX_SEG_LEN"))
    c->seg_len = std::min<int64_t>(std::max<int64_t>(std::atoll(sl), 64), INT32_MAX);
  if (const char* np = std::getenv("QMFX_PIECES"))
    c->npieces = std::min(std::max(std::atoi(np), 1), QMFX_MAX_PIECES);
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->G, (size_t)c->kp * c->kp * c->esz);
  if (e == hipSuccess)
    e = hipMalloc(&c->gpart, (size_t)c->gpart_blocks * (nt * (nt + 1) / 2) * 256 * sizeof(double));
  // sum + partials (launch_sum_f64: 1 + kSumBlocks), then the half status block
  if (e == hipSuccess) e = hipMalloc(&c->dsum, (kHalfStatus + 4) * sizeof(double));
  if (e == hipSuccess) e = hipHostMalloc(&c->hsum, 4 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&c->bad, sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&c->eval_partial, 1024 * sizeof(double));
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  for (int i = 0; i < 4 && e == hipSuccess; ++i) e = hipEventCreate(&c->evh[i]);
  for (int i = 0; i < QMFX_MAX_PIECES && e == hipSuccess; ++i)
    for (int j = 0; j < 3 && e == hipSuccess; ++j) e = hipEventCreate(&c->evp[i][j]);
  for (int i = 0; i < QMFX_MAX_PIECES && e == hipSuccess; ++i)
    for (int j = 0; j < 2 && e == hipSuccess; ++j) e = hipEventCreate(&c->evx[i][j]);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_sum, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_comm, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc(&c->Linv, (size_t)c->kp * c->kp * c->esz);
  if (e == hipSuccess) e = hipMalloc(&c->Gimg, (size_t)(nt * (nt + 1) / 2) * 256 * c->esz);
  if (e == hipSuccess) e = hipMalloc(&c->chol_status, sizeof(int32_t));
  if (e == hipSuccess && c->kp > 128)
    e = hipMalloc(&c->chol_scratch, (size_t)c->kp * (c->kp + 1) * sizeof(double));
  if (e == hipSuccess)
    e = hipMalloc(&c->fb_scratch, (size_t)FB_MAX_GRID * (c->kp + 3) * c->kp * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&c->fb_cnt, 2 * sizeof(unsigned long long));
  if (e != hipSuccess) {
    g_err = std::string("qmfx_create: ") + hipGetErrorString(e);
    delete c;
    return -2;
  }
  *out = c;
  return 0;
}

int qmfx_destroy(qmfx_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
  for (auto& row : c->evp)
    for (auto& ev : row)
      if (ev) (void)hipEventDestroy(ev);
  for (auto& row : c->evx)
    for (auto& ev : row)
      if (ev) (void)hipEventDestroy(ev);
  if (c->ev_sum) (void)hipEventDestroy(c->ev_sum);
  if (c->ev_comm) (void)hipEventDestroy(c->ev_comm);
  for (auto& sb : c->s) {
    drop_csr(sb, true);
    dfree(sb.F);
    dfree_t(sb.d_order);
    dfree_t(sb.d_desc);
    dfree_t(sb.d_seg);
    dfree_t(sb.d_heavy);
    dfree_t(sb.d_hseg);
  }
  dfree(c->part);
  dfree(c->partb);
  dfree_t(c->partc);
  dfree(c->G);
  dfree_t(c->gpart);
  dfree_t(c->rowloss);
  dfree_t(c->status);
  dfree_t(c->dsum);
  if (c->hsum) (void)hipHostFree(c->hsum);
  dfree_t(c->bad);
  dfree_t(c->eval_partial);
  dfree_t(c->ev_users);
  dfree_t(c->ev_slot);
  dfree_t(c->ev_item);
  dfree_t(c->ev_pidx);
  dfree_t(c->ev_pptr);
  dfree_t(c->ev_lscore);
  dfree_t(c->ev_pscore);
  dfree_t(c->ev_above);
  dfree_t(c->ev_sq);
  dfree_t(c->ev_udbl);
  dfree_t(c->pos_user);
  dfree_t(c->pos_item);
  dfree_t(c->urowptr);
  dfree_t(c->uitems);
  dfree(c->bias);
  dfree_t(c->trip[0]);
  dfree_t(c->trip[1]);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  for (auto& ev : c->evh)
    if (ev) (void)hipEventDestroy(ev);
  dfree(c->Z);
  dfree(c->Linv);
  dfree(c->Gimg);
  dfree_t(c->trace);
  dfree_t(c->chol_status);
  dfree_t(c->chol_scratch);
  dfree_t(c->fb_scratch);
  dfree_t(c->fb_cnt);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int qmfx_sync(qmfx_ctx* c) {
  if (set_dev(c)) return -2;
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int qmfx_set_shape(qmfx_ctx* c, int64_t nusers, int64_t nitems) {
  if (nusers <= 0 || nitems <= 0) return fail("empty shape: nusers and nitems must be > 0");
  if (nitems > 0x7fffffffll || nusers > 0x7fffffffll) return fail("more than 2^31 rows");
  if (set_dev(c)) return -2;
  for (int side = 0; side < 2; ++side) {
    const int64_t n = side == 0 ? nusers : nitems;
    c->s[side].h_ids.clear();
    if (c->s[side].n != n) {
      dfree(c->s[side].F);
      drop_csr(c->s[side], true);
      c->s[side].h_rowptr.clear();
      c->s[side].n = n;
    }
  }
  return 0;
}

int qmfx_get_shape(qmfx_ctx* c, int64_t* nusers, int64_t* nitems, int64_t* nnz) {
  if (nusers) *nusers = c->s[0].n;
  if (nitems) *nitems = c->s[1].n;
  if (nnz) *nnz = c->nnz;
  return 0;
}

int qmfx_upload_csr(qmfx_ctx* c, int side, const int64_t* rowptr, const int32_t* colidx,
                    const double* values, int64_t nnz) {
  if (side != 0 && side != 1) return fail("side must be 0 or 1");
  SideBuf& sb = c->s[side];
  if (sb.n <= 0) return fail("shape not set (qmfx_set_shape)");
  sb.h_ids.clear();
  const int64_t nother = c->s[1 - side].n;
  if (rowptr[0] != 0 || rowptr[sb.n] != nnz) return fail("rowptr inconsistent with nnz");
  for (int64_t r = 0; r < sb.n; ++r)
    if (rowptr[r + 1] < rowptr[r]) return fail("rowptr not monotone");
  for (int64_t e = 0; e < nnz; ++e)
    if (colidx[e] < 0 || colidx[e] >= nother) return fail("column index out of range");
  if (set_dev(c)) return -2;
  drop_csr(sb, true);
  HIPCHK(hipMalloc(&sb.rowptr, (size_t)(sb.n + 1) * sizeof(int64_t)));
  HIPCHK(hipMalloc(&sb.col, (size_t)std::max<int64_t>(nnz, 1) * sizeof(int32_t)));
  HIPCHK(hipMalloc(&sb.val, (size_t)std::max<int64_t>(nnz, 1) * c->esz));
  HIPCHK(scopy(c, sb.rowptr, rowptr, (size_t)(sb.n + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (nnz > 0) {
    HIPCHK(scopy(c, sb.col, colidx, (size_t)nnz * sizeof(int32_t), hipMemcpyHostToDevice));
    if (c->prec == 32) {
      auto v = convert<float>(values, (size_t)nnz);
      HIPCHK(scopy(c, sb.val, v.data(), (size_t)nnz * 4, hipMemcpyHostToDevice));
    } else {
      HIPCHK(scopy(c, sb.val, values, (size_t)nnz * 8, hipMemcpyHostToDevice));
    }
  }
  sb.nnz = nnz;
  c->nnz = nnz;
  sb.h_rowptr.assign(rowptr, rowptr + sb.n + 1);
  set_default_bounds(sb, c->world, c->rank);
  if (int rc = build_buckets(c, side)) return rc;
  return 0;
}

int qmfx_group_signals(qmfx_ctx* c, const void* records, int64_t nnz, int64_t* nusers,
                       int64_t* nitems) {
  if (nnz <= 0) return fail("empty dataset");
  if (nnz > 0x7fffffffll) return fail("device ingest takes at most 2^31-1 interactions");
  if (set_dev(c)) return -2;
  void* d_rec = nullptr;
  HIPCHK(hipMalloc(&d_rec, (size_t)nnz * 24));
  hipError_t e = scopy(c, d_rec, records, (size_t)nnz * 24, hipMemcpyHostToDevice);
  IngestOut o;
  if (e == hipSuccess) e = group_records(d_rec, nnz, c->prec, o, c->stream);
  (void)hipFree(d_rec);
  auto release = [&]() {
    for (int s = 0; s < 2; ++s) {
      dfree_t(o.ids[s]);
      dfree_t(o.rowptr[s]);
      dfree_t(o.col[s]);
      dfree(o.val[s]);
    }
  };
  if (e != hipSuccess) {
    release();
    return fail(std::string("device ingest: ") + hipGetErrorString(e), -2);
  }
  if (int rc = qmfx_set_shape(c, o.n[0], o.n[1])) {
    release();
    return rc;
  }
  for (int side = 0; side < 2; ++side) {
    SideBuf& sb = c->s[side];
    drop_csr(sb, true);
    sb.rowptr = o.rowptr[side];
    sb.col = o.col[side];
    sb.val = o.val[side];
    o.rowptr[side] = nullptr;
    o.col[side] = nullptr;
    o.val[side] = nullptr;
    sb.nnz = nnz;
    sb.h_ids.resize((size_t)sb.n);
    sb.h_rowptr.resize((size_t)sb.n + 1);
    e = scopy(c, sb.h_ids.data(), o.ids[side], (size_t)sb.n * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess)
      e = scopy(c, sb.h_rowptr.data(), sb.rowptr, (size_t)(sb.n + 1) * 8, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      release();
      return fail(std::string("device ingest: ") + hipGetErrorString(e), -2);
    }
    set_default_bounds(sb, c->world, c->rank);
  }
  release();
  c->nnz = nnz;
  for (int side = 0; side < 2; ++side)
    if (int rc = build_buckets(c, side)) return rc;
  if (nusers) *nusers = c->s[0].n;
  if (nitems) *nitems = c->s[1].n;
  return 0;
}

int qmfx_import_signals(qmfx_ctx* dst, qmfx_ctx* src) {
  if (!dst || !src || dst == src) return fail("qmfx_import_signals: two distinct contexts needed");
  if (dst->prec != src->prec) return fail("qmfx_import_signals: contexts differ in precision");
  for (int side = 0; side < 2; ++side) {
    const SideBuf& s = src->s[side];
    if (!s.rowptr || !s.col || s.h_rowptr.empty()) return fail("qmfx_import_signals: the source has no CSR");
    if (s.sharded) return fail("qmfx_import_signals: the source CSR is sharded");
  }
  // the destination takes a whole CSR: one already partitioned into ranks would be overwritten
  if (dst->comm || dst->world > 1 || dst->s[0].sharded || dst->s[1].sharded)
    return fail("qmfx_import_signals: the destination already went through qmfx_dist_init");
  // the source's CSR writes (its own stream) complete before the copies on dst's stream
  if (set_dev(src)) return -2;
  HIPCHK(hipStreamSynchronize(src->stream));
  if (int rc = qmfx_set_shape(dst, src->s[0].n, src->s[1].n)) return rc;
  if (set_dev(dst)) return -2;
  for (int side = 0; side < 2; ++side) {
    const SideBuf& s = src->s[side];
    SideBuf& d = dst->s[side];
    drop_csr(d, true);
    const size_t m = (size_t)std::max<int64_t>(s.nnz, 1);
    HIPCHK(hipMalloc(&d.rowptr, (size_t)(s.n + 1) * sizeof(int64_t)));
    HIPCHK(hipMalloc(&d.col, m * sizeof(int32_t)));
    HIPCHK(hipMalloc(&d.val, m * dst->esz));
    // device to device over xGMI (the same device: a plain copy)
    HIPCHK(hipMemcpyPeerAsync(d.rowptr, dst->device, s.rowptr, src->device,
                              (size_t)(s.n + 1) * sizeof(int64_t), dst->stream));
    if (s.nnz > 0) {
      HIPCHK(hipMemcpyPeerAsync(d.col, dst->device, s.col, src->device,
                                (size_t)s.nnz * sizeof(int32_t), dst->stream));
      HIPCHK(hipMemcpyPeerAsync(d.val, dst->device, s.val, src->device, (size_t)s.nnz * dst->esz,
                                dst->stream));
    }
    d.nnz = s.nnz;
    d.h_rowptr = s.h_rowptr;
    d.h_ids = s.h_ids;
  }
  HIPCHK(hipStreamSynchronize(dst->stream));
  dst->nnz = src->nnz;
  for (int side = 0; side < 2; ++side) {
    set_default_bounds(dst->s[side], dst->world, dst->rank);
    if (int rc = build_buckets(dst, side)) return rc;
  }
  return 0;
}

int qmfx_get_ids(qmfx_ctx* c, int side, int64_t* ids) {
  if (side != 0 && side != 1) return fail("side must be 0 or 1");
  const SideBuf& sb = c->s[side];
  if ((int64_t)sb.h_ids.size() != sb.n) return fail("no id table: the CSR was not built by qmfx_group_signals");
  std::copy(sb.h_ids.begin(), sb.h_ids.end(), ids);
  return 0;
}

int qmfx_download_csr(qmfx_ctx* c, int side, int64_t* rowptr, int32_t* colidx, double* values) {
  SideBuf& sb = c->s[side];
  if (!sb.rowptr) return fail("no CSR for this side");
  if (sb.sharded) return fail("the CSR is sharded over ranks (qmfx_dist_init): only this rank's rows are held");
  if (set_dev(c)) return -2;
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(scopy(c, rowptr, sb.rowptr, (size_t)(sb.n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
  if (sb.nnz > 0) {
    HIPCHK(scopy(c, colidx, sb.col, (size_t)sb.nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (c->prec == 64) {
      HIPCHK(scopy(c, values, sb.val, (size_t)sb.nnz * 8, hipMemcpyDeviceToHost));
    } else {
      // fp32 context: the device holds float values; widen exactly
      std::vector<float> v((size_t)sb.nnz);
      HIPCHK(scopy(c, v.data(), sb.val, (size_t)sb.nnz * 4, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < v.size(); ++i) values[i] = (double)v[i];
    }
  }
  return 0;
}

int qmfx_gen_synthetic(qmfx_ctx* c, int64_t nusers, int64_t nitems, int64_t nnz, uint64_t seed,
                       int64_t* nnz_out) {
  return qmfx_gen_synthetic_zipf(c, nusers, nitems, nnz, seed, 0.0, nnz_out);
}

int qmfx_gen_synthetic_zipf(qmfx_ctx* c, int64_t nusers, int64_t nitems, int64_t nnz,
                            uint64_t seed, double zipf_s, int64_t* nnz_out) {
  if (nnz <= 0) return fail("nnz must be positive");
  if (zipf_s < 0.0 || !std::isfinite(zipf_s)) return fail("zipf exponent must be >= 0");
  if (int rc = qmfx_set_shape(c, nusers, nitems)) return rc;
  const uint64_t space = (uint64_t)nusers * (uint64_t)nitems;
  if (zipf_s == 0.0 && (uint64_t)nnz > space / 2) return fail("nnz too large for the shape");
  if (nnz > 0x7fffffffll) return fail("at most 2^31-1 draws");
  int end_bit = 64 - __builtin_clzll(space);
  uint64_t *keys = nullptr, *scratch = nullptr;
  HIPCHK(hipMalloc(&keys, (size_t)nnz * 8));
  HIPCHK(hipMalloc(&scratch, (size_t)nnz * 8));
  if (zipf_s == 0.0)
    HIPCHK(launch_synth_keys(keys, nnz, space, seed, c->stream));
  else
    HIPCHK(launch_synth_keys_zipf(keys, nnz, (uint64_t)nusers, (uint64_t)nitems, zipf_s, seed,
                                  c->stream));
  int64_t m = 0;
  HIPCHK(sort_unique_keys(keys, scratch, nnz, &m, end_bit, c->stream));
  for (int side = 0; side < 2; ++side) {
    SideBuf& sb = c->s[side];
    drop_csr(sb, true);
    HIPCHK(hipMalloc(&sb.rowptr, (size_t)(sb.n + 1) * sizeof(int64_t)));
    HIPCHK(hipMalloc(&sb.col, (size_t)m * sizeof(int32_t)));
    HIPCHK(hipMalloc(&sb.val, (size_t)m * c->esz));
    sb.nnz = m;
  }
  // users: keys are u·nitems + i, sorted
  HIPCHK(build_csr_from_sorted_keys(keys, m, nusers, (uint64_t)nitems, c->s[0].rowptr,
                                    c->s[0].col, c->stream));
  HIPCHK(launch_synth_values_any(keys, m, (uint64_t)nitems, (uint64_t)nitems, 1, seed * 31 + 7,
                                 c->s[0].val, c->prec, c->stream));
  // items: transposed keys i·nusers + u, sorted
  HIPCHK(launch_transpose_keys(keys, m, (uint64_t)nitems, (uint64_t)nusers, scratch, c->stream));
  HIPCHK(sort_keys(scratch, keys, m, end_bit, c->stream));
  HIPCHK(build_csr_from_sorted_keys(scratch, m, nitems, (uint64_t)nusers, c->s[1].rowptr,
                                    c->s[1].col, c->stream));
  HIPCHK(launch_synth_values_any(scratch, m, (uint64_t)nusers, (uint64_t)nitems, 0, seed * 31 + 7,
                                 c->s[1].val, c->prec, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  (void)hipFree(keys);
  (void)hipFree(scratch);
  for (int side = 0; side < 2; ++side) {
    SideBuf& sb = c->s[side];
    sb.h_rowptr.resize(sb.n + 1);
    HIPCHK(scopy(c, sb.h_rowptr.data(), sb.rowptr, (size_t)(sb.n + 1) * 8, hipMemcpyDeviceToHost));
    set_default_bounds(sb, c->world, c->rank);
    if (int rc = build_buckets(c, side)) return rc;
  }
  c->nnz = m;
  if (nnz_out) *nnz_out = m;
  return 0;
}

int qmfx_set_factors(qmfx_ctx* c, int side, const double* f) {
  if (side != 0 && side != 1) return fail("side must be 0 or 1");
  if (set_dev(c)) return -2;
  if (int rc = ensure_side_factors(c, side)) return rc;
  SideBuf& sb = c->s[side];
  const size_t n = (size_t)sb.n, kp = c->kp, k = c->k;
  if (c->prec == 32) {
    std::vector<float> h(n * kp, 0.f);
    for (size_t r = 0; r < n; ++r)
      for (size_t j = 0; j < k; ++j) h[r * kp + j] = (float)f[r * k + j];
    HIPCHK(scopy(c, sb.F, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  } else {
    std::vector<double> h(n * kp, 0.0);
    for (size_t r = 0; r < n; ++r)
      for (size_t j = 0; j < k; ++j) h[r * kp + j] = f[r * k + j];
    HIPCHK(scopy(c, sb.F, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  }
  return 0;
}

int qmfx_get_factors(qmfx_ctx* c, int side, double* f) {
  if (side != 0 && side != 1) return fail("side must be 0 or 1");
  if (set_dev(c)) return -2;
  if (int rc = ensure_side_factors(c, side)) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  SideBuf& sb = c->s[side];
  const size_t n = (size_t)sb.n, kp = c->kp, k = c->k;
  if (c->prec == 32) {
    std::vector<float> h(n * kp);
    HIPCHK(scopy(c, h.data(), sb.F, h.size() * 4, hipMemcpyDeviceToHost));
    for (size_t r = 0; r < n; ++r)
      for (size_t j = 0; j < k; ++j) f[r * k + j] = h[r * kp + j];
  } else {
    std::vector<double> h(n * kp);
    HIPCHK(scopy(c, h.data(), sb.F, h.size() * 8, hipMemcpyDeviceToHost));
    for (size_t r = 0; r < n; ++r)
      for (size_t j = 0; j < k; ++j) f[r * k + j] = h[r * kp + j];
  }
  return 0;
}

int qmfx_fill_uniform(qmfx_ctx* c, int side, double bound, uint64_t seed) {
  if (set_dev(c)) return -2;
  if (int rc = ensure_side_factors(c, side)) return rc;
  SideBuf& sb = c->s[side];
  if (c->prec == 32)
    HIPCHK(launch_fill_uniform_f32((float*)sb.F, sb.n, c->kp, c->k, bound, seed, c->stream));
  else
    HIPCHK(launch_fill_uniform_f64((double*)sb.F, sb.n, c->kp, c->k, bound, seed, c->stream));
  return 0;
}

// ---- one WALS half-epoch in phases ------------------------------------------------------
// qmfx_wals_half runs them in order on one context; qmfx_wals_half_multi interleaves them
// over several contexts (one process driving several GPUs) so that piece j's all-gather of
// every context is one RCCL group while piece j+1 computes.
}  // extern "C"

namespace {

// G = YᵀY, the whitening and G + λI images, status resets (no collectives)
int half_begin(qmfx_ctx* c, int side, double alpha, double lambda) {
  if (side != 0 && side != 1) return fail("side must be 0 or 1");
  SideBuf& L = c->s[side];
  SideBuf& R = c->s[1 - side];
  if (!L.rowptr) return fail("no interactions uploaded for the solved side");
  if (!L.buckets_valid) return fail("row buckets not built");
  if (c->comm_aborted)
    return fail("the RCCL clique was aborted after a failed collective; recreate the contexts");
  if (set_dev(c)) return -2;
  if (int rc = ensure_side_factors(c, side)) return rc;
  if (int rc = ensure_side_factors(c, 1 - side)) return rc;
  if (int rc = ensure_rowloss(c, L.n)) return rc;
  const int64_t nW = L.wb[kMaxNTN];             // whitened rows (all buckets)
  const bool use_w = nW > 0 && lambda > 0.0;    // M = YᵀY + λI is SPD only for λ > 0
  const bool fp32 = c->prec == 32;
  c->hs = qmfx_ctx::HalfStateT{side, alpha, lambda, use_w, 0, std::getenv("QMFX_TRACE")};
  HIPCHK(hipEventRecord(c->evh[0], c->stream));
  // G = YᵀY of the fixed side (full replica on every rank)
  const bool big = use_big(c);
  if (fp32)
    HIPCHK(big ? launch_gram_big((const float*)R.F, R.n, c->nt, (float*)c->G, c->gpart,
                                 c->gpart_blocks, c->stream)
               : launch_gram((const float*)R.F, R.n, c->nt, (float*)c->G, c->gpart,
                             c->gpart_blocks, c->stream));
  else
    HIPCHK(big ? launch_gram_big((const double*)R.F, R.n, c->nt, (double*)c->G, c->gpart,
                                 c->gpart_blocks, c->stream)
               : launch_gram((const double*)R.F, R.n, c->nt, (double*)c->G, c->gpart,
                             c->gpart_blocks, c->stream));
  if (use_w) {
    if (c->z_cap < R.n) {
      // one extra all-zero row (index z_cap): the whitened kernel's padding signals
      dfree(c->Z);
      const int64_t cap = std::max(c->s[0].n, c->s[1].n);
      HIPCHK(hipMalloc(&c->Z, (size_t)(cap + 1) * c->kp * c->esz));
      HIPCHK(hipMemsetAsync((char*)c->Z + (size_t)cap * c->kp * c->esz, 0, (size_t)c->kp * c->esz,
                            c->stream));
      c->z_cap = cap;
    }
    HIPCHK(hipMemsetAsync(c->chol_status, 0, 4, c->stream));
    if (fp32) {
      HIPCHK(launch_chol_inv((const float*)c->G, c->nt, c->k, lambda, (float*)c->Linv,
                             c->chol_status, c->chol_scratch, c->stream));
      HIPCHK(launch_whiten((const float*)R.F, (float*)c->Z, nullptr, R.n, c->nt,
                           (const float*)c->Linv, nullptr, 0.0, false, c->stream));
    } else {
      HIPCHK(launch_chol_inv((const double*)c->G, c->nt, c->k, lambda, (double*)c->Linv,
                             c->chol_status, c->chol_scratch, c->stream));
      HIPCHK(launch_whiten((const double*)R.F, (double*)c->Z, nullptr, R.n, c->nt,
                           (const double*)c->Linv, nullptr, 0.0, false, c->stream));
    }
  }
  if (!use_big_rows(c)) {
    if (fp32)
      HIPCHK(launch_gimg((const float*)c->G, c->nt, c->k, lambda, (float*)c->Gimg, c->stream));
    else
      HIPCHK(launch_gimg((const double*)c->G, c->nt, c->k, lambda, (double*)c->Gimg, c->stream));
  }
  HIPCHK(hipMemsetAsync(c->status, 0, (size_t)std::max<int64_t>(L.n, 1) * sizeof(int32_t), c->stream));
  HIPCHK(hipMemsetAsync(c->fb_cnt, 0, 2 * sizeof(unsigned long long), c->stream));
  const char* trace_path = c->hs.trace_path;
  if (trace_path && c->trace_cap < L.n_ord) {
    dfree_t(c->trace);
    HIPCHK(hipMalloc(&c->trace, (size_t)L.n_ord * 64));
    c->trace_cap = L.n_ord;
  }
  if (trace_path) HIPCHK(hipMemsetAsync(c->trace, 0, (size_t)L.n_ord * 64, c->stream));
  return 0;
}

// the row solves of piece j (direct, heavy, whitened, pivoted re-solve); records evp[j][2]
int half_piece(qmfx_ctx* c, int j) {
  if (set_dev(c)) return -2;
  const int side = c->hs.side;
  const double alpha = c->hs.alpha, lambda = c->hs.lambda;
  const bool use_w = c->hs.use_w, fp32 = c->prec == 32;
  const char* trace_path = c->hs.trace_path;
  SideBuf& L = c->s[side];
  SideBuf& R = c->s[1 - side];
  const SideBuf::Piece& pc = L.pieces[j];
  // direct rows (heaviest first; the split-K heavy rows lead); all rows when the whitened
  // form is off
  const int64_t dh = pc.ord + pc.wb[kMaxNTN];
  c->hs.nD += pc.ord + pc.n_ord - (use_w ? dh : pc.ord);
  HIPCHK(hipEventRecord(c->evp[j][0], c->stream));
  if (pc.nh > 0) {
    // heavy rows: segment Grams (one wave per segment), fixed-order fp64 reduction into
    // each row's first segment, then the row solves from those images
    if (int rc = launch_direct_range(c, L, R, pc.s0, pc.ns, alpha, lambda, nullptr, 1))
      return rc;
    if (use_big_rows(c)) {
      // multi-wave tilings: G + λI's image is built here (the direct kernels' Gimg is not)
      if (fp32)
        HIPCHK(launch_heavy_reduce_big((float*)c->part, (float*)c->partb, c->partc, L.d_hseg,
                                       pc.h0, pc.nh, (const float*)c->G, (float*)c->Gimg, c->nt,
                                       c->k, lambda, c->stream));
      else
        HIPCHK(launch_heavy_reduce_big((double*)c->part, (double*)c->partb, c->partc, L.d_hseg,
                                       pc.h0, pc.nh, (const double*)c->G, (double*)c->Gimg,
                                       c->nt, c->k, lambda, c->stream));
    } else if (fp32) {
      HIPCHK(launch_heavy_reduce((float*)c->part, (float*)c->partb, c->partc, L.d_hseg, pc.h0,
                                 pc.nh, (const float*)c->Gimg, c->nt, c->stream));
    } else {
      HIPCHK(launch_heavy_reduce((double*)c->part, (double*)c->partb, c->partc, L.d_hseg,
                                 pc.h0, pc.nh, (const double*)c->Gimg, c->nt, c->stream));
    }
    if (int rc = launch_direct_range(c, L, R, pc.h0, pc.nh, alpha, lambda, nullptr, 2))
      return rc;
  }
  if (!use_w && pc.wb[kMaxNTN] > 0) {
    if (int rc = launch_direct_range(c, L, R, pc.ord, pc.wb[kMaxNTN], alpha, lambda, trace_path, 0))
      return rc;
  }
  if (int rc = launch_direct_range(c, L, R, dh + pc.nh, pc.ord + pc.n_ord - dh - pc.nh, alpha,
                                   lambda, trace_path, 0))
    return rc;
  HIPCHK(hipEventRecord(c->evp[j][1], c->stream));
  // whitened rows: per-bucket row solve, then x = L⁻ᵀ x' and −λ‖x‖²
  if (use_w && pc.wb[kMaxNTN] > 0) {
    for (int b = 0; b < kMaxNTN; ++b) {
      const int64_t cnt = pc.wb[b + 1] - pc.wb[b];
      if (cnt <= 0) continue;
      if (fp32) {
        SolveArgs<float> a{L.rowptr, colp(L), valp<float>(L), (const float*)c->Z, nullptr,
                           (float*)L.F, c->rowloss, c->status, L.d_order, pc.ord + pc.wb[b],
                           cnt, (float)alpha, (float)lambda, c->k, L.d_desc, nullptr,
                           trace_path ? c->trace : nullptr, (int32_t)c->z_cap};
        HIPCHK(launch_wals_woodbury(a, c->nt, b + 1, c->stream));
      } else {
        SolveArgs<double> a{L.rowptr, colp(L), valp<double>(L), (const double*)c->Z,
                            nullptr, (double*)L.F, c->rowloss, c->status, L.d_order,
                            pc.ord + pc.wb[b], cnt, alpha, lambda, c->k, L.d_desc,
                            nullptr, trace_path ? c->trace : nullptr, (int32_t)c->z_cap};
        HIPCHK(launch_wals_woodbury(a, c->nt, b + 1, c->stream));
      }
    }
    if (fp32)
      HIPCHK(launch_whiten((const float*)L.F, (float*)L.F, L.d_order + pc.ord, pc.wb[kMaxNTN], c->nt,
                           (const float*)c->Linv, c->rowloss, lambda, true, c->stream));
    else
      HIPCHK(launch_whiten((const double*)L.F, (double*)L.F, L.d_order + pc.ord, pc.wb[kMaxNTN],
                           c->nt, (const double*)c->Linv, c->rowloss, lambda, true, c->stream));
  }
  // rows the Cholesky kernels flagged: pivoted fp64 re-solve before the all-gather
  if (pc.n_ord > 0) {
    if (fp32)
      HIPCHK(launch_wals_fallback(
          fallback_args<float>(c, L, R, pc.ord, pc.n_ord, alpha, lambda), c->stream));
    else
      HIPCHK(launch_wals_fallback(
          fallback_args<double>(c, L, R, pc.ord, pc.n_ord, alpha, lambda), c->stream));
  }
  HIPCHK(hipEventRecord(c->evp[j][2], c->stream));
  return 0;
}

// piece j of this rank → every rank (one ncclGroup; nests inside a caller's group)
int half_comm_piece(qmfx_ctx* c, int j) {
  if (set_dev(c)) return -2;
  // fault injection for the clique's failure path (tests): QMFX_FAULT_COMM_RANK=<rank>
  if (c->comm && c->fault_comm_rank == c->rank && c->comm_pieces_done++ >= c->fault_comm_after)
    return fail("injected collective failure", -3);
  SideBuf& L = c->s[c->hs.side];
  const int P = (int)L.pieces.size();
  if (c->comm) {
    // piece j of every rank → every rank (an all-gather-v of contiguous row ranges), on
    // the collective stream while the next piece is solved
    HIPCHK(hipStreamWaitEvent(c->comm_stream, c->evp[j][2], 0));
    HIPCHK(hipEventRecord(c->evx[j][0], c->comm_stream));
    NCCLCHK(ncclGroupStart());
    for (int r = 0; r < c->world; ++r) {
      const int64_t b = L.pbounds[(size_t)r * (P + 1) + j], e = L.pbounds[(size_t)r * (P + 1) + j + 1];
      if (e <= b) continue;
      char* base = (char*)L.F + (size_t)b * c->kp * c->esz;
      NCCLCHK(ncclBroadcast(base, base, (size_t)(e - b) * c->kp, nccl_type(c->prec), r, c->comm,
                            c->comm_stream));
    }
    NCCLCHK(ncclGroupEnd());
    HIPCHK(hipEventRecord(c->evx[j][1], c->comm_stream));
  }
  return 0;
}

// trace dump (diagnostics), the loss sum and the status block
int half_tail(qmfx_ctx* c) {
  if (set_dev(c)) return -2;
  const int side = c->hs.side;
  const char* trace_path = c->hs.trace_path;
  SideBuf& L = c->s[side];
  if (trace_path) {
    std::vector<uint64_t> h((size_t)L.n_ord * 8);
    HIPCHK(scopy(c, h.data(), c->trace, h.size() * 8, hipMemcpyDeviceToHost));
    const std::string fn = std::string(trace_path) + "_side" + std::to_string(side) + ".bin";
    if (FILE* f = std::fopen(fn.c_str(), "wb")) {
      std::fwrite(h.data(), 8, h.size(), f);
      std::fclose(f);
    }
  }
  HIPCHK(launch_sum_f64(c->rowloss + L.rbeg, L.rend - L.rbeg, c->dsum, c->stream));
  // loss, re-solve counts and the factorization flag in one status block
  HIPCHK(launch_half_status(c->dsum, c->fb_cnt, c->hs.use_w ? c->chol_status : nullptr,
                            c->dsum + kHalfStatus, c->stream));
  return 0;
}

int half_comm_status(qmfx_ctx* c) {
  if (set_dev(c)) return -2;
  if (c->comm) {
    // the whole status block is summed over the ranks, so every rank sees the same
    // singular-row count and fails (-6) in the same half instead of leaving the others in
    // the next half's collectives
    HIPCHK(hipEventRecord(c->ev_sum, c->stream));
    HIPCHK(hipStreamWaitEvent(c->comm_stream, c->ev_sum, 0));
    NCCLCHK(ncclAllReduce(c->dsum + kHalfStatus, c->dsum + kHalfStatus, 4, ncclFloat64, ncclSum,
                          c->comm, c->comm_stream));
    HIPCHK(hipEventRecord(c->ev_comm, c->comm_stream));
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_comm, 0));
  }
  return 0;
}

int half_end(qmfx_ctx* c, double* loss_sum) {
  if (set_dev(c)) return -2;
  SideBuf& L = c->s[c->hs.side];
  const int P = (int)L.pieces.size();
  HIPCHK(hipEventRecord(c->evh[2], c->stream));
  // one small copy into pinned memory
  HIPCHK(hipMemcpyAsync(c->hsum, c->dsum + kHalfStatus, 4 * sizeof(double),
                        hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->fb_rows = (int64_t)c->hsum[1];
  // the reference's CHECK(info == 0) after dsysv_ (Matrix.cpp:94)
  if (c->hsum[2] != 0.0)
    return fail(std::to_string((int64_t)c->hsum[2]) + " singular row system(s) (dsysv info > 0)", -6);
  if (c->hsum[3] != 0.0) return fail("YᵀY + λI is not positive definite", -5);
  // timing and algorithmic work per kernel class (SURVEY.md §8(d) accounting)
  float ms_d = 0.f, ms_w = 0.f, ms_h = 0.f;
  for (int j = 0; j < P; ++j) {
    float t0 = 0.f, t1 = 0.f;
    HIPCHK(hipEventElapsedTime(&t0, c->evp[j][0], c->evp[j][1]));
    HIPCHK(hipEventElapsedTime(&t1, c->evp[j][1], c->evp[j][2]));
    ms_d += t0;
    ms_w += t1;
  }
  HIPCHK(hipEventElapsedTime(&ms_h, c->evh[0], c->evh[2]));
  const double k = c->k, s = (double)c->esz;
  const int sd = c->hs.side;
  if (c->comm) {
    // the exchange on the collective stream (the status all-reduce behind the last piece's
    // broadcasts has completed: the host synchronised on it above)
    float xb = 0.f, tail = 0.f;
    for (int j = 0; j < P; ++j) {
      float t = 0.f;
      HIPCHK(hipEventElapsedTime(&t, c->evx[j][0], c->evx[j][1]));
      xb += t;
    }
    HIPCHK(hipEventElapsedTime(&tail, c->evp[P - 1][2], c->evx[P - 1][1]));
    c->xch_ms[sd] += xb;
    c->xch_tail_ms[sd] += tail;
    c->xch_solve_ms[sd] += ms_d + ms_w;
    c->xch_halves[sd] += 1;
  }
  auto acc = [&](int cls, double ms, double fl, double by) {
    c->cls_ms[cls] += ms;
    c->cls_launches[cls] += 1;
    c->cls_flops[cls] += fl;
    c->cls_bytes[cls] += by;
    c->side_ms[sd][cls] += ms;
    c->side_launches[sd][cls] += 1;
    c->side_flops[sd][cls] += fl;
    c->side_bytes[sd][cls] += by;
  };
  const bool use_w = c->hs.use_w;
  const int64_t nD = c->hs.nD, nW = L.wb[kMaxNTN];
  const double nzd = use_w ? L.nnz_d : L.nnz_d + L.nnz_w, nd = (double)nD;
  const double nzw = use_w ? L.nnz_w : 0.0, nw = use_w ? (double)nW : 0.0;
  double fl_d = 0, by_d = 0, fl_w = 0, by_w = 0;
  if (nD > 0) {
    fl_d = nzd * k * (k + 1) + nzd * 2 * k + nd * (k * k * k / 3.0 + 2 * k * k);
    by_d = nzd * (4 + s) + nzd * k * s + nd * k * s + (nd + 1) * 8;
    acc(0, ms_d, fl_d, by_d);
  }
  if (nW > 0 && use_w) {
    // whitened-row flops precomputed per side in build_buckets; bytes as SURVEY.md §8(d):
    // signals, gathered rows, X write, rowptr (the x' round trip of the unwhitening pass,
    // 2·k·s per row, is reported beside them by bench.py as extra_bytes)
    fl_w = L.flops_w;
    by_w = nzw * (4 + s) + nzw * k * s + nw * k * s + (nw + 1) * 8;
    acc(1, ms_w, fl_w, by_w);
  }
  acc(2, ms_h, fl_d + fl_w, by_d + by_w);
  c->solve_ms += ms_d + ms_w;
  c->solve_launches += 1;
  c->solve_flops += fl_d + fl_w;
  c->solve_bytes += by_d + by_w;
  c->last_side = c->hs.side;
  if (loss_sum) *loss_sum = *c->hsum;
  return 0;
}

}  // namespace

extern "C" {

int qmfx_wals_half(qmfx_ctx* c, int side, double alpha, double lambda, double* loss_sum) {
  if (int rc = half_begin(c, side, alpha, lambda)) return rc;
  const int P = (int)c->s[side].pieces.size();
  for (int j = 0; j < P; ++j) {
    if (int rc = half_piece(c, j)) return rc;
    if (int rc = half_comm_piece(c, j)) return rc;
  }
  if (int rc = half_tail(c)) return rc;
  if (c->comm) {
    NCCLCHK(ncclGroupStart());
    const int rc = half_comm_status(c);
    NCCLCHK(ncclGroupEnd());
    if (rc) return rc;
  }
  return half_end(c, loss_sum);
}

int qmfx_wals_half_multi(qmfx_ctx* const* ctxs, int n, int side, double alpha, double lambda,
                         double* loss_sum) {
  if (n < 1 || !ctxs) return fail("no contexts");
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i]) return fail("null context");
    if (n > 1 && (!ctxs[i]->comm || ctxs[i]->world != n || ctxs[i]->rank != i))
      return fail("contexts must come from one qmfx_dist_init_all, in rank order");
  }
  for (int i = 0; i < n; ++i)
    if (int rc = half_begin(ctxs[i], side, alpha, lambda)) return rc;
  const int P = (int)ctxs[0]->s[side].pieces.size();
  for (int i = 1; i < n; ++i)
    if ((int)ctxs[i]->s[side].pieces.size() != P) return fail("contexts disagree on the pieces");
  // A context that fails after others have posted their part of a group would leave those
  // collectives waiting for peers that never join, and the next sync would hang: abort every
  // communicator of the clique instead (outstanding collectives are cancelled), so the call
  // returns the error and later calls on these contexts fail loudly.
  auto abort_clique = [&](int rc) {
    for (int i = 0; i < n; ++i) {
      if (ctxs[i]->comm) {
        (void)ncclCommAbort(ctxs[i]->comm);
        ctxs[i]->comm = nullptr;
        ctxs[i]->comm_aborted = true;
      }
    }
    return rc;
  };
  for (int j = 0; j < P; ++j) {
    for (int i = 0; i < n; ++i)
      if (int rc = half_piece(ctxs[i], j)) return abort_clique(rc);
    // one thread drives every communicator: all ranks' broadcasts of piece j in one group
    NCCLCHK(ncclGroupStart());
    int rc = 0;
    for (int i = 0; i < n && rc == 0; ++i) rc = half_comm_piece(ctxs[i], j);
    const ncclResult_t ge = ncclGroupEnd();
    if (rc) return abort_clique(rc);
    if (ge != ncclSuccess) return abort_clique(fail(std::string("RCCL: ") + ncclGetErrorString(ge), -4));
  }
  for (int i = 0; i < n; ++i)
    if (int rc = half_tail(ctxs[i])) return abort_clique(rc);
  {
    NCCLCHK(ncclGroupStart());
    int rc = 0;
    for (int i = 0; i < n && rc == 0; ++i)
      if (ctxs[i]->comm) rc = half_comm_status(ctxs[i]);
    const ncclResult_t ge = ncclGroupEnd();
    if (rc) return abort_clique(rc);
    if (ge != ncclSuccess) return abort_clique(fail(std::string("RCCL: ") + ncclGetErrorString(ge), -4));
  }
  double first = 0.0;
  for (int i = 0; i < n; ++i) {
    double l = 0.0;
    if (int rc = half_end(ctxs[i], &l)) return rc;
    if (i == 0) first = l;
  }
  if (loss_sum) *loss_sum = first;
  return 0;
}

int qmfx_row_classes(qmfx_ctx* c, int side, int64_t* counts) {
  if (side != 0 && side != 1) return fail("side must be 0 or 1");
  const SideBuf& sb = c->s[side];
  if (!sb.buckets_valid) return fail("row buckets not built");
  for (int i = 0; i < kMaxNTN + 3; ++i) counts[i] = 0;
  for (const auto& pc : sb.pieces) {
    for (int b = 0; b < kMaxNTN; ++b) counts[b] += pc.wb[b + 1] - pc.wb[b];
    counts[kMaxNTN] += pc.n_ord - pc.wb[kMaxNTN] - pc.nh;
    counts[kMaxNTN + 1] += pc.nh;
    counts[kMaxNTN + 2] += pc.ns;
  }
  return 0;
}

int qmfx_wals_row_losses(qmfx_ctx* c, double* out) {
  const SideBuf& L = c->s[c->last_side];
  if (!c->rowloss || c->rowloss_cap < L.n) return fail("no half solved yet");
  if (set_dev(c)) return -2;
  HIPCHK(scopy(c, out, c->rowloss, (size_t)L.n * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int qmfx_wals_failed_rows(qmfx_ctx* c, int64_t* rows, int64_t cap, int64_t* count) {
  SideBuf& L = c->s[c->last_side];
  if (set_dev(c)) return -2;
  std::vector<int32_t> st((size_t)std::max<int64_t>(L.n, 1));
  HIPCHK(scopy(c, st.data(), c->status, st.size() * 4, hipMemcpyDeviceToHost));
  int64_t cnt = 0;
  for (int64_t r = 0; r < L.n; ++r)
    if (st[r]) {
      if (cnt < cap && rows) rows[cnt] = r;
      ++cnt;
    }
  *count = cnt;
  return 0;
}

int qmfx_wals_row_system(qmfx_ctx* c, int side, int64_t row, double alpha, double lambda,
                         double* A, double* b, double* csum) {
  if (side != 0 && side != 1) return fail("side must be 0 or 1");
  SideBuf& L = c->s[side];
  SideBuf& R = c->s[1 - side];
  if (row < 0 || row >= L.n) return fail("row out of range");
  if (!L.rowptr) return fail("no interactions uploaded for this side");
  if (L.sharded && (row < L.rbeg || row >= L.rend)) return fail("row not held by this rank");
  if (set_dev(c)) return -2;
  if (int rc = ensure_side_factors(c, 1 - side)) return rc;
  const int k = c->k;
  // YᵀY of this side's fixed side (the last half may have solved the other side)
  if (c->prec == 32)
    HIPCHK(use_big(c) ? launch_gram_big((const float*)R.F, R.n, c->nt, (float*)c->G, c->gpart,
                                        c->gpart_blocks, c->stream)
                      : launch_gram((const float*)R.F, R.n, c->nt, (float*)c->G, c->gpart,
                                    c->gpart_blocks, c->stream));
  else
    HIPCHK(use_big(c) ? launch_gram_big((const double*)R.F, R.n, c->nt, (double*)c->G, c->gpart,
                                        c->gpart_blocks, c->stream)
                      : launch_gram((const double*)R.F, R.n, c->nt, (double*)c->G, c->gpart,
                                    c->gpart_blocks, c->stream));
  double* d = nullptr;
  const size_t nout = (size_t)k * k + k + 1;
  HIPCHK(hipMalloc(&d, nout * sizeof(double)));
  const int64_t beg = L.h_rowptr[row], end = L.h_rowptr[row + 1];
  hipError_t e = c->prec == 32
                     ? launch_wals_system(fallback_args<float>(c, L, R, 0, 0, alpha, lambda), beg,
                                          end, d, c->stream)
                     : launch_wals_system(fallback_args<double>(c, L, R, 0, 0, alpha, lambda), beg,
                                          end, d, c->stream);
  std::vector<double> h(nout);
  if (e == hipSuccess) e = scopy(c, h.data(), d, nout * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(std::string("qmfx_wals_row_system: ") + hipGetErrorString(e), -2);
  std::copy(h.begin(), h.begin() + (size_t)k * k, A);
  std::copy(h.begin() + (size_t)k * k, h.begin() + (size_t)k * k + k, b);
  if (csum) *csum = h[(size_t)k * k + k];
  return 0;
}

int qmfx_wals_set_row(qmfx_ctx* c, int side, int64_t row, const double* x) {
  SideBuf& L = c->s[side];
  if (row < 0 || row >= L.n) return fail("row out of range");
  if (set_dev(c)) return -2;
  const int kp = c->kp, k = c->k;
  if (c->prec == 32) {
    std::vector<float> h(kp, 0.f);
    for (int i = 0; i < k; ++i) h[i] = (float)x[i];
    HIPCHK(scopy(c, (float*)L.F + (size_t)row * kp, h.data(), kp * 4, hipMemcpyHostToDevice));
  } else {
    std::vector<double> h(kp, 0.0);
    for (int i = 0; i < k; ++i) h[i] = x[i];
    HIPCHK(scopy(c, (double*)L.F + (size_t)row * kp, h.data(), kp * 8, hipMemcpyHostToDevice));
  }
  return 0;
}

// ---- BPR ------------------------------------------------------------------------------------
int qmfx_bpr_set_positives(qmfx_ctx* c, const int64_t* users, const int64_t* items, int64_t npos) {
  const int64_t nu = c->s[0].n, ni = c->s[1].n;
  if (nu <= 0 || ni <= 0) return fail("shape not set (qmfx_set_shape)");
  if (set_dev(c)) return -2;
  std::vector<int32_t> it((size_t)std::max<int64_t>(npos, 1));
  for (int64_t e = 0; e < npos; ++e) {
    if (users[e] < 0 || users[e] >= nu || items[e] < 0 || items[e] >= ni)
      return fail("positive index out of range");
    it[e] = (int32_t)items[e];
  }
  dfree_t(c->pos_user);
  dfree_t(c->pos_item);
  dfree_t(c->urowptr);
  dfree_t(c->uitems);
  HIPCHK(hipMalloc(&c->pos_user, (size_t)std::max<int64_t>(npos, 1) * 8));
  HIPCHK(hipMalloc(&c->pos_item, (size_t)std::max<int64_t>(npos, 1) * 4));
  if (npos > 0) {
    HIPCHK(scopy(c, c->pos_user, users, (size_t)npos * 8, hipMemcpyHostToDevice));
    HIPCHK(scopy(c, c->pos_item, it.data(), (size_t)npos * 4, hipMemcpyHostToDevice));
  }
  // per-user sorted positive items (the reference's itemMap_, BPREngine.cpp:79-82)
  std::vector<uint64_t> keys((size_t)npos);
  for (int64_t e = 0; e < npos; ++e) keys[e] = (uint64_t)users[e] * (uint64_t)ni + (uint64_t)items[e];
  std::sort(keys.begin(), keys.end());
  std::vector<int64_t> rp((size_t)nu + 1, 0);
  std::vector<int32_t> ui((size_t)std::max<int64_t>(npos, 1));
  for (int64_t e = 0; e < npos; ++e) {
    rp[keys[e] / ni + 1]++;
    ui[e] = (int32_t)(keys[e] % ni);
  }
  c->max_user_pos = 0;
  for (int64_t u = 0; u < nu; ++u) c->max_user_pos = std::max(c->max_user_pos, rp[u + 1]);
  for (int64_t u = 0; u < nu; ++u) rp[u + 1] += rp[u];
  HIPCHK(hipMalloc(&c->urowptr, (size_t)(nu + 1) * 8));
  HIPCHK(hipMalloc(&c->uitems, ui.size() * 4));
  HIPCHK(scopy(c, c->urowptr, rp.data(), rp.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(scopy(c, c->uitems, ui.data(), ui.size() * 4, hipMemcpyHostToDevice));
  c->npos = npos;
  if (int rc = ensure_side_factors(c, 0)) return rc;
  if (int rc = ensure_side_factors(c, 1)) return rc;
  if (!c->bias) {
    HIPCHK(hipMalloc(&c->bias, (size_t)ni * c->esz));
    HIPCHK(hipMemsetAsync(c->bias, 0, (size_t)ni * c->esz, c->stream));
  }
  return 0;
}

int qmfx_bpr_set_biases(qmfx_ctx* c, const double* bias) {
  const int64_t ni = c->s[1].n;
  if (ni <= 0) return fail("shape not set");
  if (set_dev(c)) return -2;
  if (!c->bias) HIPCHK(hipMalloc(&c->bias, (size_t)ni * c->esz));
  if (c->prec == 32) {
    auto v = convert<float>(bias, (size_t)ni);
    HIPCHK(scopy(c, c->bias, v.data(), (size_t)ni * 4, hipMemcpyHostToDevice));
  } else {
    HIPCHK(scopy(c, c->bias, bias, (size_t)ni * 8, hipMemcpyHostToDevice));
  }
  return 0;
}

int qmfx_bpr_get_biases(qmfx_ctx* c, double* bias) {
  const int64_t ni = c->s[1].n;
  if (!c->bias) return fail("no biases");
  if (set_dev(c)) return -2;
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->prec == 32) {
    std::vector<float> v((size_t)ni);
    HIPCHK(scopy(c, v.data(), c->bias, (size_t)ni * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < ni; ++i) bias[i] = v[i];
  } else {
    HIPCHK(scopy(c, bias, c->bias, (size_t)ni * 8, hipMemcpyDeviceToHost));
  }
  return 0;
}

}  // extern "C"

static uint64_t gcd64(uint64_t a, uint64_t b) {
  while (b) {
    uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

template <typename T>
static BprArgs<T> bpr_args(qmfx_ctx* c, double lr, double bl, double ul, double il, int ub) {
  BprArgs<T> a{};
  a.U = (T*)c->s[0].F;
  a.I = (T*)c->s[1].F;
  a.bias = (T*)c->bias;
  a.pos_user = c->pos_user;
  a.pos_item = c->pos_item;
  a.npos = c->npos;
  a.urowptr = c->urowptr;
  a.uitems = c->uitems;
  a.nitems = c->s[1].n;
  a.lr = (T)lr;
  a.bias_lambda = (T)bl;
  a.user_lambda = (T)ul;
  a.item_lambda = (T)il;
  a.use_biases = ub;
  a.kp = c->kp;
  a.bad = c->bad;
  // Hogwild width: concurrent waves that touch the same user or item row read it stale (row
  // changes are added atomically, so no update is lost).  Keep the expected number of
  // concurrent waves per row small: ≈ min(nusers, nitems)/16 waves, capped at 16 waves per
  // CU (4096), at least 1 (a 3-user problem runs serially, as the reference's 1-thread
  // default does).
  const int64_t rows = std::min(c->s[0].n, c->s[1].n);
  a.waves = (int)std::max<int64_t>(1, std::min<int64_t>({4096, rows / 16, std::max<int64_t>(c->npos, 1)}));
  // The user row is stored plainly (an overwrite is the reference's Hogwild store) only while
  // two waves rarely hold the same user: the heaviest user's share of the positives times
  // the concurrent waves is the chance that another wave holds that user at a given moment.
  // Above 1% (skewed user activity) its net change is added atomically like the item rows.
  a.atomic_user = (double)a.waves * (double)c->max_user_pos > 0.01 * (double)std::max<int64_t>(c->npos, 1) ? 1 : 0;
  if (const char* f = std::getenv("QMFX_BPR_ATOMIC_USER")) a.atomic_user = std::atoi(f) ? 1 : 0;
  return a;
}

extern "C" {

int qmfx_bpr_epoch(qmfx_ctx* c, uint64_t seed, int num_neg, double lr, double bias_lambda,
                   double user_lambda, double item_lambda, int use_biases, int shuffle) {
  if (!c->pos_user) return fail("no positives (qmfx_bpr_set_positives)");
  if (c->npos == 0) return 0;
  if (set_dev(c)) return -2;
  uint64_t pa = 1, pb = 0;
  if (shuffle) {
    pa = (mix64(seed ^ 0xa5a5a5a5ull) % (uint64_t)c->npos) | 1ull;
    while (gcd64(pa, (uint64_t)c->npos) != 1) pa += 2;
    pa %= (uint64_t)c->npos;
    if (pa == 0) pa = 1;
    pb = mix64(seed ^ 0x5a5a5a5aull) % (uint64_t)c->npos;
  }
  HIPCHK(hipMemsetAsync(c->bad, 0, 4, c->stream));
  HIPCHK(hipEventRecord(c->ev0, c->stream));
  if (c->prec == 32) {
    auto a = bpr_args<float>(c, lr, bias_lambda, user_lambda, item_lambda, use_biases);
    a.num_neg = num_neg;
    a.seed = seed;
    a.perm_a = pa;
    a.perm_b = pb;
    c->bpr_waves = a.waves;
    c->bpr_atomic_user = a.atomic_user;
    HIPCHK(launch_bpr_epoch_f32(a, c->kp, c->stream));
  } else {
    auto a = bpr_args<double>(c, lr, bias_lambda, user_lambda, item_lambda, use_biases);
    a.num_neg = num_neg;
    a.seed = seed;
    a.perm_a = pa;
    a.perm_b = pb;
    c->bpr_waves = a.waves;
    c->bpr_atomic_user = a.atomic_user;
    HIPCHK(launch_bpr_epoch_f64(a, c->kp, c->stream));
  }
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  int32_t bad = 0;
  HIPCHK(hipMemcpyAsync(&bad, c->bad, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->solve_ms += ms;
  c->solve_launches += 1;
  const double upd = (double)c->npos * num_neg;
  c->solve_flops += upd * 10.0 * c->k;
  c->solve_bytes += upd * (6.0 * c->k * c->esz + 16 + 40);
  if (bad) return fail("gradients too big, try decreasing the learning rate (--init_learning_rate)", -4);
  return 0;
}

int qmfx_bpr_apply(qmfx_ctx* c, const int64_t* trip, int64_t n, double lr, double bias_lambda,
                   double user_lambda, double item_lambda, int use_biases) {
  if (set_dev(c)) return -2;
  if (int rc = ensure_side_factors(c, 0)) return rc;
  if (int rc = ensure_side_factors(c, 1)) return rc;
  if (!c->bias) {
    HIPCHK(hipMalloc(&c->bias, (size_t)c->s[1].n * c->esz));
    HIPCHK(hipMemsetAsync(c->bias, 0, (size_t)c->s[1].n * c->esz, c->stream));
  }
  for (int64_t t = 0; t < n; ++t)
    if (trip[3 * t] < 0 || trip[3 * t] >= c->s[0].n || trip[3 * t + 1] < 0 ||
        trip[3 * t + 1] >= c->s[1].n || trip[3 * t + 2] < 0 || trip[3 * t + 2] >= c->s[1].n)
      return fail("triplet index out of range");
  int64_t* d = nullptr;
  HIPCHK(hipMalloc(&d, (size_t)std::max<int64_t>(n, 1) * 24));
  HIPCHK(scopy(c, d, trip, (size_t)n * 24, hipMemcpyHostToDevice));
  HIPCHK(hipMemsetAsync(c->bad, 0, 4, c->stream));
  if (c->prec == 32) {
    auto a = bpr_args<float>(c, lr, bias_lambda, user_lambda, item_lambda, use_biases);
    HIPCHK(launch_bpr_apply_f32(a, d, n, c->kp, c->stream));
  } else {
    auto a = bpr_args<double>(c, lr, bias_lambda, user_lambda, item_lambda, use_biases);
    HIPCHK(launch_bpr_apply_f64(a, d, n, c->kp, c->stream));
  }
  int32_t bad = 0;
  HIPCHK(hipMemcpyAsync(&bad, c->bad, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  (void)hipFree(d);
  if (bad) return fail("gradients too big, try decreasing the learning rate (--init_learning_rate)", -4);
  return 0;
}

int qmfx_bpr_eval(qmfx_ctx* c, int slot, const int64_t* trip, int64_t n, int use_biases,
                  double* loss_sum) {
  if (slot != 0 && slot != 1) return fail("slot must be 0 or 1");
  if (set_dev(c)) return -2;
  if (c->trip_src[slot] != (const void*)trip || c->trip_n[slot] != n) {
    for (int64_t t = 0; t < n; ++t)
      if (trip[3 * t] < 0 || trip[3 * t] >= c->s[0].n || trip[3 * t + 1] < 0 ||
          trip[3 * t + 1] >= c->s[1].n || trip[3 * t + 2] < 0 || trip[3 * t + 2] >= c->s[1].n)
        return fail("triplet index out of range");
    dfree_t(c->trip[slot]);
    HIPCHK(hipMalloc(&c->trip[slot], (size_t)std::max<int64_t>(n, 1) * 24));
    HIPCHK(scopy(c, c->trip[slot], trip, (size_t)n * 24, hipMemcpyHostToDevice));
    c->trip_src[slot] = trip;
    c->trip_n[slot] = n;
  }
  if (c->prec == 32)
    HIPCHK(launch_bpr_eval_f32((const float*)c->s[0].F, (const float*)c->s[1].F,
                               (const float*)c->bias, c->trip[slot], n, c->kp, use_biases,
                               c->eval_partial, c->dsum, c->stream));
  else
    HIPCHK(launch_bpr_eval_f64((const double*)c->s[0].F, (const double*)c->s[1].F,
                               (const double*)c->bias, c->trip[slot], n, c->kp, use_biases,
                               c->eval_partial, c->dsum, c->stream));
  HIPCHK(hipMemcpyAsync(c->hsum, c->dsum, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *loss_sum = *c->hsum;
  return 0;
}

// ---- test-set evaluation ---------------------------------------------------------------------
int qmfx_eval_set_labels(qmfx_ctx* c, int64_t ntest, const int64_t* users, const int64_t* rowptr,
                         const int64_t* items, const double* values) {
  if (!c->s[0].F || !c->s[1].F) return fail("factors not allocated (qmfx_set_shape first)");
  if (ntest < 0) return fail("ntest out of range");
  if (c->k > 256) return fail("evaluation supports nfactors <= 256");
  if (set_dev(c)) return -2;
  const int64_t nu = c->s[0].n, ni = c->s[1].n;
  if (ntest > 0 && rowptr[0] != 0) return fail("label rowptr must start at 0");
  const int64_t nlab = ntest > 0 ? rowptr[ntest] : 0;
  std::vector<int32_t> slot((size_t)nlab);
  std::vector<int64_t> pidx((size_t)nlab), pptr((size_t)ntest + 1, 0);
  int64_t np = 0;
  for (int64_t t = 0; t < ntest; ++t) {
    if (users[t] < 0 || users[t] >= nu) return fail("test user index out of range");
    if (rowptr[t + 1] < rowptr[t]) return fail("label rowptr not ascending");
    pptr[(size_t)t] = np;
    for (int64_t e = rowptr[t]; e < rowptr[t + 1]; ++e) {
      if (items[e] < 0 || items[e] >= ni) return fail("label item index out of range");
      slot[(size_t)e] = (int32_t)t;
      pidx[(size_t)e] = values[e] > 0.0 ? np++ : -1;
    }
  }
  pptr[(size_t)ntest] = np;
  const int64_t nch = eval_chunks(ntest, ni);
  dfree_t(c->ev_users);
  dfree_t(c->ev_slot);
  dfree_t(c->ev_item);
  dfree_t(c->ev_pidx);
  dfree_t(c->ev_pptr);
  dfree_t(c->ev_lscore);
  dfree_t(c->ev_pscore);
  dfree_t(c->ev_above);
  dfree_t(c->ev_sq);
  dfree_t(c->ev_udbl);
  const size_t nl = (size_t)std::max<int64_t>(nlab, 1), npp = (size_t)std::max<int64_t>(np, 1);
  HIPCHK(hipMalloc(&c->ev_users, (size_t)std::max<int64_t>(ntest, 1) * 8));
  HIPCHK(hipMalloc(&c->ev_slot, nl * 4));
  HIPCHK(hipMalloc(&c->ev_item, nl * 8));
  HIPCHK(hipMalloc(&c->ev_pidx, nl * 8));
  HIPCHK(hipMalloc(&c->ev_pptr, ((size_t)ntest + 1) * 8));
  HIPCHK(hipMalloc(&c->ev_lscore, nl * 8));
  HIPCHK(hipMalloc(&c->ev_pscore, npp * 8));
  HIPCHK(hipMalloc(&c->ev_above, npp * 8));
  HIPCHK(hipMalloc(&c->ev_sq, (size_t)std::max<int64_t>(nch * ntest, 1) * 8));
  HIPCHK(hipMalloc(&c->ev_udbl, (size_t)std::max<int64_t>(eval_user_rows(ntest) * c->k, 1) * 8));
  HIPCHK(scopy(c, c->ev_users, users, (size_t)ntest * 8, hipMemcpyHostToDevice));
  HIPCHK(scopy(c, c->ev_slot, slot.data(), (size_t)nlab * 4, hipMemcpyHostToDevice));
  HIPCHK(scopy(c, c->ev_item, items, (size_t)nlab * 8, hipMemcpyHostToDevice));
  HIPCHK(scopy(c, c->ev_pidx, pidx.data(), (size_t)nlab * 8, hipMemcpyHostToDevice));
  HIPCHK(scopy(c, c->ev_pptr, pptr.data(), pptr.size() * 8, hipMemcpyHostToDevice));
  c->ev_ntest = ntest;
  c->ev_nlab = nlab;
  c->ev_npos = np;
  c->ev_chunks = nch;
  return 0;
}

}  // extern "C"

template <typename T>
static EvalArgs<T> eval_args(qmfx_ctx* c, int use_biases) {
  EvalArgs<T> a{};
  a.U = (const T*)c->s[0].F;
  a.I = (const T*)c->s[1].F;
  a.bias = use_biases ? (const T*)c->bias : nullptr;
  a.users = c->ev_users;
  a.ntest = c->ev_ntest;
  a.nitems = c->s[1].n;
  a.k = c->k;
  a.kp = c->kp;
  a.lab_slot = c->ev_slot;
  a.lab_item = c->ev_item;
  a.lab_pidx = c->ev_pidx;
  a.nlab = c->ev_nlab;
  a.lab_score = c->ev_lscore;
  a.pptr = c->ev_pptr;
  a.pscore = c->ev_pscore;
  a.above = c->ev_above;
  a.sq_part = c->ev_sq;
  a.udbl = c->ev_udbl;
  return a;
}

extern "C" {

int qmfx_eval_ranks(qmfx_ctx* c, int use_biases, double* label_scores, int64_t* above,
                    double* sq_sum) {
  if (!c->ev_users) return fail("no test labels (qmfx_eval_set_labels first)");
  if (use_biases && !c->bias) return fail("no item biases on the context");
  if (set_dev(c)) return -2;
  const int64_t nt = c->ev_ntest, nch = c->ev_chunks;
  HIPCHK(hipMemsetAsync(c->ev_above, 0, (size_t)std::max<int64_t>(c->ev_npos, 1) * 8, c->stream));
  if (c->prec == 32)
    HIPCHK(launch_eval_ranks(eval_args<float>(c, use_biases), c->stream));
  else
    HIPCHK(launch_eval_ranks(eval_args<double>(c, use_biases), c->stream));
  std::vector<double> part((size_t)(nch * nt));
  HIPCHK(scopy(c, label_scores, c->ev_lscore, (size_t)c->ev_nlab * 8, hipMemcpyDeviceToHost));
  HIPCHK(scopy(c, above, c->ev_above, (size_t)c->ev_npos * 8, hipMemcpyDeviceToHost));
  HIPCHK(scopy(c, part.data(), c->ev_sq, part.size() * 8, hipMemcpyDeviceToHost));
  for (int64_t t = 0; t < nt; ++t) {
    double v = 0.0;
    for (int64_t ch = 0; ch < nch; ++ch) v += part[(size_t)(ch * nt + t)];
    sq_sum[t] = v;
  }
  return 0;
}

// ---- multi-GPU -----------------------------------------------------------------------------
int qmfx_rccl_unique_id(uint8_t* id128) {
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  std::memcpy(id128, &id, 128);
  return 0;
}

}  // extern "C"

// This rank's row ranges of both sides, the row buckets, and (world > 1) the CSR shard.
static int dist_partition(qmfx_ctx* c) {
  const int rank = c->rank, world = c->world;
  for (int side = 0; side < 2; ++side) {
    SideBuf& sb = c->s[side];
    if (sb.h_rowptr.empty()) continue;
    if (sb.sharded) return fail("qmfx_dist_init: the CSR is already sharded (re-upload it first)");
    set_default_bounds(sb, world, rank);
    if (int rc = build_buckets(c, side)) return rc;
    if (world > 1)
      if (int rc = shard_csr(c, sb)) return rc;
  }
  return 0;
}

extern "C" {

int qmfx_dist_init(qmfx_ctx* c, int rank, int world, const uint8_t* id128) {
  if (world < 1 || rank < 0 || rank >= world) return fail("bad rank/world");
  if (set_dev(c)) return -2;
  c->rank = rank;
  c->world = world;
  // world = 1 with an id: a one-rank communicator, so a single GPU runs the RCCL calls of
  // the half (the self-broadcasts and the loss all-reduce) — the tests' loopback check
  if (id128) {
    ncclUniqueId id;
    std::memcpy(&id, id128, 128);
    NCCLCHK(ncclCommInitRank(&c->comm, world, id, rank));
    if (!c->comm_stream) HIPCHK(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
  }
  return dist_partition(c);
}

int qmfx_dist_init_all(qmfx_ctx* const* ctxs, int n) {
  if (n < 1 || !ctxs) return fail("qmfx_dist_init_all: no contexts");
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  std::vector<int> devs((size_t)n);
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i]) return fail("qmfx_dist_init_all: null context");
    if (ctxs[i]->comm) return fail("qmfx_dist_init_all: context already has a communicator");
    devs[(size_t)i] = ctxs[i]->device;
    for (int j = 0; j < i; ++j)
      if (devs[(size_t)j] == devs[(size_t)i])
        return fail("qmfx_dist_init_all: two contexts on device " + std::to_string(devs[(size_t)i]) +
                    " (one GPU per rank)");
    if (devs[(size_t)i] < 0 || devs[(size_t)i] >= ndev)
      return fail("qmfx_dist_init_all: " + std::to_string(n) + " ranks need device " +
                  std::to_string(devs[(size_t)i]) + " but only " + std::to_string(ndev) +
                  " GPU(s) are visible");
  }
  std::vector<ncclComm_t> comms((size_t)n);
  NCCLCHK(ncclCommInitAll(comms.data(), n, devs.data()));
  for (int i = 0; i < n; ++i) {
    qmfx_ctx* c = ctxs[i];
    if (set_dev(c)) return -2;
    c->comm = comms[(size_t)i];
    c->rank = i;
    c->world = n;
    if (!c->comm_stream) HIPCHK(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    if (int rc = dist_partition(c)) return rc;
  }
  return 0;
}

int qmfx_dist_plan(const int64_t* rowptr, int64_t nrows, int world, int npieces,
                   int64_t* pbounds) {
  if (world < 1) return fail("bad world size");
  if (npieces < 1 || npieces > QMFX_MAX_PIECES) return fail("npieces out of range");
  SideBuf sb;
  sb.n = nrows;
  sb.h_rowptr.assign(rowptr, rowptr + nrows + 1);
  set_default_bounds(sb, world, 0);
  std::vector<int64_t> pb;
  plan_pieces(sb.h_rowptr, sb.bounds, world, npieces, pb);
  std::copy(pb.begin(), pb.end(), pbounds);
  return 0;
}

int qmfx_partition_rows(const int64_t* rowptr, int64_t nrows, int world, int rank,
                        int64_t* begin, int64_t* end) {
  if (world < 1 || rank < 0 || rank >= world) return fail("bad rank/world");
  SideBuf sb;
  sb.n = nrows;
  sb.h_rowptr.assign(rowptr, rowptr + nrows + 1);
  set_default_bounds(sb, world, rank);
  *begin = sb.rbeg;
  *end = sb.rend;
  return 0;
}

// ---- measurement ---------------------------------------------------------------------------
int qmfx_solve_kernel_stats(qmfx_ctx* c, double* total_ms, int64_t* launches, double* flops,
                            double* bytes) {
  if (total_ms) *total_ms = c->solve_ms;
  if (launches) *launches = c->solve_launches;
  if (flops) *flops = c->solve_flops;
  if (bytes) *bytes = c->solve_bytes;
  return 0;
}

int qmfx_kernel_stats(qmfx_ctx* c, int cls, double* total_ms, int64_t* launches, double* flops,
                      double* bytes) {
  if (cls < 0 || cls > 2) return fail("class must be 0 (direct), 1 (whitened) or 2 (half)");
  if (total_ms) *total_ms = c->cls_ms[cls];
  if (launches) *launches = c->cls_launches[cls];
  if (flops) *flops = c->cls_flops[cls];
  if (bytes) *bytes = c->cls_bytes[cls];
  return 0;
}

int qmfx_kernel_stats_side(qmfx_ctx* c, int cls, int side, double* total_ms, int64_t* launches,
                           double* flops, double* bytes) {
  if (cls < 0 || cls > 2) return fail("class must be 0 (direct), 1 (whitened) or 2 (half)");
  if (side != 0 && side != 1) return fail("side must be 0 or 1");
  if (total_ms) *total_ms = c->side_ms[side][cls];
  if (launches) *launches = c->side_launches[side][cls];
  if (flops) *flops = c->side_flops[side][cls];
  if (bytes) *bytes = c->side_bytes[side][cls];
  return 0;
}

int qmfx_reset_stats(qmfx_ctx* c) {
  for (int sd = 0; sd < 2; ++sd) {
    c->xch_ms[sd] = c->xch_tail_ms[sd] = c->xch_solve_ms[sd] = 0;
    c->xch_halves[sd] = 0;
  }
  c->solve_ms = c->solve_flops = c->solve_bytes = 0;
  c->solve_launches = 0;
  for (int i = 0; i < 3; ++i) {
    c->cls_ms[i] = c->cls_flops[i] = c->cls_bytes[i] = 0;
    c->cls_launches[i] = 0;
    for (int sd = 0; sd < 2; ++sd) {
      c->side_ms[sd][i] = c->side_flops[sd][i] = c->side_bytes[sd][i] = 0;
      c->side_launches[sd][i] = 0;
    }
  }
  return 0;
}

int qmfx_exchange_stats(qmfx_ctx* c, int side, double* exchange_ms, double* exposed_ms,
                        double* solve_ms, int64_t* halves) {
  if (side != 0 && side != 1) return fail("side must be 0 or 1");
  if (exchange_ms) *exchange_ms = c->xch_ms[side];
  if (exposed_ms) *exposed_ms = c->xch_tail_ms[side];
  if (solve_ms) *solve_ms = c->xch_solve_ms[side];
  if (halves) *halves = c->xch_halves[side];
  return 0;
}

int qmfx_bpr_plan(qmfx_ctx* c, int* waves, int* atomic_user) {
  if (waves) *waves = c->bpr_waves;
  if (atomic_user) *atomic_user = c->bpr_atomic_user;
  return 0;
}

// A timing-variant build (tools/build_variant.sh) links an object that defines this; the
// product library does not, and reports "".
extern "C" __attribute__((weak)) const char* qmfx_variant_flags_tag(void);
const char* qmfx_build_variant(void) { return qmfx_variant_flags_tag ? qmfx_variant_flags_tag() : ""; }

int qmfx_selftest_mfma(int device, int precision, const double* A, const double* B, double* C) {
  HIPCHK(hipSetDevice(device));
  const size_t es = precision == 32 ? 4 : 8;
  void *dA, *dB, *dC;
  HIPCHK(hipMalloc(&dA, 64 * es));
  HIPCHK(hipMalloc(&dB, 64 * es));
  HIPCHK(hipMalloc(&dC, 256 * es));
  if (precision == 32) {
    auto a = convert<float>(A, 64), b = convert<float>(B, 64);
    HIPCHK(hipMemcpy(dA, a.data(), 256, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dB, b.data(), 256, hipMemcpyHostToDevice));
    HIPCHK(launch_mfma_selftest_f32((float*)dA, (float*)dB, (float*)dC, nullptr));
    std::vector<float> cc(256);
    HIPCHK(hipMemcpy(cc.data(), dC, 1024, hipMemcpyDeviceToHost));
    for (int i = 0; i < 256; ++i) C[i] = cc[i];
  } else {
    HIPCHK(hipMemcpy(dA, A, 512, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dB, B, 512, hipMemcpyHostToDevice));
    HIPCHK(launch_mfma_selftest_f64((double*)dA, (double*)dB, (double*)dC, nullptr));
    HIPCHK(hipMemcpy(C, dC, 2048, hipMemcpyDeviceToHost));
  }
  (void)hipFree(dA);
  (void)hipFree(dB);
  (void)hipFree(dC);
  return 0;
}

}  // extern "C"
