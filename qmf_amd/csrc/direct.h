// The direct row kernel (one wave64 per row: k×k Gram in registers + register-tile
// Cholesky) and its Gram loops, shared by the translation units that instantiate it:
// wals_direct_f32.hip, wals_direct_f64.hip (row solves) and wals_heavy.hip (split-K heavy
// rows).  Reference: WALSEngine::updateFactorsForOne, qmf/wals/WALSEngine.cpp:266-310, and
// linearSymmetricSolve (dsysv_), qmf/Matrix.cpp:81-96.  The math is in wals.hip's header.
#pragma once
#include <algorithm>
#include <utility>
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "rowsolve.h"
#include "chol.h"
#include "ntswitch.h"

namespace qmfx {

// (split3 / mma_split6: the fp32-accurate split-bf16 products, rowsolve.h; chol_solve: chol.h;
// the whitened row kernels: woodbury.hip)

// Factor-index permutation of the fp32 direct path.  Lane column c of "virtual" block B
// holds physical factor π(16B + c) = 16·W·(B / W) + W·c + (B mod W), so that one lane's
// W consecutive physical factors (one 16·W-byte load) feed W different MFMA blocks.  The
// Gram, the Cholesky and the right-hand side all live in the virtual order; the base
// YᵀY + λI is read through π and x is scattered back through π.
template <int NT>
struct Perm {
  static constexpr int W = (NT % 4 == 0) ? 4 : (NT % 2 == 0 ? 2 : 1);
  // the split-bf16 Gram pays from NT = 6 up; at k ≤ 64 the f32 loop keeps 3 waves/SIMD
  template <typename T>
  static constexpr bool split = sizeof(T) == 4 && NT >= 6;
  __device__ static __forceinline__ int phys(int v) {
    const int B = v >> 4, c = v & 15;
    return 16 * W * (B / W) + W * c + (B % W);
  }
};

// Direct-row Gram, fp32 on the bf16 matrix cores: 32 signals per step, lane (c, g) owns
// signals 8g..8g+7 of the step and virtual column c of every block.  Operands are √w·y
// (w = αv ≥ 0), so A and B are the same split values: A += Σ w y yᵀ; b = Σ c y from the
// raw rows.  The row's (column, value) pairs are staged through LDS 64 at a time (one
// coalesced load per lane, a chunk ahead), and each lane reads its 8 as two b128 pairs.
// Signals past the row's end point at the fixed side's all-zero row a.zrow with v = 0,
// so they add exactly nothing and need no masking.  Σc is summed at staging.  Pipeline:
// the rows of step s+1 are in flight while step s's MFMAs run.  A negative weight (1 + αv
// may still be > 0) sets `negw`; the caller flags the row for the host solve.
#ifndef QMFX_GRAM_HEAD
#define QMFX_GRAM_HEAD 100
#endif
#ifndef QMFX_GRAM_VALU
#define QMFX_GRAM_VALU 2
#endif
template <int NT>
__device__ __forceinline__ void gram_split_bf16(const SolveArgs<float>& a, int64_t beg,
                                                int64_t end, f32x4 (&acc)[NT * (NT + 1) / 2],
                                                float (&bpart)[NT], double& csum, int& negw,
                                                int lane, int (&mcol)[2][64],
                                                float (&mval)[2][64]) {
  constexpr int KP = 16 * NT;
  constexpr int W = Perm<NT>::W;
  constexpr int NG = NT / W;
  using vecW = float __attribute__((ext_vector_type(W)));
  const int c = lane & 15;
  const int g = lane >> 4;
  const int n = (int)(end - beg);
  const int nsteps = (n + 31) >> 5;
  const int nchunks = (n + 63) >> 6;
  float cs = 0.f;
  int pc = a.zrow;
  float pv = 0.f;
  // Every load below is issued unconditionally (past the row's end from a clamped address;
  // stage() then substitutes the zero row): a load skipped on some path makes the compiler's
  // waitcnt merge assume the shortest queue, and then each step waited for the gathers of
  // the step after it (the whole gather latency exposed twice per 64 signals).
  auto fetch = [&](int ch) {  // this lane's signal of chunk ch → raw (pc, pv)
    const int e = 64 * ch + lane;
    const int64_t src = beg + (e < n ? e : 0);
    pc = a.col[src];
    pv = a.val[src];
  };
  auto stage = [&](int ch) {  // (pc, pv) of chunk ch → LDS
    const bool ok = 64 * ch + lane < n;
    const float v = ok ? pv : 0.f;
    cs += ok ? 1.f + a.alpha * v : 0.f;
    mcol[ch & 1][lane] = ok ? pc : a.zrow;
    mval[ch & 1][lane] = v;
  };
  auto read_meta = [&](int st, int (&col)[8], float (&val)[8]) {
    const int o = 32 * (st & 1) + 8 * g;
    const int4 c0 = *reinterpret_cast<const int4*>(&mcol[(st >> 1) & 1][o]);
    const int4 c1 = *reinterpret_cast<const int4*>(&mcol[(st >> 1) & 1][o + 4]);
    const float4 v0 = *reinterpret_cast<const float4*>(&mval[(st >> 1) & 1][o]);
    const float4 v1 = *reinterpret_cast<const float4*>(&mval[(st >> 1) & 1][o + 4]);
    col[0] = c0.x, col[1] = c0.y, col[2] = c0.z, col[3] = c0.w;
    col[4] = c1.x, col[5] = c1.y, col[6] = c1.z, col[7] = c1.w;
    val[0] = v0.x, val[1] = v0.y, val[2] = v0.z, val[3] = v0.w;
    val[4] = v1.x, val[5] = v1.y, val[6] = v1.z, val[7] = v1.w;
  };
  auto load_rows = [&](const int (&col)[8], vecW (&y)[8][NG]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const vecW* yr =
          reinterpret_cast<const vecW*>(a.Y + (uint64_t)(uint32_t)col[j] * KP) + c;
#pragma unroll
      for (int G = 0; G < NG; ++G) y[j][G] = yr[16 * G];
    }
  };
  if (nsteps == 0) return;
  // prologue: chunks 0 and 1 staged (a chunk past the end as zero-row signals), chunk 2 in
  // flight, step 0's rows in flight
  fetch(0);
  stage(0);
  fetch(1);
  stage(1);
  fetch(2);
  // One step: the next step's rows go out first (into the other buffer, whose rows were
  // consumed one step ago), then each block is split right before the tiles of its block
  // row, so the split VALU of block I+1 issues in the free cycles of row I's MFMAs.  The
  // two buffers swap roles by a 2× unroll (no register copies).
  auto step = [&](int st, vecW (&yc)[8][NG], float (&vc)[8], vecW (&yn)[8][NG],
                  float (&vn)[8]) {
    __builtin_amdgcn_sched_barrier(0);
    {
      // (unconditional: past the last step this stages / fetches / gathers zero-row or
      // already-consumed signals whose results are never used)
      if (((st + 1) & 1) == 0) {
        // step st+1 opens chunk k = (st+1)/2: stage chunk k+1, fetch chunk k+2
        const int k = (st + 1) >> 1;
        stage(k + 1);
        fetch(k + 2);
      }
      int cn[8];
      read_meta(st + 1, cn, vn);
      load_rows(cn, yn);
    }
    // the next step's gathers all leave before this step's MFMAs start: each then has a
    // whole step to land (scheduled freely they trickled out between the MFMAs, the last
    // ones right before the next step waits on them)
    __builtin_amdgcn_sched_barrier(0);
    float sw[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float w = a.alpha * vc[j];
      const float cw = 1.f + w;
      negw |= w < 0.f;
      sw[j] = fast_sqrt(fabsf(w));
#pragma unroll
      for (int G = 0; G < NG; ++G)
#pragma unroll
        for (int m = 0; m < W; ++m) bpart[W * G + m] += cw * yc[j][G][m];
    }
    Split3 sp[NT];
#pragma unroll
    for (int I = 0; I < NT; ++I) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = sw[j] * yc[j][I / W][I % W];
      split3(x, sp[I]);
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        const int t = tile_index(I, J);
        acc[t] = mma_split6(sp[I], sp[J], acc[t]);
      }
    }
    // issue order: the sqrt/rhs VALU and block 0's split up front, then one MFMA and two
    // VALU at a time (an MFMA holds the vector issue for 8 of its 16 cycles)
    __builtin_amdgcn_sched_group_barrier(0x2, QMFX_GRAM_HEAD, 0);
#pragma unroll
    for (int i = 0; i < 6 * NT * (NT + 1) / 2; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x2, QMFX_GRAM_VALU, 0);
    }
  };
  int col0[8];
  float val0[8], val1[8];
  vecW y0[8][NG], y1[8][NG];
  read_meta(0, col0, val0);
  load_rows(col0, y0);
  // an even number of steps (a row with an odd count runs one step of zero-row signals), so
  // the loop body has no branch between the loads and their consumers
  for (int st = 0; st < 2 * nchunks; st += 2) {
    step(st, y0, val0, y1, val1);
    step(st + 1, y1, val1, y0, val0);
  }
  const double tot = wave_sum((double)cs);
  csum += lane == 0 ? tot : 0.0;  // the caller sums the cl == 0 lanes
}

// fp64 k = 112 / 128 direct Gram: the accumulator tiles are pinned to a register class by
// issuing the MFMA from inline asm — the first QMFX_F64_AG tiles in AGPRs (srcC / vdst may be
// AGPRs at full rate), the rest in VGPRs, so the step's rows, w·y and rhs stay in VGPRs.  With
// the builtin the allocator put 27 tiles in VGPRs and 9 in AGPRs, landed the gathered rows in
// AGPRs and copied them (and one rotating tile) through v_accvgpr moves at every step
// boundary.  The asm is opaque to the hazard recognizer: each MFMA carries its own 2 wait
// states for a VALU-written srcA/B/C (issued while the previous MFMA holds the pipe), and the
// loop's exit pads the f64 MFMA → VALU/VMEM read distance (gram_asm_drain).
#ifndef QMFX_F64_ASM
#define QMFX_F64_ASM 1
#endif
// Wait states the asm relies on (gfx950, MI355X_MICROARCH / the ISA's MFMA hazard table): a
// VALU write of an MFMA's srcA/B/C needs 2 before the MFMA (the `s_nop 1` in front of each
// asm MFMA; it issues while the previous MFMA holds the pipe); an f64 16x16x4 MFMA's result
// read by VALU / VMEM / a non-dependent MFMA needs up to 18 (gram_asm_drain's 3 × s_nop 7 at the
// loop exit).  tests/test_isa.py checks the compiled Gram loop: MFMAs only on pinned tiles,
// no v_accvgpr moves or scratch between them.
#ifndef QMFX_F64_AG
#define QMFX_F64_AG 24
#endif
// fp64 k > 64 row solves run gram_plain (DPP-broadcast signal pairs, a ring of PD row buffers)
// the ring depth of the other gram_plain instances (fp32 k ≤ 80, fp64 k ≤ 64)
#ifndef QMFX_PLAIN_PD
#define QMFX_PLAIN_PD 4
#endif
#ifndef QMFX_F64_PD
#define QMFX_F64_PD 2
#endif
template <bool AG>
__device__ __forceinline__ void mfma_f64_pinned(f64x4& c, double x, double y) {
  if constexpr (AG)
    asm("s_nop 1\n\tv_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(c) : "v"(x), "v"(y));
  else
    asm("s_nop 1\n\tv_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c) : "v"(x), "v"(y));
}
template <int i, int NTT>
__device__ __forceinline__ void pin_tiles(f64x4 (&acc)[NTT]) {
  if constexpr (i < NTT) {
    if constexpr (i < QMFX_F64_AG)
      asm volatile("" : "+a"(acc[i]));
    else
      asm volatile("" : "+v"(acc[i]));
    pin_tiles<i + 1, NTT>(acc);
  }
}
template <int NTT>
__device__ __forceinline__ void gram_asm_drain(f64x4 (&acc)[NTT]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  pin_tiles<0, NTT>(acc);
}
// the MFMAs of one 4-signal step, tile order (I, J ≤ I)
template <int i, int NTT, int NT>
__device__ __forceinline__ void gram_step_pinned(f64x4 (&acc)[NTT], const double (&yv)[NT],
                                                 const double (&wy)[NT]) {
  if constexpr (i < NTT) {
    constexpr int I = tile_row(i), J = i - I * (I + 1) / 2;
    mfma_f64_pinned<(i < QMFX_F64_AG)>(acc[i], yv[I], wy[J]);
    gram_step_pinned<i + 1, NTT, NT>(acc, yv, wy);
  }
}

// Direct-row Gram without the split (fp64, and fp32 at k ≤ 80): one 16x16x4 MFMA per tile
// per 4 signals, straight from the gathered rows.  Signals come in chunks of 64: lane (l, g)
// holds the (column, value) of signal 64c + g·S + l, where S = the chunk's step count (16;
// in a final partial chunk ⌈rest/4⌉ rounded up to PD), so step j's signal of lane group g
// sits in lane j of the same 16-lane row.  In the full chunks it arrives by one DPP row
// broadcast (compile-time lane, the chunk's 16 steps in straight line); the partial last
// chunk runs a loop of PD-step groups with shuffles.  The rows of step j + PD are gathered
// while step j's MFMAs run (PD register buffers); every load is issued unconditionally (past
// the end from a clamped address, replaced by the all-zero row a.zrow at use) and each step
// is its own scheduling region, so a step waits only for the buffer it consumes.  The next
// chunk's (column, value) pairs are loaded a whole chunk ahead.
template <typename T, int NT>
constexpr int plain_depth() {
  // fp64 k = 80..128 row and heavy-row solves: a ring of QMFX_F64_PD = 2 (the pinned
  // accumulators leave room for two row buffers: round 5, profiles/r05/ab_f64_pinned_gram_c3.txt,
  // 189.0 -> 180.0 ms per C3 item half); the one-step loop below remains only for the split-K
  // segment instance (MODE 1)
  return (sizeof(T) == 8 && NT > 4) ? QMFX_F64_PD : QMFX_PLAIN_PD;
}
template <int J>
__device__ __forceinline__ int row_bcast(int v) {
  // every lane has a source lane: no old operand (update_dpp(0, …) zero-initialised the
  // destination with one more v_mov per broadcast)
  return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xf, 0xf, true);
}
template <int J>
__device__ __forceinline__ float row_bcast(float v) {
  return __int_as_float(row_bcast<J>(__float_as_int(v)));
}
template <int J>
__device__ __forceinline__ double row_bcast(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = row_bcast<J>((int)(b & 0xffffffffll));
  const int hi = row_bcast<J>((int)(b >> 32));
  return __longlong_as_double(((long long)(unsigned)lo) | ((long long)hi << 32));
}

template <typename T, int NT, int PD>
__device__ __forceinline__ void gram_plain(const SolveArgs<T>& a, int64_t beg, int n,
                                           typename Mfma<T>::acc_t (&acc)[NT * (NT + 1) / 2],
                                           T (&bpart)[NT], double& csum, int lane) {
  using M = Mfma<T>;
  constexpr int KP = 16 * NT;
  constexpr bool ASM = QMFX_F64_ASM && sizeof(T) == 8 && NT * (NT + 1) / 2 > 21;
  static_assert(16 % PD == 0, "the ring must tile a chunk");
  const int cl = lane & 15;
  const int g = lane >> 4;
  if (n <= 0) return;
  const int nfull = n >> 6;
  // steps of chunk c: 16, or the partial chunk's ⌈rest/4⌉ rounded up to a multiple of PD
  // (0 past the end)
  auto steps_of = [&](int c) {
    const int rest = n - 64 * c;
    if (rest >= 64) return 16;
    const int st = rest > 0 ? (rest + 3) >> 2 : 0;
    return ((st + PD - 1) / PD) * PD;
  };
  // raw (clamped) loads of this lane's signal of chunk c; validity is re-derived at use
  auto load_chunk = [&](int c, int& cr, T& vr) {
    const int S = steps_of(c);
    const int e = 64 * c + g * S + cl;
    const int64_t src = beg + ((cl < S && e < n) ? e : 0);
    cr = a.col[src];
    vr = a.val[src];
  };
  T yb[PD][NT];
  T wb[PD], cwb[PD];
  // gather step j (its column cj / value vj broadcast from lane j of the row) into buffer b
  auto gather = [&](bool ok, int cj, T vj, int b) {
    const int col = ok ? cj : a.zrow;
    const T v = ok ? vj : T(0);
    wb[b] = a.alpha * v;
    cwb[b] = ok ? T(1) + a.alpha * v : T(0);
    const T* yrow = a.Y + (uint64_t)(uint32_t)col * KP + cl;
#pragma unroll
    for (int q = 0; q < NT; ++q) yb[b][q] = yrow[16 * q];
  };
  // step J of a chunk whose lane (l, g) signals start at base = 64c + g·S (S steps)
  auto issue = [&](auto Jc, int S, int base, int cr, T vr, int b) {
    constexpr int J = decltype(Jc)::value;
    // pinned here: hoisted to the chunk's start, 16 steps of broadcasts and addresses
    // stayed live across it (and spilled)
    int crx = cr;
    T vrx = vr;
    asm volatile("" : "+v"(crx), "+v"(vrx));
    gather(J < S && base + J < n, row_bcast<J>(crx), row_bcast<J>(vrx), b);
  };
  auto consume = [&](int b) {
    const T w = wb[b], cw = cwb[b];
    T wy[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      bpart[q] += cw * yb[b][q];
      wy[q] = w * yb[b][q];
    }
    csum += (double)cw;
    // pinned to the step: otherwise the rhs FMAs sink to the chunk's end and every step's
    // rows stay live (spilled) until then
#pragma unroll
    for (int q = 0; q < NT; ++q) asm volatile("" : "+v"(bpart[q]));
    asm volatile("" : "+v"(csum));
    if constexpr (ASM) {
      gram_step_pinned<0, NT * (NT + 1) / 2, NT>(acc, yb[b], wy);
    } else {
#pragma unroll
      for (int I = 0; I < NT; ++I) {
#pragma unroll
        for (int J2 = 0; J2 <= I; ++J2) {
          const int t = tile_index(I, J2);
          acc[t] = M::mma(yb[b][I], wy[J2], acc[t]);
        }
      }
    }
  };
  int cr, crn;
  T vr, vrn;
  load_chunk(0, cr, vr);
  load_chunk(1, crn, vrn);
  {
    const int S0 = steps_of(0);
    const int base0 = g * S0;
    [&]<int... P>(std::integer_sequence<int, P...>) {
      (issue(std::integral_constant<int, P>{}, S0, base0, cr, vr, P), ...);
    }(std::make_integer_sequence<int, PD>{});
  }
  // full chunks: 16 steps in straight line
  for (int c = 0; c < nfull; ++c) {
    const int base = 64 * c + 16 * g;
    const int Sn = steps_of(c + 1);
    const int basen = 64 * (c + 1) + g * Sn;
    [&]<int... J>(std::integer_sequence<int, J...>) {
      auto one = [&](auto Jc) {
        constexpr int j = decltype(Jc)::value;
        __builtin_amdgcn_sched_barrier(0);
        consume(j % PD);
        if constexpr (j + PD < 16)
          issue(std::integral_constant<int, j + PD>{}, 16, base, cr, vr, j % PD);
        else
          issue(std::integral_constant<int, j + PD - 16>{}, Sn, basen, crn, vrn, j % PD);
      };
      (one(std::integral_constant<int, J>{}), ...);
    }(std::make_integer_sequence<int, 16>{});
    __builtin_amdgcn_sched_barrier(0);
    cr = crn;
    vr = vrn;
    load_chunk(c + 2, crn, vrn);
  }
  // the partial chunk (its first PD steps already in the buffers)
  const int St = steps_of(nfull);
  const int baset = 64 * nfull + g * St;
  for (int j0 = 0; j0 < St; j0 += PD) {
    [&]<int... P>(std::integer_sequence<int, P...>) {
      auto one = [&](auto Pc) {
        constexpr int b = decltype(Pc)::value;
        __builtin_amdgcn_sched_barrier(0);
        consume(b);
        const int j = j0 + b + PD;  // next step for this buffer (lane j of the row)
        const int src = (g << 4) + (j & 15);
        gather(j < St && baset + j < n, __shfl(cr, src, 64), __shfl(vr, src, 64), b);
      };
      (one(std::integral_constant<int, P>{}), ...);
    }(std::make_integer_sequence<int, PD>{});
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (ASM) gram_asm_drain<NT * (NT + 1) / 2>(acc);
}

// ---------------------------------------------------------------------------------------
// Direct row kernel: one wave64 per row (slot order heaviest-first).  Gram
// A = G + λI + Σ w y yᵀ accumulated into the lower tiles held in registers, starting from
// the tile image of G + λI (gimg_kernel: one coalesced 16-B load per tile and lane);
// b = Σ c y and Σc on the side.  (A persistent variant that prefetched the next row's
// descriptor measured slower: the trace showed the gathers' latency is a small part of a
// row, and a fixed grid loses the dispatcher's balancing.)
// ---------------------------------------------------------------------------------------
#ifndef QMFX_WAVES_NT8
#define QMFX_WAVES_NT8 1
#endif
// waves per SIMD the direct kernel is compiled for: fp32 split-Gram and fp64 k > 64 tilings
// keep their accumulators in the whole (VGPR + AGPR) register file of one wave
template <typename T, int NT>
constexpr int direct_waves() {
  // fp64 k = 48 / 64: 3 / 2 waves (asked for 4, the row solve settled there anyway and the
  // split-K segment instance spilled 896 VGPRs)
  if constexpr (sizeof(T) == 8 && NT >= 3 && NT <= 4) return NT == 3 ? 3 : 2;
  return Perm<NT>::template split<T> ? QMFX_WAVES_NT8 : (sizeof(T) == 8 && NT > 4 ? 1 : (NT <= 4 ? 4 : 2));
}

// MODE (compile time, so the row-solve instance keeps its register allocation): 0 = row
// solve, 1 = split-K segment Gram, 2 = split-K heavy-row solve (SolveArgs::seg_mode)
template <typename T, int NT, bool TRACE, int MODE = 0>
__global__ __launch_bounds__(64, (direct_waves<T, NT>()))
void wals_direct_kernel(SolveArgs<T> a) {
  // fp32 at NT = 8: the split-bf16 Gram keeps 144 accumulator + 96 operand + 128 row
  // registers live: one wave per SIMD with the whole register file (QMFX_WAVES_NT8 = 1)
  using M = Mfma<T>;
  using acc_t = typename M::acc_t;
  constexpr int KP = 16 * NT;
  constexpr int NTT = NT * (NT + 1) / 2;
  __shared__ __attribute__((aligned(16))) CholShared<T, NT> S;
  __shared__ __attribute__((aligned(16))) T borig[KP];
  __shared__ __attribute__((aligned(16))) int mcol[2][64];
  __shared__ __attribute__((aligned(16))) float mval[2][64];

  const int lane = threadIdx.x;
  const int cl = lane & 15;
  const int kk = lane >> 4;
  {
    const RowDesc d = a.desc[a.row_begin + blockIdx.x];
    const int64_t row = d.row;
    const int64_t beg = d.beg;
    const int64_t end = beg + d.n;
    uint64_t tr[5] = {0, 0, 0, 0, 0};
    if (TRACE) tr[0] = __builtin_amdgcn_s_memtime();

    acc_t acc[NTT];
    // split-K heavy rows (SolveArgs::seg_mode): 1 = one segment's Gram from zero, 2 = the
    // row's reduced image (G + λI + Σ segments) in place of G + λI, with no signals
    if constexpr (MODE == 1) {
#pragma unroll
      for (int t = 0; t < NTT; ++t) acc[t] = acc_t{0, 0, 0, 0};
    } else {
      // buffer loads: the tile offset rides in the scalar offset, so no per-tile address
      // registers are kept
      constexpr int AB = (int)sizeof(acc_t);
      const T* src = MODE == 2 ? a.part + d.beg * (NTT * 256) : a.Gimg;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, NTT * 64 * AB, 0x00020000);
#pragma unroll
      for (int t = 0; t < NTT; ++t) {
#pragma unroll
        for (int h = 0; h < AB / 16; ++h) {
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * AB + 16 * h,
                                                                t * 64 * AB, 0);
          if constexpr (sizeof(T) == 4) {
            acc[t] = __builtin_bit_cast(acc_t, v);
          } else {
            const double lo = __builtin_bit_cast(double, (unsigned long long)v[0] |
                                                             ((unsigned long long)v[1] << 32));
            const double hi = __builtin_bit_cast(double, (unsigned long long)v[2] |
                                                             ((unsigned long long)v[3] << 32));
            acc[t][2 * h] = lo;
            acc[t][2 * h + 1] = hi;
          }
        }
      }
    }
    if (TRACE) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tr[1] = __builtin_amdgcn_s_memtime();
    }
    T bpart[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) bpart[c] = T(0);
    double csum = 0.0;
    int negw = 0;
    if constexpr (MODE == 2) {
      // the reduced rhs / Σc / flag of the row (lanes of group 0 and lane 0; the reductions
      // below then reproduce them)
      if (kk == 0) {
#pragma unroll
        for (int c = 0; c < NT; ++c) bpart[c] = a.partb[d.beg * KP + 16 * c + cl];
      }
      if (lane == 0) {
        csum = a.partc[2 * d.beg];
        negw = a.partc[2 * d.beg + 1] != 0.0;
      }
    }
    if constexpr (Perm<NT>::template split<T>) {
      gram_split_bf16<NT>(a, beg, end, acc, bpart, csum, negw, lane, mcol, mval);
    } else if constexpr (sizeof(T) == 8 && NT > 4 && MODE == 1) {
      // fp64 k > 64, split-K segment Grams (MODE 1): the
      // one-step loop, one step ahead (the row solves take gram_plain's ring above);
      // signals past the row's end gather the fixed side's all-zero row a.zrow with v = 0,
      // so they contribute exactly nothing without per-value selects (only Σc needs the
      // validity)
      // (the split-K segment instance keeps the builtin: pinned, its zero-initialised tiles
      // and the partial-image stores spilled 208 VGPRs)
      constexpr bool ASM = QMFX_F64_ASM && NTT > 21 && MODE != 1;
      for (int64_t base = beg; base < end; base += 64) {
        const int nst = (int)(end - base < 64 ? end - base : 64);
        const int cr = lane < nst ? a.col[base + lane] : a.zrow;
        const T vr = lane < nst ? a.val[base + lane] : T(0);
        bool valid = kk < nst;
        T v = __shfl(vr, kk, 64);
        T yn[NT];
        {
          const T* yrow = a.Y + (uint64_t)(uint32_t)__shfl(cr, kk, 64) * KP + cl;
#pragma unroll
          for (int q = 0; q < NT; ++q) yn[q] = yrow[16 * q];
        }
        for (int s = 0; 4 * s < nst; ++s) {
          T yv[NT];
#pragma unroll
          for (int q = 0; q < NT; ++q) yv[q] = yn[q];
          const T w = a.alpha * v;
          const T cw = valid ? T(1) + w : T(0);
          const int jn = 4 * (s + 1) + kk;
          const bool vn = jn < nst;
          if (4 * (s + 1) < nst) {
            // (lanes ≥ nst hold the zero row and v = 0)
            const int cn = __shfl(cr, jn < 64 ? jn : 63, 64);
            v = __shfl(vr, jn < 64 ? jn : 63, 64);
            const T* yrow = a.Y + (uint64_t)(uint32_t)cn * KP + cl;
#pragma unroll
            for (int q = 0; q < NT; ++q) yn[q] = yrow[16 * q];
          }
          valid = vn;
#pragma unroll
          for (int q = 0; q < NT; ++q) bpart[q] += cw * yv[q];
          csum += (double)cw;
          if constexpr (ASM) {
            T wy[NT];
#pragma unroll
            for (int q = 0; q < NT; ++q) wy[q] = w * yv[q];
            gram_step_pinned<0, NTT, NT>(acc, yv, wy);
          } else {
#pragma unroll
            for (int I = 0; I < NT; ++I) {
#pragma unroll
              for (int J = 0; J <= I; ++J) {
                const int t = tile_index(I, J);
                acc[t] = M::mma(yv[I], w * yv[J], acc[t]);
              }
            }
          }
        }
      }
      if constexpr (ASM) gram_asm_drain<NTT>(acc);
    } else {
      gram_plain<T, NT, plain_depth<T, NT>()>(a, beg, (int)(end - beg), acc, bpart, csum, lane);
    }
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      bpart[q] += shfl_xor(bpart[q], 16);
      bpart[q] += shfl_xor(bpart[q], 32);
      if (kk == 0 && MODE != 1) {
        borig[16 * q + cl] = bpart[q];
        S.bw[16 * q + cl] = bpart[q];
      }
    }
    csum = wave_sum(cl == 0 ? csum : 0.0);  // each k-slot row counted once
    int bad = __any(negw) ? 1 : 0;  // split Gram with a negative weight: solved on the host
    if constexpr (MODE == 1) {
      // one segment of a heavy row: its partial tiles, rhs, Σc and flag to the segment's slot
      const int64_t seg = a.row_begin + blockIdx.x;
      acc_t* o = reinterpret_cast<acc_t*>(a.part + seg * (NTT * 256));
#pragma unroll
      for (int t = 0; t < NTT; ++t) o[t * 64 + lane] = acc[t];
      if (kk == 0) {
#pragma unroll
        for (int q = 0; q < NT; ++q) a.partb[seg * KP + 16 * q + cl] = bpart[q];
      }
      if (lane == 0) {
        a.partc[2 * seg] = csum;
        a.partc[2 * seg + 1] = (double)bad;
      }
      return;
    }
    __syncthreads();
    if (TRACE) tr[2] = __builtin_amdgcn_s_memtime();
    row_chol<T, NT>(acc, S, lane, bad);
    if (TRACE) tr[3] = __builtin_amdgcn_s_memtime();

    double xb = 0.0, xx = 0.0;
    for (int j = lane; j < KP; j += 64) {
      const T xj = S.xs[j];
      // a failed row stores x = 0 (loss term 0), like the whitened kernel; the caller
      // re-solves it
      a.X[row * KP + (Perm<NT>::template split<T> ? Perm<NT>::phys(j) : j)] = bad ? T(0) : xj;
      xb += (double)xj * (double)borig[j];
      xx += (double)xj * (double)xj;
    }
    xb = wave_sum(xb);
    xx = wave_sum(xx);
    if (lane == 0) {
      a.rowloss[row] = bad ? 0.0 : csum - xb - (double)a.lambda * xx;
      if (bad && a.status) a.status[row] = 1;
    }
    if (TRACE && lane == 0) {
      tr[4] = __builtin_amdgcn_s_memtime();
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint64_t* o = a.trace + 8 * (a.row_begin + blockIdx.x);
#pragma unroll
      for (int j = 0; j < 5; ++j) o[j] = tr[j];
      o[5] = hw | ((uint64_t)xcc << 32);
      o[6] = (uint64_t)d.n;
      o[7] = (uint64_t)row;
    }
  }
}

// One launch (in row chunks) of wals_direct_kernel in a compile-time mode.
template <typename T, int NT, int MODE>
hipError_t launch_direct_mode(const SolveArgs<T>& a, hipStream_t s) {
  if (a.nrows <= 0) return hipSuccess;
  if (!a.desc || !a.Gimg) return hipErrorInvalidValue;
  return launch_row_chunks(a, 64, [&](const SolveArgs<T>& c) {
    if constexpr (MODE != 0)
      hipLaunchKernelGGL((wals_direct_kernel<T, NT, false, MODE>), dim3((unsigned)c.nrows), dim3(64), 0, s, c);
    else if (c.trace)
      hipLaunchKernelGGL((wals_direct_kernel<T, NT, true>), dim3((unsigned)c.nrows), dim3(64), 0, s, c);
    else
      hipLaunchKernelGGL((wals_direct_kernel<T, NT, false>), dim3((unsigned)c.nrows), dim3(64), 0, s, c);
  });
}

}  // namespace qmfx
