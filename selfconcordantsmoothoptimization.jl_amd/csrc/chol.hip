// Blocked Cholesky G = UᵀU (upper, column-major, in place) and the two
// triangular solves, for the m x m system of ProxNSCORE / ProxGGNSCORE
// (`(H + λ·Diagonal(Hr)) \ ∇q`, prox-N-SCORE.jl:204; `qr(JQJ) \ Je`,
// prox-GGN-SCORE.jl:131 -- the system is SPD whenever Q ⪰ 0, the LU
// fallback in scsopt.cpp covers the rest).
//
// Why upper: in column-major storage the block row k of U (U_kj, j > k) has
// its 128 rows contiguous per column, which is exactly the operand layout of
// the MFMA Gram kernel (contraction along the contiguous index).  So
//   panel solve      U_kj = U_kk⁻ᵀ A_kj     = Gram(P = U_kk⁻¹, Q = A_kj), in place
//   trailing update  A_ij -= U_kiᵀ U_kj     = Gram(row panel k, w = -1), accumulate,
//                                               transposed store (upper triangle)
// both run on gram_f64_kernel (MFMA); only the 128 x 128 diagonal block is
// factorized (and inverted) by a single workgroup in LDS.  The diagonal-block
// inverses are kept, so both triangular solves become 128 x 128 matvecs plus a
// streaming panel update per block step.
//
// Layout: G is m_pad x m_pad, ld = m_pad, m_pad % 128 == 0; the padded tail of
// the diagonal is set to 1 by the caller (block-diag(A, I)).
#include <algorithm>
#include <cstdlib>
#include <functional>
#include <vector>

#include "common.h"
#include "gram_strip.h"
#include "kernels.h"

namespace scs {

constexpr int CB = 128;          // block size (= Gram tile edge)
constexpr int CLD = CB + 1;      // LDS row pitch (doubles) -> conflict-light column access

// Factor the diagonal block U_kk (upper) of G in place and write W_k = U_kk⁻¹
// (upper, column-major 128 x 128).  info: first non-positive pivot (1-based,
// global); the caller then takes the LU path.
//
// Inner-blocked (b = 16) right-looking factorization of the LDS copy S:
//   A  wave 0 factors the 16 x 16 diagonal sub-block in registers (lane c =
//      column c; row values broadcast with v_readlane), reciprocal pivots to LDS;
//   B  panel: forward substitution Dᵀ P = S(o:o+16, c), one column per thread;
//   C  trailing update of the upper triangle with 4 x 4 register tiles.
// Then W = U⁻¹: the eight 16 x 16 diagonal inverses (two per wave, in
// registers), and recursive doubling W12 = -W11 · (U12 · W22) at block sizes
// 16 -> 32 -> 64 -> 128 on MFMA (chol_inv_double_mfma); the intermediate T = U12·W22
// lives in the (unused) strictly-lower triangle of S.  Only the factorization steps
// are a serial chain.
constexpr int SB = 16;

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

#ifdef CHOL_PROF
// probe_chol -DCHOL_PROF: thread 0 records s_memrealtime (100 MHz) at phase boundaries
__device__ long long chol_prof[128];
#define PROF_MARK(i) \
  if (threadIdx.x == 0 && k == 0) chol_prof[i] = (long long)__builtin_amdgcn_s_memrealtime()
#define PROF_MARK_T(i, t) \
  if (threadIdx.x == (t) && k == 0) chol_prof[i] = (long long)__builtin_amdgcn_s_memrealtime()
#else
#define PROF_MARK(i)
#define PROF_MARK_T(i, t)
#endif
#ifdef CHOL_DTIME
// probe_chol -DCHOL_DTIME: every diagonal-kernel launch's entry / exit (s_memrealtime, 100 MHz) by
// block index, to split its traced duration into waiting for a CU and running
__device__ long long chol_dtime[2 * 1024];
#define DTIME_MARK(i) \
  if (threadIdx.x == 0) chol_dtime[2 * k + (i)] = (long long)__builtin_amdgcn_s_memrealtime()
#else
#define DTIME_MARK(i)
#endif

constexpr int DNT = 256;
// W = U⁻¹ by block columns beside the factor (w_column_t) instead of the recursive doubling after it
// (chol_inv_double_mfma, kept for tri_inv_kernel / wy_t_kernel); compile-time A/B switch
#ifndef CHOL_W_DOUBLING
constexpr bool W_BY_COLUMNS = true;
#else
constexpr bool W_BY_COLUMNS = false;
#endif          // threads of chol_diag_kernel (4 waves; 512 spills: measured slower)

// One doubling level of W = U⁻¹ for every pair (i0 = 2pS, j0 = i0 + S):
//   step 1  T(r, c) = Σ_{t <= c} U(i0+r, j0+t) W(j0+t, j0+c)   -> S[j0 + r][i0 + c] (strictly lower)
//   step 2  W(i0+r, j0+c) = -Σ_{t >= r} W(i0+r, i0+t) T(t, c)  -> S[i0 + r][j0 + c]
// on MFMA: S x S products as 16 x 16 output tiles (S/4 MFMAs each), (pair, tile) items round-robin
// over the waves.  Fragment maps as in phase C; the triangular operands are masked per lane (W22:
// k <= j; W11: k >= i) AFTER unconditional LDS reads: a masked read compiles to a branch the
// compiler cannot hoist, one LDS wait per MFMA (doubling + W store 17.4 -> 11.5 us).  (Skipping the
// k blocks that lie wholly in the zero part of the triangle -- 5/8 of the MFMAs at S = 64 -- with a
// run-time trip count measured slower, 13.0 us: the reads of a block then wait in front of its MFMAs.)
template <int S>
__device__ __forceinline__ void chol_inv_double_mfma(double* su, int tid) {
  constexpr int NP = CB / (2 * S), NT16 = (S / 16) * (S / 16);
  const int wv = tid >> 6, lane = tid & 63, li = lane & 15, lk = lane >> 4;
  for (int it = wv; it < NP * NT16; it += DNT / 64) {   // step 1: T = U12 · W22 -> strictly lower
    const int pair = it / NT16, tt = it % NT16;
    const int i0 = 2 * S * pair, j0 = i0 + S;
    const int ti = 16 * (tt / (S / 16)), tj = 16 * (tt % (S / 16));
    v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t0 = 0; t0 < S; t0 += 4) {
      const int k = t0 + lk;
      const double a = su[(j0 + k) * CLD + i0 + ti + li];
      const double bl = su[(j0 + tj + li) * CLD + j0 + k];
      const double b = (k <= tj + li) ? bl : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) su[(i0 + tj + li) * CLD + j0 + ti + lk + 4 * r] = acc[r];
  }
  __syncthreads();
  for (int it = wv; it < NP * NT16; it += DNT / 64) {   // step 2: W12 = -W11 · T
    const int pair = it / NT16, tt = it % NT16;
    const int i0 = 2 * S * pair, j0 = i0 + S;
    const int ti = 16 * (tt / (S / 16)), tj = 16 * (tt % (S / 16));
    v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t0 = 0; t0 < S; t0 += 4) {
      const int k = t0 + lk;
      const double al = su[(i0 + k) * CLD + i0 + ti + li];
      const double a = (k >= ti + li) ? al : 0.0;
      const double b = su[(i0 + tj + li) * CLD + j0 + k];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) su[(j0 + tj + li) * CLD + i0 + ti + lk + 4 * r] = -acc[r];
  }
  __syncthreads();
}

// 64-bit DPP lane move within each quad: lane 4c + t takes lane 4c + Q (quad_perm Q,Q,Q,Q)
template <int Q>
__device__ __forceinline__ double quad_bcast(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, Q * 0x55, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), Q * 0x55, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// LDS layouts of the diagonal block S (upper triangle + zeros below the diagonal of the 16 x 16
// diagonal sub-blocks).  idxb(I, C, rr, cc) = S(16 I + rr, 16 C + cc), I <= C.
//   LayFull: the whole 128 x 128 block column-major with pitch CLD = 129 (132 KiB).
//   LayPack (r06): only the 36 upper 16 x 16 blocks, block (I, C) at (C (C + 1) / 2 + I)·272, each
//     column-major with pitch 17 (the same bank spread as CLD within a block): 76.5 KiB, so that with
//     the rest (~96 KiB) the kernel fits beside one workgroup of the trailing-update Gram kernel
//     (32 KiB LDS, 256 VGPRs per lane) instead of waiting for a whole CU to drain.
// Every element takes the same arithmetic in the same order in both: the same U, W and pivots.
constexpr int PBP = 17, PBS = SB * PBP, NPB = (CB / SB) * (CB / SB + 1) / 2;
struct LayFull {
  static constexpr bool packed = false;
  static constexpr int words = CB * CLD;
  __device__ static __forceinline__ int idxb(int I, int C, int rr, int cc) { return (16 * C + cc) * CLD + 16 * I + rr; }
};
struct LayPack {
  static constexpr bool packed = true;
  static constexpr int words = NPB * PBS;
  __device__ static __forceinline__ int idxb(int I, int C, int rr, int cc) {
    return (C * (C + 1) / 2 + I) * PBS + cc * PBP + rr;
  }
};

// Phase A: wave 0 factors the 16 x 16 diagonal sub-block at o in registers, reciprocal pivots to
// srinv.  Lane 4c + q holds rows 4q .. 4q+3 of column c (a[s] = S(o+4q+s, o+c)), so all 64 lanes
// work and a column step is ~35 instructions instead of ~80 (the one-column-per-lane form
// broadcast each of the 15 row-j values with a v_readlane pair and spilled SGPRs).  Per column j:
// the pivot by v_readlane; row j scaled in the lanes of quarter j/4; U(j, c) to the other lanes of
// the column's quad by DPP; U(j, i) of the lane's own rows from a 16-double LDS row copy (urow).
// The serial chain is pivot -> rsq -> row scale -> DPP -> the next pivot's update (pnext), computed
// ahead of the LDS-fed updates.  Every element takes the same fused multiply-subtracts in the same
// j order as the one-column-per-lane form: bitwise the same U and pivots.
template <class L>
__device__ __forceinline__ void diag_factor16(double* su, double* srinv, double* urow, int o, int k, int* info,
                                              int tid) {
  const int kb = o >> 4;
  int c = (tid & 63) >> 2, q = tid & 3;
  // opaque per call: keeps the compiler from hoisting the lane masks out of the inner-block loop
  asm volatile("" : "+v"(c), "+v"(q));
  double a[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) a[s] = su[L::idxb(kb, kb, 4 * q + s, c)];   // zero below the diagonal
  double pnext = a[0];   // S(j, j) of the next pivot, in lane 4j + j/4
  double rr[SB];         // the reciprocal pivots (wave-uniform), to srinv after the loop
  int bad = -1;
#pragma unroll
  for (int j = 0; j < SB; ++j) {
    const int jq = j >> 2, js = j & 3;
    const double ajj = readlane_d(pnext, 4 * j + jq);
    bad = (bad < 0 && !(ajj > 0.0)) ? j : bad;   // the first non-positive pivot, off the chain
    // 1/sqrt(ajj): v_rsq_f64 + two Newton steps (6 dependent FMAs instead of the
    // sqrt + divide sequences on this serial chain); d = ajj * r
    double r = __builtin_amdgcn_rsq(ajj);
    const double hj = 0.5 * ajj;
#pragma unroll
    for (int it = 0; it < 2; ++it) r = fma(r, fma(-hj * r, r, 0.5), r);
    const double d = ajj * r;
    rr[j] = r;
    // row j of U, U(j, c), in the lanes of quarter jq (slot js)
    const double ar = a[js] * r;
    const double sc = (c > j) ? ar : ((c == j) ? d : a[js]);
    a[js] = (q == jq) ? sc : a[js];
    if (j == SB - 1) break;
    // U(j, c) in every lane of column c's quad, straight from the product (the selects above are off
    // the chain: in columns c <= j it feeds only rows i > c, which are never stored)
    double ujc;
    switch (jq) {
      case 0: ujc = quad_bcast<0>(ar); break;
      case 1: ujc = quad_bcast<1>(ar); break;
      case 2: ujc = quad_bcast<2>(ar); break;
      default: ujc = quad_bcast<3>(ar); break;
    }
    // the next pivot first: S(j+1, j+1) -= U(j, j+1)² (its lane holds U(j, j+1) as ujc)
    const int s1 = (j + 1) & 3;
    pnext = fma(-ujc, ujc, a[s1]);
    if (q == jq) urow[c] = ar;   // = U(j, c) wherever it is read (columns c > j)
    // the other lanes' row-j values: without a (wavefront-scope, instruction-free) fence the compiler
    // may reuse a lane's previous-iteration loads where that lane did not store itself
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const v2d u01 = *(const v2d*)(urow + 4 * q), u23 = *(const v2d*)(urow + 4 * q + 2);
    const double uji[4] = {u01[0], u01[1], u23[0], u23[1]};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (4 * q + s > j) a[s] = fma(-uji[s], ujc, a[s]);   // rows i > j: S(i, c) -= U(j, i) U(j, c)
  }
#pragma unroll
  for (int s = 0; s < 4; ++s)
    if (4 * q + s <= c) su[L::idxb(kb, kb, 4 * q + s, c)] = a[s];
  if (tid == 0) {
#pragma unroll
    for (int j = 0; j < SB; ++j) srinv[o + j] = rr[j];
    if (bad >= 0 && *info == 0) *info = k * CB + o + bad + 1;
  }
}

// Phase B: panel, forward substitution Dᵀ p = x per column (D(u, t) reads are wave-uniform)
template <class L>
__device__ __forceinline__ void diag_panel16(double* su, const double* srinv, int o, int np, int tid) {
  if (tid < np) {
    const int kb = o >> 4;
    const int c = o + SB + tid, C = c >> 4, cc = c & 15;
    double X[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) X[u] = su[L::idxb(kb, C, u, cc)];
    // right-looking: X[t] takes D(u, t) X[u] as soon as X[u] is final -- the same fused
    // multiply-subtracts in the same u order as the dot-product form (bit-identical), but the
    // dependent chain is 16 x (fma + mul) instead of all 120 fmas in a row
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      X[u] *= srinv[o + u];
#pragma unroll
      for (int t = u + 1; t < SB; ++t) X[t] -= su[L::idxb(kb, kb, u, t)] * X[u];
    }
#pragma unroll
    for (int u = 0; u < SB; ++u) su[L::idxb(kb, C, u, cc)] = X[u];
  }
}

// Phase C, one 16 x 16 upper tile `id` (C-major: id = C(C+1)/2 + I, I <= C) of the trailing
// update S(i, c) -= Σ_t U(o + t, i) U(o + t, c), o+16 <= i <= c, as 4 x v_mfma_f64_16x16x4
// (A[i][k] = U(o+t0+k, i0+i), B[k][j] = U(o+t0+k, c0+j); lane l feeds i|j = l&15, k = l>>4;
// D row = (l>>4) + 4r, col = l&15).  Diagonal tiles update only i <= c: phase A reads the
// zeros below the diagonal.  Tile 0 is the next diagonal sub-block.
template <class L>
__device__ __forceinline__ void diag_trail_tile(double* su, int o, int id, int lane) {
  const int li = lane & 15, lk = lane >> 4;
  int C = 0;
  while ((C + 1) * (C + 2) / 2 <= id) ++C;
  const int I = id - C * (C + 1) / 2;
  const int kb = o >> 4, BI = kb + 1 + I, BC = kb + 1 + C;   // the tile's block row / column of S
  v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t0 = 0; t0 < SB; t0 += 4) {
    const double a = su[L::idxb(kb, BI, t0 + lk, li)];
    const double b = su[L::idxb(kb, BC, t0 + lk, li)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (I < C || lk + 4 * r <= li) su[L::idxb(BI, BC, lk + 4 * r, li)] -= acc[r];   // i <= c
  }
}

// W = U⁻¹ by block columns (r04; replaces the recursive doubling on the chain): block column J of W
// (16 columns, rows of blocks 0..J) by ONE wave, in registers: W_JJ = inv(U_JJ) (swinv), then
// W_iJ = -inv(U_ii) · Σ_{l=i+1..J} U_il W_lJ for i = J-1 .. 0, right-looking -- as soon as W_lJ is
// final every pending sum S_i (i < l) takes U_il W_lJ (l descending), so the dependent chain is
// W_l -> S_{l-1} -> W_{l-1}, 8 MFMAs per block.  The accumulator of an MFMA (acc[r] = D[(lane>>4) +
// 4r][lane & 15]) is directly the B operand of the next one's k-chunk r, so W never goes through
// LDS; U_il are A operands read from su (final: written before the barrier of step i), swinv[i] too.
// Column J needs U rows 0..J and swinv[0..J]: it can run in the step after inv16(J), beside the
// factor (the doubling needed all of U first: 11.5 us after the loop).  The column goes straight to
// global W (zeros below its diagonal block).  Fixed order per element: bitwise run to run, and the
// same bits in both kernel schedules (PIPE or not).
template <int J, class L>
__device__ __forceinline__ void w_column_t(const double* su, const double* swv /*[CB/SB][SB*SB]*/, double* Wk,
                                           int lane, double* su_w) {
  const int li = lane & 15, lk = lane >> 4;
  v4d W[J + 1], S[J + 1];
#pragma unroll
  for (int r = 0; r < 4; ++r) W[J][r] = swv[J * SB * SB + li * SB + lk + 4 * r];
#pragma unroll
  for (int i = 0; i < J; ++i) S[i] = (v4d){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int l = J; l >= 1; --l) {
#pragma unroll
    for (int i = l - 1; i >= 0; --i)   // S_i += U_il W_lJ (i = l - 1 first: the chain)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        S[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(su[L::idxb(i, l, li, 4 * q + lk)], W[l][q], S[i], 0, 0, 0);
    v4d acc = {0.0, 0.0, 0.0, 0.0};   // W_{l-1,J} = -inv(U_{l-1,l-1}) S_{l-1}
#pragma unroll
    for (int q = 0; q < 4; ++q)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(swv[(l - 1) * SB * SB + (4 * q + lk) * SB + li], S[l - 1][q], acc, 0, 0, 0);
    W[l - 1] = -acc;
  }
  double* col = Wk + (int64_t)(16 * J + li) * CB + lk;
#pragma unroll
  for (int i = 0; i < CB / SB; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) col[16 * i + 4 * r] = (i <= J) ? W[i <= J ? i : 0][r] : 0.0;
  // the off-diagonal blocks also into the (unused, zero) strictly-lower triangle of su, transposed:
  // W(r, c) at su[r·CLD + c] -- w_last_column_par reads them there (r05).  LayPack has no lower
  // triangle: w_last_column_par reads them back from Wk
  if (!L::packed && J < CB / SB - 1) {
#pragma unroll
    for (int i = 0; i < J; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) su_w[(16 * i + lk + 4 * r) * CLD + 16 * J + li] = W[i][r];
  }
}

template <class L>
__device__ __forceinline__ void w_column(double* su, const double* swv, double* Wk, int J, int lane) {
  switch (J) {
    case 0: w_column_t<0, L>(su, swv, Wk, lane, su); break;
    case 1: w_column_t<1, L>(su, swv, Wk, lane, su); break;
    case 2: w_column_t<2, L>(su, swv, Wk, lane, su); break;
    case 3: w_column_t<3, L>(su, swv, Wk, lane, su); break;
    case 4: w_column_t<4, L>(su, swv, Wk, lane, su); break;
    case 5: w_column_t<5, L>(su, swv, Wk, lane, su); break;
    case 6: w_column_t<6, L>(su, swv, Wk, lane, su); break;
    default: w_column_t<7, L>(su, swv, Wk, lane, su); break;
  }
}

// W's last block column J = 7 by all four waves (r05; was w_column_t<7> on one wave after the loop,
// 7 dependent steps, 5.7 us): the block inverse of an upper-triangular matrix,
//   W_{0:J, J} = -W_{0:J, 0:J} · (U_{0:J, J} · W_JJ),
// so V_l = U_lJ W_JJ (W_JJ = swinv[J] as the B operand; every wave forms all J of them, 4 MFMAs each,
// and the accumulator layout D[(lane>>4) + 4r][lane & 15] is the next MFMA's B operand), then
// W_iJ = -Σ_{l=i}^{J-1} W_il V_l for the wave's row blocks (W_ii = swinv[i]; W_il, l > i, from the
// transposed copies w_column_t left in su's strictly-lower triangle).  Row blocks {w, 6-w} per wave
// w < 3 and {3} for wave 3: 32 / 32 / 32 / 16 MFMAs of the second level.  Fixed order per element.
template <class L>
__device__ __forceinline__ void w_last_column_par(const double* su, const double* swv, double* Wk, int tid) {
  constexpr int J = CB / SB - 1;
  const int lane = tid & 63, wv = tid >> 6, li = lane & 15, lk = lane >> 4;
  // LayPack: W_il (i < l < J) from Wk, where w_column_t<l> stored it before the kernel's last barrier;
  // all of a wave's loads are issued first, so their latency runs under the V products
  const int i1 = wv < 3 ? wv : 3, i2 = wv < 3 ? J - 1 - wv : -1;
  double g1[J][4], g2[J][4];
  if (L::packed) {
#pragma unroll
    for (int l = 0; l < J; ++l)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t off = (int64_t)(16 * l + 4 * q + lk) * CB + li;
        g1[l][q] = (l > i1) ? Wk[off + 16 * i1] : 0.0;
        g2[l][q] = (i2 >= 0 && l > i2) ? Wk[off + 16 * i2] : 0.0;
      }
  }
  v4d V[J];
#pragma unroll
  for (int l = 0; l < J; ++l) {
    v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(su[L::idxb(l, J, li, 4 * q + lk)],
                                                 swv[J * SB * SB + li * SB + 4 * q + lk], acc, 0, 0, 0);
    V[l] = acc;
  }
  auto rowblock = [&](int i, const double (*g)[4]) {
    v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int l = 0; l < J; ++l) {
      if (l < i) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double a = (l == i) ? swv[i * SB * SB + (4 * q + lk) * SB + li]
                                  : (L::packed ? g[l][q] : su[(16 * i + li) * CLD + 16 * l + 4 * q + lk]);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, V[l][q], acc, 0, 0, 0);
      }
    }
    double* col = Wk + (int64_t)(16 * J + li) * CB + 16 * i + lk;
#pragma unroll
    for (int r = 0; r < 4; ++r) col[4 * r] = -acc[r];
  };
  if (wv < 3) {
    rowblock(i1, g1);
    rowblock(i2, g2);
  } else {
    rowblock(3, g1);
    double* col = Wk + (int64_t)(16 * J + li) * CB + 16 * J + lk;   // W_JJ, the column's diagonal block
#pragma unroll
    for (int r = 0; r < 4; ++r) col[4 * r] = swv[J * SB * SB + li * SB + lk + 4 * r];
  }
}

// PIPE (default): wave 0 takes tile 0 of C(kb) -- the next diagonal sub-block -- and goes straight
// on to A(kb+1) while waves 1..3 run the rest of C(kb); one barrier per inner block instead of
// three.  Every element receives the same updates in the same order, so U and W are bitwise those
// of the phase-serial kernel (PIPE = false, SCS_CHOL_DIAG=0).
// LayPack (r06, default): launch bounds for two workgroups per CU, i.e. <= 256 registers per lane
// (VGPRs + AGPRs): with ~96 KiB of LDS the kernel then fits beside one workgroup of the bulk stream's
// gram_sia_kernel (32 KiB, 256 registers); LayFull (SCS_CHOL_DIAG_PACK=0) keeps r05's bounds.
template <bool PIPE, class L>
__global__ __launch_bounds__(DNT, L::packed ? 2 : 1) void chol_diag_kernel(double* __restrict__ G, int64_t ld, int k,
                                                        double* __restrict__ W, int* __restrict__ info, int wpar) {
  // S(r, c) = su[L::idxb(r / 16, c / 16, r % 16, c % 16)]; swinv: inverses of the 16 x 16 diagonal blocks
  // (col-major).  LayPack takes both as DYNAMIC LDS (CHOL_DIAG_PACK_LDS bytes at launch): with ~94 KiB of
  // static LDS the backend infers one wave per SIMD and pads the descriptor's VGPRs to 264 to match
  // (NumVGPRsForWavesPerEU), which no bulk workgroup's 256 registers leave room for; with the LDS dynamic
  // the descriptor carries the 235 the kernel uses
  extern __shared__ double chol_dlds[];
  __shared__ double su_st[L::packed ? 1 : L::words];
  __shared__ double swinv_st[L::packed ? 1 : CB / SB][SB * SB];
  double* su = L::packed ? chol_dlds : su_st;
  double (*swinv)[SB * SB] = L::packed ? reinterpret_cast<double (*)[SB * SB]>(chol_dlds + L::words) : swinv_st;
  __shared__ double srinv[CB];      // 1 / U(j, j)
  __shared__ __attribute__((aligned(16))) double urow[SB];   // phase A's row-j copy
  __shared__ int tctr;                                        // phase C's tile counter
  if (wpar & 2) __builtin_amdgcn_s_setprio(3);   // SCS_CHOL_PRIO: beside bulk waves (the packed form) it wins issue
  double* blk = G + (int64_t)k * CB * ld + (int64_t)k * CB;
  double* Wk = W + (int64_t)k * CB * CB;
  const int tid = threadIdx.x;
  DTIME_MARK(0);
  // the block into LDS: all 32 16-B loads per thread in flight before their LDS stores, and
  // unconditional (the block is whole in memory; the lower triangle is masked after the load -- a
  // masked load compiled to a branch with a kernel-argument reload and an lgkmcnt wait per element)
  if (!L::packed) {
    v2d t[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int e = tid + DNT * i, c = e >> 6, r = 2 * (e & 63);
      t[i] = *(const v2d*)(blk + (int64_t)c * ld + r);
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int e = tid + DNT * i, c = e >> 6, r = 2 * (e & 63);
      su[c * CLD + r] = (r <= c) ? t[i][0] : 0.0;
      su[c * CLD + r + 1] = (r + 1 <= c) ? t[i][1] : 0.0;
    }
  } else {
    // the 36 upper blocks only: 128 row pairs per block (8 threads read one column's 16 rows, 128 B),
    // item e = tid + 256 i lies in block 2 i + (tid >> 7); the diagonal blocks' lower parts are zeroed
    constexpr int NI = NPB * SB * SB / 2 / DNT;   // 18
    v2d t[NI];
    const int h = tid >> 7, cc = (tid >> 3) & 15, rp = 2 * (tid & 7);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int b = 2 * i + h;
      int C = 0;
      while ((C + 1) * (C + 2) / 2 <= b) ++C;
      const int I = b - C * (C + 1) / 2;
      t[i] = *(const v2d*)(blk + (int64_t)(16 * C + cc) * ld + 16 * I + rp);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int b = 2 * i + h;
      int C = 0;
      while ((C + 1) * (C + 2) / 2 <= b) ++C;
      const int I = b - C * (C + 1) / 2;
      su[b * PBS + cc * PBP + rp] = (I < C || rp <= cc) ? t[i][0] : 0.0;
      su[b * PBS + cc * PBP + rp + 1] = (I < C || rp + 1 <= cc) ? t[i][1] : 0.0;
    }
  }
  // inverse of the (final) 16 x 16 diagonal block kb by one wave (lane c = column c)
  auto inv16 = [&](int kb) {
    // U(o+i, o+t) as a wave-uniform LDS read (broadcast), not v_readlane of a register copy: the
    // 120 independent readlanes were hoisted into SGPRs and spilled to VGPR lanes
    const int o = kb * SB;
    const int c = tid & 15;
    double w[SB];
#pragma unroll
    for (int i = 0; i < SB; ++i) w[i] = (i == c) ? 1.0 : 0.0;
#pragma unroll
    for (int t = SB - 1; t >= 0; --t) {
      w[t] *= srinv[o + t];
#pragma unroll
      for (int i = 0; i < t; ++i) w[i] -= su[L::idxb(kb, kb, i, t)] * w[t];
    }
    if ((tid & 63) < SB) {
#pragma unroll
      for (int i = 0; i < SB; ++i) swinv[kb][c * SB + i] = (i <= c) ? w[i] : 0.0;
    }
  };
  // row block rb of U (rows 16 rb .. 16 rb + 15, columns from 16 rb) from S to G by threads t0, t0 + nt,
  // ...: 16-B stores of row pairs, the diagonal element of an even pair alone
  auto store_urows = [&](int rb, int t0, int nt) {
    const int o = rb * SB, n = (CB - o) * (SB / 2);
    for (int e = t0; e < n; e += nt) {
      const int c = o + (e >> 3), r = o + 2 * (e & 7);
      const int sidx = L::idxb(rb, c >> 4, r & 15, c & 15);
      if (r + 1 <= c) {
        v2d v;
        v[0] = su[sidx];
        v[1] = su[sidx + 1];
        *(v2d*)(blk + (int64_t)c * ld + r) = v;
      } else if (r == c) {
        blk[(int64_t)c * ld + r] = su[sidx];
      }
    }
  };
  __syncthreads();

  PROF_MARK(0);
  const int wv = tid >> 6, lane = tid & 63;
  if (PIPE) {
    if (tid < 64) diag_factor16<L>(su, srinv, urow, 0, k, info, tid);
    __syncthreads();
  }
  for (int kb = 0; kb < CB / SB; ++kb) {
    const int o = kb * SB;
    PROF_MARK(1 + 4 * kb);
    if (!PIPE) {
      if (tid < 64) diag_factor16<L>(su, srinv, urow, o, k, info, tid);
      __syncthreads();
    }
    PROF_MARK(2 + 4 * kb);
    const int np = CB - o - SB;  // columns right of the sub-block
    if (np == 0) break;
    diag_panel16<L>(su, srinv, o, np, tid);
    if (tid == 0) tctr = 1;   // C(kb)'s tile counter (tile 0 is wave 0's)
    __syncthreads();
    PROF_MARK(3 + 4 * kb);
    const int n16 = np >> 4, ntl = n16 * (n16 + 1) / 2;
    if (PIPE) {
      // tiles 1.. of C(kb) are claimed from an LDS counter: waves 1..3 at once (the one that inverts
      // block kb after its inverse), wave 0 once it has factored sub-block kb+1
      auto claim_tiles = [&]() {
        for (;;) {
          int id = 0;
          if (lane == 0) id = __hip_atomic_fetch_add(&tctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          id = __builtin_amdgcn_readfirstlane(id);
          if (id >= ntl) break;
          diag_trail_tile<L>(su, o, id, lane);
        }
      };
      if (wv == 0) {
        diag_trail_tile<L>(su, o, 0, lane);
        PROF_MARK_T(36 + kb, 0);
        // tile 0's elements go from the lanes that updated them to the lanes that factor them (lane
        // 4c + q reads rows 4q.. of column c): an intra-wave LDS hand-off with no barrier, so order it
        // for the compiler (instruction-free wavefront fence + wave barrier, as in diag_factor16)
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        diag_factor16<L>(su, srinv, urow, o + SB, k, info, tid);
        PROF_MARK_T(43 + kb, 0);
#ifndef CHOL_NO_W0CLAIM
        claim_tiles();
#endif
      } else {
        if (wv == 1 + kb % 3) {
          inv16(kb);   // U_kb,kb is final: its inverse beside the update
          PROF_MARK_T(50 + kb, 64 * wv);
        }
        // W's block column kb - 1 (its last input, swinv[kb - 1], came before this step's barrier)
        if (W_BY_COLUMNS && kb >= 1 && wv == 1 + (kb + 1) % 3) w_column<L>(su, &swinv[0][0], Wk, kb - 1, lane);
        claim_tiles();
        // row blocks of U are final after their panel step: waves 1..3 store them while wave 0 is
        // on the chain (kb = 3: blocks 0, 1; 4: 2, 3; 5: 4, 5; 6: 6 -- where these waves have slack)
        if (kb >= 3) {
          store_urows(2 * (kb - 3), tid - 64, DNT - 64);
          if (kb < 6) store_urows(2 * (kb - 3) + 1, tid - 64, DNT - 64);
        }
        PROF_MARK_T(57 + 3 * kb + wv - 1, 64 * wv);
      }
    } else {
      for (int id = wv; id < ntl; id += DNT / 64) diag_trail_tile<L>(su, o, id, lane);
    }
    __syncthreads();
  }
  PROF_MARK(33);
  // ---- store U (PIPE: the last row block; the others went out during the loop).  (Running inv16
  // beside phase B on the idle last wave measured slower: B waits for it; PIPE runs inv16(kb) beside
  // C(kb), so only the last block's is left.)
  if (PIPE) {
    if (wv == DNT / 64 - 1) inv16(CB / SB - 1);
    else store_urows(CB / SB - 1, tid, DNT - 64);
    if (W_BY_COLUMNS && wv == 1) w_column<L>(su, &swinv[0][0], Wk, CB / SB - 2, lane);   // swinv[6]: step 6
  } else {
    for (int rb = 0; rb < CB / SB; ++rb) store_urows(rb, tid, DNT);
    for (int kb = tid >> 6; kb < CB / SB; kb += DNT / 64) inv16(kb);
  }
  __syncthreads();   // storeU has read the diagonal blocks; swinv complete
  if (W_BY_COLUMNS) {
    PROF_MARK(34);
    if (PIPE) {
      if (wpar & 1) w_last_column_par<L>(su, &swinv[0][0], Wk, tid);
      else if (wv == 0) w_column<L>(su, &swinv[0][0], Wk, CB / SB - 1, lane);
    } else if (wpar & 1) {   // columns 0..6 (wave w: w and 6 - w), then the last one by all waves, as PIPE
      w_column<L>(su, &swinv[0][0], Wk, wv, lane);
      if (wv < 3) w_column<L>(su, &swinv[0][0], Wk, CB / SB - 2 - wv, lane);
      __syncthreads();   // the transposed off-diagonal blocks w_last_column_par reads
      w_last_column_par<L>(su, &swinv[0][0], Wk, tid);
    } else {   // every column here: wave w takes columns w and 7 - w
      w_column<L>(su, &swinv[0][0], Wk, wv, lane);
      w_column<L>(su, &swinv[0][0], Wk, CB / SB - 1 - wv, lane);
    }
    PROF_MARK(35);
    DTIME_MARK(1);
    return;
  }
  if constexpr (L::packed) return;   // (W_BY_COLUMNS only)
  // ---- diagonal 16 x 16 inverses into the diagonal blocks of S (start of the doubling)
  for (int e = tid; e < CB * SB; e += DNT) {
    const int kb = e >> 8, c = (e >> 4) & 15, i = e & 15;
    if (i <= c) su[(kb * SB + c) * CLD + kb * SB + i] = swinv[kb][c * SB + i];
  }
  __syncthreads();
  PROF_MARK(34);
  chol_inv_double_mfma<16>(su, tid);
  chol_inv_double_mfma<32>(su, tid);
  chol_inv_double_mfma<64>(su, tid);
#pragma unroll 8
  for (int i = 0; i < 32; ++i) {
    const int e = tid + DNT * i, c = e >> 6, r = 2 * (e & 63);
    const double w0 = su[c * CLD + r], w1 = su[c * CLD + r + 1];   // unconditional reads, then the mask
    v2d v;
    v[0] = (r <= c) ? w0 : 0.0;
    v[1] = (r + 1 <= c) ? w1 : 0.0;
    *(v2d*)(Wk + (int64_t)c * CB + r) = v;
  }
  PROF_MARK(35);
}

// the inverse of an upper 128 x 128 block already in su (S(r, c) = su[c·CLD + r], zero below the diagonal)
// with its reciprocal pivots in srinv: the 16 x 16 diagonal inverses (one wave each, in registers), then
// the doubling levels 16 -> 32 -> 64 on MFMA; W = S⁻¹ ends in su's upper triangle (the strictly-lower
// triangle is the doubling's scratch)
__device__ __forceinline__ void tri_inv_loaded(double* su, const double* srinv, double (*swinv)[SB * SB], int tid) {
  for (int kb = tid >> 6; kb < CB / SB; kb += DNT / 64) {
    const int o = kb * SB, c = tid & 15;
    double w[SB];
#pragma unroll
    for (int i = 0; i < SB; ++i) w[i] = (i == c) ? 1.0 : 0.0;
#pragma unroll
    for (int t = SB - 1; t >= 0; --t) {
      w[t] *= srinv[o + t];
#pragma unroll
      for (int i = 0; i < t; ++i) w[i] -= su[(o + t) * CLD + o + i] * w[t];
    }
    if ((tid & 63) < SB) {
#pragma unroll
      for (int i = 0; i < SB; ++i) swinv[kb][c * SB + i] = (i <= c) ? w[i] : 0.0;
    }
  }
  __syncthreads();
  for (int e = tid; e < CB * SB; e += DNT) {
    const int kb = e >> 8, c = (e >> 4) & 15, i = e & 15;
    if (i <= c) su[(kb * SB + c) * CLD + kb * SB + i] = swinv[kb][c * SB + i];
  }
  __syncthreads();
  chol_inv_double_mfma<16>(su, tid);
  chol_inv_double_mfma<32>(su, tid);
  chol_inv_double_mfma<64>(su, tid);
}

// W_k = R_kk⁻¹ for the upper 128 x 128 diagonal blocks of a triangular R (the QR solve): the
// inverse part of chol_diag_kernel (the 16 x 16 inverses, then recursive doubling on MFMA) on a
// block whose factor is given; the strictly lower part of the block is ignored.
__global__ __launch_bounds__(DNT) void tri_inv_kernel(const double* __restrict__ R, int64_t ld,
                                                      double* __restrict__ W) {
  __shared__ double su[CB * CLD];
  __shared__ double srinv[CB];
  __shared__ double swinv[CB / SB][SB * SB];
  const int k = blockIdx.x, tid = threadIdx.x;
  const double* blk = R + (int64_t)k * CB * ld + (int64_t)k * CB;
  for (int e = tid; e < CB * CB; e += DNT) {
    const int c = e >> 7, r = e & 127;
    su[c * CLD + r] = (r <= c) ? blk[(int64_t)c * ld + r] : 0.0;
  }
  __syncthreads();
  if (tid < CB) srinv[tid] = 1.0 / su[tid * CLD + tid];
  __syncthreads();
  tri_inv_loaded(su, srinv, swinv, tid);
  double* Wk = W + (int64_t)k * CB * CB;
  for (int e = tid; e < CB * CB; e += DNT) {
    const int c = e >> 7, r = e & 127;
    Wk[(int64_t)c * CB + r] = (r <= c) ? su[c * CLD + r] : 0.0;
  }
}

// L11⁻¹ and U11⁻¹ of the LU's factored 128 x 128 diagonal block (lu.hip: row-major, unit-lower L and
// upper U sharing the block) by the same 16 x 16 inverses + MFMA doubling (r05; the r02 kernel
// eliminated one row per barrier, 128 of them: 226 us per launch, 14 % of the n = 8192 factor).
// Workgroup 0 inverts Lᵀ (upper, unit diagonal; S column c = row c of L), workgroup 1 U; both write
// row-major 128 x 128: Linv = (Lᵀ)⁻¹ transposed, Uinv = U⁻¹.  A zero pivot of U gives inf / NaN, as
// the elimination did (info already holds it).
__global__ __launch_bounds__(DNT) void lu_tri_inv_kernel(const double* __restrict__ A, int64_t ld, int64_t r0,
                                                         double* __restrict__ Linv, double* __restrict__ Uinv) {
  __shared__ double su[CB * CLD];
  __shared__ double srinv[CB];
  __shared__ double swinv[CB / SB][SB * SB];
  const bool lower = blockIdx.x == 0;
  const int tid = threadIdx.x;
  const double* blk = A + r0 * ld + r0;
  for (int e = tid; e < CB * CB; e += DNT) {
    const int i = e >> 7, j = e & 127;   // block row i, column j (coalesced over j)
    const double v = blk[(int64_t)i * ld + j];
    if (lower) su[i * CLD + j] = (j < i) ? v : ((j == i) ? 1.0 : 0.0);   // S(j, i) = L(i, j)
    else su[j * CLD + i] = (i <= j) ? v : 0.0;                             // S(i, j) = U(i, j)
  }
  __syncthreads();
  if (tid < CB) srinv[tid] = lower ? 1.0 : 1.0 / su[tid * CLD + tid];
  __syncthreads();
  tri_inv_loaded(su, srinv, swinv, tid);
  double* out = lower ? Linv : Uinv;
  for (int e = tid; e < CB * CB; e += DNT) {
    const int i = e >> 7, j = e & 127;   // out(i, j); W(r, c) = su[c·CLD + r], r <= c
    const double v = lower ? ((j <= i) ? su[i * CLD + j] : 0.0) : ((i <= j) ? su[j * CLD + i] : 0.0);
    out[(int64_t)i * CB + j] = v;
  }
}

hipError_t launch_lu_tri_inv(const double* A, int64_t ld, int64_t r0, double* Linv, double* Uinv, hipStream_t st) {
  hipLaunchKernelGGL(lu_tri_inv_kernel, dim3(2), dim3(DNT), 0, st, A, ld, r0, Linv, Uinv);
  return hipGetLastError();
}


// T of a 128-column compact WY block (dlarft forward, columnwise; qr.hip) from Gv = VᵀV and tau,
// by the same doubling as W = U⁻¹: T = [T11, -T11 G12 T22; 0, T22] with G12 = V1ᵀV2 in the place
// of U12.  The 16 x 16 diagonal blocks come from dlarft's recurrence T(0:i, i) = -tau_i T(0:i, 0:i)
// Gv(0:i, i) (one wave per block, lane t = row t); the doubling levels 16 -> 32 -> 64 on MFMA.
__global__ __launch_bounds__(DNT) void wy_t_kernel(const double* __restrict__ Gv, const double* __restrict__ tau,
                                                   double* __restrict__ T) {
  __shared__ double su[CB * CLD];
  const int tid = threadIdx.x;
  for (int e = tid; e < CB * CB; e += DNT) {   // G12 entries (different 16-blocks) in the upper part
    const int c = e >> 7, r = e & 127;
    su[c * CLD + r] = (r < c && (r >> 4) != (c >> 4)) ? Gv[(int64_t)c * CB + r] : 0.0;
  }
  __syncthreads();
  const int wv = tid >> 6, lane = tid & 63, t = lane & 15;
  for (int kb = wv; kb < CB / SB; kb += DNT / 64) {
    const int o = kb * SB;
    double tc[SB];
#pragma unroll
    for (int q = 0; q < SB; ++q) tc[q] = 0.0;
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const double ti = tau[o + i];
      const double z = (t < i) ? -ti * Gv[(int64_t)(o + i) * CB + o + t] : 0.0;   // lane q: z_q
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < SB; ++q) {
        const double zq = __shfl(z, q, 64);
        if (q < i && q >= t) s += tc[q] * zq;   // T(t, q), q >= t (upper)
      }
      tc[i] = (t < i) ? s : ((t == i) ? ti : 0.0);
    }
    if (lane < SB) {
#pragma unroll
      for (int q = 0; q < SB; ++q) su[(o + q) * CLD + o + t] = (t <= q) ? tc[q] : 0.0;
    }
  }
  __syncthreads();
  chol_inv_double_mfma<16>(su, tid);
  chol_inv_double_mfma<32>(su, tid);
  chol_inv_double_mfma<64>(su, tid);
  for (int e = tid; e < CB * CB; e += DNT) {
    const int c = e >> 7, r = e & 127;
    T[(int64_t)c * CB + r] = (r <= c) ? su[c * CLD + r] : 0.0;
  }
}

hipError_t wy_t_build(const double* Gv, const double* tau, double* T, hipStream_t st) {
  hipLaunchKernelGGL(wy_t_kernel, dim3(1), dim3(DNT), 0, st, Gv, tau, T);
  return hipGetLastError();
}

hipError_t chol_tri_inverse(const double* R, int64_t ld, int nblk, double* W, hipStream_t st) {
  if (nblk <= 0) return hipSuccess;
  hipLaunchKernelGGL(tri_inv_kernel, dim3((unsigned)nblk), dim3(DNT), 0, st, R, ld, W);
  return hipGetLastError();
}

static int chol_prio();   // SCS_CHOL_PRIO (below)

static bool chol_diag_pipe() {   // read per call (A/B within one process)
  const char* e = getenv("SCS_CHOL_DIAG");
  return !(e && e[0] == '0');
}

// SCS_CHOL_WPAR (read per call; default on): W's last block column by all four waves
// (w_last_column_par, r05); 0 = the one-wave recursion (w_column_t<7>)
static int chol_wpar() {
  const char* e = getenv("SCS_CHOL_WPAR");
  return (e && e[0] == '0') ? 0 : 1;
}

// SCS_CHOL_DIAG_PACK (read per call; default off): 1 = the packed-LDS diagonal kernel (LayPack, r06),
// else r05's full 128 x 129 LDS copy (LayFull).  The same U, W and pivots either way (probe bit sums).
// Measured (profiles/r06/chol_pack/): LayPack fits beside one bulk workgroup and starts sooner, but
// sharing the CU's SIMDs with the bulk's MFMA waves it runs 128 us instead of 51 (in-kernel, m = 16384):
// factor 33.0-33.3 vs 31.9-32.1 ms, m = 8192 8.3 vs 7.6 ms -- so LayFull stays the default.
static bool chol_diag_pack() {
  const char* e = getenv("SCS_CHOL_DIAG_PACK");
  return e && e[0] == '1';
}

constexpr int CHOL_DIAG_PACK_LDS = (LayPack::words + (CB / SB) * SB * SB) * (int)sizeof(double);   // 94,720 B

static hipError_t chol_diag_pack_attr() {   // the dynamic LDS above the 64 KiB default, once per process
  static hipError_t done = [] {
    hipError_t e = hipFuncSetAttribute((const void*)chol_diag_kernel<true, LayPack>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, CHOL_DIAG_PACK_LDS);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)chol_diag_kernel<false, LayPack>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              CHOL_DIAG_PACK_LDS);
    if (e != hipSuccess) (void)hipGetLastError();   // the LayFull kernel runs instead
    return e;
  }();
  return done;
}

hipError_t launch_chol_diag(double* G, int64_t ld, int k, double* W, int* info, hipStream_t st) {
  const bool pipe = chol_diag_pipe(), pack = chol_diag_pack() && chol_diag_pack_attr() == hipSuccess;
  const int dflag = chol_wpar() | (chol_prio() ? 2 : 0);
  if (pipe && pack)
    hipLaunchKernelGGL((chol_diag_kernel<true, LayPack>), dim3(1), dim3(DNT), CHOL_DIAG_PACK_LDS, st, G, ld, k, W, info,
                       dflag);
  else if (pipe)
    hipLaunchKernelGGL((chol_diag_kernel<true, LayFull>), dim3(1), dim3(DNT), 0, st, G, ld, k, W, info, dflag);
  else if (pack)
    hipLaunchKernelGGL((chol_diag_kernel<false, LayPack>), dim3(1), dim3(DNT), CHOL_DIAG_PACK_LDS, st, G, ld, k, W,
                       info, dflag);
  else
    hipLaunchKernelGGL((chol_diag_kernel<false, LayFull>), dim3(1), dim3(DNT), 0, st, G, ld, k, W, info, dflag);
  return hipGetLastError();
}

__global__ void diag_pad_kernel(double* __restrict__ G, int64_t ld, int64_t m, int64_t mpad) {
  const int64_t i = m + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < mpad) G[i * ld + i] = 1.0;
}

// ---------------------------------------------------------------------------
// Two-level blocked factorization.  Outer blocks of OB (default 8) inner 128-blocks:
//   A  inner factor of the outer diagonal block (the single-level loop below, restricted
//      to the block: chol_diag_kernel + panel solve + trailing update with K = 128);
//   B  forward solve of the outer row strip X = U_D⁻ᵀ R (rows of the block, all columns to
//      its right), recursively: X1 = solve(D11, R1); R2 -= U12ᵀ X1 (one Gram launch over
//      an (rows of R2) x (strip columns) rectangle, K = rows of X1); X2 = solve(D22, R2);
//      leaves are the in-place W_kᵀ multiplies;
//   C  trailing update of everything right of / below the block with K = OB·128:
//      A_rest -= Xᵀ X (upper store).
// Moving the bulk of the m³/3 flops into C with K = 1024 instead of 128 cuts the
// read-modify-write of the trailing matrix 8x (the single-level update is HBM-bound on
// that C tile traffic: 2·128 KiB per 4.2 MFLOP tile).
static int outer_block();

// SCS_CHOL_PRIO (read per call; r06): the chain's latency launches (row panels, in-block updates, Ba's strip
// steps, C1a) run their waves at s_setprio 3, so that on a SIMD shared with the bulk stream's MFMA waves
// they win the issue arbitration (MI355X_MICROARCH.md: priority, then age).  Default on: the same bits;
// probe factor, three rounds per arm on one box (profiles/r06/prio/): m = 16384 31.37-31.83 vs 32.17-32.58 ms,
// m = 8192 7.17-7.28 vs 7.23-7.30 ms.  0 = r05's normal priority.
static int chol_prio() {
  const char* e = getenv("SCS_CHOL_PRIO");
  return e ? atoi(e) : 1;
}

// The bulk stream (the lookahead's trailing updates) is a plain non-blocking stream.  (r02 kept 32
// CUs from it with a CU-masked queue, hipExtStreamCreateWithCUMask; a process that created one
// faulted at exit under rocprofv3 -- in librocprofiler-sdk's static destructors, profiles/r03/segv/
// -- so the profiled configuration could not be the benchmarked one.  Removed in r04: the CU-bounded
// persistent bulk launches below keep the same CUs free.)
// SCS_CHOL_BULK_SKIP: the CU ids (within a shader engine, HW_REG_HW_ID bits 11:8; a bit mask,
// hex accepted) whose workgroup slots the bulk stream's launches leave to the chain
// (gram_launch_bounded); 0 = plain launches.  Default: CU id 5 (present in every shader engine
// of the measured boxes: 4 CUs per XCD, 32 in all -- the r02 CU reserve) up to m = 8192, where
// the chain's launches waited for slots the trailing update held (C2 solve 10.20 -> 9.55 ms);
// none above: m = 16384 38.6 vs 39.3 ms, m = 32768 212.6 vs 228.8 ms with it (the bulk stream
// bounds those factors; profiles/r03/chol/bounded/).  Which CUs a harvested part lacks only
// changes how many are left free.
// SCS_CHOL_BULK_SKIP_XCC (r06, A/B): a bit mask of the XCDs where the skip set applies (default all)
static unsigned bulk_skip_mask(int nblk) {
  const char* e = getenv("SCS_CHOL_BULK_SKIP");
  const char* x = getenv("SCS_CHOL_BULK_SKIP_XCC");
  const unsigned xm = x ? ((unsigned)strtoul(x, nullptr, 0) & 0xffu) << 24 : 0u;
  if (e) return ((unsigned)strtoul(e, nullptr, 0) & 0xffffu) | xm;
  return nblk <= 64 ? (0x20u | xm) : 0u;
}

static hipError_t create_bulk_stream(hipStream_t* s) { return hipStreamCreateWithFlags(s, hipStreamNonBlocking); }

// The lookahead's two streams must sit on different hardware queues (r05).  The runtime gives each
// stream priority its own pool of hardware queues and, once a pool holds GPU_MAX_HW_QUEUES (4) queues,
// maps a new stream onto the least-used queue of its pool -- so in a process where torch and RCCL have
// created streams, the caller's stream (the chain) and the bulk stream could land on ONE hardware queue
// and the two halves of the factor then ran back to back: +6.8 ms of solve per C3-shaped step with the
// exchange forced at world 1, every kernel of the step on one queue in the trace
// (profiles/r05/rccltrace/).  Streams of different priority cannot share a queue.  Modes: 2 the bulk
// stream at the device's greatest priority, the chain on the caller's stream (the default where the
// context holds an RCCL communicator: CholAux::chain_mode, set by scsopt.cpp); 1 the chain on a stream
// of its own at the greatest priority, joined to the caller's by events; 0 both at normal priority (r04;
// the default elsewhere: a high-priority bulk stream wins the dispatcher's free slots over the chain's
// latency launches, which shows under a kernel tracer -- the m = 8192 probe factor 7.6 -> 13.4 ms under
// rocprofv3 -- though not in the untraced C2 line).  SCS_CHOL_CHAIN (read per call) overrides.
static hipError_t create_hiprio_stream(hipStream_t* s) {
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e == hipSuccess) e = hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
  return e;
}

static int chol_chain_mode(const CholAux* a) {
  const char* e = getenv("SCS_CHOL_CHAIN");
  return e ? atoi(e) : a->chain_mode;
}

// SCS_CHOL_SKIP_MAXTILES (A/B; unset = no limit): bulk launches of more tiles than this run on every
// CU (skip set 0) -- the bulk-bound early outer blocks -- and only the smaller ones keep the skip set
static unsigned bulk_skip_for(const CholAux* a, int ntiles) {
  const char* e = getenv("SCS_CHOL_SKIP_MAXTILES");
  if (e && ntiles > atoi(e)) return 0u;
  return a->bskip;
}

// SCS_CHOL_BULK_RESERVE (read per call): where no CU is skipped (m >= 16384), the bulk stream's
// launches as persistent launches of 2·CUs − r workgroups, r slots left to the chain.  A plain bulk
// launch of thousands of tiles refills every slot it frees, and the chain's diagonal kernel -- which
// (packed, r06) fits in one free slot beside a bulk workgroup -- then waited for the whole trailing
// update (up to 3.3 ms, once per outer block, profiles/r06/pack/).  BULK_BND_ONLY marks a persistent
// launch that skips no CU (bits above 15 match no CU id).
constexpr unsigned BULK_BND_ONLY = 1u << 16;
static int bulk_reserve(const CholAux* a) {
  const char* e = getenv("SCS_CHOL_BULK_RESERVE");
  (void)a;
  return e ? atoi(e) : 0;
}
static unsigned bulk_mask(const CholAux* a, int ntiles) {
  const unsigned s = bulk_skip_for(a, ntiles);
  return (s == 0 && bulk_reserve(a) > 0) ? BULK_BND_ONLY : s;
}
static int bulk_slots(const CholAux* a, unsigned mask) {
  return mask == BULK_BND_ONLY ? a->bslots - bulk_reserve(a) : a->bslots;
}

// The bulk stream's bounded launches take counter sets from a->bctr in turn, each zero when taken
// (r04: a 9-counter memset in front of every bounded launch was 38 fill kernels, 0.21 ms of the
// bulk stream, per m = 8192 factor -- profiles/r03/chol/trace_end/).  All bounded launches run on
// st2, so re-zeroing the array there when the sets run out is ordered after every launch that used
// them.
constexpr int BCTR_SLOTS = 1024;
static unsigned* bulk_ctr(const CholAux* a, hipStream_t st2, hipError_t* e) {
  if (a->bslot >= BCTR_SLOTS) {
    const hipError_t z = hipMemsetAsync(a->bctr, 0, (size_t)BCTR_SLOTS * 16 * sizeof(unsigned), st2);
    if (z != hipSuccess) *e = z;
    a->bslot = 0;
  }
  return a->bctr + 16 * (a->bslot++);
}

hipError_t chol_aux_init(CholAux* a, int64_t mpad, hipStream_t st) {
  const int nblk = (int)(mpad / CB);
  a->nblk = nblk;
  std::vector<double> hw((size_t)CB + mpad, -1.0);
  for (int i = 0; i < CB; ++i) hw[i] = 1.0;
  std::vector<int2> rl;
  for (int R = 1; R <= 8; ++R)
    for (int j = 0; j < nblk; ++j)
      for (int i = 0; i < R; ++i) rl.push_back(make_int2(i, j));   // bj-major: first R*C = R x C rectangle
  std::vector<int2> sb;   // 8 x 8 super-blocks of the lower triangle, super-rows ascending
  for (int R = 0; R < (nblk + 7) / 8; ++R)
    for (int C = 0; C <= R; ++C)
      for (int i = 8 * R; i < 8 * R + 8 && i < nblk; ++i)
        for (int j = 8 * C; j < 8 * C + 8 && j <= i; ++j) sb.push_back(make_int2(i, j));
  hipError_t e = hipMalloc(&a->w, sizeof(double) * hw.size());
  if (e == hipSuccess) e = hipMalloc(&a->rect, sizeof(int2) * rl.size());
  if (e == hipSuccess) e = hipMemcpyAsync(a->w, hw.data(), sizeof(double) * hw.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(a->rect, rl.data(), sizeof(int2) * rl.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess && !sb.empty()) e = hipMalloc(&a->sbl, sizeof(int2) * sb.size());
  if (e == hipSuccess && !sb.empty())
    e = hipMemcpyAsync(a->sbl, sb.data(), sizeof(int2) * sb.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = create_bulk_stream(&a->st2);
  if (e == hipSuccess) e = create_hiprio_stream(&a->stc);
  if (e == hipSuccess) e = create_hiprio_stream(&a->st2h);
  if (e == hipSuccess) e = hipMalloc(&a->bctr, (size_t)BCTR_SLOTS * 16 * sizeof(unsigned));
  if (e == hipSuccess) e = hipMemsetAsync(a->bctr, 0, (size_t)BCTR_SLOTS * 16 * sizeof(unsigned), st);
  a->bslot = 0;
  if (e == hipSuccess) e = hipMalloc(&a->sscr, sizeof(double) * 2 * (size_t)CB * 16 * CB);
  if (e == hipSuccess) {
    a->bskip = bulk_skip_mask(nblk);
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      a->bslots = 2 * ncu;   // the 128 x 128 throughput kernels: 2 workgroups per CU
    else
      a->bslots = 0;
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&a->ev1, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&a->ev2, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&a->ev3, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&a->ev4, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&a->ev0, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&a->ev5, hipEventDisableTiming);
  // the one-launch triangular solves' block flags (generation-stamped: never reset) and error flag
  if (e == hipSuccess) e = hipMalloc(&a->sflags, sizeof(unsigned) * 2 * (size_t)nblk + sizeof(int));
  if (e == hipSuccess) e = hipMemsetAsync(a->sflags, 0, sizeof(unsigned) * 2 * (size_t)nblk + sizeof(int), st);
  if (e == hipSuccess) a->serr = (int*)(a->sflags + 2 * nblk);
  a->sgen = 0;
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  return e;
}

void chol_aux_free(CholAux* a) {
  if (a->st2) (void)hipStreamSynchronize(a->st2);
  if (a->stc) (void)hipStreamSynchronize(a->stc);
  if (a->st2h) (void)hipStreamSynchronize(a->st2h);
  if (a->w) (void)hipFree(a->w);
  if (a->rect) (void)hipFree(a->rect);
  if (a->ev1) (void)hipEventDestroy(a->ev1);
  if (a->ev2) (void)hipEventDestroy(a->ev2);
  if (a->ev3) (void)hipEventDestroy(a->ev3);
  if (a->ev4) (void)hipEventDestroy(a->ev4);
  if (a->ev0) (void)hipEventDestroy(a->ev0);
  if (a->ev5) (void)hipEventDestroy(a->ev5);
  for (auto& q : a->ssched) {
    if (q.work) (void)hipFree(q.work);
    if (q.comb) (void)hipFree(q.comb);
  }
  a->ssched.clear();
  if (a->spart) (void)hipFree(a->spart);
  a->spart = nullptr;
  if (a->sflags) (void)hipFree(a->sflags);
  a->sflags = nullptr;
  if (a->bctr) (void)hipFree(a->bctr);
  a->bctr = nullptr;
  if (a->sbl) (void)hipFree(a->sbl);
  a->sbl = nullptr;
  if (a->sscr) (void)hipFree(a->sscr);
  a->sscr = nullptr;
  a->serr = nullptr;
  for (void* p : {(void*)a->dtasks, (void*)a->ddeps, (void*)a->dcnt, (void*)a->dper})
    if (p) (void)hipFree(p);
  a->dtasks = nullptr;
  a->ddeps = nullptr;
  a->dcnt = a->dper = nullptr;
  a->dag_ob = 0;
  a->dstep.clear();
  a->dnext.clear();
  if (a->st2) (void)hipStreamDestroy(a->st2);
  if (a->stc) (void)hipStreamDestroy(a->stc);
  if (a->st2h) (void)hipStreamDestroy(a->st2h);
  a->w = nullptr;
  a->rect = nullptr;
  a->ev1 = a->ev2 = a->ev3 = a->ev4 = a->ev0 = a->ev5 = nullptr;
  a->st2 = a->stc = a->st2h = nullptr;
}

static const int2* rect_list(const CholAux* a, int R) { return a->rect + (int64_t)a->nblk * (R - 1) * R / 2; }
int chol_outer_block();

// Outer block (inner 128-blocks per outer step) of chol_factor: SCS_CHOL_OB (1..16, read per call),
// else 8.  (16 at m = 32768, where the bulk stream's K = 1024 trailing updates bound the factor,
// measured slower: C4-half cached solve 221.5 -> 229.8 ms, profiles/r02/chol/ob16/.)  The
// strip-solve recursion needs rectangle lists of up to OB/2 block rows (chol_aux_init: R <= 8).
// Default since the r03 chain (faster diagonal kernel, strip-solve steps): 4 up to m = 8192, where
// the chain bounds the factor and shorter outer blocks put less of it on the critical path (C2
// factor 8.45 -> 8.08 ms), else 8 (m = 16384: 34.8 with 8, 36.3 with 4, 38.3 with 16;
// profiles/r03/chol/ob/).
static int outer_block_for(int nblk) {
  const char* e = getenv("SCS_CHOL_OB");
  const int v = e ? atoi(e) : (nblk <= 64 ? 4 : 8);
  return v < 1 ? 1 : (v > 16 ? 16 : v);
}

// the strip pipeline's outer strip (SCS_CHOL_PIPE): 8, or SCS_CHOL_OB up to 8
static int outer_block() {
  static const int ob = [] {
    const char* e = getenv("SCS_CHOL_OB");
    const int v = e ? atoi(e) : 8;
    return v < 1 ? 1 : (v > 8 ? 8 : v);
  }();
  return ob;
}

// forward solve of the strip rows [lo, hi) (inner blocks) x nc columns starting at block c0
// (bulk: the bulk stream's CU-bounded launches, gram_launch_bounded)
static hipError_t strip_solve(double* G, int64_t ld, const double* W, const CholAux* a, int lo, int hi, int c0, int nc,
                              hipStream_t st, bool bulk = false) {
  auto launch = [&](const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w, int64_t k1,
                    const int2* tiles, int ntiles, double* R, int flags) {
    if (bulk) {
      hipError_t ez = hipSuccess;
      unsigned* ctr = bulk_ctr(a, st, &ez);
      if (ez != hipSuccess) return ez;
      const unsigned mk = bulk_mask(a, ntiles);
      return gram_launch_bounded(A1, lda1, A2, lda2, w, 0, k1, tiles, ntiles, R, ld, flags, ctr, mk, bulk_slots(a, mk),
                                 st, true);
    }
    return gram_launch_gen(A1, lda1, A2, lda2, w, 0, k1, tiles, ntiles, R, ld, flags, st);
  };
  if (hi - lo == 1) {
    double* R = G + (int64_t)c0 * CB * ld + (int64_t)lo * CB;
    return launch(W + (int64_t)lo * CB * CB, CB, R, ld, a->w, CB, rect_list(a, 1), nc, R, 0);
  }
  const int mid = (lo + hi) / 2;
  hipError_t e = strip_solve(G, ld, W, a, lo, mid, c0, nc, st, bulk);
  if (e != hipSuccess) return e;
  // R2 -= U12ᵀ X1: A1 = U[lo:mid, mid:hi] (panels mid.., rows from lo), A2 = X1 (panels c0.., rows from lo)
  const double* U12 = G + (int64_t)mid * CB * ld + (int64_t)lo * CB;
  const double* X1 = G + (int64_t)c0 * CB * ld + (int64_t)lo * CB;
  double* R2 = G + (int64_t)c0 * CB * ld + (int64_t)mid * CB;
  e = launch(U12, ld, X1, ld, a->w + CB, (int64_t)(mid - lo) * CB, rect_list(a, hi - mid), (hi - mid) * nc, R2,
             /*GRAM_ACCUMULATE*/ 2);
  if (e != hipSuccess) return e;
  return strip_solve(G, ld, W, a, mid, hi, c0, nc, st, bulk);
}

// The chain's strip solve (Ba, and the same columns of the serial order) as right-looking steps:
// step r is ONE launch in which every workgroup takes a 16-column strip s of column tile j and forms
// Y = W_rᵀ R_rj[:, s] (row r's leaf, 128 x 16, in LDS); for row q = r that is X_rj's strip (to a
// scratch row, in place at the last step), for q > r it updates R_qj[:, s] -= U_rqᵀ Y.  The leaf is
// recomputed per strip (bitwise the leaf's own value: the same latency-kernel body) instead of being a
// launch of its own; extra workgroups copy the previous step's scratch row into G (row r - 1 is read
// by no one in this launch).  OB steps instead of the recursion's 2 OB - 1 launches; every R_qj takes
// its updates in row order with K = 128 each (the recursion groups them by K = 128 .. OB/2·128).
__global__ __launch_bounds__(256) void strip_step_kernel(double* G, int64_t ld, const double* __restrict__ W,
                                                         const double* __restrict__ wv, int r, int hi, int c0,
                                                         int nc, double* __restrict__ scur,
                                                         const double* __restrict__ sprev, int prio) {
  __shared__ __attribute__((aligned(16))) double lds[2 * (GT + 16) * GBK];
  __shared__ __attribute__((aligned(16))) double Y[GT * 16];
  if (prio) __builtin_amdgcn_s_setprio(3);
  const int nitem = (hi - r) * nc * 8, it = blockIdx.x;
  if (it >= nitem) {   // copy-back of the previous step's row r - 1: one 128 x 16 strip
    const int ci = it - nitem, j = ci >> 3, s = ci & 7;
    for (int e = threadIdx.x; e < GT * 8; e += 256) {
      const int col = j * GT + 16 * s + (e >> 6), rr = 2 * (e & 63);
      *(v2d*)(G + ((int64_t)c0 * GT + col) * ld + (int64_t)(r - 1) * GT + rr) = *(const v2d*)(sprev + (int64_t)col * GT + rr);
    }
    return;
  }
  const int q = r + it / (nc * 8), j = (it >> 3) % nc, s = it & 7;
  const int64_t col0 = (int64_t)(c0 + j) * GT + 16 * s;   // the strip's first column of G
  const double* Wr = W + (int64_t)r * GT * GT;
  const double* Rr = G + col0 * ld + (int64_t)r * GT;
  if (q == r) {   // the leaf: X_rj[:, s] (in place at the last step)
    double* out = scur ? scur + ((int64_t)j * GT + 16 * s) * GT : G + col0 * ld + (int64_t)r * GT;
    gram_small_strip<16>(Wr, GT, Rr, ld, wv, 0, GT, out, scur ? GT : ld, 0, lds);
    return;
  }
  gram_small_strip<16>(Wr, GT, Rr, ld, wv, 0, GT, Y, GT, 0, lds);
  __syncthreads();   // Y complete; the staging buffer free again
  gram_small_strip<16>(G + (int64_t)q * GT * ld + (int64_t)r * GT, ld, Y, GT, wv + GT, 0, GT,
                       G + col0 * ld + (int64_t)q * GT, ld, GRAM_ACCUMULATE, lds);
}

static hipError_t strip_solve_steps(double* G, int64_t ld, const double* W, const CholAux* a, int lo, int hi, int c0,
                                    int nc, hipStream_t st) {
  if (nc <= 0) return hipSuccess;
  if (nc > 16 || !a->sscr) return hipErrorInvalidValue;
  const size_t row = (size_t)CB * 16 * CB;
  for (int r = lo; r < hi; ++r) {
    const bool last = r == hi - 1;
    double* scur = last ? nullptr : a->sscr + row * ((r - lo) & 1);
    const double* sprev = a->sscr + row * ((r - lo + 1) & 1);
    const unsigned grid = (unsigned)((hi - r) * nc * 8 + (r > lo ? nc * 8 : 0));
    hipLaunchKernelGGL(strip_step_kernel, dim3(grid), dim3(256), 0, st, G, ld, W, a->w, r, hi, c0, nc, scur, sprev,
                       chol_prio());
  }
  return hipGetLastError();
}

// SCS_CHOL_BA_STEPS (default 1): the chain's strip solve by strip_solve_steps; 0 = the recursion
// (also whenever the dependency-driven launches replay it, SCS_CHOL_DAG=1)
static bool ba_steps() {
  const char* e = getenv("SCS_CHOL_BA_STEPS");
  return !(e && e[0] == '0');
}

// Lookahead (default; SCS_CHOL_LA=0 off).  Outer block t's strip solve B and trailing update C
// are cut so that only what outer block t+1's serial diagonal steps need stays on the chain
// stream st:
//   Ba  (st)  strip solve of the next block's OB columns;
//   C1a (st)  the next outer block's diagonal triangle -= X_tᵀ X_t (latency kernel);
//   Bb  (st2) strip solve of the columns beyond the next block (starts when A_t is done);
//   C12 (st2) everything else of the trailing update in ONE launch: the rest of the next
//             block's strip and all pairs beyond it (the full trailing tile list minus its
//             first OB(OB+1)/2 entries, which are C1a's).
// st2 is the bulk stream (create_bulk_stream; CU-bounded launches) and streams Bb_t, C12_t, Bb_{t+1}, ...
// back to back whenever the chain (A + Ba + C1a) is shorter than C12 (large m); the chain's
// Ba_{t+1} / C1a_{t+1} wait for C12_t (same elements).  Every element still receives its
// updates in block order with the same per-tile arithmetic (the kernels share one MFMA order),
// so U is bit-identical to the serial order.
static bool chol_lookahead() {
  const char* e = getenv("SCS_CHOL_LA");
  return !(e && e[0] == '0');
}

// ---------------------------------------------------------------------------
// Dependency-driven chain launches (opt-in SCS_CHOL_DAG=1; default: one launch per operation).
// The serial chain of the factor was ~300 small launches at m = 8192 (per inner block a row
// panel and a trailing-update launch; per outer block the next block's recursive strip solve, 15
// launches, and its diagonal triangle), each paying a launch and a ramp (~17 us) for 2-3 us of
// MFMA work.  Here each of those groups is ONE launch of independent 256-thread workgroups, each
// a strip task (a 16-column strip of one 128 x 128 tile of the operation, gram_small_strip<16>:
// the per-tile MFMA order of every Gram kernel, so U is bitwise that of the launch-per-operation
// schedule).  A task first waits for the counters of the tasks it reads (a completed task
// releases its stores, then advances its counters), so the recursion of the strip solve and the
// panel -> trailing dependency run inside one launch.  Tasks are listed in a topological order
// and a task waits only on tasks listed before it -- dispatched before it -- so the grid always
// progresses whatever is resident; a wait over ~30 s sets the error flag and drains.  Counters
// only grow: run g of a list waits for (g - 1)·period + target.
// Measured at C2 (profiles/r03/chol/dag/): bitwise identical, but SLOWER -- a step list (row panel +
// trailing, 280 strip tasks) takes 79 us against 2 x 17 us for the two launches it replaces (61 us
// even with the agent-scope fences removed, which is not coherent across XCDs and was a timing
// probe only: SCS_CHOL_DAG_FENCE=0); C2 solve 10.35 -> 11.3 ms.  Kept opt-in for the record.
template <int FENCE>
__global__ __launch_bounds__(256) void chol_dag_kernel(const DagTask* __restrict__ tasks, const DagDep* __restrict__ deps,
                                                       double* G, int64_t ld, const double* __restrict__ W,
                                                       const double* __restrict__ wv, unsigned* cnt,
                                                       const unsigned* __restrict__ period, unsigned gen,
                                                       int* __restrict__ err, int nap) {
  __shared__ __attribute__((aligned(16))) double lds[2 * (GT + 16) * GBK];
  const DagTask t = tasks[blockIdx.x];
  if (threadIdx.x == 0 && t.ndep > 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int d = 0; d < t.ndep; ++d) {
      const DagDep q = deps[t.dep0 + d];
      const unsigned target = (gen - 1u) * period[q.c] + (unsigned)q.target;
      while ((int)(__hip_atomic_load(cnt + q.c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
        for (int z = 0; z < nap; ++z) __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull) {   // 30 s at 100 MHz
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  gram_small_strip<16>((t.a1w ? W : G) + t.a1, t.lda1, G + t.a2, ld, wv + (t.wneg ? CB : 0), t.k0, t.k0 + t.nk,
                       G + t.out, ld, t.flags, lds);
  if (t.sig0 < 0 && t.sig1 < 0) return;
  if (FENCE) __threadfence();   // every thread's stores of the strip, then the counters
  else __builtin_amdgcn_s_waitcnt(0);   // A/B timing only (SCS_CHOL_DAG_FENCE=0): NOT coherent across XCDs
  __syncthreads();
  if (threadIdx.x == 0) {
    if (t.sig0 >= 0) __hip_atomic_fetch_add(cnt + t.sig0, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (t.sig1 >= 0) __hip_atomic_fetch_add(cnt + t.sig1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static bool chol_dag_on();
bool chol_dag_active(const CholAux* a) { return chol_dag_on() && a->serr && !a->no_dag; }

static bool chol_dag_on() {
  const char* e = getenv("SCS_CHOL_DAG");
  return e && e[0] == '1';
}

namespace {
struct DagBuilder {
  std::vector<DagTask> t;
  std::vector<DagDep> d;
  std::vector<unsigned> per;
  int counter() {
    per.push_back(0);
    return (int)per.size() - 1;
  }
  void add(DagTask x, const std::vector<DagDep>& dep) {
    x.dep0 = (int)d.size();
    x.ndep = (int)dep.size();
    for (const DagDep& q : dep) d.push_back(q);
    if (x.sig0 >= 0) ++per[(size_t)x.sig0];
    if (x.sig1 >= 0) ++per[(size_t)x.sig1];
    t.push_back(x);
  }
};

DagTask strip_task(int64_t a1, int lda1, bool a1w, int64_t a2, int64_t out, int k0, int nk, bool neg, int flags) {
  DagTask x;
  x.a1 = a1;
  x.a2 = a2;
  x.out = out;
  x.lda1 = lda1;
  x.a1w = a1w ? 1 : 0;
  x.k0 = k0;
  x.nk = nk;
  x.wneg = neg ? 1 : 0;
  x.flags = flags;
  x.dep0 = x.ndep = 0;
  x.sig0 = x.sig1 = -1;
  return x;
}
}  // namespace

// The task lists of one factorization shape (nblk inner blocks, outer block OB, ld):
//   step k (k not the last of its outer block [i0, i1)), nb = i1 - k - 1 blocks right of it:
//     row panel  U_kj = W_kᵀ A_kj, j = k+1 .. i1-1 (8 strips each, counter rp_j);
//     trailing   A_xy -= U_kxᵀ U_ky over the outer block (upper), after rp_x and rp_y;
//   next t (outer block t, columns c0 = i1 .. i1 + OB - 1 of the next block):
//     the strip solve X = U_Dᵀ⁻¹ R of strip_solve(i0, i1, c0, OB) -- its recursion replayed
//     per strip: every update / leaf of output strip (row r, column j, strip s) waits for the
//     previous operation on that strip and for the leaves of the X rows it reads;
//     C1a  the next diagonal triangle -= Xᵀ X (K = the block's rows, upper), after every leaf of
//     its two column blocks.
static hipError_t chol_dag_build(const CholAux* a, int nblk, int OB, int64_t ld, hipStream_t st) {
  if (a->dag_ob == OB && a->dag_ld == ld && a->dtasks) return hipSuccess;
  DagBuilder B;
  a->dstep.assign((size_t)nblk, DagList());
  a->dnext.assign((size_t)((nblk + OB - 1) / OB), DagList());
  const int up = GRAM_ACCUMULATE | GRAM_UPPER;
  for (int i0 = 0; i0 < nblk; i0 += OB) {
    const int i1 = std::min(i0 + OB, nblk);
    for (int k = i0; k + 1 < i1; ++k) {
      const int nb = i1 - k - 1;
      DagList L;
      L.t0 = (int)B.t.size();
      std::vector<int> rp((size_t)nb);
      for (int j = 0; j < nb; ++j) {
        rp[(size_t)j] = B.counter();
        for (int sq = 0; sq < 8; ++sq) {
          const int64_t a2 = ((int64_t)(k + 1 + j) * CB + 16 * sq) * ld + (int64_t)k * CB;
          DagTask x = strip_task((int64_t)k * CB * CB, CB, true, a2, a2, 0, CB, false, 0);
          x.sig0 = rp[(size_t)j];
          B.add(x, {});
        }
      }
      for (int x = 0; x < nb; ++x)
        for (int y = 0; y <= x; ++y)
          for (int sq = 0; sq < 8; ++sq) {
            const int64_t a1 = (int64_t)(k + 1 + x) * CB * ld + (int64_t)k * CB;
            const int64_t a2 = ((int64_t)(k + 1 + y) * CB + 16 * sq) * ld + (int64_t)k * CB;
            const int64_t out = (int64_t)(k + 1 + x) * CB * ld + (int64_t)(k + 1 + y) * CB + 16 * sq;
            std::vector<DagDep> dep{{rp[(size_t)x], 8}};
            if (y != x) dep.push_back({rp[(size_t)y], 8});
            B.add(strip_task(a1, (int)ld, false, a2, out, 0, CB, true, up), dep);
          }
      L.nt = (int)B.t.size() - L.t0;
      a->dstep[(size_t)k] = L;
    }
    const int nc = nblk - i1;
    if (nc <= OB) continue;   // the serial tail (chol_factor's !la branch) has no next-block list
    const int c0 = i1, R = i1 - i0;
    DagList L;
    L.t0 = (int)B.t.size();
    // per output strip (row r in [0, R), column j in [0, OB), strip s): its operation counter and
    // how many operations it has seen so far; per column the count of finished leaves
    std::vector<int> sc((size_t)R * OB * 8), nops((size_t)R * OB * 8, 0), col((size_t)OB);
    for (auto& c : sc) c = B.counter();
    for (auto& c : col) c = B.counter();
    auto sid = [&](int r, int j, int sq) { return ((size_t)r * OB + j) * 8 + sq; };
    std::vector<int> nleaf_ops((size_t)R * OB * 8, 0);   // operations of a strip including its leaf
    // first pass: count the operations each output strip receives (updates + its leaf)
    std::function<void(int, int, bool)> walk = [&](int lo, int hi, bool emit) {
      if (hi - lo == 1) {
        for (int j = 0; j < OB; ++j)
          for (int sq = 0; sq < 8; ++sq) {
            const size_t id = sid(lo - i0, j, sq);
            if (!emit) {
              ++nleaf_ops[id];
              continue;
            }
            const int64_t a2 = ((int64_t)c0 * CB + (int64_t)j * CB + 16 * sq) * ld + (int64_t)lo * CB;
            DagTask x = strip_task((int64_t)lo * CB * CB, CB, true, a2, a2, 0, CB, false, 0);
            x.sig0 = sc[id];
            x.sig1 = col[(size_t)j];
            std::vector<DagDep> dep;
            if (nops[id] > 0) dep.push_back({sc[id], nops[id]});
            B.add(x, dep);
            ++nops[id];
          }
        return;
      }
      const int mid = (lo + hi) / 2;
      walk(lo, mid, emit);
      for (int i = 0; i < hi - mid; ++i)
        for (int j = 0; j < OB; ++j)
          for (int sq = 0; sq < 8; ++sq) {
            const size_t id = sid(mid + i - i0, j, sq);
            if (!emit) {
              ++nleaf_ops[id];
              continue;
            }
            const int64_t a1 = ((int64_t)mid * CB + (int64_t)i * CB) * ld + (int64_t)lo * CB;
            const int64_t a2 = ((int64_t)c0 * CB + (int64_t)j * CB + 16 * sq) * ld + (int64_t)lo * CB;
            const int64_t out = ((int64_t)c0 * CB + (int64_t)j * CB + 16 * sq) * ld + (int64_t)(mid + i) * CB;
            DagTask x = strip_task(a1, (int)ld, false, a2, out, 0, (mid - lo) * CB, true, GRAM_ACCUMULATE);
            x.sig0 = sc[id];
            std::vector<DagDep> dep;
            if (nops[id] > 0) dep.push_back({sc[id], nops[id]});
            for (int r = lo; r < mid; ++r) {   // the X1 rows it reads: their leaves, strip s of column j
              const size_t rid = sid(r - i0, j, sq);
              dep.push_back({sc[rid], nleaf_ops[rid]});
            }
            B.add(x, dep);
            ++nops[id];
          }
      walk(mid, hi, emit);
    };
    walk(i0, i1, false);
    walk(i0, i1, true);
    // C1a: the next block's diagonal triangle (tiles x >= y < OB, row-major), K = rows [i0, i1)
    for (int x = 0; x < OB; ++x)
      for (int y = 0; y <= x; ++y)
        for (int sq = 0; sq < 8; ++sq) {
          const int64_t a1 = ((int64_t)c0 * CB + (int64_t)x * CB) * ld;
          const int64_t a2 = ((int64_t)c0 * CB + (int64_t)y * CB + 16 * sq) * ld;
          const int64_t out = ((int64_t)c0 * CB + (int64_t)x * CB) * ld + (int64_t)c0 * CB + (int64_t)y * CB + 16 * sq;
          std::vector<DagDep> dep{{col[(size_t)x], 8 * R}};
          if (y != x) dep.push_back({col[(size_t)y], 8 * R});
          B.add(strip_task(a1, (int)ld, false, a2, out, i0 * CB, R * CB, true, up), dep);
        }
    L.nt = (int)B.t.size() - L.t0;
    a->dnext[(size_t)(i0 / OB)] = L;
  }
  if (a->dtasks) (void)hipFree(a->dtasks);
  if (a->ddeps) (void)hipFree(a->ddeps);
  if (a->dcnt) (void)hipFree(a->dcnt);
  if (a->dper) (void)hipFree(a->dper);
  a->dtasks = nullptr;
  a->ddeps = nullptr;
  a->dcnt = a->dper = nullptr;
  hipError_t e = hipMalloc(&a->dtasks, sizeof(DagTask) * std::max<size_t>(B.t.size(), 1));
  if (e == hipSuccess) e = hipMalloc(&a->ddeps, sizeof(DagDep) * std::max<size_t>(B.d.size(), 1));
  if (e == hipSuccess) e = hipMalloc(&a->dcnt, sizeof(unsigned) * std::max<size_t>(B.per.size(), 1));
  if (e == hipSuccess) e = hipMalloc(&a->dper, sizeof(unsigned) * std::max<size_t>(B.per.size(), 1));
  if (e == hipSuccess && !B.t.empty())
    e = hipMemcpyAsync(a->dtasks, B.t.data(), sizeof(DagTask) * B.t.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess && !B.d.empty())
    e = hipMemcpyAsync(a->ddeps, B.d.data(), sizeof(DagDep) * B.d.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess && !B.per.empty()) {
    e = hipMemsetAsync(a->dcnt, 0, sizeof(unsigned) * B.per.size(), st);
    if (e == hipSuccess)
      e = hipMemcpyAsync(a->dper, B.per.data(), sizeof(unsigned) * B.per.size(), hipMemcpyHostToDevice, st);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess) {
    a->dag_ob = OB;
    a->dag_ld = ld;
  }
  return e;
}

static hipError_t chol_dag_launch(const CholAux* a, DagList& L, double* G, int64_t ld, const double* W, hipStream_t st) {
  if (L.nt <= 0) return hipSuccess;
  ++L.gen;
  static const int nap = [] { const char* e = getenv("SCS_CHOL_DAG_SLEEP"); return e ? atoi(e) : 1; }();
  const char* fe = getenv("SCS_CHOL_DAG_FENCE");
  if (fe && fe[0] == '0')
    hipLaunchKernelGGL(chol_dag_kernel<0>, dim3((unsigned)L.nt), dim3(256), 0, st, a->dtasks + L.t0, a->ddeps, G, ld, W,
                       a->w, a->dcnt, a->dper, L.gen, a->serr, nap);
  else
    hipLaunchKernelGGL(chol_dag_kernel<1>, dim3((unsigned)L.nt), dim3(256), 0, st, a->dtasks + L.t0, a->ddeps, G, ld, W,
                       a->w, a->dcnt, a->dper, L.gen, a->serr, nap);
  return hipGetLastError();
}

// SCS_CHOL_C12_SPLIT (default 1): the lookahead's trailing update C12_t as two bulk launches,
// C12a_t -- the upper triangle of the next two blocks' square less C1a_t: rows of block t+1 x
// columns of block t+2 (what Ba_{t+1} solves) and block t+2's diagonal triangle (what C1a_{t+1}
// updates next) -- then C12b_t, the rest.  The chain waits for C12a_t only, i.e. for C12b_{t-1}
// one outer block later than before (stream order on st2), so in the bulk-bound outer blocks the
// bulk stream no longer idles while the chain's Ba waits for a whole C12 (r03 trace at m = 8192:
// 6.19 ms of chain and 6.18 ms of bulk work in an 8.23 ms span).  Every element still takes its
// updates in block order with the per-tile-identical kernels: U bitwise the serial order's.  0 = one
// C12 launch.
static bool c12_split() {
  const char* e = getenv("SCS_CHOL_C12_SPLIT");
  return !(e && e[0] == '0');
}

// SCS_CHOL_SBL (read per call; default on, 0 = row-major): the bulk trailing update C12b takes its
// tiles in 8 x 8 super-blocks (a->sbl) where the slice is exact (8 | 2OB, 8 | nc).  A workgroup
// takes tile tix of its XCD's contiguous segment, so an XCD's 64 concurrent tiles are one super-block
// sharing 8 + 8 operand panels instead of one row sharing 1 + 64: at K = 1024 a panel is 1 MiB, so
// the row-major band re-fetched its A2 panels from HBM.  m = 65536 factor 1498-1510 -> 1427-1436 ms,
// m = 32768 204.0-204.7 -> 201.8-202.8 ms, U / W bitwise equal (profiles/r04/sbl/).
// SCS_CHOL_C12B_CHUNK (read per call; 0 = one launch): where the bulk stream launches plainly (no skip
// set: m >= 16384), C12b as launches of this many tiles.  One launch of thousands of tiles refills every
// slot it frees, and the chain's diagonal kernel then waited for all of it, once per outer block
// (profiles/r06/chol_pack/); between launches of about one round the CUs drain and the chain gets one.
static int c12b_chunk() {
  const char* e = getenv("SCS_CHOL_C12B_CHUNK");
  return e ? atoi(e) : 0;
}

static bool chol_sbl() {
  const char* e = getenv("SCS_CHOL_SBL");
  return !(e && e[0] == '0');
}

hipError_t chol_factor(double* G, int64_t ld, int64_t m, int64_t mpad, double* W, const CholAux* a,
                       const int2* trilist, int* info, hipStream_t st_caller) {
  const int nblk = (int)(mpad / CB);
  const int OB = outer_block_for(nblk);
  const bool la = chol_lookahead() && a->st2 && nblk > 2 * OB;
  // the chain's and the bulk stream (create_hiprio_stream): never one hardware queue
  const int cmode = chol_chain_mode(a);
  hipStream_t st = st_caller;
  hipStream_t sb = (cmode == 2 && a->st2h) ? a->st2h : a->st2;
  if (la && cmode == 1 && a->stc && a->ev0 && a->ev5) {
    hipError_t ej = hipEventRecord(a->ev0, st_caller);
    if (ej == hipSuccess) ej = hipStreamWaitEvent(a->stc, a->ev0, 0);
    if (ej != hipSuccess) return ej;
    st = a->stc;
  }
  const bool dag = chol_dag_on() && a->serr && !a->no_dag;
  const bool steps = !dag && ba_steps() && a->sscr && OB <= 16;
  const bool split = la && c12_split() && a->ev4;
  if (dag) {
    const hipError_t eb = chol_dag_build(a, nblk, OB, ld, st);
    if (eb != hipSuccess) return eb;
  }
  bool c12_pending = false;
  const int pf = (la && chol_prio()) ? GRAM_PRIO : 0;   // the chain's latency launches (SCS_CHOL_PRIO)
  hipError_t e = hipSuccess;
  auto wait = [&](hipStream_t s, hipEvent_t ev) {
    if (e == hipSuccess) e = hipStreamWaitEvent(s, ev, 0);
  };
  if (mpad > m) hipLaunchKernelGGL(diag_pad_kernel, dim3((unsigned)ceil_div(mpad - m, 256)), dim3(256), 0, st, G, ld,
                                   m, mpad);
  for (int i0 = 0; i0 < nblk; i0 += OB) {
    const int i1 = i0 + OB < nblk ? i0 + OB : nblk;
    // A: inner factor of the outer diagonal block
    for (int k = i0; k < i1; ++k) {
      e = launch_chol_diag(G, ld, k, W, info, st);
      if (e != hipSuccess) return e;
      const int nb = i1 - k - 1;
      if (nb == 0) break;
      if (dag) {   // the row panel and the trailing update of step k as one launch
        e = chol_dag_launch(a, a->dstep[(size_t)k], G, ld, W, st);
        if (e != hipSuccess) return e;
        continue;
      }
      double* rowpanel = G + (int64_t)(k + 1) * CB * ld + (int64_t)k * CB;   // U_k,(k+1..i1-1)
      e = gram_launch_gen(W + (int64_t)k * CB * CB, CB, rowpanel, ld, a->w, 0, CB, rect_list(a, 1), nb, rowpanel, ld,
                          pf, st);
      if (e != hipSuccess) return e;
      double* trail = G + (int64_t)(k + 1) * CB * ld + (int64_t)(k + 1) * CB;
      e = gram_launch_gen(rowpanel, ld, rowpanel, ld, a->w + CB, 0, CB, trilist, nb * (nb + 1) / 2, trail, ld,
                          /*GRAM_ACCUMULATE|GRAM_UPPER*/ 2 | 4 | pf, st);
      if (e != hipSuccess) return e;
    }
    const int nc = nblk - i1;
    if (nc == 0) break;
    const double* X = G + (int64_t)i1 * CB * ld;
    double* trail = G + (int64_t)i1 * CB * ld + (int64_t)i1 * CB;
    const int ntri = nc * (nc + 1) / 2;
    if (!la || nc <= OB) {
      if (c12_pending) {   // the previous block's bulk update reaches these elements first
        wait(st, a->ev2);
        c12_pending = false;
      }
      // B: strip solve, C: trailing update with K = (i1 - i0)·128.  With the step launches for the
      // chain's columns, the first OB columns take them here too (the lookahead's Ba) and the rest
      // the recursion (its Bb): the same operations per element in both orders
      if (e == hipSuccess) {
        if (steps) {
          const int nb = nc < OB ? nc : OB;
          e = strip_solve_steps(G, ld, W, a, i0, i1, i1, nb, st);
          if (e == hipSuccess && nc > nb) e = strip_solve(G, ld, W, a, i0, i1, i1 + nb, nc - nb, st);
        } else {
          e = strip_solve(G, ld, W, a, i0, i1, i1, nc, st);
        }
      }
      if (e == hipSuccess)
        e = gram_launch_gen(X, ld, X, ld, a->w + CB, (int64_t)i0 * CB, (int64_t)i1 * CB, trilist, ntri, trail, ld,
                            2 | 4, st);
      if (e != hipSuccess) return e;
      continue;
    }
    // Bb on st2 once A_t is done (stream order keeps C12_{t-1} before it)
    if (e == hipSuccess) e = hipEventRecord(a->ev3, st);
    wait(sb, a->ev3);
    if (e == hipSuccess) e = strip_solve(G, ld, W, a, i0, i1, i1 + OB, nc - OB, sb, true);
    // Ba, C1a on the chain after C12a_{t-1} (and so after everything before it on st2)
    if (c12_pending) wait(st, split ? a->ev4 : a->ev2);
    const int n1a = (OB * (OB + 1)) / 2;
    if (dag) {   // the recursive strip solve and the next diagonal triangle as one launch
      if (e == hipSuccess) e = chol_dag_launch(a, a->dnext[(size_t)(i0 / OB)], G, ld, W, st);
    } else {
      if (e == hipSuccess)
        e = steps ? strip_solve_steps(G, ld, W, a, i0, i1, i1, OB, st) : strip_solve(G, ld, W, a, i0, i1, i1, OB, st);
      if (e == hipSuccess)
        e = gram_launch_small(X, ld, X, ld, a->w + CB, (int64_t)i0 * CB, (int64_t)i1 * CB, trilist, n1a, trail, ld,
                              2 | 4 | pf, st);
    }
    // C12 on st2 after Ba (it reads X's columns of the next block); split: C12a (the tiles the
    // chain's next Ba and C1a read) as a latency launch, its event, then C12b
    if (e == hipSuccess) e = hipEventRecord(a->ev1, st);
    wait(sb, a->ev1);
    const int n2a = split ? std::min(ntri, OB * (2 * OB + 1)) : n1a;   // 2OB(2OB+1)/2 tiles
    if (split) {
      if (e == hipSuccess && n2a > n1a)
        e = gram_launch_small(X, ld, X, ld, a->w + CB, (int64_t)i0 * CB, (int64_t)i1 * CB, trilist + n1a, n2a - n1a,
                              trail, ld, 2 | 4, sb);
      if (e == hipSuccess) e = hipEventRecord(a->ev4, sb);
    }
    if (e == hipSuccess && ntri > n2a) {
      unsigned* ctr = bulk_ctr(a, sb, &e);
      const bool sbo = split && a->sbl && (2 * OB) % 8 == 0 && nc % 8 == 0 && chol_sbl();
      const unsigned mk = bulk_mask(a, ntri - n2a);
      const int2* tl = (sbo ? a->sbl : trilist) + n2a;
      const int tot = ntri - n2a, ck = c12b_chunk();
      if (ck > 0 && mk == 0) {   // (r06, A/B) C12b as launches of ck tiles: the chain finds CUs between them
        for (int t0 = 0; t0 < tot && e == hipSuccess; t0 += ck)
          e = gram_launch_gen(X, ld, X, ld, a->w + CB, (int64_t)i0 * CB, (int64_t)i1 * CB, tl + t0,
                              std::min(ck, tot - t0), trail, ld, 2 | 4, sb);
      } else if (e == hipSuccess) {
        e = gram_launch_bounded(X, ld, X, ld, a->w + CB, (int64_t)i0 * CB, (int64_t)i1 * CB, tl, tot, trail, ld, 2 | 4,
                                ctr, mk, bulk_slots(a, mk), sb, true);
      }
    }
    if (e == hipSuccess) e = hipEventRecord(a->ev2, sb);
    if (e != hipSuccess) return e;
    c12_pending = true;
  }
  if (c12_pending) wait(st, a->ev2);
  if (e == hipSuccess && st != st_caller) {   // the caller's stream continues behind the whole factor
    e = hipEventRecord(a->ev5, st);
    wait(st_caller, a->ev5);
  }
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Strip pipeline.  Where the Gram is computed strip by strip (scsopt.cpp), the factor runs
// LEFT-looking behind it: strip s receives the updates of all earlier strips in one launch
// (K = i0·128 rows of U) once its own Gram strip has landed, then its diagonal block (A) and
// row strip (B) are factored exactly as in chol_factor.  There is no trailing update: the
// later strips pull theirs.  Few tiles with a long K (the last strips) are what
// gram_schedule's K-split tail pieces are for.
int chol_outer_block() { return outer_block(); }

hipError_t chol_pipe_init(CholAux* a, int64_t mpad, hipStream_t st) {
  if (!a->ssched.empty()) return hipSuccess;
  const int nblk = (int)(mpad / CB), OB = outer_block();
  const int ns = (nblk + OB - 1) / OB;
  std::vector<int2> lst;   // (i >= j, j < OB), row-major in i: a strip's list is a prefix
  for (int i = 0; i < nblk; ++i)
    for (int j = 0; j <= i && j < OB; ++j) lst.push_back(make_int2(i, j));
  a->ssched.resize(ns);
  int npart_max = 0;
  hipError_t e = hipSuccess;
  for (int s = 1; s < ns && e == hipSuccess; ++s) {
    const int nc = nblk - s * OB;
    int n = 0;
    for (int i = 0; i < nc; ++i) n += std::min(i + 1, OB);
    std::vector<int4> wk, cb;
    int nsplit = 1, npart = 0;
    const int seglen = gram_schedule(lst.data(), n, 64, wk, cb, &nsplit, &npart);
    CholAux::StripSched& q = a->ssched[s];
    q.seglen = seglen;
    q.nsplit = nsplit;
    q.ncomb = (int)cb.size();
    npart_max = std::max(npart_max, npart);
    e = hipMalloc(&q.work, sizeof(int4) * wk.size());
    if (e == hipSuccess) e = hipMemcpyAsync(q.work, wk.data(), sizeof(int4) * wk.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess && !cb.empty()) {
      e = hipMalloc(&q.comb, sizeof(int4) * cb.size());
      if (e == hipSuccess) e = hipMemcpyAsync(q.comb, cb.data(), sizeof(int4) * cb.size(), hipMemcpyHostToDevice, st);
    }
  }
  if (e == hipSuccess && npart_max > 0) e = hipMalloc(&a->spart, sizeof(double) * (size_t)npart_max * CB * CB);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  return e;
}

hipError_t chol_strip_update(double* G, int64_t ld, int s, const CholAux* a, hipStream_t st) {
  if (s <= 0 || s >= (int)a->ssched.size()) return hipSuccess;
  const int i0 = s * outer_block();
  const CholAux::StripSched& q = a->ssched[s];
  const double* X = G + (int64_t)i0 * CB * ld;
  double* trail = G + (int64_t)i0 * CB * ld + (int64_t)i0 * CB;
  return gram_launch_sched_cm(X, ld, a->w + CB, 0, (int64_t)i0 * CB, q.work, q.seglen, q.nsplit, q.comb, q.ncomb,
                              a->spart, trail, ld, /*GRAM_ACCUMULATE*/ 2, st);
}

hipError_t chol_strip_factor(double* G, int64_t ld, int s, double* W, const CholAux* a, const int2* trilist, int* info,
                             hipStream_t st) {
  const int nblk = a->nblk, OB = outer_block();
  const int i0 = s * OB, i1 = std::min(i0 + OB, nblk);
  for (int k = i0; k < i1; ++k) {
    hipError_t e = launch_chol_diag(G, ld, k, W, info, st);
    if (e != hipSuccess) return e;
    const int nb = i1 - k - 1;
    if (nb == 0) break;
    double* rowpanel = G + (int64_t)(k + 1) * CB * ld + (int64_t)k * CB;
    e = gram_launch_gen(W + (int64_t)k * CB * CB, CB, rowpanel, ld, a->w, 0, CB, rect_list(a, 1), nb, rowpanel, ld, 0,
                        st);
    if (e != hipSuccess) return e;
    double* trail = G + (int64_t)(k + 1) * CB * ld + (int64_t)(k + 1) * CB;
    e = gram_launch_gen(rowpanel, ld, rowpanel, ld, a->w + CB, 0, CB, trilist, nb * (nb + 1) / 2, trail, ld, 2 | 4, st);
    if (e != hipSuccess) return e;
  }
  const int nc = nblk - i1;
  if (nc > 0) {
    hipError_t e = strip_solve(G, ld, W, a, i0, i1, i1, nc, st);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

// dst(r0:r1, c) = src(r0:r1, c) for c in [c0, c1) (column-major, ld): a strip of the upper system.
// One workgroup per column run of 8 columns, the rows contiguous (hipMemcpy2DAsync's rectangle blit
// moved these 64 MB strips at 13 GB/s).
__global__ void copy_rows_kernel(double* __restrict__ dst, const double* __restrict__ src, int64_t ld, int64_t r0,
                                 int64_t r1, int64_t c0, int64_t c1) {
  const int64_t nr = r1 - r0;
  for (int64_t c = c0 + (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); c < c1; c += (int64_t)gridDim.x * 8) {
    const double* s = src + c * ld + r0;
    double* d = dst + c * ld + r0;
    for (int64_t i = 2 * (threadIdx.x & 31); i + 1 < nr; i += 64) *(v2d*)(d + i) = *(const v2d*)(s + i);
    if ((nr & 1) && (threadIdx.x & 31) == 0) d[nr - 1] = s[nr - 1];
  }
}

hipError_t chol_copy_rows(double* dst, const double* src, int64_t ld, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                          hipStream_t st) {
  if (r1 <= r0 || c1 <= c0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(c1 - c0, 8), 2048);
  hipLaunchKernelGGL(copy_rows_kernel, dim3(grid), dim3(256), 0, st, dst, src, ld, r0, r1, c0, c1);
  return hipGetLastError();
}

__global__ void diag_pad_range_kernel(double* __restrict__ G, int64_t ld, int64_t lo, int64_t hi) {
  const int64_t i = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < hi) G[i * ld + i] = 1.0;
}

hipError_t chol_diag_pad(double* G, int64_t ld, int64_t lo, int64_t hi, hipStream_t st) {
  if (hi <= lo) return hipSuccess;
  hipLaunchKernelGGL(diag_pad_range_kernel, dim3((unsigned)ceil_div(hi - lo, 256)), dim3(256), 0, st, G, ld, lo, hi);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Triangular solves, two-level: per outer block one single-workgroup kernel runs the
// (≤ OB) serial 128-block steps with the block's right-hand side in LDS, and one
// many-workgroup kernel applies the block's contribution to the rest of the vector
// (a (OB·128) x rest transposed GEMV).  2 launches per outer block instead of
// 2 per 128-block, and the W_k products are coalesced.
constexpr int SOLVE_NT = 1024;
constexpr int SOLVE_MAXB = 16;   // max inner blocks per outer block held in LDS

// Uᵀ y = b restricted to rows [i0, i1) (inner blocks): b is already reduced by the
// contributions of earlier outer blocks.  Writes y[i0..i1).
__global__ __launch_bounds__(SOLVE_NT) void chol_fwd_inner_kernel(const double* __restrict__ G, int64_t ld,
                                                                   const double* __restrict__ W, int i0, int i1,
                                                                   const double* __restrict__ b,
                                                                   double* __restrict__ y) {
  __shared__ double bs[SOLVE_MAXB * CB];
  __shared__ double yk[CB];
  const int tid = threadIdx.x;
  const int nr = (i1 - i0) * CB;
  for (int r = tid; r < nr; r += SOLVE_NT) bs[r] = b[(int64_t)i0 * CB + r];
  __syncthreads();
  for (int k = i0; k < i1; ++k) {
    const int ko = (k - i0) * CB;
    {  // y_k[t] = Σ_u W(u, t) b_k(u): 8 threads per output t, 16 contiguous u each (column t of W)
      const int t = tid >> 3, p = tid & 7;
      const double* col = W + (int64_t)k * CB * CB + (int64_t)t * CB + 16 * p;
      double sacc = 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) sacc += col[u] * bs[ko + 16 * p + u];
      sacc += __shfl_xor(sacc, 1, 64);
      sacc += __shfl_xor(sacc, 2, 64);
      sacc += __shfl_xor(sacc, 4, 64);
      if (p == 0) yk[t] = sacc;
    }
    __syncthreads();
    if (tid < CB) y[(int64_t)k * CB + tid] = yk[tid];
    // b_j -= U_kjᵀ y_k for the columns of the later blocks of this outer block
    const int ncol = (i1 - k - 1) * CB;
    for (int cb = 0; cb < ncol; cb += SOLVE_NT / 8) {
      const int cl = cb + (tid >> 3), p = tid & 7;
      double sacc = 0.0;
      if (cl < ncol) {
        const double* col = G + (int64_t)((k + 1) * CB + cl) * ld + (int64_t)k * CB + 16 * p;
#pragma unroll
        for (int u = 0; u < 16; ++u) sacc += col[u] * yk[16 * p + u];
      }
      sacc += __shfl_xor(sacc, 1, 64);
      sacc += __shfl_xor(sacc, 2, 64);
      sacc += __shfl_xor(sacc, 4, 64);
      if (p == 0 && cl < ncol) bs[ko + CB + cl] -= sacc;
    }
    __syncthreads();
  }
}

// b[c] -= Σ_{r in rows [r0, r1)} U(r, c) y(r) for columns c in [c0, c0 + nc): one wave per column
// (contiguous rows), fixed-order wave reduction.
__global__ __launch_bounds__(256) void chol_fwd_update_kernel(const double* __restrict__ G, int64_t ld, int64_t r0,
                                                              int64_t r1, const double* __restrict__ y, int64_t c0,
                                                              int64_t nc, double* __restrict__ b) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nc) return;
  const double* col = G + (c0 + c) * ld;
  double sacc = 0.0;
  for (int64_t r = r0 + 2 * lane; r < r1; r += 128) {
    const v2d u = *(const v2d*)(col + r);
    const v2d yy = *(const v2d*)(y + r);
    sacc += u[0] * yy[0] + u[1] * yy[1];
  }
  sacc = wave_sum(sacc);
  if (lane == 0) b[c0 + c] -= sacc;
}

// U x = y restricted to rows [i0, i1), descending; y already reduced by the later outer
// blocks.  Writes x[i0..i1).
__global__ __launch_bounds__(SOLVE_NT) void chol_bwd_inner_kernel(const double* __restrict__ G, int64_t ld,
                                                                   const double* __restrict__ W, int i0, int i1,
                                                                   const double* __restrict__ yv,
                                                                   double* __restrict__ x) {
  __shared__ double ys[SOLVE_MAXB * CB];
  __shared__ double part[8][CB];
  __shared__ double xk[CB];
  const int tid = threadIdx.x;
  const int nr = (i1 - i0) * CB;
  for (int r = tid; r < nr; r += SOLVE_NT) ys[r] = yv[(int64_t)i0 * CB + r];
  __syncthreads();
  for (int k = i1 - 1; k >= i0; --k) {
    const int ko = (k - i0) * CB;
    {  // x_k[t] = Σ_{u} W(t, u) y_k(u): thread (p, t), u in [16p, 16p+16), coalesced over t
      const int t = tid & 127, p = tid >> 7;
      const double* Wk = W + (int64_t)k * CB * CB;
      double sacc = 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) sacc += Wk[(int64_t)(16 * p + u) * CB + t] * ys[ko + 16 * p + u];
      part[p][t] = sacc;
    }
    __syncthreads();
    if (tid < CB) {
      double sacc = 0.0;
#pragma unroll
      for (int p = 0; p < 8; ++p) sacc += part[p][tid];
      xk[tid] = sacc;
      x[(int64_t)k * CB + tid] = sacc;
    }
    __syncthreads();
    // y_r -= Σ_t U(r, k·128 + t) x_k(t) for the rows of the earlier blocks of this outer block
    const int nrow = ko;
    for (int r = tid; r < nrow; r += SOLVE_NT) {
      const double* row = G + (int64_t)k * CB * ld + (int64_t)i0 * CB + r;
      double sacc = 0.0;
#pragma unroll 8
      for (int t = 0; t < CB; ++t) sacc += row[(int64_t)t * ld] * xk[t];
      ys[r] -= sacc;
    }
    __syncthreads();
  }
}

// y[r] -= Σ_{c in [c0, c1)} U(r, c) x(c) for rows r in [0, nr): 64 rows per workgroup,
// 4 waves split the column range, partials summed in wave order.
__global__ __launch_bounds__(256) void chol_bwd_update_kernel(const double* __restrict__ G, int64_t ld, int64_t c0,
                                                              int64_t c1, const double* __restrict__ x, int64_t nr,
                                                              double* __restrict__ y) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * 64 + lane;
  const int64_t len = (c1 - c0 + 3) / 4;
  const int64_t ca = c0 + wv * len, cz = ca + len < c1 ? ca + len : c1;
  double sacc = 0.0;
  if (r < nr)
    for (int64_t c = ca; c < cz; ++c) sacc += G[c * ld + r] * x[c];
  part[wv][lane] = sacc;
  __syncthreads();
  if (wv == 0 && r < nr) y[r] -= ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
}

// ---------------------------------------------------------------------------
// Triangular solves as ONE launch per direction (default; SCS_SOLVE_PERSIST=0: the two-launch-per-
// block form above).  The per-block form is launch-bound: m = 8192 has 64 blocks x 2 launches x 2
// directions = 256 launches, ~7 us each (1.9 ms).  Here workgroup j owns block j of the
// right-hand side for the whole solve: it applies the earlier blocks' contributions as their
// results appear -- each published by its owner with a release store of the solve's generation
// number into flags[block] -- and then publishes its own.  A workgroup waits only on blocks
// dispatched before it (forward: lower ids; backward: blockIdx b owns block nblk-1-b), so the grid
// always progresses whatever is resident; a wait longer than ~30 s sets *err and drains.
//   forward  Uᵀ y = b:  acc = b_j - Σ_{k<j} U_kjᵀ y_k (k ascending), y_j = W_jᵀ acc
//   backward U x = y:   acc = y_k - Σ_{j>k} U_kj x_j (j descending), x_k = W_k acc
// Fixed summation orders: bitwise run to run.
constexpr int PS_NT = 256;

__device__ __forceinline__ bool ps_wait(const unsigned* flag, unsigned gen, int* err) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull) {   // 30 s at 100 MHz
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  return true;
}

__device__ __forceinline__ void ps_publish(unsigned* flag, unsigned gen) {
  __threadfence();   // every thread's stores of the block's result, then the flag
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// A 128 x 128 column-major tile held in registers for the two GEMV forms below, loaded before the
// vector it multiplies is published (the load latency leaves the serial chain).
//   column form  out[c] += sign · Σ_r T(r, c) v[r] (ps_load_col / ps_apply_col below);
//   row form     out[r] += sign · Σ_t T(r, t) v[t]: wave w holds columns [32w, 32w + 32), lane l
//                rows l and l + 64 (coalesced, no lane reduction); the four wave partials are
//                summed in wave order through LDS.
// Fixed summation orders: bitwise run to run.
struct PsTile {
  double a[32][2];
};

// column form: wave w holds columns [32w, 32w + 32) as 8 groups of 4; in group g the 16 lanes of
// row ρ = l >> 4 hold column 32w + 4g + ρ, lane l its rows [8(l & 15), 8(l & 15) + 8) (four 16-B
// loads: each column's 1 KiB read by 16 lanes).  After the 8-row partial sums, a transposing
// butterfly inside each 16-lane row needs only DPP: row_mirror (lane bit 3), row_half_mirror (bit
// 2), quad_perm xor 2, xor 1 -- 8 value moves for 8 columns -- and lane l (bit 0 clear) ends with
// the column of group ((l>>3)&1)·4 + ((l>>2)&1)·2 + ((l>>1)&1).
template <int CTRL>
__device__ __forceinline__ double ps_dpp(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
constexpr int DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141, DPP_XOR2 = 0x4E, DPP_XOR1 = 0xB1;

__device__ __forceinline__ void ps_load_col(const double* __restrict__ T, int64_t ld, PsTile& R) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = 8 * (lane & 15), cq = lane >> 4;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const double* col = T + (int64_t)(32 * wv + 4 * g + cq) * ld + r0;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const v2d t = *(const v2d*)(col + 2 * h);
      R.a[4 * g + h][0] = t[0];
      R.a[4 * g + h][1] = t[1];
    }
  }
}

__device__ __forceinline__ void ps_apply_col(const PsTile& R, const double* v, double* out, double sign) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = 8 * (lane & 15);
  double vv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) vv[i] = v[r0 + i];
  double p[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    double t = 0.0;
#pragma unroll
    for (int h = 0; h < 4; ++h) t += R.a[4 * g + h][0] * vv[2 * h] + R.a[4 * g + h][1] * vv[2 * h + 1];
    p[g] = t;
  }
  {  // row_mirror: bit 3, 8 -> 4 values
    const bool hi = (lane & 8) != 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double send = hi ? p[i] : p[i + 4], keep = hi ? p[i + 4] : p[i];
      p[i] = keep + ps_dpp<DPP_ROW_MIRROR>(send);
    }
  }
  {  // row_half_mirror: bit 2, 4 -> 2
    const bool hi = (lane & 4) != 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const double send = hi ? p[i] : p[i + 2], keep = hi ? p[i + 2] : p[i];
      p[i] = keep + ps_dpp<DPP_ROW_HALF_MIRROR>(send);
    }
  }
  {  // xor 2: bit 1, 2 -> 1
    const bool hi = (lane & 2) != 0;
    const double send = hi ? p[0] : p[1], keep = hi ? p[1] : p[0];
    p[0] = keep + ps_dpp<DPP_XOR2>(send);
  }
  const double t = p[0] + ps_dpp<DPP_XOR1>(p[0]);   // xor 1: the whole 16-lane sum
  if ((lane & 1) == 0) {
    const int g = ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
    out[32 * wv + 4 * g + (lane >> 4)] += sign * t;
  }
}

__device__ __forceinline__ void ps_load_row(const double* __restrict__ T, int64_t ld, PsTile& R) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const double* col = T + (int64_t)(32 * wv + q) * ld;
    R.a[q][0] = col[lane];
    R.a[q][1] = col[lane + 64];
  }
}

__device__ __forceinline__ void ps_apply_row(const PsTile& R, const double* v, double* part, double* out,
                                             double sign) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const double vt = v[32 * wv + q];
    s0 += R.a[q][0] * vt;
    s1 += R.a[q][1] * vt;
  }
  part[wv * CB + lane] = s0;
  part[wv * CB + lane + 64] = s1;
  __syncthreads();
  if (threadIdx.x < CB) {
    const int r = threadIdx.x;
    out[r] += sign * (((part[r] + part[CB + r]) + part[2 * CB + r]) + part[3 * CB + r]);
  }
  __syncthreads();
}

__global__ __launch_bounds__(PS_NT) void chol_fwd_persist_kernel(const double* __restrict__ G, int64_t ld,
                                                                 const double* __restrict__ W,
                                                                 const double* __restrict__ b, double* __restrict__ y,
                                                                 unsigned* __restrict__ flags, unsigned gen,
                                                                 int* __restrict__ err) {
  __shared__ double acc[CB], yk[CB], yj[CB];
  const int j = blockIdx.x, tid = threadIdx.x;
  PsTile Wr, Tr;
  ps_load_col(W + (int64_t)j * CB * CB, CB, Wr);
  if (tid < CB) {
    acc[tid] = b[(int64_t)j * CB + tid];
    yj[tid] = 0.0;
  }
  for (int k = 0; k < j; ++k) {
    ps_load_col(G + (int64_t)j * CB * ld + (int64_t)k * CB, ld, Tr);   // U_kj, before y_k is out
    ps_wait(flags + k, gen, err);
    if (tid < CB) yk[tid] = __hip_atomic_load(y + (int64_t)k * CB + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    ps_apply_col(Tr, yk, acc, -1.0);
    __syncthreads();
  }
  __syncthreads();
  ps_apply_col(Wr, acc, yj, 1.0);   // y_j[t] = Σ_u W(u, t) acc[u]
  __syncthreads();
  if (tid < CB) __hip_atomic_store(y + (int64_t)j * CB + tid, yj[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ps_publish(flags + j, gen);
}

__global__ __launch_bounds__(PS_NT) void chol_bwd_persist_kernel(const double* __restrict__ G, int64_t ld,
                                                                 const double* __restrict__ W,
                                                                 const double* __restrict__ y, double* __restrict__ x,
                                                                 unsigned* __restrict__ flags, unsigned gen,
                                                                 int* __restrict__ err, int nblk) {
  __shared__ double acc[CB], xj[CB], xk[CB], part[4 * CB];
  const int k = nblk - 1 - (int)blockIdx.x, tid = threadIdx.x;
  PsTile Wr, Tr;
  ps_load_row(W + (int64_t)k * CB * CB, CB, Wr);
  if (tid < CB) {
    acc[tid] = y[(int64_t)k * CB + tid];
    xk[tid] = 0.0;
  }
  __syncthreads();
  for (int j = nblk - 1; j > k; --j) {
    ps_load_row(G + (int64_t)j * CB * ld + (int64_t)k * CB, ld, Tr);   // U_kj, before x_j is out
    ps_wait(flags + j, gen, err);
    if (tid < CB) xj[tid] = __hip_atomic_load(x + (int64_t)j * CB + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    ps_apply_row(Tr, xj, part, acc, -1.0);
  }
  ps_apply_row(Wr, acc, part, xk, 1.0);   // x_k[t] = Σ_u W(t, u) acc[u]
  if (tid < CB) __hip_atomic_store(x + (int64_t)k * CB + tid, xk[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ps_publish(flags + k, gen);
}

static bool solve_persist() {
  const char* e = getenv("SCS_SOLVE_PERSIST");
  return !(e && e[0] == '0');
}

hipError_t chol_back_solve(const double* U, int64_t ld, int64_t mpad, const double* W, double* y, double* x,
                           unsigned* flags, unsigned gen, int* err, hipStream_t st) {
  const int nblk = (int)(mpad / CB);
  if (!solve_persist()) return chol_back_blocks(U, ld, mpad, W, y, x, st);   // SCS_SOLVE_PERSIST=0 (y consumed)
  if (!flags || !err || gen == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(chol_bwd_persist_kernel, dim3((unsigned)nblk), dim3(PS_NT), 0, st, U, ld, W, y, x, flags, gen,
                     err, nblk);
  return hipGetLastError();
}

// U x = y by outer blocks of OB 128-blocks in descending order: the x of block [i0, i1) to x, y
// updated in place (the per-block form of chol_bwd_persist_kernel)
static hipError_t chol_back_blocks_ob(const double* G, int64_t ld, int nblk, const double* W, double* y, double* b,
                                      int OB, hipStream_t st) {
  const int nout = (nblk + OB - 1) / OB;
  for (int q = nout - 1; q >= 0; --q) {
    const int i0 = q * OB, i1 = i0 + OB < nblk ? i0 + OB : nblk;
    hipLaunchKernelGGL(chol_bwd_inner_kernel, dim3(1), dim3(SOLVE_NT), 0, st, G, ld, W, i0, i1, y, b);
    const int64_t nr = (int64_t)i0 * CB;
    if (nr > 0)
      hipLaunchKernelGGL(chol_bwd_update_kernel, dim3((unsigned)ceil_div(nr, 64)), dim3(256), 0, st, G, ld,
                         (int64_t)i0 * CB, (int64_t)i1 * CB, b, nr, y);
  }
  return hipGetLastError();
}

// Solve G x = b given the factor; b (length mpad, zero-padded) is overwritten by x; y is
// scratch (mpad).
hipError_t chol_solve(const double* G, int64_t ld, int64_t mpad, const double* W, double* b, double* y,
                      CholAux* a, hipStream_t st) {
  const int nblk = (int)(mpad / CB);
  if (a && a->sflags && solve_persist() && !a->no_persist) {
    // y (forward) then b := x (backward); flags [0, nblk) forward, [nblk, 2 nblk) backward
    const unsigned gen = ++a->sgen == 0 ? ++a->sgen : a->sgen;
    hipLaunchKernelGGL(chol_fwd_persist_kernel, dim3((unsigned)nblk), dim3(PS_NT), 0, st, G, ld, W, b, y, a->sflags,
                       gen, a->serr);
    hipLaunchKernelGGL(chol_bwd_persist_kernel, dim3((unsigned)nblk), dim3(PS_NT), 0, st, G, ld, W, y, b,
                       a->sflags + nblk, gen, a->serr, nblk);
    return hipGetLastError();
  }
  // one 128-block per outer step measured fastest for the solves (m = 16384: 4.2 ms vs 6.6 ms
  // with 8); SCS_SOLVE_OB overrides (A/B)
  static const int sob = [] {
    const char* e = getenv("SCS_SOLVE_OB");
    const int v = e ? atoi(e) : 1;
    return v < 1 ? 1 : (v > SOLVE_MAXB ? SOLVE_MAXB : v);
  }();
  const int OB = sob;
  for (int i0 = 0; i0 < nblk; i0 += OB) {
    const int i1 = i0 + OB < nblk ? i0 + OB : nblk;
    hipLaunchKernelGGL(chol_fwd_inner_kernel, dim3(1), dim3(SOLVE_NT), 0, st, G, ld, W, i0, i1, b, y);
    const int64_t nc = (int64_t)(nblk - i1) * CB;
    if (nc > 0)
      hipLaunchKernelGGL(chol_fwd_update_kernel, dim3((unsigned)ceil_div(nc, 4)), dim3(256), 0, st, G, ld,
                         (int64_t)i0 * CB, (int64_t)i1 * CB, y, (int64_t)i1 * CB, nc, b);
  }
  // backward: outer blocks in descending order; the x of block [i0, i1) goes to b
  return chol_back_blocks_ob(G, ld, nblk, W, y, b, OB, st);
}

hipError_t chol_back_blocks(const double* U, int64_t ld, int64_t mpad, const double* W, double* y, double* x,
                            hipStream_t st) {
  return chol_back_blocks_ob(U, ld, (int)(mpad / CB), W, y, x, 1, st);
}

}  // namespace scs
