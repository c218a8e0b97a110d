// Blocked LU with partial pivoting (GEPP), in place, ROW-major, for the systems the
// reference solves with a general factorization:
//   * `(H + λ·Diagonal(Hr)) \ ∇q` (prox-N-SCORE.jl:70, Julia `\` on a dense Matrix = LAPACK
//     getrf/getrs) when the hand-written Cholesky (chol.hip) meets a non-positive pivot --
//     the indefinite Q of a cross-entropy GGN on ±1 labels (test/test_algs.jl:10) and the
//     NSCORE box QP;
//   * the GGN sample-space system `qr(I + Q'(Jt'H⁻¹)Jt) \ [r; 1]` (prox-GGN-SCORE.jl:124-127),
//     non-symmetric, (N+1) x (N+1).
// Pivots follow LAPACK getf2: the first row of maximal |a| in the column; a zero pivot
// is recorded (info, 1-based) and its column is neither swapped nor scaled.
//
// Why row-major: a row interchange then moves contiguous bytes, the panel rows are 1 KiB
// contiguous pieces (the panel is factored in place, no copy), and the L21 rows are
// directly the "contiguous K" operand of the MFMA Gram kernels (gram.hip):
//   panel      128 launches of lu_panel_step_kernel (one per column: the argmax of the
//              column needs every row of the panel, so each column step is one grid-wide
//              hand-off -- a kernel boundary here, cheaper than an in-launch grid barrier,
//              MI355X_MICROARCH.md "boundary" vs "barrier-xcd");
//   swaps      the block's 128 interchanges composed into <= 256 (dst, src) row moves
//              (lu_perm_kernel) and applied to the columns right of the panel in one pass;
//   inverses   L11⁻¹ (unit lower) and U11⁻¹ of the diagonal block (lu_diag_inv_kernel);
//   TRSM       U12 = L11⁻¹ A12 = Gram(L11⁻¹ rows, A12ᵀ) on MFMA (A12ᵀ staged by a transpose);
//   update     A22 -= L21 U12 = Gram(L21 rows, U12ᵀ, w = -1), accumulate, row-major store.
// The column interchanges of later blocks are NOT applied to the L columns of earlier
// blocks; lu_solve applies each block's interchanges to b just before that block's
// forward step (the order getrf's left swaps would have produced).
//
// Layout: A is npad x npad, row stride ld >= npad, npad % 128 == 0.  Rows/columns
// [n, npad) must be zero on entry; lu_factor puts ones on their diagonal (block-diag(A, I)).
#include <climits>
#include <utility>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace scs {

constexpr int LB = 128;           // block / panel width
constexpr int LU_MAXWG = 256;     // workgroups of a panel step at most
constexpr int LU_NT = 256;        // panel step: 32 rows x 8 lanes (16 columns each) per pass
constexpr int LU_MAXPAIRS = 2 * LB;
constexpr int LU_OB = 4;          // panels per outer block (SCS_LU_OB)
constexpr int LU_LCTR = 256;      // counter sets of the lookahead bulk's bounded launches (per factorization)

__device__ __forceinline__ bool lu_better(double v1, int i1, double v2, int i2) {
  return v1 > v2 || (v1 == v2 && i1 < i2);
}

// One DPP combine step of the wave argmax below: every lane takes the better of its (v, i, w) and the one
// CTRL moves to it (lanes without a source, or outside ROWMASK, compare with themselves).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void lu_dpp_step(double& v, int& i, int& w) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const int lo = (int)(unsigned)u, hi = (int)(unsigned)(u >> 32);
  const int lo2 = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROWMASK, 0xF, false);
  const int hi2 = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROWMASK, 0xF, false);
  const int i2 = __builtin_amdgcn_update_dpp(i, i, CTRL, ROWMASK, 0xF, false);
  const int w2 = __builtin_amdgcn_update_dpp(w, w, CTRL, ROWMASK, 0xF, false);
  const double v2 = __longlong_as_double((long long)(((unsigned long long)(unsigned)hi2 << 32) | (unsigned)lo2));
  if (lu_better(v2, i2, v, i)) {
    v = v2;
    i = i2;
    w = w2;
  }
}

// (v, i, w) argmax over the wave (larger v, then smaller i) by DPP -- the quad swaps, the half-row and
// row mirrors, the row-15 / row-31 broadcasts leave the wave's best in lane 63, read back into every lane
// (r05; was six ds_bpermute rounds).  The rule is associative and commutative and the rows are distinct,
// so the result is the same as any reduction order's.
__device__ __forceinline__ void lu_wave_argmax(double& v, int& i, int& w) {
  lu_dpp_step<0xB1, 0xF>(v, i, w);    // quad_perm [1, 0, 3, 2]
  lu_dpp_step<0x4E, 0xF>(v, i, w);    // quad_perm [2, 3, 0, 1]
  lu_dpp_step<0x141, 0xF>(v, i, w);   // row_half_mirror
  lu_dpp_step<0x140, 0xF>(v, i, w);   // row_mirror
  lu_dpp_step<0x142, 0xA>(v, i, w);   // row_bcast:15 into rows 1, 3
  lu_dpp_step<0x143, 0xC>(v, i, w);   // row_bcast:31 into rows 2, 3
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)u, 63), hi = __builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 63);
  v = __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
  i = __builtin_amdgcn_readlane(i, 63);
  w = __builtin_amdgcn_readlane(w, 63);
}

// (v, i) argmax over the workgroup (larger |a|, then smaller row); every thread gets the result.
// sv / si hold NT / 64 entries.
template <int NT = LU_NT>
__device__ __forceinline__ void lu_block_argmax(double& v, int& i, int& w, double* sv, int* si, int* sw) {
  lu_wave_argmax(v, i, w);
  const int wv = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    sv[wv] = v;
    si[wv] = i;
    sw[wv] = w;
  }
  __syncthreads();
  v = sv[0];
  i = si[0];
  w = sw[0];
#pragma unroll
  for (int k = 1; k < NT / 64; ++k)
    if (lu_better(sv[k], si[k], v, i)) {
      v = sv[k];
      i = si[k];
      w = sw[k];
    }
}

template <int NV>
__device__ __forceinline__ double sel(const double (&v)[NV], int k) {
  double r = 0.0;
#pragma unroll
  for (int t = 0; t < NV; ++t) r = (t == k) ? v[t] : r;
  return r;
}

// One column step j of the panel (columns c0 .. c0+127, rows r0 .. r0+h-1 = local 0 .. h-1).
// Workgroup g owns local rows [g·R, g·R + R).
//   1. pivot: the best of the per-workgroup candidates of column j (written by step j-1 into
//      slot j&1): row p, pivot row u = that candidate's full panel row (a copy: no race with
//      this launch's stores);
//   2. row j <- u, row p <- the previous row j (rowj copy), every row i > j:
//      l = a_ij / u_j (column j <- l), a_ic -= l·u_c for c > j;
//   3. candidates of column j+1 over this workgroup's rows > j (post-update) -> slot (j+1)&1,
//      with the row's full copy; the owner of row j+1 also copies it to rowj.
// j = -1: only step 3 for column 0.
__global__ __launch_bounds__(LU_NT) void lu_panel_step_kernel(double* A, int64_t ld, int64_t r0, int64_t c0,
                                                              int64_t h, int R, int j, double* cand, int* candi,
                                                              double* candrow, double* rowj, int* ipiv, int* info) {
  __shared__ double sv[LU_NT / 64];
  __shared__ int si[LU_NT / 64], sw[LU_NT / 64];
  const int tid = threadIdx.x, g = blockIdx.x, nwg = gridDim.x;
  const int q = tid & 7, rr = tid >> 3, cq = 16 * q;
  const int par = j & 1, npar = (j + 1) & 1;
  int p = j;
  double piv = 0.0, rp = 0.0;
  bool scale = false;
  const double* urow = nullptr;
  if (j >= 0) {
    double v = -1.0;
    int i = INT_MAX, w = -1;
    if (tid < nwg) {
      v = cand[par * LU_MAXWG + tid];
      i = candi[par * LU_MAXWG + tid];
      w = tid;
      if (!(v >= 0.0)) {   // no candidate (or NaN): never wins
        v = -1.0;
        i = INT_MAX;
      }
    }
    lu_block_argmax(v, i, w, sv, si, sw);
    if (v < 0.0) {   // no valid candidate anywhere (NaN column): keep row j
      p = j;
      urow = rowj + par * LB;
    } else {
      p = i;
      urow = candrow + ((int64_t)par * LU_MAXWG + w) * LB;
    }
    piv = urow[j];
    scale = (piv != 0.0);
    if (!scale) {   // getf2: zero pivot -> no interchange, no scaling (the column below is zero)
      p = j;
      urow = rowj + par * LB;
      piv = urow[j];
    }
    rp = 1.0 / piv;
    if (g == 0 && tid == 0) {
      ipiv[r0 + j] = (int)(r0 + p);
      if (!scale && *info == 0) *info = (int)(r0 + j + 1);
    }
  }
  const int jn = j + 1;
  double u[16];
  const bool need_u = (j >= 0) && (cq + 15 > j);
  if (need_u) {
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(u + c) = *(const v2d*)(urow + cq + c);
  }
  double bv = -1.0;
  int bi = INT_MAX;
  const int npass = R / 32;
  for (int pass = 0; pass < npass; ++pass) {
    const int64_t i = (int64_t)g * R + pass * 32 + rr;
    if (i >= h || i < j) continue;
    double* row = A + (r0 + i) * ld + c0;
    if (j < 0) {   // column-0 candidates
      if (q == 0) {
        const double a = fabs(row[0]);
        if (lu_better(a, (int)i, bv, bi)) {
          bv = a;
          bi = (int)i;
        }
      }
      continue;
    }
    const bool top = (i == j) && (p != j);
    const bool bot = (i == p) && (p != j);
    if (i == j) {   // the pivot row: U(j, :) = u
      if (top) {
#pragma unroll
        for (int c = 0; c < 16; c += 2) *(v2d*)(row + cq + c) = *(const v2d*)(urow + cq + c);
      }
      continue;
    }
    const double* src = bot ? (rowj + par * LB) : row;
    if (!(bot || cq + 15 >= j)) continue;   // columns < j of an unmoved row are final
    double v[16];
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(v + c) = *(const v2d*)(src + cq + c);
    const double x = src[j];
    const double l = scale ? (fabs(piv) >= 2.2250738585072014e-308 ? x * rp : x / piv) : x;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int col = cq + c;
      if (col > j) v[c] -= l * u[c];
      else if (col == j) v[c] = l;
    }
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(row + cq + c) = *(const v2d*)(v + c);
    if (jn < LB && q == (jn >> 4)) {
      const double a = fabs(sel(v, jn & 15));
      if (lu_better(a, (int)i, bv, bi)) {
        bv = a;
        bi = (int)i;
      }
    }
  }
  if (jn >= LB) return;
  int bw = g;
  lu_block_argmax(bv, bi, bw, sv, si, sw);   // (its __syncthreads also orders this workgroup's row stores)
  if (tid == 0) {
    cand[npar * LU_MAXWG + g] = (bi == INT_MAX) ? -1.0 : bv;
    candi[npar * LU_MAXWG + g] = bi;
  }
  if (bi != INT_MAX && tid < LB) candrow[((int64_t)npar * LU_MAXWG + g) * LB + tid] = A[(r0 + bi) * ld + c0 + tid];
  if ((int64_t)g * R <= jn && jn < (int64_t)g * R + R && tid < LB) rowj[npar * LB + tid] = A[(r0 + jn) * ld + c0 + tid];
}

// The same column step with one memory round trip less on each side of the pivot choice (r05; bitwise
// the same arithmetic).  The r02 kernel issued its loads in dependency order: the candidates, then (after
// the argmax) the pivot row, then its own rows, and at the end re-read the rows it had just stored to
// publish the next candidate row and row j + 1 -- four global round trips per column, 7.9 us per step at
// n = 8192 (63 % of the factor).  Here every thread loads its rows (all columns: NP passes of 32 rows x
// 8 lanes) together with the candidate reads, before the argmax, and publishes the candidate row and row
// j + 1 from its registers.  A displaced row j (the pivot's old row) is still read after the argmax.
template <int NP>
__global__ __launch_bounds__(LU_NT) void lu_panel_step2_kernel(double* A, int64_t ld, int64_t r0, int64_t c0,
                                                               int64_t h, int R, int j, double* cand, int* candi,
                                                               double* candrow, double* rowj, int* ipiv, int* info) {
  __shared__ double sv[LU_NT / 64];
  __shared__ int si[LU_NT / 64], sw[LU_NT / 64];
  const int tid = threadIdx.x, g = blockIdx.x, nwg = gridDim.x;
  const int q = tid & 7, rr = tid >> 3, cq = 16 * q;
  const int par = j & 1, npar = (j + 1) & 1;
  const int jn = j + 1;
  // 1. this thread's row pieces (rows > j; the pivot row j itself is only ever overwritten), in flight
  //    together with the candidate reads below
  // (only the lanes whose 16 columns reach column j: the others' columns of an unmoved row are final,
  // as in the r02 step -- loading them too measured slower, profiles/r05/lu_prefetch/)
  double v[NP][16];
  bool have[NP];
#pragma unroll
  for (int ps = 0; ps < NP; ++ps) {
    const int64_t i = (int64_t)g * R + ps * 32 + rr;
    have[ps] = i < h && i > j && (j < 0 || cq + 15 >= j);
    const double* row = A + (r0 + (have[ps] ? i : 0)) * ld + c0 + cq;
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(v[ps] + c) = have[ps] ? *(const v2d*)(row + c) : (v2d){0.0, 0.0};
  }
  int p = j;
  double piv = 0.0, rp = 0.0;
  bool scale = false;
  const double* urow = nullptr;
  if (j >= 0) {
    double cv = -1.0;
    int ci = INT_MAX, w = -1;
    if (tid < nwg) {
      cv = cand[par * LU_MAXWG + tid];
      ci = candi[par * LU_MAXWG + tid];
      w = tid;
      if (!(cv >= 0.0)) {
        cv = -1.0;
        ci = INT_MAX;
      }
    }
    lu_block_argmax(cv, ci, w, sv, si, sw);
    if (cv < 0.0) {
      p = j;
      urow = rowj + par * LB;
    } else {
      p = ci;
      urow = candrow + ((int64_t)par * LU_MAXWG + w) * LB;
    }
    piv = urow[j];
    scale = (piv != 0.0);
    if (!scale) {
      p = j;
      urow = rowj + par * LB;
      piv = urow[j];
    }
    rp = 1.0 / piv;
    if (g == 0 && tid == 0) {
      ipiv[r0 + j] = (int)(r0 + p);
      if (!scale && *info == 0) *info = (int)(r0 + j + 1);
    }
  }
  double u[16];
  const bool need_u = (j >= 0) && (cq + 15 > j);
  if (need_u) {
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(u + c) = *(const v2d*)(urow + cq + c);
  }
  double bv = -1.0;
  int bi = INT_MAX;
#pragma unroll
  for (int ps = 0; ps < NP; ++ps) {
    const int64_t i = (int64_t)g * R + ps * 32 + rr;
    if (i >= h || i < j) continue;
    double* row = A + (r0 + i) * ld + c0;
    if (j < 0) {   // column-0 candidates
      if (q == 0) {
        const double a = fabs(v[ps][0]);
        if (lu_better(a, (int)i, bv, bi)) {
          bv = a;
          bi = (int)i;
        }
      }
      continue;
    }
    if (i == j) {   // the pivot row: U(j, :) = u
      if (p != j) {
#pragma unroll
        for (int c = 0; c < 16; c += 2) *(v2d*)(row + cq + c) = *(const v2d*)(urow + cq + c);
      }
      continue;
    }
    const bool bot = (i == p) && (p != j);
    if (bot) {   // the displaced row j takes row p's place
#pragma unroll
      for (int c = 0; c < 16; c += 2) *(v2d*)(v[ps] + c) = *(const v2d*)(rowj + par * LB + cq + c);
      have[ps] = true;
    }
    if (!(bot || cq + 15 >= j)) continue;   // columns < j of an unmoved row are final
    const double x = bot ? rowj[par * LB + j] : __shfl(sel(v[ps], j & 15), (tid & ~7) | (j >> 4), 64);
    const double l = scale ? (fabs(piv) >= 2.2250738585072014e-308 ? x * rp : x / piv) : x;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int col = cq + c;
      if (col > j) v[ps][c] -= l * u[c];
      else if (col == j) v[ps][c] = l;
    }
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(row + cq + c) = *(const v2d*)(v[ps] + c);
    if (jn < LB && q == (jn >> 4)) {
      const double a = fabs(sel(v[ps], jn & 15));
      if (lu_better(a, (int)i, bv, bi)) {
        bv = a;
        bi = (int)i;
      }
    }
  }
  if (jn >= LB) return;
  int bw = g;
  lu_block_argmax(bv, bi, bw, sv, si, sw);
  if (tid == 0) {
    cand[npar * LU_MAXWG + g] = (bi == INT_MAX) ? -1.0 : bv;
    candi[npar * LU_MAXWG + g] = bi;
  }
  // the candidate row and row j + 1 from the registers of the 8 lanes that hold them (a lane whose
  // columns were final and not loaded copies them from the row itself)
#pragma unroll
  for (int ps = 0; ps < NP; ++ps) {
    const int64_t i = (int64_t)g * R + ps * 32 + rr;
    if (i >= h || i < jn || (i != bi && i != jn)) continue;
    if (!have[ps]) {
      const double* row = A + (r0 + i) * ld + c0 + cq;
#pragma unroll
      for (int c = 0; c < 16; c += 2) *(v2d*)(v[ps] + c) = *(const v2d*)(row + c);
    }
    if (i == bi) {
#pragma unroll
      for (int c = 0; c < 16; c += 2)
        *(v2d*)(candrow + ((int64_t)npar * LU_MAXWG + g) * LB + cq + c) = *(const v2d*)(v[ps] + c);
    }
    if (i == jn) {
#pragma unroll
      for (int c = 0; c < 16; c += 2) *(v2d*)(rowj + npar * LB + cq + c) = *(const v2d*)(v[ps] + c);
    }
  }
}

// ---- the cooperative panel (r05) ---------------------------------------------------------------------
// The whole 128-column panel as ONE launch of G = h / 128 workgroups (one per CU and all resident: G <=
// 128, h <= 16384), each holding its 128 rows in registers through the 128 column steps (4 passes x 32
// rows x 8 lanes of 16 columns, the step kernels' layout).  The per-column grid-wide hand-off is the
// candidate exchange itself, as data-tagged 8-byte granules {tag, 32-bit word} (MI355X_MICROARCH.md
// § visibility: R2, one sc1 store each, no flag and no ordering; tag = panel·256 + column + 1, unique in
// the factorization, the granules zeroed once per factorization):
//   * each workgroup publishes its candidate of the next column -- |a| and its row, three granules --
//     and the candidate's whole panel row (two granules per double), and the owner of row j + 1 that
//     row (the one a pivot displaces), straight after its argmax (no drain, no barrier);
//   * every wave sweeps all G candidate triples (relaxed sc1 loads, bounded spin) until every tag is
//     the column's, takes the pivot by the step kernels' rule (larger |a|, then the smaller row), then
//     reads its 16 columns of the pivot row (and, at the pivot's old position, of the displaced row)
//     as granules, re-reading until their tags are the column's.
// Two slots by column parity: a workgroup publishes column j + 2 only after every workgroup has
// published column j + 1, i.e. after all have read column j.  The arithmetic per element is the step
// kernels' (l = x·(1/u_j), or x / u_j below DBL_MIN; a_ic -= l·u_c): the same factor and pivots bit for
// bit; the rows go back to A once, after the last column.  A sweep past its bound (a workgroup that
// never became resident) stores info = -1 and the abort word, and every later panel leaves at once.
constexpr int LUC_MAXWG = 128;                // workgroups (= CUs) at most
constexpr int LUC_LDS = 96 * 1024;            // dynamic LDS that keeps a second workgroup off the CU
constexpr unsigned LUC_SPIN_MAX = 1u << 19;   // sweeps before giving up (~0.5 s; SCS_LU_COOP_SPIN overrides)
// granule words (u64): candidates [2][MAXWG][4] | abort word (+pad) | candidate rows [2][MAXWG][128][2]
// | row j + 1 [2][128][2]
constexpr int64_t LUC_CAND = 0, LUC_ABORT = 2 * LUC_MAXWG * 4, LUC_CROW = LUC_ABORT + 16;
constexpr int64_t LUC_ROWJ = LUC_CROW + 2 * LUC_MAXWG * LB * 2, LUC_WORDS = LUC_ROWJ + 2 * LB * 2;
typedef __attribute__((address_space(1))) unsigned long long luc_gu64;

#ifdef LU_PROF
// probe_lu -DLU_PROF: workgroup 0's thread 0 splits each column of every cooperative panel into
// sweep | pick + stage | barrier | update | publish (s_memrealtime, 100 MHz ticks, summed) + columns
__device__ unsigned long long lu_prof[8];
#define LUP_MARK(v) const long long v = (g == 0 && tid == 0) ? (long long)__builtin_amdgcn_s_memrealtime() : 0
#define LUP_SET(v) v = (g == 0 && tid == 0) ? (long long)__builtin_amdgcn_s_memrealtime() : 0
#else
#define LUP_MARK(v)
#define LUP_SET(v)
#endif

__device__ __forceinline__ void luc_put(unsigned long long* p, unsigned long long x) {
  __hip_atomic_store((luc_gu64*)p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long luc_get(const unsigned long long* p) {
  return __hip_atomic_load((luc_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a double as two granules {tag, low word}, {tag, high word}
__device__ __forceinline__ void luc_put_d(unsigned long long* p, unsigned tag, double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v), t = (unsigned long long)tag << 32;
  luc_put(p, t | (b & 0xffffffffull));
  luc_put(p + 1, t | (b >> 32));
}
__device__ __forceinline__ double luc_get_d(const unsigned long long* p, unsigned tag, bool& ok) {
  const unsigned long long x0 = luc_get(p), x1 = luc_get(p + 1);
  ok = ok && (unsigned)(x0 >> 32) == tag && (unsigned)(x1 >> 32) == tag;
  return __longlong_as_double((long long)((x0 & 0xffffffffull) | (x1 << 32)));
}

// WIDE (SCS_LU_COOP_WIDE=1; measured slower at NT = 256, 84.9 vs 83.2 ms at n = 8192): the candidate row
// and row j + 1 go through LDS and are stored by a whole wave each (4 granules per lane instead of 32 per
// holding lane), before the candidate's own granules
// NT: threads per workgroup -- 256 (128 rows, up to 128 workgroups) or 512 (256 rows, up to 64 workgroups:
// half the grid to sweep and to wait for, two waves per SIMD)
// EARLY (r06, default; SCS_LU_COOP_EARLY=0 off; !WIDE only): each column step updates column j + 1 of
// its rows first, publishes the column's candidate RECORD, then updates the other columns and
// publishes the rows -- so the records every workgroup's sweep waits for leave ~1 update earlier,
// and the rows (fetched after the sweep, or prefetched) land while the sweep runs.  Every element
// takes the same operations: the same factor and pivots bit for bit.
template <bool WIDE, int NT, bool EARLY = false>
__global__ __launch_bounds__(NT) void lu_panel_coop_kernel(double* __restrict__ A, int64_t ld, int64_t r0,
                                                              int64_t c0, int64_t h, unsigned long long* gran,
                                                              unsigned tagbase,
                                                              int* ipiv, int* info, int2* pairs, int* npairs,
                                                              int pf_on, unsigned spin_max) {
  constexpr int RW = NT / 2, RP = NT / 8;   // rows per workgroup, rows per pass
  __shared__ double sv[NT / 64];
  __shared__ int si[NT / 64], sw[NT / 64];
  __shared__ double su_u[LB], su_rj[LB];   // the pivot row, the displaced row j (staged by wave 0)
  __shared__ double su_c[LB], su_n[LB];    // WIDE: this workgroup's candidate row and row j + 1 to publish
  __shared__ int s_p, s_alive;
  __shared__ double ev[2][NT / 64];   // EARLY: the wave argmax partials by column parity
  __shared__ int ei[2][NT / 64];
  // workgroup 0: the block's interchanges composed into row moves as the pivots come (lu_perm_kernel's
  // bookkeeping, one swap per column behind the column's publication): rows r0 .. r0+127, and the
  // touched rows below the block as (row, content)
  __shared__ int ptop[LB], pbrow[LB], pbval[LB], pnb;
  const int tid = threadIdx.x, g = blockIdx.x, nwg = gridDim.x, lane = tid & 63;
  const int q = tid & 7, rr = tid >> 3, cq = 16 * q;
  const int base = g * RW + rr;   // this thread's panel position in pass ps: base + RP ps
  if (gran[LUC_ABORT] != 0) return;   // an earlier panel of this factorization gave up (info = -1)
  if (spin_max == 0) {   // (tests: SCS_LU_COOP_SPIN=0 gives up at once, as a never-resident workgroup would)
    if (threadIdx.x == 0) {
      *info = -1;
      gran[LUC_ABORT] = 1;
    }
    return;
  }
  double v[4][16];
#pragma unroll
  for (int ps = 0; ps < 4; ++ps) {
    const bool in = base + RP * ps < h;   // (NT = 512: the last workgroup may hold only 128 rows)
    const double* row = A + (r0 + (in ? base + RP * ps : 0)) * ld + c0 + cq;
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(v[ps] + c) = in ? *(const v2d*)(row + c) : (v2d){0.0, 0.0};
  }
  bool alive = true;
  auto give_up = [&]() {   // a spin past its bound: this wave leaves, later panels leave at once
    if (lane == 0) {
      *info = -1;
      gran[LUC_ABORT] = 1;
    }
    alive = false;
  };
  // this workgroup's candidate of column jn (rows >= jn) and its row, and row jn: granules
  auto publish = [&](int jn) {
    double bv = -1.0;
    int bi = INT_MAX;
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
      const int i = base + RP * ps;
      if (i >= jn && i < h && q == (jn >> 4)) {
        const double a = fabs(sel(v[ps], jn & 15));
        if (lu_better(a, i, bv, bi)) {
          bv = a;
          bi = i;
        }
      }
    }
    int bw = g;
    lu_block_argmax<NT>(bv, bi, bw, sv, si, sw);
    const int par = jn & 1;
    const unsigned tag = tagbase + (unsigned)(jn + 1);
    if (WIDE) {
      const bool hold_jn = jn >= g * RW && jn < g * RW + RW;
#pragma unroll
      for (int ps = 0; ps < 4; ++ps) {
        const int i = base + RP * ps;
        if (i == bi) {
#pragma unroll
          for (int c = 0; c < 16; ++c) su_c[cq + c] = v[ps][c];
        }
        if (i == jn) {
#pragma unroll
          for (int c = 0; c < 16; ++c) su_n[cq + c] = v[ps][c];
        }
      }
      __syncthreads();
      const int wv = tid >> 6;
      if (wv == 1 && bi != INT_MAX) {
        unsigned long long* rp = gran + LUC_CROW + ((int64_t)par * LUC_MAXWG + g) * LB * 2;
        luc_put_d(rp + 4 * lane, tag, su_c[2 * lane]);
        luc_put_d(rp + 4 * lane + 2, tag, su_c[2 * lane + 1]);
      }
      if (wv == 2 && hold_jn) {
        unsigned long long* rp = gran + LUC_ROWJ + (int64_t)par * LB * 2;
        luc_put_d(rp + 4 * lane, tag, su_n[2 * lane]);
        luc_put_d(rp + 4 * lane + 2, tag, su_n[2 * lane + 1]);
      }
      __syncthreads();   // the rows' granules issued ahead of the candidate's (the tags decide anyway)
    }
#pragma unroll
    for (int ps = 0; ps < 4 && !WIDE; ++ps) {
      const int i = base + RP * ps;
      if (i == bi) {
        unsigned long long* rp = gran + LUC_CROW + (((int64_t)par * LUC_MAXWG + g) * LB + cq) * 2;
#pragma unroll
        for (int c = 0; c < 16; ++c) luc_put_d(rp + 2 * c, tag, v[ps][c]);
      }
      if (i == jn) {
        unsigned long long* rp = gran + LUC_ROWJ + ((int64_t)par * LB + cq) * 2;
#pragma unroll
        for (int c = 0; c < 16; ++c) luc_put_d(rp + 2 * c, tag, v[ps][c]);
      }
    }
    // the record after the rows (a barrier apart): a consumer that prefetches the best row so far
    // usually finds it landed (the tags decide either way)
    if (!WIDE) __syncthreads();
    if (tid == 0) {
      const unsigned long long t = (unsigned long long)tag << 32;
      const unsigned long long bits = (unsigned long long)__double_as_longlong(bi == INT_MAX ? -1.0 : bv);
      unsigned long long* gp = gran + LUC_CAND + ((int64_t)par * LUC_MAXWG + g) * 4;
      luc_put(gp + 0, t | (bits & 0xffffffffull));
      luc_put(gp + 1, t | (bits >> 32));
      luc_put(gp + 2, t | (unsigned)bi);
    }
  };
  // EARLY: the candidate record of column jn (column jn of the rows already updated), returning the
  // workgroup's candidate row; then, after the rest of the update, its row and row jn
  auto publish_record = [&](int jn) -> int {
    double bv = -1.0;
    int bi = INT_MAX, bw_dummy = g;
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
      const int i = base + RP * ps;
      if (i >= jn && i < h && q == (jn >> 4)) {
        const double a = fabs(sel(v[ps], jn & 15));
        if (lu_better(a, i, bv, bi)) {
          bv = a;
          bi = i;
        }
      }
    }
    // the workgroup's argmax with ONE barrier: the wave partials go to a slot by column parity, last
    // read two columns ago (the column loop's barrier lies between), so no barrier before the writes
    lu_wave_argmax(bv, bi, bw_dummy);
    {
      const int wv = tid >> 6, sl = jn & 1;
      if (lane == 0) {
        ev[sl][wv] = bv;
        ei[sl][wv] = bi;
      }
      __syncthreads();
      bv = ev[sl][0];
      bi = ei[sl][0];
#pragma unroll
      for (int k = 1; k < NT / 64; ++k)
        if (lu_better(ev[sl][k], ei[sl][k], bv, bi)) {
          bv = ev[sl][k];
          bi = ei[sl][k];
        }
    }
    if (tid == 0) {
      const unsigned long long t = (unsigned long long)(tagbase + (unsigned)(jn + 1)) << 32;
      const unsigned long long bits = (unsigned long long)__double_as_longlong(bi == INT_MAX ? -1.0 : bv);
      unsigned long long* gp = gran + LUC_CAND + ((int64_t)(jn & 1) * LUC_MAXWG + g) * 4;
      luc_put(gp + 0, t | (bits & 0xffffffffull));
      luc_put(gp + 1, t | (bits >> 32));
      luc_put(gp + 2, t | (unsigned)bi);
    }
    return bi;
  };
  auto publish_rows = [&](int jn, int bi) {
    const int par = jn & 1;
    const unsigned tag = tagbase + (unsigned)(jn + 1);
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
      const int i = base + RP * ps;
      if (i == bi) {
        unsigned long long* rp = gran + LUC_CROW + (((int64_t)par * LUC_MAXWG + g) * LB + cq) * 2;
#pragma unroll
        for (int c = 0; c < 16; ++c) luc_put_d(rp + 2 * c, tag, v[ps][c]);
      }
      if (i == jn) {
        unsigned long long* rp = gran + LUC_ROWJ + ((int64_t)par * LB + cq) * 2;
#pragma unroll
        for (int c = 0; c < 16; ++c) luc_put_d(rp + 2 * c, tag, v[ps][c]);
      }
    }
  };
  if (g == 0) {
    if (tid < LB) ptop[tid] = (int)r0 + tid;
    if (tid == 0) pnb = 0;
  }
  publish(0);   // (its barriers order the initialisation above)
#ifdef LU_PROF
  long long lp_acc[5] = {0, 0, 0, 0, 0};
  long long lp_t1 = 0, lp_t2 = 0;
#endif
  for (int j = 0; j < LB; ++j) {
    const int par = j & 1;
    const unsigned tag = tagbase + (unsigned)(j + 1);
    LUP_MARK(lp_t0);
    // 1. wave 0 alone: sweep the G candidates of column j until all carry this column's tag, pick the
    //    pivot, and stage the pivot row (and the displaced row j where this workgroup holds row p) in LDS
    if (tid < 64) {
      double cv = -1.0;
      int ci = INT_MAX, cw = -1;
      const unsigned long long* gp = gran + LUC_CAND + (int64_t)par * LUC_MAXWG * 4;
      // the row of the best candidate among those already arrived, prefetched while the sweep waits for
      // the rest (lane l: granules 4l .. 4l+3 = columns 2l, 2l+1); used if that candidate wins
      int pf_w = -1;
      unsigned long long pf0 = 0, pf1 = 0, pf2 = 0, pf3 = 0;
      for (unsigned spins = 0;;) {
        bool ok = true;
        cv = -1.0;
        ci = INT_MAX;
        cw = -1;
        double bv = -2.0;   // the best arrived candidate (every lane's arrived records)
        int bi = INT_MAX, bw = -1;
#pragma unroll
        for (int t = 0; t < LUC_MAXWG / 64; ++t) {
          const int w = lane + 64 * t;
          if (w < nwg) {
            const unsigned long long x0 = luc_get(gp + 4 * w + 0), x1 = luc_get(gp + 4 * w + 1),
                                     x2 = luc_get(gp + 4 * w + 2);
            const bool okw = (unsigned)(x0 >> 32) == tag && (unsigned)(x1 >> 32) == tag && (unsigned)(x2 >> 32) == tag;
            ok = ok && okw;
            double a = __longlong_as_double((long long)((x0 & 0xffffffffull) | (x1 << 32)));
            int r = (int)(unsigned)x2;
            if (!(a >= 0.0)) {   // no candidate (or NaN): never wins
              a = -1.0;
              r = INT_MAX;
            }
            if (lu_better(a, r, cv, ci)) {
              cv = a;
              ci = r;
              cw = w;
            }
            if (okw && a >= 0.0 && lu_better(a, r, bv, bi)) {
              bv = a;
              bi = r;
              bw = w;
            }
          }
        }
        if (__all(ok)) break;
        lu_wave_argmax(bv, bi, bw);
        if (pf_on && bw >= 0 && bw != pf_w) {   // (wave-uniform)
          const unsigned long long* rp = gran + LUC_CROW + ((int64_t)par * LUC_MAXWG + bw) * LB * 2 + 4 * lane;
          pf0 = luc_get(rp);
          pf1 = luc_get(rp + 1);
          pf2 = luc_get(rp + 2);
          pf3 = luc_get(rp + 3);
          pf_w = bw;
        }
        if (++spins > spin_max) {
          give_up();
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#ifdef LU_PROF
      if (g == 0 && tid == 0) lp_t1 = (long long)__builtin_amdgcn_s_memrealtime();
#endif
      lu_wave_argmax(cv, ci, cw);
      // a row of 128 doubles as 256 granules: lane l takes columns 2l, 2l + 1
      auto stage = [&](const unsigned long long* rp, double* dst) {
        for (unsigned spins = 0; alive;) {
          bool ok = true;
          const double d0 = luc_get_d(rp + 4 * lane, tag, ok), d1 = luc_get_d(rp + 4 * lane + 2, tag, ok);
          if (__all(ok)) {
            dst[2 * lane] = d0;
            dst[2 * lane + 1] = d1;
            return;
          }
          if (++spins > spin_max) give_up();
          __builtin_amdgcn_s_sleep(1);
        }
      };
      const unsigned long long* rowj_g = gran + LUC_ROWJ + (int64_t)par * LB * 2;
      int p = ci;
      const unsigned long long* urow = gran + LUC_CROW + ((int64_t)par * LUC_MAXWG + cw) * LB * 2;
      if (cv < 0.0) {   // no valid candidate anywhere (NaN column): keep row j
        p = j;
        urow = rowj_g;
      }
      if (alive) {
        const bool hit = cv >= 0.0 && cw == pf_w &&
                         __all((unsigned)(pf0 >> 32) == tag && (unsigned)(pf1 >> 32) == tag &&
                               (unsigned)(pf2 >> 32) == tag && (unsigned)(pf3 >> 32) == tag);
        if (hit) {
          su_u[2 * lane] = __longlong_as_double((long long)((pf0 & 0xffffffffull) | (pf1 << 32)));
          su_u[2 * lane + 1] = __longlong_as_double((long long)((pf2 & 0xffffffffull) | (pf3 << 32)));
        } else {
          stage(urow, su_u);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");   // this wave's LDS writes, then its reads
      __builtin_amdgcn_wave_barrier();
      if (alive && su_u[j] == 0.0) {   // getf2: zero pivot -> no interchange, no scaling (row j's u_j
        p = j;                           // is then zero too: the column's largest |a| was)
        stage(rowj_g, su_u);
      }
      if (alive && p != j && p >= g * RW && p < g * RW + RW) stage(rowj_g, su_rj);
      if (lane == 0) {
        s_p = p;
        s_alive = alive ? 1 : 0;
      }
#ifdef LU_PROF
      if (g == 0 && tid == 0) lp_t2 = (long long)__builtin_amdgcn_s_memrealtime();
#endif
    }
    __syncthreads();
    if (!s_alive) return;   // (every wave: the abort word and info are set)
    LUP_MARK(lp_t3);
    const int p = s_p;
    double u[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) u[c] = su_u[cq + c];
    const double piv = su_u[j];
    const bool scale = (piv != 0.0);
    const double rp = 1.0 / piv;
    if (g == 0 && tid == 0) {
      ipiv[r0 + j] = (int)(r0 + p);
      if (!scale && *info == 0) *info = (int)(r0 + j + 1);
    }
    // 2. row j <- u, row p <- the displaced row j, every row i > j: l = a_ij / u_j, a_ic -= l·u_c
    //    (EARLY: column j + 1 first, its record, then the other columns)
    const int jn = j + 1;
    double lv[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
      const int i = base + RP * ps;
      if (i < j || i >= h) continue;
      if (i == j) {
        if (p != j) {
#pragma unroll
          for (int c = 0; c < 16; ++c) v[ps][c] = u[c];
        }
        continue;
      }
      if (i == p) {   // (p != j here)
#pragma unroll
        for (int c = 0; c < 16; ++c) v[ps][c] = su_rj[cq + c];
      }
      const double x = __shfl(sel(v[ps], j & 15), (tid & ~7) | (j >> 4), 64);
      const double l = scale ? (fabs(piv) >= 2.2250738585072014e-308 ? x * rp : x / piv) : x;
      lv[ps] = l;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int col = cq + c;
        if (EARLY) {
          if (col == jn) v[ps][c] -= l * u[c];
          else if (col == j) v[ps][c] = l;
        } else {
          if (col > j) v[ps][c] -= l * u[c];
          else if (col == j) v[ps][c] = l;
        }
      }
    }
#ifdef LU_PROF
    long long lp_t4 = 0;
#endif
    if constexpr (EARLY) {
      const int bi = jn < LB ? publish_record(jn) : INT_MAX;
      // the rest of the update -- first the two rows the next column's consumers fetch (the candidate row
      // bi and row jn), published at once, then the others
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int ps = 0; ps < 4; ++ps) {
          const int i = base + RP * ps;
          if (i <= j || i >= h || ((i == bi || i == jn) != (pass == 0))) continue;
#pragma unroll
          for (int c = 0; c < 16; ++c) {
            const int col = cq + c;
            if (col > j && col != jn) v[ps][c] -= lv[ps] * u[c];
          }
        }
        if (pass == 0 && jn < LB) publish_rows(jn, bi);
      }
      LUP_SET(lp_t4);
    } else {
      LUP_SET(lp_t4);
      if (j + 1 < LB) publish(j + 1);
    }
#ifdef LU_PROF
    if (g == 0 && tid == 0) {
      const long long t5 = (long long)__builtin_amdgcn_s_memrealtime();
      lp_acc[0] += lp_t1 - lp_t0;
      lp_acc[1] += lp_t2 - lp_t1;
      lp_acc[2] += lp_t3 - lp_t2;
      lp_acc[3] += lp_t4 - lp_t3;
      lp_acc[4] += t5 - lp_t4;
    }
#endif
    if (g == 0 && tid < 64 && p != j) {   // compose interchange j (rows r0+j <-> r0+p)
      if (p < LB) {
        if (lane == 0) {
          const int t = ptop[j];
          ptop[j] = ptop[p];
          ptop[p] = t;
        }
      } else {
        const int pr = (int)r0 + p;
        int slot = -1;
        for (int b = lane; b < pnb; b += 64)
          if (pbrow[b] == pr) slot = b;
        const unsigned long long hit = __ballot(slot >= 0);   // rows are unique in the list
        const int found = hit ? __shfl(slot, __ffsll((long long)hit) - 1, 64) : -1;
        if (lane == 0) {
          int sl = found;
          if (sl < 0) {
            sl = pnb;
            pbrow[sl] = pr;
            pbval[sl] = pr;
            pnb = sl + 1;
          }
          const int t = ptop[j];
          ptop[j] = pbval[sl];
          pbval[sl] = t;
        }
      }
    }
  }
#ifdef LU_PROF
  if (g == 0 && tid == 0) {
    for (int q = 0; q < 5; ++q) atomicAdd(&lu_prof[q], (unsigned long long)lp_acc[q]);
    atomicAdd(&lu_prof[5], (unsigned long long)LB);
  }
#endif
  if (g == 0 && tid < 64) {   // the moves: top rows (ascending), then the rows below (list order)
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int n = 0;
    for (int t0 = 0; t0 < LB; t0 += 64) {
      const int t = t0 + lane;
      const bool mv = ptop[t] != (int)r0 + t;
      const unsigned long long bm = __ballot(mv);
      if (mv) pairs[n + __popcll(bm & ((1ull << lane) - 1))] = make_int2((int)r0 + t, ptop[t]);
      n += __popcll(bm);
    }
    for (int b0 = 0; b0 < pnb; b0 += 64) {
      const int b = b0 + lane;
      const bool mv = b < pnb && pbval[b] != pbrow[b];
      const unsigned long long bm = __ballot(mv);
      if (mv) pairs[n + __popcll(bm & ((1ull << lane) - 1))] = make_int2(pbrow[b], pbval[b]);
      n += __popcll(bm);
    }
    if (lane == 0) *npairs = n;
  }
#pragma unroll
  for (int ps = 0; ps < 4; ++ps) {
    if (base + RP * ps >= h) continue;
    double* row = A + (r0 + base + RP * ps) * ld + c0 + cq;
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(row + c) = *(const v2d*)(v[ps] + c);
  }
}

// ---- the cooperative panel, block-deferred (r06; SCS_LU_COOP_BLK) -------------------------------------
// The exchange, records, rows and interchanges of lu_panel_coop_kernel, but a column step j updates only
// the columns of its 16-column block b = j / 16 right of j -- held, for each row, by ONE lane (q = b),
// whose multiplier l = a_ij / u_j it forms itself (no shuffle) at compile-time register indices (the
// block's 16 steps are unrolled).  The columns right of the block take the block's 16 rank-1 updates at
// its end, in step order (what the column steps would have done to them, delayed):
//   * the pivot rows as staged (sU) carry the block's columns current and the columns right of it as
//     they stood at the block's start; their final values there are the 16-row unit-lower solve
//     u_kc -= l_kk'·u_k'c (k' < k, ascending), formed by every workgroup from sU itself (no exchange);
//   * a row at position i then takes a_ic -= l_ik·u_kc for the steps k < i of the block, ascending
//     (the rows above the block: none; the block's pivot rows: those before them; all others: 16).
// Every element sees the column steps' operations (x - l·u, contracted alike) in the same order: the
// factor and pivots bit for bit (test_lu_panel_variants_bit_identical).  A row published for the next
// column (its candidate, or row j + 1) is current in the block and stale right of it, which is what the
// consumers' own deferred updates expect.  The column step costs ~(15 - j % 16) FMAs on one lane of eight
// instead of 16 masked FMAs on all; the block's updates ~1024 FMAs per thread on the lanes right of it.
template <class F, int... I>
__device__ __forceinline__ void luc_unroll(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}

// wave 0 of a cooperative panel's workgroup, column j: sweep the G candidate records until all carry the
// column's tag (prefetching the best arrived candidate's row), pick the pivot by the step kernels' rule,
// stage its row in su and, where this workgroup holds row p, the displaced row j in srj; returns p
// (lu_panel_coop_kernel's step 1; a sweep past spin_max clears alive and sets info = -1 and the abort word)
__device__ __forceinline__ int luc_sweep_stage(unsigned long long* gran, int j, unsigned tag, int nwg, int lane,
                                               int lo, int hi, int pf_on, unsigned spin_max, int* info,
                                               bool& alive, double* su, double* srj) {
  const int par = j & 1;
  auto give_up = [&]() {
    if (lane == 0) {
      *info = -1;
      gran[LUC_ABORT] = 1;
    }
    alive = false;
  };
  double cv = -1.0;
  int ci = INT_MAX, cw = -1;
  const unsigned long long* gp = gran + LUC_CAND + (int64_t)par * LUC_MAXWG * 4;
  int pf_w = -1;
  unsigned long long pf0 = 0, pf1 = 0, pf2 = 0, pf3 = 0;
  for (unsigned spins = 0;;) {
    bool ok = true;
    cv = -1.0;
    ci = INT_MAX;
    cw = -1;
    double bv = -2.0;
    int bi = INT_MAX, bw = -1;
#pragma unroll
    for (int t = 0; t < LUC_MAXWG / 64; ++t) {
      const int w = lane + 64 * t;
      if (w < nwg) {
        const unsigned long long x0 = luc_get(gp + 4 * w + 0), x1 = luc_get(gp + 4 * w + 1),
                                 x2 = luc_get(gp + 4 * w + 2);
        const bool okw = (unsigned)(x0 >> 32) == tag && (unsigned)(x1 >> 32) == tag && (unsigned)(x2 >> 32) == tag;
        ok = ok && okw;
        double a = __longlong_as_double((long long)((x0 & 0xffffffffull) | (x1 << 32)));
        int r = (int)(unsigned)x2;
        if (!(a >= 0.0)) {
          a = -1.0;
          r = INT_MAX;
        }
        if (lu_better(a, r, cv, ci)) {
          cv = a;
          ci = r;
          cw = w;
        }
        if (okw && a >= 0.0 && lu_better(a, r, bv, bi)) {
          bv = a;
          bi = r;
          bw = w;
        }
      }
    }
    if (__all(ok)) break;
    lu_wave_argmax(bv, bi, bw);
    if (pf_on && bw >= 0 && bw != pf_w) {
      const unsigned long long* rp = gran + LUC_CROW + ((int64_t)par * LUC_MAXWG + bw) * LB * 2 + 4 * lane;
      pf0 = luc_get(rp);
      pf1 = luc_get(rp + 1);
      pf2 = luc_get(rp + 2);
      pf3 = luc_get(rp + 3);
      pf_w = bw;
    }
    if (++spins > spin_max) {
      give_up();
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  lu_wave_argmax(cv, ci, cw);
  auto stage = [&](const unsigned long long* rp, double* dst) {
    for (unsigned spins = 0; alive;) {
      bool ok = true;
      const double d0 = luc_get_d(rp + 4 * lane, tag, ok), d1 = luc_get_d(rp + 4 * lane + 2, tag, ok);
      if (__all(ok)) {
        dst[2 * lane] = d0;
        dst[2 * lane + 1] = d1;
        return;
      }
      if (++spins > spin_max) give_up();
      __builtin_amdgcn_s_sleep(1);
    }
  };
  const unsigned long long* rowj_g = gran + LUC_ROWJ + (int64_t)par * LB * 2;
  int p = ci;
  const unsigned long long* urow = gran + LUC_CROW + ((int64_t)par * LUC_MAXWG + cw) * LB * 2;
  if (cv < 0.0) {
    p = j;
    urow = rowj_g;
  }
  if (alive) {
    const bool hit = cv >= 0.0 && cw == pf_w &&
                     __all((unsigned)(pf0 >> 32) == tag && (unsigned)(pf1 >> 32) == tag &&
                           (unsigned)(pf2 >> 32) == tag && (unsigned)(pf3 >> 32) == tag);
    if (hit) {
      su[2 * lane] = __longlong_as_double((long long)((pf0 & 0xffffffffull) | (pf1 << 32)));
      su[2 * lane + 1] = __longlong_as_double((long long)((pf2 & 0xffffffffull) | (pf3 << 32)));
    } else {
      stage(urow, su);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (alive && su[j] == 0.0) {   // getf2: zero pivot -> row j, no interchange, no scaling
    p = j;
    stage(rowj_g, su);
  }
  if (alive && p != j && p >= lo && p < hi) stage(rowj_g, srj);
  return p;
}

template <int NT>
__global__ __launch_bounds__(NT) void lu_panel_blk_kernel(double* __restrict__ A, int64_t ld, int64_t r0,
                                                             int64_t c0, int64_t h, unsigned long long* gran,
                                                             unsigned tagbase, int* ipiv, int* info, int2* pairs,
                                                             int* npairs, int pf_on, unsigned spin_max) {
  constexpr int RW = NT / 2, RP = NT / 8, NBK = LB / 16;
  __shared__ double sU[16][LB];    // the block's pivot rows as staged; at its end, final right of it
  __shared__ double sL[RW][17];    // at a block's end: its multipliers of this workgroup's rows
  __shared__ double su_rj[LB];
  __shared__ double ev[2][NT / 64];
  __shared__ int ei[2][NT / 64];
  __shared__ int s_p, s_alive;
  __shared__ int ptop[LB], pbrow[LB], pbval[LB], pnb;
  const int tid = threadIdx.x, g = blockIdx.x, lane = tid & 63;
  const int q = tid & 7, rr = tid >> 3, cq = 16 * q;
  const int base = g * RW + rr;
  if (gran[LUC_ABORT] != 0) return;
  if (spin_max == 0) {
    if (threadIdx.x == 0) {
      *info = -1;
      gran[LUC_ABORT] = 1;
    }
    return;
  }
  double v[4][16];
#pragma unroll
  for (int ps = 0; ps < 4; ++ps) {
    const bool in = base + RP * ps < h;
    const double* row = A + (r0 + (in ? base + RP * ps : 0)) * ld + c0 + cq;
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(v[ps] + c) = in ? *(const v2d*)(row + c) : (v2d){0.0, 0.0};
  }
  bool alive = true;
  // the candidate record of column jn (its column K = jn % 16 on the lanes q = jn / 16), one barrier
  // (lu_panel_coop_kernel's publish_record); returns the workgroup's candidate row
  auto record = [&](int jn, auto Kc) __attribute__((always_inline)) -> int {
    constexpr int K = decltype(Kc)::value;
    double bv = -1.0;
    int bi = INT_MAX, bw_dummy = g;
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
      const int i = base + RP * ps;
      if (i >= jn && i < h && q == (jn >> 4)) {
        const double a = fabs(v[ps][K]);
        if (lu_better(a, i, bv, bi)) {
          bv = a;
          bi = i;
        }
      }
    }
    lu_wave_argmax(bv, bi, bw_dummy);
    {
      const int wv = tid >> 6, sl = jn & 1;
      if (lane == 0) {
        ev[sl][wv] = bv;
        ei[sl][wv] = bi;
      }
      __syncthreads();
      bv = ev[sl][0];
      bi = ei[sl][0];
#pragma unroll
      for (int k = 1; k < NT / 64; ++k)
        if (lu_better(ev[sl][k], ei[sl][k], bv, bi)) {
          bv = ev[sl][k];
          bi = ei[sl][k];
        }
    }
    if (tid == 0) {
      const unsigned long long t = (unsigned long long)(tagbase + (unsigned)(jn + 1)) << 32;
      const unsigned long long bits = (unsigned long long)__double_as_longlong(bi == INT_MAX ? -1.0 : bv);
      unsigned long long* gp = gran + LUC_CAND + ((int64_t)(jn & 1) * LUC_MAXWG + g) * 4;
      luc_put(gp + 0, t | (bits & 0xffffffffull));
      luc_put(gp + 1, t | (bits >> 32));
      luc_put(gp + 2, t | (unsigned)bi);
    }
    return bi;
  };
  auto publish_rows = [&](int jn, int bi) __attribute__((always_inline)) {
    const int par = jn & 1;
    const unsigned tag = tagbase + (unsigned)(jn + 1);
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
      const int i = base + RP * ps;
      if (i == bi) {
        unsigned long long* rp = gran + LUC_CROW + (((int64_t)par * LUC_MAXWG + g) * LB + cq) * 2;
#pragma unroll
        for (int c = 0; c < 16; ++c) luc_put_d(rp + 2 * c, tag, v[ps][c]);
      }
      if (i == jn) {
        unsigned long long* rp = gran + LUC_ROWJ + ((int64_t)par * LB + cq) * 2;
#pragma unroll
        for (int c = 0; c < 16; ++c) luc_put_d(rp + 2 * c, tag, v[ps][c]);
      }
    }
  };
  if (g == 0) {
    if (tid < LB) ptop[tid] = (int)r0 + tid;
    if (tid == 0) pnb = 0;
  }
  publish_rows(0, record(0, std::integral_constant<int, 0>{}));   // (its barrier orders the initialisation)
  bool dead = false;
  for (int b = 0; b < NBK; ++b) {
    luc_unroll(
        [&](auto JJc) __attribute__((always_inline)) {
          constexpr int jj = decltype(JJc)::value;
          if (dead) return;
          const int j = 16 * b + jj;
          const unsigned tag = tagbase + (unsigned)(j + 1);
          if (tid < 64) {
            const int p = luc_sweep_stage(gran, j, tag, (int)gridDim.x, lane, g * RW, g * RW + RW, pf_on, spin_max,
                                          info, alive, sU[jj], su_rj);
            if (lane == 0) {
              s_p = p;
              s_alive = alive ? 1 : 0;
            }
          }
          __syncthreads();
          if (!s_alive) {   // (every wave: the abort word and info are set)
            dead = true;
            return;
          }
          const int p = s_p;
          const double piv = sU[jj][j];
          const bool scale = (piv != 0.0);
          const double rp = 1.0 / piv;
          if (g == 0 && tid == 0) {
            ipiv[r0 + j] = (int)(r0 + p);
            if (!scale && *info == 0) *info = (int)(r0 + j + 1);
          }
          const bool mine = q == b;   // this lane holds the block's columns of its rows
          double u[16];
#pragma unroll
          for (int c = jj + 1; c < 16; ++c) u[c] = sU[jj][16 * b + c];
#pragma unroll
          for (int ps = 0; ps < 4; ++ps) {
            const int i = base + RP * ps;
            if (i < j || i >= h) continue;
            if (i == j) {
              if (p != j) {
#pragma unroll
                for (int c = 0; c < 16; ++c) v[ps][c] = sU[jj][cq + c];
              }
              continue;
            }
            if (i == p) {
#pragma unroll
              for (int c = 0; c < 16; ++c) v[ps][c] = su_rj[cq + c];
            }
            if (mine) {
              const double x = v[ps][jj];
              const double l = scale ? (fabs(piv) >= 2.2250738585072014e-308 ? x * rp : x / piv) : x;
              v[ps][jj] = l;
#pragma unroll
              for (int c = jj + 1; c < 16; ++c) v[ps][c] -= l * u[c];
            }
          }
          if constexpr (jj == 15) {
            if (b + 1 < NBK) {   // the block's 16 updates of the columns right of it
              if (mine) {
#pragma unroll
                for (int ps = 0; ps < 4; ++ps)
#pragma unroll
                  for (int k = 0; k < 16; ++k) sL[rr + RP * ps][k] = v[ps][k];
              }
              if (tid >= 16 * (b + 1) && tid < LB) {   // the pivot rows' final values right of the block
                double col[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) col[k] = sU[k][tid];
#pragma unroll
                for (int k = 1; k < 16; ++k)
#pragma unroll
                  for (int kk = 0; kk < k; ++kk) col[k] -= sU[k][16 * b + kk] * col[kk];
#pragma unroll
                for (int k = 1; k < 16; ++k) sU[k][tid] = col[k];
              }
              __syncthreads();
              if (q > b) {
#pragma unroll 2
                for (int k = 0; k < 16; ++k) {
                  double uk[16];
#pragma unroll
                  for (int c = 0; c < 16; ++c) uk[c] = sU[k][cq + c];
#pragma unroll
                  for (int ps = 0; ps < 4; ++ps) {
                    const int i = base + RP * ps;
                    if (i > 16 * b + k && i < h) {
                      const double lk = sL[rr + RP * ps][k];
#pragma unroll
                      for (int c = 0; c < 16; ++c) v[ps][c] -= lk * uk[c];
                    }
                  }
                }
              }
            }
          }
          const int jn = j + 1;
          if (jn < LB) publish_rows(jn, record(jn, std::integral_constant<int, (jj + 1) & 15>{}));
          if (g == 0 && tid < 64 && p != j) {   // compose interchange j (rows r0+j <-> r0+p)
            if (p < LB) {
              if (lane == 0) {
                const int t = ptop[j];
                ptop[j] = ptop[p];
                ptop[p] = t;
              }
            } else {
              const int pr = (int)r0 + p;
              int slot = -1;
              for (int bb = lane; bb < pnb; bb += 64)
                if (pbrow[bb] == pr) slot = bb;
              const unsigned long long hit = __ballot(slot >= 0);
              const int found = hit ? __shfl(slot, __ffsll((long long)hit) - 1, 64) : -1;
              if (lane == 0) {
                int sl = found;
                if (sl < 0) {
                  sl = pnb;
                  pbrow[sl] = pr;
                  pbval[sl] = pr;
                  pnb = sl + 1;
                }
                const int t = ptop[j];
                ptop[j] = pbval[sl];
                pbval[sl] = t;
              }
            }
          }
        },
        std::make_integer_sequence<int, 16>{});
    if (dead) return;
  }
  if (g == 0 && tid < 64) {   // the moves (lu_panel_coop_kernel's)
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int n = 0;
    for (int t0 = 0; t0 < LB; t0 += 64) {
      const int t = t0 + lane;
      const bool mv = ptop[t] != (int)r0 + t;
      const unsigned long long bm = __ballot(mv);
      if (mv) pairs[n + __popcll(bm & ((1ull << lane) - 1))] = make_int2((int)r0 + t, ptop[t]);
      n += __popcll(bm);
    }
    for (int b0 = 0; b0 < pnb; b0 += 64) {
      const int bb = b0 + lane;
      const bool mv = bb < pnb && pbval[bb] != pbrow[bb];
      const unsigned long long bm = __ballot(mv);
      if (mv) pairs[n + __popcll(bm & ((1ull << lane) - 1))] = make_int2(pbrow[bb], pbval[bb]);
      n += __popcll(bm);
    }
    if (lane == 0) *npairs = n;
  }
#pragma unroll
  for (int ps = 0; ps < 4; ++ps) {
    if (base + RP * ps >= h) continue;
    double* row = A + (r0 + base + RP * ps) * ld + c0 + cq;
#pragma unroll
    for (int c = 0; c < 16; c += 2) *(v2d*)(row + c) = *(const v2d*)(v[ps] + c);
  }
}

// Compose block k's 128 interchanges (rows r0+s <-> ipiv[r0+s], in order) into row moves
// "row dst <- previous row src" (<= 256 of them).  One wave.
__global__ __launch_bounds__(64) void lu_perm_kernel(const int* __restrict__ ipiv, int r0, int2* __restrict__ pairs,
                                                     int* __restrict__ npairs) {
  __shared__ int top[LB];         // content of rows r0 .. r0+127
  __shared__ int brow[LB], bval[LB];   // touched rows below the block: (row, content)
  __shared__ int nb;
  __shared__ int sp[LB];   // the block's pivots, loaded once (r02 read one per step: 64 us per launch)
  const int lane = threadIdx.x;
  for (int t = lane; t < LB; t += 64) {
    top[t] = r0 + t;
    sp[t] = ipiv[r0 + t];
  }
  if (lane == 0) nb = 0;
  __syncthreads();
  for (int s = 0; s < LB; ++s) {
    const int pr = sp[s];
    if (pr == r0 + s) continue;
    if (pr < r0 + LB) {
      if (lane == 0) {
        const int t = top[s];
        top[s] = top[pr - r0];
        top[pr - r0] = t;
      }
    } else {
      int slot = -1;
      for (int b = lane; b < nb; b += 64)
        if (brow[b] == pr) slot = b;
      // rows are unique in the list: at most one lane matches
      const unsigned long long hit = __ballot(slot >= 0);
      const int found = hit ? __shfl(slot, __ffsll((long long)hit) - 1, 64) : -1;
      if (lane == 0) {
        int sl;
        if (found >= 0) {
          sl = found;
        } else {
          sl = nb;
          brow[sl] = pr;
          bval[sl] = pr;
          nb = nb + 1;
        }
        const int t = top[s];
        top[s] = bval[sl];
        bval[sl] = t;
      }
    }
    __syncthreads();
  }
  if (lane == 0) {
    int n = 0;
    for (int t = 0; t < LB; ++t)
      if (top[t] != r0 + t) pairs[n++] = make_int2(r0 + t, top[t]);
    for (int b = 0; b < nb; ++b)
      if (bval[b] != brow[b]) pairs[n++] = make_int2(brow[b], bval[b]);
    *npairs = n;
  }
}

// Apply the row moves to columns [c_lo, c_lo + w): all sources read before any store.
constexpr int SW_COLS = 64;
__global__ __launch_bounds__(256) void lu_swap_cols_kernel(double* A, int64_t ld, int64_t c_lo, int64_t w,
                                                           const int2* __restrict__ pairs,
                                                           const int* __restrict__ npairs) {
  __shared__ double buf[LU_MAXPAIRS * SW_COLS];
  __shared__ int2 sp[LU_MAXPAIRS];
  const int np = *npairs;
  if (np == 0) return;
  // the moves to LDS first, then the row loads eight at a time in flight (r02 chained a pairs[] load in
  // front of every row load: 52 us per launch)
  for (int k = threadIdx.x; k < np; k += 256) sp[k] = pairs[k];
  __syncthreads();
  const int col = threadIdx.x & (SW_COLS - 1), kg = threadIdx.x / SW_COLS;
  const int64_t c = c_lo + (int64_t)blockIdx.x * SW_COLS + col;
  const bool ok = (int64_t)blockIdx.x * SW_COLS + col < w;
  constexpr int KS = 256 / SW_COLS;
  if (ok) {
    for (int k0 = kg; k0 < np; k0 += 8 * KS) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * KS;
        v[u] = (k < np) ? A[(int64_t)sp[k].y * ld + c] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * KS;
        if (k < np) buf[k * SW_COLS + col] = v[u];
      }
    }
  }
  __syncthreads();
  if (ok)
    for (int k = kg; k < np; k += KS) A[(int64_t)sp[k].x * ld + c] = buf[k * SW_COLS + col];
}

// L11⁻¹ (block 0) and U11⁻¹ (block 1) of the factored 128 x 128 diagonal block, row-major.
// X in registers (8 x 8 per thread: rows 8·(tid>>4), columns 8·(tid&15)); one row of X is
// broadcast through LDS per elimination step.
__global__ __launch_bounds__(256) void lu_diag_inv_kernel(const double* __restrict__ A, int64_t ld, int64_t r0,
                                                          double* __restrict__ Linv, double* __restrict__ Uinv) {
  constexpr int SP = LB + 1;
  __shared__ double S[LB * SP];
  __shared__ double rb[2][LB];
  const int tid = threadIdx.x, ti = tid >> 4, tc = tid & 15;
  for (int e = tid; e < LB * LB; e += 256) {
    const int i = e >> 7, c = e & 127;
    S[i * SP + c] = A[(r0 + i) * ld + r0 + c];
  }
  double X[8][8];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) X[r][c] = (8 * ti + r == 8 * tc + c) ? 1.0 : 0.0;
  __syncthreads();
  const bool lower = blockIdx.x == 0;
  for (int s = 0; s < LB; ++s) {
    const int k = lower ? s : LB - 1 - s;
    const int b = s & 1;
    if (ti == (k >> 3)) {
      const double dinv = lower ? 1.0 : 1.0 / S[k * SP + k];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        double xv = 0.0;
#pragma unroll
        for (int r = 0; r < 8; ++r) xv = (r == (k & 7)) ? X[r][c] : xv;
        xv *= dinv;
        rb[b][8 * tc + c] = xv;
        if (!lower) {
#pragma unroll
          for (int r = 0; r < 8; ++r)
            if (r == (k & 7)) X[r][c] = xv;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int i = 8 * ti + r;
      if (lower ? (i > k) : (i < k)) {
        const double f = S[i * SP + k];
#pragma unroll
        for (int c = 0; c < 8; ++c) X[r][c] -= f * rb[b][8 * tc + c];
      }
    }
  }
  double* out = lower ? Linv : Uinv;
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) out[(8 * ti + r) * LB + 8 * tc + c] = X[r][c];
}

// T[j][k] = A(r0 + k, c_lo + j): the block row's 128 rows as columns (K-contiguous operand)
__global__ __launch_bounds__(256) void lu_transpose_kernel(const double* __restrict__ A, int64_t ld, int64_t r0,
                                                           int64_t c_lo, int64_t w, double* __restrict__ T) {
  __shared__ double t[64][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t j0 = (int64_t)blockIdx.x * 64, k0 = (int64_t)blockIdx.y * 64;
  for (int kk = ty; kk < 64; kk += 4) t[kk][tx] = (j0 + tx < w) ? A[(r0 + k0 + kk) * ld + c_lo + j0 + tx] : 0.0;
  __syncthreads();
  for (int jj = ty; jj < 64; jj += 4)
    if (j0 + jj < w) T[(j0 + jj) * LB + k0 + tx] = t[tx][jj];
}

__global__ void lu_pad_kernel(double* A, int64_t ld, int64_t n, int64_t npad) {
  const int64_t i = n + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < npad) A[i * ld + i] = 1.0;
}

// ---- solve -------------------------------------------------------------------------
// forward block k: apply the block's row moves to b, then b_k <- L11⁻¹ b_k
// a block's row moves applied to b (all sources read before any store)
__global__ __launch_bounds__(256) void lu_moves_kernel(const int2* __restrict__ pairs, const int* __restrict__ npairs,
                                                       double* b) {
  const int tid = threadIdx.x, np = *npairs;
  double v = 0.0;
  if (tid < np) v = b[pairs[tid].y];
  __syncthreads();
  if (tid < np) b[pairs[tid].x] = v;
}

__global__ __launch_bounds__(256) void lu_fwd_block_kernel(const int2* __restrict__ pairs,
                                                           const int* __restrict__ npairs,
                                                           const double* __restrict__ Linv, int64_t r0, double* b,
                                                           int moves) {
  __shared__ double bs[LB];
  __shared__ double part[2][LB];
  const int tid = threadIdx.x, np = moves ? *npairs : 0;
  double v = 0.0;
  if (tid < np) v = b[pairs[tid].y];
  __syncthreads();
  if (tid < np) b[pairs[tid].x] = v;
  __syncthreads();
  if (tid < LB) bs[tid] = b[r0 + tid];
  __syncthreads();
  {  // y_i = Σ_c Linv(i, c) b_c: two threads per row, 64 columns each
    const int i = tid >> 1, h = tid & 1;
    const double* lr = Linv + (int64_t)i * LB + 64 * h;
    double s = 0.0;
    for (int c = 0; c < 64; c += 2) {
      const v2d a = *(const v2d*)(lr + c);
      s += a[0] * bs[64 * h + c] + a[1] * bs[64 * h + c + 1];
    }
    part[h][i] = s;
  }
  __syncthreads();
  if (tid < LB) b[r0 + tid] = part[0][tid] + part[1][tid];
}

// backward block k: b_k <- U11⁻¹ b_k
__global__ __launch_bounds__(256) void lu_bwd_block_kernel(const double* __restrict__ Uinv, int64_t r0, double* b) {
  __shared__ double bs[LB];
  __shared__ double part[2][LB];
  const int tid = threadIdx.x;
  if (tid < LB) bs[tid] = b[r0 + tid];
  __syncthreads();
  {
    const int i = tid >> 1, h = tid & 1;
    const double* ur = Uinv + (int64_t)i * LB + 64 * h;
    double s = 0.0;
    for (int c = 0; c < 64; c += 2) {
      const v2d a = *(const v2d*)(ur + c);
      s += a[0] * bs[64 * h + c] + a[1] * bs[64 * h + c + 1];
    }
    part[h][i] = s;
  }
  __syncthreads();
  if (tid < LB) b[r0 + tid] = part[0][tid] + part[1][tid];
}

// b[r] -= Σ_t A(r, c0 + t) b[c0 + t] for rows r in [rlo, rlo + nr): 8 lanes per row (16 columns
// each), fixed-order butterfly over the 8 lanes.
__global__ __launch_bounds__(256) void lu_rank_update_kernel(const double* __restrict__ A, int64_t ld, int64_t rlo,
                                                             int64_t nr, int64_t c0, double* b) {
  __shared__ double xs[LB];
  const int tid = threadIdx.x;
  if (tid < LB) xs[tid] = b[c0 + tid];
  __syncthreads();
  const int q = tid & 7;
  const int64_t r = (int64_t)blockIdx.x * 32 + (tid >> 3);
  double s = 0.0;
  if (r < nr) {
    const double* row = A + (rlo + r) * ld + c0 + 16 * q;
#pragma unroll
    for (int c = 0; c < 16; c += 2) {
      const v2d a = *(const v2d*)(row + c);
      s += a[0] * xs[16 * q + c] + a[1] * xs[16 * q + c + 1];
    }
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  if (r < nr && q == 0) b[rlo + r] -= s;
}

// ---------------------------------------------------------------------------
hipError_t lu_aux_init(LUAux* a, int64_t npad, hipStream_t st) {
  if (a->npad >= npad) return hipSuccess;
  lu_aux_free(a);
  const int nblk = (int)(npad / LB);
  std::vector<double> hw(LB + LU_OB * LB, -1.0);   // [128 x +1 | 512 x -1]
  for (int i = 0; i < LB; ++i) hw[i] = 1.0;
  // square-shell order: the first t² entries are the t x t leading block
  std::vector<int2> sq;
  sq.reserve((size_t)nblk * nblk);
  for (int s = 0; s < nblk; ++s) {
    for (int j = 0; j <= s; ++j) sq.push_back(make_int2(s, j));
    for (int i = 0; i < s; ++i) sq.push_back(make_int2(i, s));
  }
  std::vector<int2> row1(nblk);
  for (int j = 0; j < nblk; ++j) row1[j] = make_int2(0, j);
  // row-major nblk x c rectangles, c = 1 .. LU_OB (the updates inside an outer block; LU_OB: the
  // lookahead's update of the next outer block's columns)
  std::vector<int2> rect;
  for (int c = 1; c <= LU_OB; ++c)
    for (int i = 0; i < nblk; ++i)
      for (int j = 0; j < c; ++j) rect.push_back(make_int2(i, j));
  // column-major LU_OB x nblk (the lookahead bulk's rows of the next outer block)
  std::vector<int2> col4;
  for (int j = 0; j < nblk; ++j)
    for (int i = 0; i < LU_OB; ++i) col4.push_back(make_int2(i, j));
  hipError_t e = hipSuccess;
  auto al = [&](void** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, bytes);
    if (e == hipSuccess) e = hipMemsetAsync(*p, 0, bytes, st);
  };
  al((void**)&a->cand, sizeof(double) * 2 * LU_MAXWG);
  al((void**)&a->candi, sizeof(int) * 2 * LU_MAXWG);
  al((void**)&a->candrow, sizeof(double) * 2 * LU_MAXWG * LB);
  al((void**)&a->rowj, sizeof(double) * 2 * LB);
  al((void**)&a->gran, sizeof(unsigned long long) * LUC_WORDS);
  al((void**)&a->ipiv, sizeof(int) * npad);
  al((void**)&a->pairs, sizeof(int2) * (size_t)nblk * LU_MAXPAIRS);
  al((void**)&a->npairs, sizeof(int) * nblk);
  al((void**)&a->Linv, sizeof(double) * (size_t)nblk * LB * LB);
  al((void**)&a->Uinv, sizeof(double) * (size_t)nblk * LB * LB);
  al((void**)&a->T, sizeof(double) * (size_t)npad * LB);
  al((void**)&a->UT, sizeof(double) * (size_t)npad * LB);
  al((void**)&a->UTo, sizeof(double) * (size_t)npad * LU_OB * LB);
  al((void**)&a->rect, sizeof(int2) * rect.size());
  al((void**)&a->w, sizeof(double) * hw.size());
  al((void**)&a->sq, sizeof(int2) * sq.size());
  al((void**)&a->row1, sizeof(int2) * row1.size());
  al((void**)&a->T2, sizeof(double) * (size_t)npad * LB);
  al((void**)&a->col4, sizeof(int2) * col4.size());
  al((void**)&a->lctr, sizeof(unsigned) * 16 * LU_LCTR);
  if (e == hipSuccess) e = hipMemcpyAsync(a->w, hw.data(), sizeof(double) * hw.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(a->sq, sq.data(), sizeof(int2) * sq.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = hipMemcpyAsync(a->row1, row1.data(), sizeof(int2) * row1.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = hipMemcpyAsync(a->rect, rect.data(), sizeof(int2) * rect.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = hipMemcpyAsync(a->col4, col4.data(), sizeof(int2) * col4.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess) a->npad = npad;
  return e;
}

void lu_aux_free(LUAux* a) {
  void* ps[] = {a->cand, a->candi, a->candrow, a->rowj, a->gran, a->ipiv, a->pairs, a->npairs, a->Linv,
                a->Uinv, a->T,     a->UT,      a->UTo,  a->rect, a->w,    a->sq,   a->row1,
                a->T2,   a->col4,  a->lctr};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  if (a->st2) (void)hipStreamDestroy(a->st2);
  if (a->evp) (void)hipEventDestroy(a->evp);
  if (a->evb) (void)hipEventDestroy(a->evb);
  *a = LUAux();
}

// SCS_LU_PANEL (read per call): unset / 3 = the cooperative one-launch panel where G = h / 128 <= 128
// (lu_panel_coop_kernel, r05), else the column steps; 2 = lu_panel_step2_kernel up to two 32-row passes
// per workgroup (n <= 16384); 1 = the r02 column step everywhere (all bitwise the same factor)
static int lu_panel_mode() {
  const char* e = getenv("SCS_LU_PANEL");
  return e ? atoi(e) : 3;
}

static hipError_t lu_coop_attr() {   // the dynamic LDS above the 64 KiB default, once per process
  static hipError_t done = [] {
    const void* ks[] = {(const void*)lu_panel_coop_kernel<true, 256>, (const void*)lu_panel_coop_kernel<false, 256>,
                        (const void*)lu_panel_coop_kernel<true, 512>, (const void*)lu_panel_coop_kernel<false, 512>,
                        (const void*)lu_panel_coop_kernel<false, 256, true>,
                        (const void*)lu_panel_coop_kernel<false, 512, true>, (const void*)lu_panel_blk_kernel<256>,
                        (const void*)lu_panel_blk_kernel<512>};
    hipError_t e = hipSuccess;
    for (const void* f : ks)
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LUC_LDS);
    if (e != hipSuccess) (void)hipGetLastError();   // the step kernels run instead: no error left behind
    return e;
  }();
  return done;
}

static int lu_device_cus() {   // compute units of the current device (per call: contexts may switch devices)
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return ncu;
}

static bool lu_coop_pf() {   // read per call (A/B): SCS_LU_COOP_PF=0 stages the pivot row only after the sweep
  const char* e = getenv("SCS_LU_COOP_PF");
  return !(e && e[0] == '0');
}

static int lu_coop_nt() {   // read per call (A/B): SCS_LU_COOP_NT = 256 | 512
  const char* e = getenv("SCS_LU_COOP_NT");
  return (e && atoi(e) == 512) ? 512 : 256;
}

static unsigned lu_coop_spin() {   // read per call: SCS_LU_COOP_SPIN (sweeps; 0 = give up at once, tests)
  const char* e = getenv("SCS_LU_COOP_SPIN");
  return e ? (unsigned)strtoul(e, nullptr, 10) : LUC_SPIN_MAX;
}

// SCS_LU_COOP_LAUNCH (read per call; default 1): the one-launch panel through hipLaunchCooperativeKernel,
// which guarantees that all its workgroups are resident together or refuses the launch (the panel then
// runs as column steps); 0 = a plain launch, residency by the 96 KiB of LDS and the CU-count check only
static bool lu_coop_api() {
  const char* e = getenv("SCS_LU_COOP_LAUNCH");
  return !(e && e[0] == '0');
}

static bool lu_coop_early() {   // read per call (A/B): SCS_LU_COOP_EARLY=0 publishes rows before the record
  const char* e = getenv("SCS_LU_COOP_EARLY");
  return !(e && e[0] == '0');
}

// SCS_LU_COOP_BLK (read per call; default 1): the block-deferred panel (lu_panel_blk_kernel; n = 8192
// factor + solve 77.0 -> 55.9 ms, 16384 197.4-198.5 -> 159.8-160.1 ms, same bits); 0 = lu_panel_coop_kernel
static bool lu_coop_blk() {
  const char* e = getenv("SCS_LU_COOP_BLK");
  return !(e && e[0] == '0');
}

static bool lu_coop_wide() {   // read per call (A/B): SCS_LU_COOP_WIDE=1 (n = 8192: 84.9 vs 83.2 ms narrow)
  const char* e = getenv("SCS_LU_COOP_WIDE");
  return e && e[0] == '1';
}

// SCS_LU_INV (read per call): unset / 2 = the diagonal block's inverses by 16 x 16 inverses + MFMA doubling
// (lu_tri_inv_kernel, chol.hip), 1 = the r02 row-by-row elimination (lu_diag_inv_kernel)
static int lu_inv_mode() {
  const char* e = getenv("SCS_LU_INV");
  return e ? atoi(e) : 2;
}

// SCS_LU_OB (read per call): an on/off switch -- 1 = per-panel updates, any other value (default) = outer
// blocks of LU_OB = 4 panels (the only outer size built: 2, 3 or 8 also run with 4).  With 4 the trailing matrix takes ONE update per
// four panels with K = 512 (r05; the K = 128 updates ran at ~26 TF/s on the C read-modify-write: the
// n = 8192 updates 13.8 -> 8.0 ms, factor + solve 83.7-83.9 -> 82.0-82.9 ms, n = 16384 250.8-251.2 ->
// 216.8-217.1 ms); 1: the r02 per-panel updates.  Recorded in the aux for lu_solve (its forward steps follow the
// factor's row order).
static int lu_outer_block() {
  const char* e = getenv("SCS_LU_OB");
  const int v = e ? atoi(e) : LU_OB;
  return v >= 2 ? LU_OB : 1;
}

// the panel of block k: its 128 column steps (one cooperative launch, or the step launches), the composed
// row moves and the diagonal block's inverses
static hipError_t lu_panel(double* A, int64_t ld, int64_t npad, int k, const LUAux* a, int* info, hipStream_t st) {
  const int64_t r0 = (int64_t)k * LB, c0 = r0, h = npad - r0;
  const int R = 32 * (int)ceil_div(h, 32 * LU_MAXWG);
  const int nwg = (int)ceil_div(h, R);
  const int npass = R / 32, mode = lu_panel_mode();
  const int cnt = lu_coop_nt();
  const int64_t gco = ceil_div(h, (int64_t)(cnt / 2));
  // (a runtime that refuses the dynamic-LDS attribute gets the step kernels, and so does a device with
  // fewer than twice as many CUs as the panel needs workgroups -- a partitioned MI355X -- where they
  // could not all be resident at once)
  bool coop = mode == 3 && !a->no_coop && gco <= (cnt == 512 ? 64 : LUC_MAXWG) && 2 * gco <= lu_device_cus() &&
              lu_coop_attr() == hipSuccess;
  if (coop) {
    const bool wide = lu_coop_wide();
    const bool early = !wide && lu_coop_early();
    auto kern = cnt == 512 ? (wide ? lu_panel_coop_kernel<true, 512>
                                   : (early ? lu_panel_coop_kernel<false, 512, true> : lu_panel_coop_kernel<false, 512>))
                           : (wide ? lu_panel_coop_kernel<true, 256>
                                   : (early ? lu_panel_coop_kernel<false, 256, true> : lu_panel_coop_kernel<false, 256>));
    if (!wide && lu_coop_blk()) kern = cnt == 512 ? lu_panel_blk_kernel<512> : lu_panel_blk_kernel<256>;
    double* pA = A;
    int64_t pld = ld, pr0 = r0, pc0 = c0, ph = h;
    unsigned long long* pgran = a->gran;
    unsigned ptag = (unsigned)k << 8, pspin = lu_coop_spin();
    int* pipiv = a->ipiv;
    int* pinfo = info;
    int2* ppairs = a->pairs + (int64_t)k * LU_MAXPAIRS;
    int* pnp = a->npairs + k;
    int ppf = lu_coop_pf() ? 1 : 0;
    if (lu_coop_api()) {
      void* args[] = {&pA, &pld, &pr0, &pc0, &ph, &pgran, &ptag, &pipiv, &pinfo, &ppairs, &pnp, &ppf, &pspin};
      if (hipLaunchCooperativeKernel((const void*)kern, dim3((unsigned)gco), dim3(cnt), args, LUC_LDS, st) != hipSuccess) {
        (void)hipGetLastError();   // refused (the grid cannot be resident at once): this panel by column steps
        ++a->coop_refused;
        coop = false;
      }
    } else {
      hipLaunchKernelGGL(kern, dim3((unsigned)gco), dim3(cnt), LUC_LDS, st, pA, pld, pr0, pc0, ph, pgran, ptag, pipiv,
                         pinfo, ppairs, pnp, ppf, pspin);
    }
  }
  if (!coop)
    for (int j = -1; j < LB; ++j) {
      if (mode == 2 && npass == 1)
        hipLaunchKernelGGL(lu_panel_step2_kernel<1>, dim3(nwg), dim3(LU_NT), 0, st, A, ld, r0, c0, h, R, j, a->cand,
                           a->candi, a->candrow, a->rowj, a->ipiv, info);
      else if (mode == 2 && npass == 2)
        hipLaunchKernelGGL(lu_panel_step2_kernel<2>, dim3(nwg), dim3(LU_NT), 0, st, A, ld, r0, c0, h, R, j, a->cand,
                           a->candi, a->candrow, a->rowj, a->ipiv, info);
      else
        hipLaunchKernelGGL(lu_panel_step_kernel, dim3(nwg), dim3(LU_NT), 0, st, A, ld, r0, c0, h, R, j, a->cand,
                           a->candi, a->candrow, a->rowj, a->ipiv, info);
    }
  if (!coop)   // (the cooperative panel composes its interchanges itself)
    hipLaunchKernelGGL(lu_perm_kernel, dim3(1), dim3(64), 0, st, a->ipiv, (int)r0, a->pairs + (int64_t)k * LU_MAXPAIRS,
                       a->npairs + k);
  if (lu_inv_mode() == 1)
    hipLaunchKernelGGL(lu_diag_inv_kernel, dim3(2), dim3(256), 0, st, A, ld, r0, a->Linv + (int64_t)k * LB * LB,
                       a->Uinv + (int64_t)k * LB * LB);
  else
    (void)launch_lu_tri_inv(A, ld, r0, a->Linv + (int64_t)k * LB * LB, a->Uinv + (int64_t)k * LB * LB, st);
  return hipGetLastError();
}

static void lu_swap(double* A, int64_t ld, int64_t c_lo, int64_t w, const LUAux* a, int k, hipStream_t st) {
  if (w <= 0) return;
  hipLaunchKernelGGL(lu_swap_cols_kernel, dim3((unsigned)ceil_div(w, SW_COLS)), dim3(256), 0, st, A, ld, c_lo, w,
                     a->pairs + (int64_t)k * LU_MAXPAIRS, a->npairs + k);
}

// SCS_LU_LA (read per call; default 1, 0 = the one-stream outer step): the lookahead outer step.  After an outer block's panels, the
// trailing columns of the NEXT outer block (the next panels' input) are updated on the caller's stream
// and every column beyond them on a bulk stream, which runs beside the next outer block's panels --
// the panels (37 of the 55 ms of an n = 8192 factor + solve, r06) hold a cooperative launch of one
// workgroup per CU on h / 128 of the 256 CUs, the rest idle.  Per tile the same kernels and K order as
// the one-stream step: the same factor bit for bit (test_lu_lookahead_bit_identical).
static bool lu_lookahead() {
  const char* e = getenv("SCS_LU_LA");
  return !(e && e[0] == '0');
}

// SCS_LU_LA_SKIP (read per call): CU ids per shader engine the bulk's throughput launches leave free
// (gram_launch_bounded; 0 = full-grid launches).  Unset: full-grid launches while the bulk outweighs
// the next outer block's panels -- more than SCS_LU_LA_FULL (default 8192) trailing columns: its
// update is 2·h²·512 flop, 4.6 ms at h = 16384 against ~2.3 ms of panels (~0.58 ms each, latency-bound)
// -- then a skip set sized to the next panel's cooperative launch of h / 128 CUs: k = ceil(h / 4096)
// ids (1..4) of each of the 32 shader engines, from id 4 up.  Measured (r06, factor + solve, 3 rounds
// alternated): n = 8192 55.6-57.4 -> 54.3-54.4 ms, 16384 157.7-159.2 -> 147.3-148.1 ms; full grid
// throughout 54.6-55.7 / 148.9-150.3, threshold 4096 55.4-55.9 / 149.1-150.5, 12288 53.9-54.3 /
// 146.7-147.6; sized skip sets throughout 16384 178-180 (profiles/r06/lu_la/).
static unsigned lu_la_skip(int64_t h_next) {
  const char* e = getenv("SCS_LU_LA_SKIP");
  if (e) return (unsigned)strtoul(e, nullptr, 0) & 0xffffu;
  const char* f = getenv("SCS_LU_LA_FULL");
  if (h_next > (f ? atoll(f) : 8192)) return 0u;
  const int k = (int)std::min<int64_t>(4, std::max<int64_t>(1, ceil_div(h_next, (int64_t)32 * LB)));
  return ((1u << k) - 1u) << 4;
}

// The trailing columns [cb1 + coff, cb1 + coff + w) of the outer block [b0, b1) on stream s: the block's
// row moves in order, its U rows by block forward substitution (X_t = L_tt⁻¹ (A_t - Σ_{s<t} L_ts X_s),
// X into A and, K-contiguous, into UTo), then A22 -= L21 X with K = (b1 - b0)·128 over all the rows
// below the block.  coff = 0: the columns from cb1 (rect / square tile lists); coff = LU_OB·128: the
// lookahead bulk (the square below the next outer block's rows + those rows' LU_OB x nc strip), its
// throughput launches CU-bounded when ctr is given.
static hipError_t lu_outer_trailing(double* A, int64_t ld, int64_t npad, int b0, int b1, int64_t coff, int64_t w,
                                    double* Tb, const LUAux* a, unsigned* ctr, hipStream_t s) {
  const int64_t cb0 = (int64_t)b0 * LB, cb1 = (int64_t)b1 * LB, c_lo = cb1 + coff;
  const int ncr = (int)(w / LB), nr = (int)((npad - cb1) / LB), KO = (b1 - b0) * LB;
  const int64_t ncap = a->npad / LB;   // the lists were built for the aux's capacity
  double* U = a->UTo + coff * (LU_OB * LB);
  hipError_t e = hipSuccess;
  for (int k = b0; k < b1; ++k) lu_swap(A, ld, c_lo, w, a, k, s);
  for (int k = b0; k < b1; ++k) {
    const int64_t r0 = (int64_t)k * LB;
    const int t = k - b0;
    if (t > 0)
      e = gram_launch_gen(A + r0 * ld + cb0, ld, U, LU_OB * LB, a->w + LB, 0, (int64_t)t * LB, a->row1, ncr,
                          A + r0 * ld + c_lo, ld, /*GRAM_ACCUMULATE|GRAM_UPPER*/ 2 | 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lu_transpose_kernel, dim3((unsigned)ceil_div(w, 64), LB / 64), dim3(256), 0, s, A, ld, r0, c_lo,
                       w, Tb);
    const double* Lk = a->Linv + (int64_t)k * LB * LB;
    e = gram_launch_gen(Lk, LB, Tb, LB, a->w, 0, LB, a->row1, ncr, A + r0 * ld + c_lo, ld, /*GRAM_UPPER*/ 4, s);
    if (e == hipSuccess)
      e = gram_launch_gen(Lk, LB, Tb, LB, a->w, 0, LB, a->row1, ncr, U + (int64_t)t * LB, LU_OB * LB, 0, s);
    if (e != hipSuccess) return e;
  }
  if (coff == 0) {
    const int2* tl = ncr == nr ? a->sq : a->rect + ncap * (ncr - 1) * ncr / 2;
    return gram_launch_gen(A + cb1 * ld + cb0, ld, U, LU_OB * LB, a->w + LB, 0, KO, tl, ncr == nr ? nr * nr : nr * ncr,
                           A + cb1 * ld + c_lo, ld, /*GRAM_ACCUMULATE|GRAM_UPPER*/ 2 | 4, s);
  }
  // (coff = LU_OB·128 and ncr = nr - LU_OB: the rows below the next outer block form a square)
  const unsigned skip = ctr ? lu_la_skip(npad - cb1) : 0u;
  const int slots = 2 * lu_device_cus();
  e = gram_launch_bounded(A + c_lo * ld + cb0, ld, U, LU_OB * LB, a->w + LB, 0, KO, a->sq, ncr * ncr,
                          A + c_lo * ld + c_lo, ld, 2 | 4, ctr, skip, slots, s, true);
  if (e == hipSuccess)
    e = gram_launch_bounded(A + cb1 * ld + cb0, ld, U, LU_OB * LB, a->w + LB, 0, KO, a->col4, LU_OB * ncr,
                            A + cb1 * ld + c_lo, ld, 2 | 4, ctr ? ctr + 16 : nullptr, skip, slots, s, true);
  return e;
}

hipError_t lu_factor(double* A, int64_t ld, int64_t n, int64_t npad, const LUAux* a, int* info, hipStream_t st) {
  if (npad % LB != 0 || npad > a->npad || ld < npad) return hipErrorInvalidValue;
  const int nblk = (int)(npad / LB);
  const int OB = lu_outer_block();
  a->ob = OB;
  if (lu_panel_mode() == 3) {   // the cooperative panels' granules and abort word, once per factorization
    const hipError_t e = hipMemsetAsync(a->gran, 0, sizeof(unsigned long long) * LUC_WORDS, st);
    if (e != hipSuccess) return e;
  }
  // the lookahead: only where some outer block has columns beyond the next one
  const bool la = lu_lookahead() && OB == LU_OB && nblk > 2 * LU_OB;
  if (la) {
    hipError_t e = hipSuccess;
    if (!a->st2) e = hipStreamCreateWithFlags(&a->st2, hipStreamNonBlocking);
    if (e == hipSuccess && !a->evp) e = hipEventCreateWithFlags(&a->evp, hipEventDisableTiming);
    if (e == hipSuccess && !a->evb) e = hipEventCreateWithFlags(&a->evb, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMemsetAsync(a->lctr, 0, sizeof(unsigned) * 16 * LU_LCTR, st);
    if (e != hipSuccess) return e;
    a->lslot = 0;
  }
  if (npad > n)
    hipLaunchKernelGGL(lu_pad_kernel, dim3((unsigned)ceil_div(npad - n, 256)), dim3(256), 0, st, A, ld, n, npad);
  hipError_t e = hipSuccess;
  bool bulk = false;   // a bulk update is in flight on st2 (evb recorded after it)
  for (int b0 = 0; b0 < nblk; b0 += OB) {
    const int b1 = std::min(b0 + OB, nblk);
    const int64_t cb0 = (int64_t)b0 * LB, cb1 = (int64_t)b1 * LB;
    // the outer block's panels, right-looking inside it: each panel's moves to the block's other columns
    // (the earlier panels' L columns too, so the block's L rows end in the block's final order) and its
    // U rows / update over the block's later columns only (OB = 1: the whole trailing matrix)
    for (int k = b0; k < b1; ++k) {
      const int64_t r0 = (int64_t)k * LB, c0 = r0;
      e = lu_panel(A, ld, npad, k, a, info, st);
      if (e != hipSuccess) return e;
      const int64_t wr = (OB == 1 ? npad : cb1) - c0 - LB;   // columns right of the panel it updates now
      lu_swap(A, ld, c0 + LB, wr, a, k, st);
      lu_swap(A, ld, cb0, c0 - cb0, a, k, st);
      if (wr == 0) continue;
      // TRSM: U12 = L11⁻¹ A12 (row-major into A) and U12ᵀ-as-columns into UT
      hipLaunchKernelGGL(lu_transpose_kernel, dim3((unsigned)ceil_div(wr, 64), LB / 64), dim3(256), 0, st, A, ld, r0,
                         c0 + LB, wr, a->T);
      const int nc = (int)(wr / LB), nr = (int)((npad - r0 - LB) / LB);
      const double* Lk = a->Linv + (int64_t)k * LB * LB;
      e = gram_launch_gen(Lk, LB, a->T, LB, a->w, 0, LB, a->row1, nc, A + r0 * ld + c0 + LB, ld, /*GRAM_UPPER*/ 4, st);
      if (e == hipSuccess) e = gram_launch_gen(Lk, LB, a->T, LB, a->w, 0, LB, a->row1, nc, a->UT, LB, 0, st);
      // A22 -= L21 U12 over the rows below and the columns it updates now (square: OB = 1; nr x nc rows-major:
      // inside an outer block)
      if (e == hipSuccess && nr > 0) {
        const int64_t ncap = a->npad / LB;   // the lists were built for the aux's capacity
        const int2* tl = (OB == 1) ? a->sq : a->rect + ncap * (nc - 1) * nc / 2;
        e = gram_launch_gen(A + (r0 + LB) * ld + c0, ld, a->UT, LB, a->w + LB, 0, LB, tl, (OB == 1) ? nc * nc : nr * nc,
                            A + (r0 + LB) * ld + c0 + LB, ld, /*GRAM_ACCUMULATE|GRAM_UPPER*/ 2 | 4, st);
      }
      if (e != hipSuccess) return e;
    }
    if (OB == 1 || cb1 == npad) continue;
    // the trailing columns (lu_outer_trailing).  Lookahead: the previous bulk update wrote the columns
    // this step starts from, so the caller's stream waits for it here -- after this block's panels, which
    // ran beside it -- and columns beyond the next outer block go to the bulk stream
    const int64_t wt = npad - cb1;
    if (bulk) {
      e = hipStreamWaitEvent(st, a->evb, 0);
      if (e != hipSuccess) return e;
      bulk = false;
    }
    if (la && wt > (int64_t)LU_OB * LB) {
      const int64_t wa = (int64_t)LU_OB * LB;
      unsigned* ctr = nullptr;
      if (a->lslot + 2 <= LU_LCTR) {
        ctr = a->lctr + 16 * a->lslot;
        a->lslot += 2;
      }
      e = hipEventRecord(a->evp, st);
      if (e == hipSuccess) e = hipStreamWaitEvent(a->st2, a->evp, 0);
      if (e == hipSuccess) e = lu_outer_trailing(A, ld, npad, b0, b1, wa, wt - wa, a->T2, a, ctr, a->st2);
      if (e == hipSuccess) e = hipEventRecord(a->evb, a->st2);
      if (e != hipSuccess) return e;
      bulk = true;
      e = lu_outer_trailing(A, ld, npad, b0, b1, 0, wa, a->T, a, nullptr, st);
    } else {
      e = lu_outer_trailing(A, ld, npad, b0, b1, 0, wt, a->T, a, nullptr, st);
    }
    if (e != hipSuccess) return e;
  }
  if (bulk) {
    e = hipStreamWaitEvent(st, a->evb, 0);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

hipError_t lu_solve(const double* A, int64_t ld, int64_t npad, const LUAux* a, double* b, hipStream_t st) {
  const int nblk = (int)(npad / LB);
  const int OB = a->ob;
  for (int k = 0; k < nblk; ++k) {
    const int64_t r0 = (int64_t)k * LB;
    // an outer block's L rows are in the block's final row order: all its moves to b before its first
    // forward step (OB = 1: each block's moves just before its own step)
    if (OB > 1 && k % OB == 0)
      for (int kk = k; kk < std::min(k + OB, nblk); ++kk)
        hipLaunchKernelGGL(lu_moves_kernel, dim3(1), dim3(256), 0, st, a->pairs + (int64_t)kk * LU_MAXPAIRS,
                           a->npairs + kk, b);
    hipLaunchKernelGGL(lu_fwd_block_kernel, dim3(1), dim3(256), 0, st, a->pairs + (int64_t)k * LU_MAXPAIRS,
                       a->npairs + k, a->Linv + (int64_t)k * LB * LB, r0, b, OB == 1 ? 1 : 0);
    const int64_t nr = npad - r0 - LB;
    if (nr > 0)
      hipLaunchKernelGGL(lu_rank_update_kernel, dim3((unsigned)ceil_div(nr, 32)), dim3(256), 0, st, A, ld, r0 + LB, nr,
                         r0, b);
  }
  for (int k = nblk - 1; k >= 0; --k) {
    const int64_t r0 = (int64_t)k * LB;
    hipLaunchKernelGGL(lu_bwd_block_kernel, dim3(1), dim3(256), 0, st, a->Uinv + (int64_t)k * LB * LB, r0, b);
    if (r0 > 0)
      hipLaunchKernelGGL(lu_rank_update_kernel, dim3((unsigned)ceil_div(r0, 32)), dim3(256), 0, st, A, ld, (int64_t)0,
                         r0, r0, b);
  }
  return hipGetLastError();
}

}  // namespace scs
