// Householder QR solve x = qr(A) \ b -- the reference's solver for ProxGGNSCORE's systems
// (`qr(JQJ) \ Je`, prox-GGN-SCORE.jl:131; `qr(I + A) \ residual`, :126), behind the opt-in
// reference-solver mode (scs_set_solver(ctx, SCS_SOLVER_REFERENCE)); the default path solves the
// same systems by Cholesky / LU, equal to O(cond·eps).
//
// LAPACK's conventions (dgeqrf / dlarfg / dlarft, what Julia's qr on a dense Matrix calls):
// column c of the panel gets H_c = I - tau v vᵀ with v(c) = 1, beta = -sign(alpha) ||(alpha, x)||,
// tau = (beta - alpha) / beta, v(c+1:) = x / (alpha - beta); tau = 0 (H = I) when x = 0.  Blocked
// by 128-column panels (compact WY, T from dlarft forward / columnwise):
//   panel, per column c:  qr_col_partials  -- per (row chunk, column j) the partial Σ x_r A_rj
//                                            (j = c: Σ x_r²), fixed chunks, one wave sum each;
//                         qr_col_reflect   -- one workgroup: the chunk partials in chunk order,
//                                            beta, tau, w_j = vᵀ A_j, R(c, c) = beta, v -> V;
//                         qr_col_update    -- A_j -= tau w_j v over the panel's later columns and
//                                            b (Qᵀ b is applied reflector by reflector);
//   trailing columns:     Wm = Vᵀ A_trail, Y = Tᵀ Wm, A_trail -= V Y, on the Gram kernels (MFMA).
// Then R x = Qᵀ b: the inverses of R's 128 x 128 diagonal blocks and the Cholesky's one-launch
// backward solve (chol.hip).  A is column-major npad x npad (ld), rows / columns [n, npad) the
// identity (the caller pads); A and b are overwritten (R above the diagonal, x in b).
#include <cmath>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace scs {

constexpr int QB = 128;         // panel width
constexpr int QR_RC = 1024;     // rows per partial-sum chunk
constexpr int QR_KS = 512;      // rows per K piece of the panel's Vᵀ products (qr_ksplit)
constexpr int QR_KMAXITEMS = 1024;   // K-split work items per launch at most (partial buffer: 128 MiB)
constexpr int QR_MAXRC = 64;         // chunks whose partials qr_col_step stages in LDS (npad <= 65536)

// partial[(j - c) * nrc + rc]: Σ_{r in chunk rc, r > c} A[r, c] · A[r, j] for the panel's columns
// j = c .. c1-1, and (j = c1) the right-hand side b
__global__ __launch_bounds__(256) void qr_col_partials(const double* __restrict__ A, int64_t ld, int64_t npad, int64_t c,
                                                       int64_t c1, const double* __restrict__ b,
                                                       double* __restrict__ part, int nrc) {
  const int rc = blockIdx.x, jj = blockIdx.y;
  const int64_t j = c + jj;
  const double* col = (j < c1) ? A + j * ld : b;
  const double* x = A + c * ld;
  const int64_t r0 = c + 1 + (int64_t)rc * QR_RC, r1 = min(r0 + QR_RC, npad);
  double s = 0.0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) s += x[r] * col[r];
  __shared__ double ws[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[(int64_t)jj * nrc + rc] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

// one workgroup: reduce the partials (chunk order), the reflector (dlarfg), tw_j = tau · vᵀ A_j
// for the later panel columns and b; R(c, c) = beta; V's column: zeros above, 1 on the diagonal
__global__ __launch_bounds__(256) void qr_col_reflect(double* __restrict__ A, int64_t ld, int64_t c, int64_t c1, int64_t c0,
                                                      const double* __restrict__ b, const double* __restrict__ part,
                                                      int nrc, double* __restrict__ tw, double* __restrict__ tau,
                                                      double* __restrict__ scal, double* __restrict__ V, int64_t ldv) {
  __shared__ double sh[3];
  const int ncol = (int)(c1 - c) + 1;   // column c, the later panel columns, b
  const int tid = threadIdx.x;
  if (tid == 0) {
    double xx = 0.0;
    for (int rc = 0; rc < nrc; ++rc) xx += part[rc];
    const double alpha = A[c * ld + c];
    double t = 0.0, sc = 0.0, beta = alpha;
    if (xx > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + xx), alpha);
      t = (beta - alpha) / beta;
      sc = 1.0 / (alpha - beta);
    }
    sh[0] = t;
    sh[1] = sc;
    sh[2] = beta;
    tau[c - c0] = t;
    scal[0] = sc;
  }
  __syncthreads();
  const double t = sh[0], sc = sh[1];
  for (int jj = 1 + tid; jj < ncol; jj += 256) {
    double d = 0.0;
    for (int rc = 0; rc < nrc; ++rc) d += part[(int64_t)jj * nrc + rc];
    const double arc = (c + jj < c1) ? A[(c + jj) * ld + c] : b[c];   // row c of column j (v(c) = 1)
    tw[jj] = t * (arc + sc * d);
  }
  // V column (c - c0): rows [c0, c) zero, row c one (the rows below come from qr_col_update)
  for (int64_t r = c0 + tid; r <= c; r += 256) V[(c - c0) * ldv + (r - c0)] = (r == c) ? 1.0 : 0.0;
  __syncthreads();
  if (tid == 0) A[c * ld + c] = sh[2];
}

// rows r >= c: v_r (1 at r = c, A[r, c]·scal below) into V; A[r, j] -= tw_j v_r for the later panel
// columns j, and b[r] -= tw_b v_r
__global__ __launch_bounds__(256) void qr_col_update(double* __restrict__ A, int64_t ld, int64_t npad, int64_t c, int64_t c1,
                                                     int64_t c0, double* __restrict__ b, const double* __restrict__ tw,
                                                     const double* __restrict__ scal, double* __restrict__ V, int64_t ldv) {
  const int64_t r = c + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= npad) return;
  const int jj = blockIdx.y;   // 0: V; 1 .. c1-c-1: panel columns; c1-c: b
  const double sc = scal[0];
  const double v = (r == c) ? 1.0 : A[c * ld + r] * sc;
  if (jj == 0) {
    if (r > c) V[(c - c0) * ldv + (r - c0)] = v;
    return;
  }
  const int64_t j = c + jj;
  if (j < c1) A[j * ld + r] -= tw[jj] * v;
  else b[r] -= tw[jj] * v;
}

// One launch per column step (the default; SCS_QR_STEP=0 the three launches above): launch c applies
// the reflector of column c-1 (its partials came from launch c-1) and forms the partials of column c,
// as the LU's panel steps pipeline the pivot search (lu.hip).  Workgroup (rc, jj): row chunk rc of
// rows [rbeg, npad) (rbeg = c-1, or c for the panel's first column) and
//   jj = 0        column c-1's reflector: v (V), beta = R(c-1, c-1), R(c-2, c-1), tau;
//   jj = 1 + q    column j = c + q of the panel (q = c1 - c: b): a_j -= tw_j v over its rows, then
//                 the partial Σ_{r > c} a'_rc a'_rj with the UPDATED column c, recomputed here from
//                 the unmodified A column c, and row c of a'_j (rowc) for the next launch's alpha
//                 and w.
// Column c's updated values go to the scratch column xs (by column parity), not into A, so no
// workgroup reads what another one of the same launch writes; the next launch takes its x from xs
// and writes column c's R entries.  Every workgroup reduces the previous column's partials itself,
// in chunk order: the same beta, tau and w_j everywhere.  Launch c1 only finishes column c1-1.
__global__ __launch_bounds__(256) void qr_col_step(double* __restrict__ A, int64_t ld, int64_t npad, int64_t c,
                                                   int64_t c0, int64_t c1, double* __restrict__ b,
                                                   double* __restrict__ part, int64_t pslot, int nrc, int nrc_prev,
                                                   double* __restrict__ rowc, double* __restrict__ xs,
                                                   double* __restrict__ tau, double* __restrict__ V, int64_t ldv,
                                                   int stage) {
  const int rc = blockIdx.x;
  const int jj = (int)blockIdx.y - 1;
  const int tid = threadIdx.x;
  const bool has_prev = c > c0;
  const int64_t pv = c - 1;
  const int64_t rbeg = has_prev ? pv : c;
  const int64_t r0 = rbeg + (int64_t)rc * QR_RC, r1 = min(r0 + QR_RC, npad);
  __shared__ double sh[5];
  __shared__ double ws[4];
  const double* x = xs + (pv & 1) * npad;   // column pv as launch pv left it
  const int64_t j = c + jj;
  double* colj = (jj >= 0 && j < c1) ? A + j * ld : b;
  const double* colc = (c < c1) ? A + c * ld : b;
  // this thread's (at most QR_RC/256) rows of colj, colc and x are loaded before thread 0's serial
  // reduction of the previous column's partials (r05; the same arithmetic, 98 vs 100 ms at n = 8192)
  constexpr int NPF = QR_RC / 256;
  double paj[NPF], pac[NPF], px[NPF];
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int64_t r = r0 + tid + 256 * k;
    const bool in = r < r1;
    paj[k] = (in && jj >= 0) ? colj[r] : 0.0;
    pac[k] = (in && jj >= 0) ? colc[r] : 0.0;
    px[k] = (in && has_prev) ? x[r] : 0.0;
  }
  // r06: the previous column's chunk partials (its xnorm², w_j, w_c) are fetched by wave 0's lanes at once
  // into LDS and summed by thread 0 in chunk order as before -- one memory latency instead of up to
  // 3·nrc_prev dependent loads in thread 0's loops; the same sums and bits (SCS_QR_STAGE=0: the r05
  // loops).  probe_qr, same box, two rounds: n = 16384 307.4-310.0 -> 291.5-292.3 ms, 8192 85.8-86.3 ->
  // 85.1-85.5 ms (profiles/r06/qrstage/); from 8 chunks on (n = 2048, two chunks: 13.4-13.5 vs 14.1 ms)
  __shared__ double sxx[QR_MAXRC], sbj[QR_MAXRC], sbc[QR_MAXRC];
  const bool staged = has_prev && nrc_prev >= 8 && nrc_prev <= QR_MAXRC && stage;   // (2 chunks: the loop is cheaper)
  if (staged && tid < 64) {
    const double* pp = part + (pv & 1) * pslot;
    for (int q = tid; q < nrc_prev; q += 64) {
      sxx[q] = pp[q];
      if (jj >= 0) sbj[q] = pp[(c + jj - pv) * nrc_prev + q];
      if (c < c1) sbc[q] = pp[(c - pv) * nrc_prev + q];
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (tid == 0) {
    double t = 0.0, sc = 0.0, beta = 0.0, twj = 0.0, twc = 0.0;
    if (has_prev) {
      const double* pp = part + (pv & 1) * pslot;
      const double* rp = rowc + (pv & 1) * (QB + 2);
      const double alpha = rp[0], rpj = jj >= 0 ? rp[c + jj - pv] : 0.0, rpc = c < c1 ? rp[c - pv] : 0.0;
      double xx = 0.0;
      if (staged)
        for (int q = 0; q < nrc_prev; ++q) xx += sxx[q];
      else
        for (int q = 0; q < nrc_prev; ++q) xx += pp[q];
      beta = alpha;
      if (xx > 0.0) {
        beta = -copysign(sqrt(alpha * alpha + xx), alpha);
        t = (beta - alpha) / beta;
        sc = 1.0 / (alpha - beta);
      }
      auto twf = [&](int64_t j, const double* sb, double rpv) {   // tau · vᵀ a_j, v(pv) = 1
        double d = 0.0;
        if (staged)
          for (int q = 0; q < nrc_prev; ++q) d += sb[q];
        else
          for (int q = 0; q < nrc_prev; ++q) d += pp[(j - pv) * nrc_prev + q];
        return t * (rpv + sc * d);
      };
      if (jj >= 0) twj = twf(c + jj, sbj, rpj);
      if (c < c1) twc = twf(c, sbc, rpc);
    }
    sh[0] = t;
    sh[1] = sc;
    sh[2] = beta;
    sh[3] = twj;
    sh[4] = twc;
  }
  __syncthreads();
  const double t = sh[0], sc = sh[1];
  if (jj < 0) {   // column pv: V, its R entries, tau
    if (!has_prev) return;
    const int64_t vc = (pv - c0) * ldv;
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int64_t r = r0 + tid + 256 * k;
      if (r < r1 && r > pv) V[vc + (r - c0)] = px[k] * sc;
    }
    if (rc == 0) {
      for (int64_t r = c0 + tid; r <= pv; r += 256) V[vc + (r - c0)] = (r == pv) ? 1.0 : 0.0;
      if (tid == 0) {
        A[pv * ld + pv] = sh[2];
        if (pv - 1 >= c0) A[pv * ld + pv - 1] = x[pv - 1];   // R(pv-1, pv): updated by launch pv
        tau[pv - c0] = t;
      }
    }
    return;
  }
  double* xo = xs + (c & 1) * npad;
  const double twj = sh[3], twc = sh[4];
  double s = 0.0;
  auto row = [&](int64_t r, double aj, double ac, double xr) {
    if (has_prev) {
      const double v = (r == pv) ? 1.0 : xr * sc;
      aj -= twj * v;
      ac -= twc * v;
    }
    if (jj == 0 && c < c1) xo[r] = aj;       // column c itself: to the scratch column
    else if (has_prev) colj[r] = aj;         // later columns and b: in place
    if (r == c) rowc[(c & 1) * (QB + 2) + jj] = aj;
    if (r > c) s += ac * aj;
  };
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int64_t r = r0 + tid + 256 * k;
    if (r < r1) row(r, paj[k], pac[k], px[k]);
  }
  if (c >= c1) return;
  s = wave_sum(s);
  if ((tid & 63) == 0) ws[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) part[(c & 1) * pslot + (int64_t)jj * nrc + rc] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

// qr_col_step with CPW of the panel's columns per workgroup (r06, late; SCS_QR_CPW): workgroup (rc, 0)
// is column c-1's reflector as before, workgroup (rc, 1 + g) takes columns jj = g·CPW .. g·CPW + CPW-1
// (jj = c1 - c: b) of row chunk rc.  Column c and x (the previous column) are loaded once for the CPW
// columns instead of once per column, and the launch has CPW times fewer workgroups; per column the
// same operations in the same order (each thread's rows, wave sums, the ws combine, the previous
// column's partials summed in chunk order by one lane each), so the same bits.
template <int CPW, int RC>
__global__ __launch_bounds__(256) void qr_col_step_g(double* __restrict__ A, int64_t ld, int64_t npad, int64_t c,
                                                     int64_t c0, int64_t c1, double* __restrict__ b,
                                                     double* __restrict__ part, int64_t pslot, int nrc, int nrc_prev,
                                                     double* __restrict__ rowc, double* __restrict__ xs,
                                                     double* __restrict__ tau, double* __restrict__ V, int64_t ldv) {
  const int rc = blockIdx.x;
  const int g = (int)blockIdx.y - 1;
  const int tid = threadIdx.x;
  const bool has_prev = c > c0;
  const int64_t pv = c - 1;
  const int64_t rbeg = has_prev ? pv : c;
  const int64_t r0 = rbeg + (int64_t)rc * RC, r1 = min(r0 + RC, npad);
  const int jmax = (int)(c1 - c);   // jj = jmax: b
  __shared__ double sh[3 + CPW + 1];
  __shared__ double ws[CPW][4];
  __shared__ double sxx[QR_MAXRC], sbc[QR_MAXRC], sbj[CPW][QR_MAXRC];
  const double* x = xs + (pv & 1) * npad;
  const double* colc = (c < c1) ? A + c * ld : b;
  constexpr int NPF = RC / 256;
  double pac[NPF], px[NPF], paj[CPW][NPF];
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int64_t r = r0 + tid + 256 * k;
    const bool in = r < r1;
    pac[k] = (in && g >= 0) ? colc[r] : 0.0;
    px[k] = (in && has_prev) ? x[r] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < CPW; ++q) {
    const int jj = g * CPW + q;
    const bool live = g >= 0 && jj <= jmax;
    const double* colj = (jj < jmax) ? A + (c + jj) * ld : b;
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int64_t r = r0 + tid + 256 * k;
      paj[q][k] = (live && r < r1) ? colj[r] : 0.0;
    }
  }
  // the previous column's chunk partials: staged by wave 0 into LDS (any chunk count up to QR_MAXRC)
  const bool staged = has_prev && nrc_prev <= QR_MAXRC;
  const double* pp = part + (pv & 1) * pslot;
  if (staged && tid < 64) {
    for (int q = tid; q < nrc_prev; q += 64) {
      sxx[q] = pp[q];
      if (c < c1) sbc[q] = pp[(c - pv) * nrc_prev + q];
#pragma unroll
      for (int u = 0; u < CPW; ++u) {
        const int jj = g * CPW + u;
        if (g >= 0 && jj <= jmax) sbj[u][q] = pp[(c + jj - pv) * nrc_prev + q];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // lanes 0 .. CPW of wave 0: the reflector (every lane the same sums in the same order) and one
  // tau · vᵀ a_j each (lane CPW: column c's)
  if (tid <= CPW) {
    double t = 0.0, sc = 0.0, beta = 0.0, tw = 0.0;
    if (has_prev) {
      const double* rp = rowc + (pv & 1) * (QB + 2);
      const double alpha = rp[0];
      double xx = 0.0;
      if (staged)
        for (int q = 0; q < nrc_prev; ++q) xx += sxx[q];
      else
        for (int q = 0; q < nrc_prev; ++q) xx += pp[q];
      beta = alpha;
      if (xx > 0.0) {
        beta = -copysign(sqrt(alpha * alpha + xx), alpha);
        t = (beta - alpha) / beta;
        sc = 1.0 / (alpha - beta);
      }
      const int jj = tid < CPW ? g * CPW + tid : 0;   // lane CPW: column c (jj = 0)
      const bool want = tid < CPW ? (g >= 0 && jj <= jmax) : (c < c1);
      if (want) {
        const double* sb = tid < CPW ? sbj[tid] : sbc;
        const int64_t j = c + jj;
        double d = 0.0;
        if (staged)
          for (int q = 0; q < nrc_prev; ++q) d += sb[q];
        else
          for (int q = 0; q < nrc_prev; ++q) d += pp[(j - pv) * nrc_prev + q];
        tw = t * (rp[j - pv] + sc * d);
      }
    }
    if (tid == 0) {
      sh[0] = t;
      sh[1] = sc;
      sh[2] = beta;
    }
    sh[3 + tid] = tw;
  }
  __syncthreads();
  const double t = sh[0], sc = sh[1];
  if (g < 0) {   // column pv: V, its R entries, tau
    if (!has_prev) return;
    const int64_t vc = (pv - c0) * ldv;
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int64_t r = r0 + tid + 256 * k;
      if (r < r1 && r > pv) V[vc + (r - c0)] = px[k] * sc;
    }
    if (rc == 0) {
      for (int64_t r = c0 + tid; r <= pv; r += 256) V[vc + (r - c0)] = (r == pv) ? 1.0 : 0.0;
      if (tid == 0) {
        A[pv * ld + pv] = sh[2];
        if (pv - 1 >= c0) A[pv * ld + pv - 1] = x[pv - 1];   // R(pv-1, pv): updated by launch pv
        tau[pv - c0] = t;
      }
    }
    return;
  }
  double* xo = xs + (c & 1) * npad;
  const double twc = sh[3 + CPW];
  double s[CPW];
#pragma unroll
  for (int q = 0; q < CPW; ++q) s[q] = 0.0;
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int64_t r = r0 + tid + 256 * k;
    if (r >= r1) continue;
    const double v = has_prev ? ((r == pv) ? 1.0 : px[k] * sc) : 0.0;
    const double ac = has_prev ? pac[k] - twc * v : pac[k];
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const int jj = g * CPW + q;
      if (jj > jmax) continue;
      double aj = paj[q][k];
      if (has_prev) aj -= sh[3 + q] * v;
      if (jj == 0 && c < c1) xo[r] = aj;              // column c itself: to the scratch column
      else if (has_prev) ((jj < jmax) ? A + (c + jj) * ld : b)[r] = aj;   // later columns and b: in place
      if (r == c) rowc[(c & 1) * (QB + 2) + jj] = aj;
      if (r > c) s[q] += ac * aj;
    }
  }
  if (c >= c1) return;
#pragma unroll
  for (int q = 0; q < CPW; ++q) {
    const double w = wave_sum(s[q]);
    if ((tid & 63) == 0) ws[q][tid >> 6] = w;
  }
  __syncthreads();
  if (tid < CPW) {
    const int jj = g * CPW + tid;
    if (jj <= jmax) part[(c & 1) * pslot + (int64_t)jj * nrc + rc] = ((ws[tid][0] + ws[tid][1]) + ws[tid][2]) + ws[tid][3];
  }
}

// SCS_QR_CPW (read per call): panel columns per workgroup of the column step, unset / 2 (default) | 4 | 8,
// 1 = qr_col_step.  probe_qr alternated, same box (profiles/r06/qr_cpw/): n = 16384 292.9 -> 277.8-278.0 ms,
// 8192 84.9-85.3 -> 83.1-83.8 ms; 4: 300-301 / 95 ms, 8: 361 / 123 ms (a quarter / an eighth of the
// workgroups, each thread's loads in series: too little memory parallelism per launch)
// SCS_QR_RC (read per call; the grouped step only): rows per partial-sum chunk, 256 | unset / 512 | 1024.
// Another chunking is another summation order of the column norms and dots (checked against LAPACK, as
// every QR here).  probe_qr alternated with CPW = 2 (profiles/r06/qr_rc/): n = 8192 83.2-83.5 -> 79.7 ms,
// 2048 14.6 -> 13.5 ms, 16384 277.7-279.9 -> 277.7-277.8 ms; 256: 82.2-82.8 / 13.1 / 304.8-305.3 ms;
// CPW = 4 slower at every chunk
static int qr_rc() {
  const char* e = getenv("SCS_QR_RC");
  const int v = e ? atoi(e) : 512;
  return (v == 256 || v == 1024) ? v : 512;
}

template <int CPW, int RC>
static void qr_step_launch(int nrc_c, unsigned gy, hipStream_t st, double* A, int64_t ld, int64_t npad, int64_t c,
                           int64_t c0, int64_t c1, double* b, double* part, int64_t pslot, int nrc_prev, double* rowc,
                           double* xs, double* tau, double* V) {
  hipLaunchKernelGGL((qr_col_step_g<CPW, RC>), dim3((unsigned)nrc_c, gy), dim3(256), 0, st, A, ld, npad, c, c0, c1, b,
                     part, pslot, nrc_c, nrc_prev, rowc, xs, tau, V, npad);
}

static int qr_cpw() {
  const char* e = getenv("SCS_QR_CPW");
  const int v = e ? atoi(e) : 2;
  return (v == 2 || v == 4 || v == 8) ? v : 1;
}

static bool qr_stage() {   // read per call (A/B): SCS_QR_STAGE=0 thread 0 loads the partials itself (r05)
  const char* e = getenv("SCS_QR_STAGE");
  return !(e && e[0] == '0');
}

static bool qr_step_fused() {   // read per call (A/B)
  const char* e = getenv("SCS_QR_STEP");
  return !(e && e[0] == '0');
}

// ---- the panel as ONE cooperative launch (r06, opt-in: SCS_QR_COOP=1; measured slower than the per-column
// launches above, see qr_coop_mode).  The LU's cooperative panel (lu.hip) transposed to the QR: workgroup g
// (NT = 512 threads: 4 row groups x 128 columns) holds the panel's rows [128 g, 128 g + 128) in registers,
// column-major -- thread (j, rg) column j, rows 32 rg .. 32 rg + 31 (a wave: one row range, 64 columns) --
// and b in LDS, through the 128 column steps.  Per column c ONE grid-wide hand-off: every workgroup
// publishes its record (c) -- for the panel's columns j >= c the partial Σ_{r > c} a_rc a_rj over its rows
// (j = c: Σ x_r², dlarfg's xnorm²) and the same for b -- as data-tagged 8-byte granules (tag = panel·256 +
// c + 1, zeroed once per factorization, two slots by column parity as the LU's records), and workgroup 0 the
// row c itself (alpha = a_cc, a_cj, b_c).  Every workgroup sweeps all G records (4 threads per slot,
// records part, part + 4, ...; the parts then in order: the same sums, beta, tau and w_j = vᵀ a_j in every
// workgroup), then applies reflector c to its rows of columns j > c and b (A_j -= tau (a_cj + sc d_j) v,
// v_c = 1, v_r = x_r sc: LAPACK's dlarf arithmetic), and in the same pass forms record (c + 1) from the
// UPDATED column c + 1 (x'_r recomputed from an LDS copy of column c + 1, so no barrier separates the update
// from the next column's partials).  Three LDS barriers + one memory hop per column instead of a kernel
// boundary.  A sweep past its bound (a workgroup that never became resident) stores info = -1 and the abort
// word; the host then redoes the whole solve from a saved copy by the per-column launches (scsopt.cpp
// qr_run).  Sums differ from the per-column launches' order (the QR is checked against LAPACK within
// tolerance, not bitwise).
constexpr int QC_RPT = 32;               // rows per thread
constexpr int QC_MAXWG = 512;            // workgroups at most
constexpr int QC_SWK = 4;                // records per sweep thread in flight (16: slower, the fabric's load rate)
constexpr int QC_SL = 130;               // record slots: the panel's columns, b (128), pad
constexpr int QC_BS = QB;                // b's slot
constexpr int64_t QC_REC = 0;                                    // records [2][MAXWG][SL] x 2 granules
constexpr int64_t QC_ROW = QC_REC + 2LL * QC_MAXWG * QC_SL * 2;   // row c [2][SL] x 2
constexpr int64_t QC_ABORT = QC_ROW + 2LL * QC_SL * 2;
constexpr int64_t QC_WORDS = QC_ABORT + 16;
constexpr unsigned QC_SPIN_MAX = 1u << 19;   // sweeps before giving up (~0.5 s; SCS_QR_COOP_SPIN overrides)
typedef __attribute__((address_space(1))) unsigned long long qc_gu64;

#ifdef QR_PROF
// probe_qr -DQR_PROF: workgroup 0's thread 0 splits each column of every cooperative panel into
// sweep | reflector + v | rows | B2 | publish (s_memrealtime, 100 MHz ticks, summed) + columns
__device__ unsigned long long qr_prof[32];
#define QRP_MARK(v) const long long v = (g == 0 && tid == 0) ? (long long)__builtin_amdgcn_s_memrealtime() : 0
#define QRP_ADD(k, a, b) if (g == 0 && tid == 0) qr_prof[k] += (unsigned long long)((b) - (a))
// the last wave's column pass (slot 6)
#define QRP_MARK2(v) const long long v = (g == 0 && (tid & 63) == 0) ? (long long)__builtin_amdgcn_s_memrealtime() : 0
#define QRP_ADD2(k, a, b) if (g == 0 && (tid & 63) == 0) qr_prof[k] += (unsigned long long)((b) - (a))
#else
#define QRP_MARK2(v)
#define QRP_ADD2(k, a, b)
#define QRP_MARK(v)
#define QRP_ADD(k, a, b)
#endif

__device__ __forceinline__ void qc_put(unsigned long long* p, unsigned long long x) {
  __hip_atomic_store((qc_gu64*)p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long qc_get(const unsigned long long* p) {
  return __hip_atomic_load((qc_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a double as two granules {tag, low word}, {tag, high word}
__device__ __forceinline__ void qc_put_d(unsigned long long* p, unsigned tag, double v) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(v), t = (unsigned long long)tag << 32;
  qc_put(p, t | (bits & 0xffffffffull));
  qc_put(p + 1, t | (bits >> 32));
}
__device__ __forceinline__ double qc_get_d(const unsigned long long* p, unsigned tag, bool& ok) {
  const unsigned long long x0 = qc_get(p), x1 = qc_get(p + 1);
  ok = ok && (unsigned)(x0 >> 32) == tag && (unsigned)(x1 >> 32) == tag;
  return __longlong_as_double((long long)((x0 & 0xffffffffull) | (x1 << 32)));
}

// Panel [c0, c0 + 128) of the column-major A (rows c0 .. c0 + h - 1), b rows likewise; tau[0 .. 128) and V
// (rows relative to c0: zeros above the diagonal, one on it, v below) as qr_col_step leaves them; A gets R
// on and above the diagonal (below it the columns as they stood before their own reflector: unused, as with
// the column steps).  Per column, after the sweep: the ROW PASS (thread r < 256: row r of the workgroup)
// forms v_r (into LDS and V), column c + 1's updated x'_r, and b's update and partial; then the COLUMN PASS
// (thread (j, rg)) updates its 32 rows of column j > c and forms its partial of record (c + 1) -- two
// fma per element, no branch, the owner lane idle (tw = 0).
template <int NT>
__global__ __launch_bounds__(NT) void qr_panel_coop_kernel(double* __restrict__ A, int64_t ld, int64_t c0, int64_t h,
                                                              double* __restrict__ b, unsigned long long* gran,
                                                              unsigned tagbase, double* __restrict__ tau,
                                                              double* __restrict__ V, int64_t ldv, int* info,
                                                              unsigned spin_max) {
  constexpr int QC_RG = NT / QB;             // row groups (and sweep parts)
  constexpr int QC_RW = QC_RG * QC_RPT;      // rows per workgroup (>= QB: row c is always workgroup 0's)
  __shared__ double sX[2][QC_RW];      // column c as its owner holds it (x_r), by column parity
  __shared__ double sN[2][QC_RW];      // column c + 1 before reflector c
  __shared__ double sb[QC_RW];         // b (row r: the row pass's thread r)
  __shared__ double sV[QC_RW], sXN[QC_RW];   // this column's v_r; column c + 1's updated x'_r (0 at r <= c + 1)
  __shared__ double sp[QC_RG][QC_SL];  // the row groups' partials of the next record
  __shared__ double red[QC_SL][QC_RG]; // the sweep: per slot, per part
  __shared__ double srow[QC_SL];       // row c
  __shared__ double sbeta[QB];         // R(c, c)
  __shared__ int s_dead;
  const int tid = threadIdx.x, g = blockIdx.x, G = gridDim.x;
  const int j = tid & (QB - 1);
  const int rg = __builtin_amdgcn_readfirstlane(tid >> 7), jlo = __builtin_amdgcn_readfirstlane(tid & 64);   // per wave
  const int r0w = g * QC_RW;                // the workgroup's first row (panel-local; h <= 65536)
  const int rw0 = rg * QC_RPT;              // this thread's first row within the workgroup
  const int rb = r0w + rw0;                 // ... panel-local
  const bool rows_in = rb < h;              // (h and rb are multiples of 32: all of a thread's rows or none)
  const int rr = r0w + tid;                 // the row pass: this thread's row (tid < QC_RW)
  if (gran[QC_ABORT] != 0) return;
  if (spin_max == 0) {   // (tests: every workgroup gives up at once, as one that never became resident would)
    if (tid == 0) {
      *info = -1;
      gran[QC_ABORT] = 1;
    }
    return;
  }
  double v[QC_RPT];
  {
    const double* src = A + (c0 + j) * ld + c0 + (rows_in ? rb : 0);
#pragma unroll
    for (int i = 0; i < QC_RPT; ++i) v[i] = src[i];
    if (!rows_in)
#pragma unroll
      for (int i = 0; i < QC_RPT; ++i) v[i] = 0.0;
  }
  if (tid < QC_RW) sb[tid] = rr < h ? b[c0 + rr] : 0.0;
  if (tid == 0) s_dead = 0;
  if (j == 0)
#pragma unroll
    for (int i = 0; i < QC_RPT; ++i) sX[0][rw0 + i] = v[i];
  if (j == 1)
#pragma unroll
    for (int i = 0; i < QC_RPT; ++i) sN[1][rw0 + i] = v[i];
  __syncthreads();
  auto rec_at = [&](int c, int gg, int s) { return gran + QC_REC + (((int64_t)(c & 1) * QC_MAXWG + gg) * QC_SL + s) * 2; };
  auto row_at = [&](int c, int s) { return gran + QC_ROW + ((int64_t)(c & 1) * QC_SL + s) * 2; };
  auto publish_record = [&](int c) {   // after the barrier that completes sp: slots c .. 127 and b
    if (tid >= c && tid <= QC_BS) {
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < QC_RG; ++q) s += sp[q][tid];
      qc_put_d(rec_at(c, g, tid), tagbase + (unsigned)c + 1, s);
    }
  };
  auto b_partial = [&](double pb) {   // the row pass: b's partial per row group (32 rows: half a wave)
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) pb += __shfl_xor(pb, o, 64);
    if ((tid & 31) == 0) sp[tid >> 5][QC_BS] = pb;
  };
  {   // record (0): the panel's columns as loaded
    double p = 0.0;
#pragma unroll
    for (int i = 0; i < QC_RPT; ++i) p = fma(rb + i > 0 ? sX[0][rw0 + i] : 0.0, v[i], p);
    sp[rg][j] = p;
    if (tid < QC_RW) b_partial((rr > 0 ? sX[0][tid] : 0.0) * sb[tid]);
    if (g == 0 && rg == 0) qc_put_d(row_at(0, j), tagbase + 1, v[0]);   // row 0
    if (g == 0 && tid == 0) qc_put_d(row_at(0, QC_BS), tagbase + 1, sb[0]);
  }
  __syncthreads();
  publish_record(0);
  for (int c = 0; c < QB; ++c) {
    const unsigned tag = tagbase + (unsigned)c + 1;
    QRP_MARK(t_a);
    {   // the sweep of record (c) and row c: thread (slot s, part) sums records part, part + 8, ... of slot s
      const int s = tid / QC_RG, part = tid % QC_RG;
      const int sa = s >= c ? s : -1;
      const bool hb = s == 0;   // and b's slot
      const int rs = (part == 1 && s >= c) ? s : ((part == 2 && s == 0) ? QC_BS : -1);
      double aa = 0.0, ab = 0.0, rv = 0.0;
      for (unsigned spins = 0;;) {
        bool ok = true;
        aa = 0.0;
        ab = 0.0;
        for (int k0 = part; k0 < G; k0 += QC_SWK * QC_RG) {   // QC_SWK records in flight
          double xs[QC_SWK];
#pragma unroll
          for (int q = 0; q < QC_SWK; ++q) {
            const int k = k0 + q * QC_RG;
            xs[q] = (sa >= 0 && k < G) ? qc_get_d(rec_at(c, k, sa), tag, ok) : 0.0;
          }
#pragma unroll
          for (int q = 0; q < QC_SWK; ++q) aa += xs[q];
          if (hb) {
#pragma unroll
            for (int q = 0; q < QC_SWK; ++q) {
              const int k = k0 + q * QC_RG;
              xs[q] = k < G ? qc_get_d(rec_at(c, k, QC_BS), tag, ok) : 0.0;
            }
#pragma unroll
            for (int q = 0; q < QC_SWK; ++q) ab += xs[q];
          }
        }
        if (rs >= 0) rv = qc_get_d(row_at(c, rs), tag, ok);
        if (ok) break;
        if (++spins > spin_max) {
          *info = -1;
          gran[QC_ABORT] = 1;
          s_dead = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (sa >= 0) red[sa][part] = aa;
      if (hb) red[QC_BS][part] = ab;
      if (rs >= 0) srow[rs] = rv;
    }
    __syncthreads();
    if (s_dead) return;
    QRP_MARK(t_b);
    // the reflector (dlarfg) -- every thread the same sums in the same order
    double xx = 0.0;
#pragma unroll
    for (int q = 0; q < QC_RG; ++q) xx += red[c][q];
    const double alpha = srow[c];
    double t = 0.0, sc = 0.0, beta = alpha;
    if (xx > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + xx), alpha);
      t = (beta - alpha) / beta;
      sc = 1.0 / (alpha - beta);
    }
    auto twf = [&](int s) {   // tau · vᵀ a_s (v_c = 1)
      double d = 0.0;
#pragma unroll
      for (int q = 0; q < QC_RG; ++q) d += red[s][q];
      return t * (srow[s] + sc * d);
    };
    const bool last = c + 1 >= QB;
    const double tw = j > c ? twf(j) : 0.0;
    if (tid < QC_RW) {   // the row pass
      const double vr = rr < c ? 0.0 : (rr == c ? 1.0 : sX[c & 1][tid] * sc);
      sV[tid] = vr;
      if (rr < h) V[(int64_t)c * ldv + rr] = vr;
      const double bb = fma(-twf(QC_BS), vr, sb[tid]);
      sb[tid] = bb;
      if (!last) {
        const double xn = rr > c + 1 ? fma(-twf(c + 1), vr, sN[(c + 1) & 1][tid]) : 0.0;
        sXN[tid] = xn;
        b_partial(xn * bb);
        if (g == 0 && rr == c + 1) qc_put_d(row_at(c + 1, QC_BS), tag + 1, bb);
      }
    }
    if (tid == 0) {
      sbeta[c] = beta;
      if (g == 0) tau[c] = t;
    }
    __syncthreads();
    QRP_MARK(t_c);
    QRP_MARK2(u_c);
    double p = 0.0;
    if (rows_in && jlo + 63 > c && rb + QC_RPT - 1 >= c) {   // the column pass: lanes j > c, rows >= c
      double rowv = 0.0, pq[4] = {0.0, 0.0, 0.0, 0.0};   // four partial chains, summed in order at the end
#pragma unroll
      for (int i0 = 0; i0 < QC_RPT; i0 += 8) {   // 8 rows' v_r and x'_r loaded before their updates
        v2d vv[4], xv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          vv[q] = *(const v2d*)(sV + rw0 + i0 + 2 * q);
          xv[q] = *(const v2d*)(sXN + rw0 + i0 + 2 * q);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int i = i0 + q;
          const double a = fma(-tw, vv[q >> 1][q & 1], v[i]);
          pq[q & 3] = fma(xv[q >> 1][q & 1], a, pq[q & 3]);
          rowv = (rb + i == c + 1) ? a : rowv;
          v[i] = a;
        }
      }
      p = (pq[0] + pq[1]) + (pq[2] + pq[3]);
      if (g == 0 && !last && rb <= c + 1 && c + 1 < rb + QC_RPT && j > c)   // row c + 1 for the next step
        qc_put_d(row_at(c + 1, j), tag + 1, rowv);
    }
    QRP_MARK(t_d);
    QRP_MARK2(u_d);
    QRP_ADD2(8 + (tid >> 6), u_c, u_d);
    if (last) break;
    if (j == c + 1)
#pragma unroll
      for (int i = 0; i < QC_RPT; ++i) sX[(c + 1) & 1][rw0 + i] = v[i];
    if (j == c + 2)
#pragma unroll
      for (int i = 0; i < QC_RPT; ++i) sN[(c + 2) & 1][rw0 + i] = v[i];
    sp[rg][j] = p;
    QRP_MARK2(u_e);
    QRP_ADD2(16 + (tid >> 6), u_d, u_e);
    __syncthreads();
    QRP_MARK(t_e);
    publish_record(c + 1);
    QRP_MARK(t_f);
    QRP_ADD(0, t_a, t_b);
    QRP_ADD(1, t_b, t_c);
    QRP_ADD(2, t_c, t_d);
    QRP_ADD(3, t_d, t_e);
    QRP_ADD(4, t_e, t_f);
    QRP_ADD(5, 0, 1);
  }
  __syncthreads();   // (the last row pass's b, sbeta, before they go back)
  if (rows_in) {
    double* dst = A + (c0 + j) * ld + c0 + rb;
#pragma unroll
    for (int i = 0; i < QC_RPT; ++i) dst[i] = (rb + i == j) ? sbeta[j] : v[i];
  }
  if (tid < QC_RW && rr < h) b[c0 + rr] = sb[tid];
}

// T (QB x QB, column-major, upper) of the panel's compact WY form from Gv = VᵀV (dlarft forward,
// columnwise): T(i, i) = tau_i, T(0:i, i) = -tau_i T(0:i, 0:i) Gv(0:i, i)
__global__ __launch_bounds__(QB) void qr_build_t(const double* __restrict__ Gv, const double* __restrict__ tau, int nb,
                                                 double* __restrict__ T) {
  __shared__ double Ts[QB * QB];
  __shared__ double z[QB];
  const int t = threadIdx.x;
  for (int e = t; e < QB * QB; e += QB) Ts[e] = 0.0;
  __syncthreads();
  for (int i = 0; i < nb; ++i) {
    const double ti = tau[i];
    if (t < i) z[t] = -ti * Gv[(int64_t)i * QB + t];   // -tau_i Vᵀ v_i (rows 0..i-1)
    __syncthreads();
    if (t < i) {   // T(0:i,0:i) upper: Σ_{q >= t} T(t, q) z(q), eight independent partial sums
      double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      int q = t;
      for (; q + 7 < i; q += 8)
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u] += Ts[(q + u) * QB + t] * z[q + u];
      for (; q < i; ++q) s[0] += Ts[q * QB + t] * z[q];
      Ts[i * QB + t] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    }
    if (t == i) Ts[i * QB + i] = ti;
    __syncthreads();
  }
  for (int e = t; e < QB * QB; e += QB) T[e] = Ts[e];
}

// Vt (QB x rows, column-major: Vt[i + r QB]) = Vᵀ for the trailing update's A1 operand
__global__ __launch_bounds__(256) void qr_transpose_v(const double* __restrict__ V, int64_t ldv, int64_t rows,
                                                      double* __restrict__ Vt) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  for (int i = 0; i < QB; ++i) Vt[r * QB + i] = V[(int64_t)i * ldv + r];
}

__global__ void qr_fill_kernel(double* __restrict__ p, int64_t n, double v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// the column-major system with the identity padding the QR expects: from a symmetric (or
// symmetrized) column-major matrix in place (pad only), or transposed from a row-major one
__global__ void qr_pad_kernel(double* __restrict__ A, int64_t ld, int64_t n, int64_t npad) {
  const int64_t i = n + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < npad) A[i * ld + i] = 1.0;
}

__global__ void qr_transpose_sq(const double* __restrict__ S, int64_t lds, double* __restrict__ D, int64_t ldd, int64_t n,
                                int64_t npad) {
  const int64_t j = blockIdx.y;   // destination column
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npad; i += (int64_t)gridDim.x * blockDim.x)
    D[j * ldd + i] = (i < n && j < n) ? S[i * lds + j] : (i == j ? 1.0 : 0.0);
}

hipError_t qr_prepare(double* A, int64_t ld, int64_t n, int64_t npad, hipStream_t st) {
  if (npad > n)
    hipLaunchKernelGGL(qr_pad_kernel, dim3((unsigned)((npad - n + 255) / 256)), dim3(256), 0, st, A, ld, n, npad);
  return hipGetLastError();
}

hipError_t qr_from_rowmajor(const double* S, int64_t lds, double* D, int64_t ldd, int64_t n, int64_t npad,
                            hipStream_t st) {
  hipLaunchKernelGGL(qr_transpose_sq, dim3((unsigned)((npad + 255) / 256 > 64 ? 64 : (npad + 255) / 256), (unsigned)npad),
                     dim3(256), 0, st, S, lds, D, ldd, n, npad);
  return hipGetLastError();
}

static void qr_free_bufs(QRAux* a) {
  for (double** p : {&a->part, &a->tw, &a->tau, &a->scal, &a->V, &a->Vt, &a->Wm, &a->Ym, &a->Gv, &a->T, &a->ones,
                     &a->W, &a->rowc, &a->xs, &a->kpart, &a->V2, &a->T2, &a->Wm2, &a->Ym2, &a->Vt2, &a->kpart2})
    if (*p) {
      (void)hipFree(*p);
      *p = nullptr;
    }
  if (a->tiles) (void)hipFree(a->tiles);
  a->tiles = nullptr;
  a->rect_off.clear();
  if (a->kwork) (void)hipFree(a->kwork);
  a->kwork = nullptr;
  a->klists.clear();
  if (a->flags) (void)hipFree(a->flags);
  a->flags = nullptr;
  a->err = nullptr;
  if (a->gran) (void)hipFree(a->gran);
  a->gran = nullptr;
  a->cinfo = nullptr;
  if (a->st2) (void)hipStreamDestroy(a->st2);
  if (a->evp) (void)hipEventDestroy(a->evp);
  if (a->evb) (void)hipEventDestroy(a->evb);
  a->st2 = nullptr;
  a->evp = a->evb = nullptr;
  a->gen = 0;
  a->npad = 0;
}

hipError_t qr_aux_init(QRAux* a, int64_t npad, hipStream_t st) {
  if (a->npad == npad) return hipSuccess;
  qr_free_bufs(a);
  const int64_t nrc = (npad + 255) / 256;   // (the partials' slots: the smallest chunk, SCS_QR_RC = 256)
  const int nbk = (int)(npad / QB);
  hipError_t e = hipSuccess;
  auto al = [&](double** p, size_t n) {
    if (e == hipSuccess) e = hipMalloc(p, sizeof(double) * std::max<size_t>(n, 1));
  };
  al(&a->part, 2 * (size_t)(QB + 2) * (nrc + 1));   // the fused step: two parity slots of (QB + 1)(nrc + 1)
  al(&a->rowc, 2 * (size_t)(QB + 2));
  al(&a->xs, 2 * (size_t)npad);
  al(&a->tw, QB + 2);
  al(&a->tau, QB);
  al(&a->scal, 2);
  al(&a->V, (size_t)npad * QB);
  al(&a->Vt, (size_t)npad * QB);
  al(&a->Wm, (size_t)npad * QB);
  al(&a->Ym, (size_t)npad * QB);
  al(&a->Gv, (size_t)QB * QB);
  al(&a->T, (size_t)QB * QB);
  al(&a->ones, (size_t)npad + QB);
  al(&a->W, (size_t)npad * QB);
  // tile lists, one launch per product of a panel: [row 0: (0, j), j < nbk] then, per panel p, the
  // rectangle (i, j), i < nbk - p (rows of the panel's reflectors), j < nbk - p - 1 (trailing column
  // blocks), j-major -- the update A_trail -= V Y as ONE launch (was one launch per column block)
  std::vector<int2> tl;
  for (int j = 0; j < nbk; ++j) tl.push_back(make_int2(0, j));
  a->rect_off.assign((size_t)nbk, 0);
  for (int p = 0; p < nbk; ++p) {
    a->rect_off[(size_t)p] = (int64_t)tl.size();
    for (int j = 0; j < nbk - p - 1; ++j)
      for (int i = 0; i < nbk - p; ++i) tl.push_back(make_int2(i, j));
  }
  // K-split work lists (qr_ksplit): per panel p, list 2p = Gv (one tile), 2p + 1 = Wm (ntr tiles); item
  // (0, j, piece s, slot j·nsplit + s) at position (i % 8)·seglen + i / 8 (the Gram kernel's XCD
  // segments), padding bi = -1; at most QR_KMAXITEMS items per list
  std::vector<int4> kw;
  a->klists.clear();
  size_t kmax = 1;
  for (int p = 0; p < nbk; ++p) {
    const int64_t rows = npad - (int64_t)p * QB;
    for (int nj : {1, std::max(nbk - p - 1, 1)}) {
      int ns = (int)((rows + QR_KS - 1) / QR_KS);
      ns = std::max(1, std::min(ns, QR_KMAXITEMS / nj));
      const int n = nj * ns, seglen = (n + 7) / 8;
      QRAux::KList L;
      L.off = (int64_t)kw.size();
      L.seglen = seglen;
      L.nsplit = ns;
      L.nj = nj;
      a->klists.push_back(L);
      kw.resize(kw.size() + (size_t)8 * seglen, make_int4(-1, 0, 0, 0));
      for (int i = 0; i < n; ++i) {
        const int j = i / ns, s = i % ns;
        kw[(size_t)L.off + (size_t)(i % 8) * seglen + i / 8] = make_int4(0, j, s, j * ns + s);
      }
      kmax = std::max(kmax, (size_t)n);
    }
  }
  // the lookahead's Wm lists, klists[2 nbk + 2p + {0, 1}]: the next panel's column block and the
  // trailing column blocks beyond it, K split as the whole update's list 2p + 1 (the same pieces and
  // combine order per column block: the same bits)
  for (int p = 0; p < 2 * nbk; ++p) {
    const int pp = p / 2;
    const int64_t rows = npad - (int64_t)pp * QB;
    const int nj = (p & 1) ? std::max(nbk - pp - 2, 1) : 1;
    int ns = (int)((rows + QR_KS - 1) / QR_KS);
    ns = std::max(1, std::min(ns, QR_KMAXITEMS / std::max(nbk - pp - 1, 1)));
    const int n = nj * ns, seglen = (n + 7) / 8;
    QRAux::KList L;
    L.off = (int64_t)kw.size();
    L.seglen = seglen;
    L.nsplit = ns;
    L.nj = nj;
    a->klists.push_back(L);
    kw.resize(kw.size() + (size_t)8 * seglen, make_int4(-1, 0, 0, 0));
    for (int i = 0; i < n; ++i) {
      const int j = i / ns, s = i % ns;
      kw[(size_t)L.off + (size_t)(i % 8) * seglen + i / 8] = make_int4(0, j, s, j * ns + s);
    }
    kmax = std::max(kmax, (size_t)n);
  }
  if (e == hipSuccess) e = hipMalloc(&a->kwork, sizeof(int4) * std::max<size_t>(kw.size(), 1));
  if (e == hipSuccess && !kw.empty())
    e = hipMemcpyAsync(a->kwork, kw.data(), sizeof(int4) * kw.size(), hipMemcpyHostToDevice, st);
  al(&a->kpart, kmax * QB * QB);
  al(&a->kpart2, kmax * QB * QB);
  al(&a->V2, (size_t)npad * QB);
  al(&a->T2, (size_t)QB * QB);
  al(&a->Wm2, (size_t)npad * QB);
  al(&a->Ym2, (size_t)npad * QB);
  al(&a->Vt2, (size_t)npad * QB);
  if (e == hipSuccess) e = hipMalloc(&a->tiles, sizeof(int2) * std::max<size_t>(tl.size(), 1));
  if (e == hipSuccess && !tl.empty())
    e = hipMemcpyAsync(a->tiles, tl.data(), sizeof(int2) * tl.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMalloc(&a->flags, sizeof(unsigned) * (size_t)nbk + sizeof(int));
  if (e == hipSuccess) e = hipMemsetAsync(a->flags, 0, sizeof(unsigned) * (size_t)nbk + sizeof(int), st);
  if (e == hipSuccess) a->err = (int*)(a->flags + nbk);
  // the cooperative panel's granules + its info word (zeroed per solve)
  if (e == hipSuccess) e = hipMalloc(&a->gran, sizeof(unsigned long long) * (QC_WORDS + 2));
  if (e == hipSuccess) a->cinfo = (int*)(a->gran + QC_WORDS);
  if (e == hipSuccess) {
    // ones[0, npad) = +1, ones[npad, npad + QB) = -1 (the Gram kernels' weights)
    hipLaunchKernelGGL(qr_fill_kernel, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, st, a->ones, npad, 1.0);
    hipLaunchKernelGGL(qr_fill_kernel, dim3(1), dim3(QB), 0, st, a->ones + npad, (int64_t)QB, -1.0);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess) a->npad = npad;
  return e;
}

void qr_aux_free(QRAux* a) { qr_free_bufs(a); }

// out(:, 128 j .. 128 j + 127) = Σ_s P[slot j·nsplit + s] (pieces in order): the K-split products
__global__ __launch_bounds__(256) void qr_combine_kernel(const double* __restrict__ P, int nsplit,
                                                         double* __restrict__ out, int64_t ldo) {
  const int j = blockIdx.y;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < QB * QB; e += gridDim.x * 256) {
    const int jl = e / QB, il = e % QB;
    double s = 0.0;
    for (int sp = 0; sp < nsplit; ++sp) s += P[((int64_t)(j * nsplit + sp) * QB + jl) * QB + il];
    out[((int64_t)j * QB + jl) * ldo + il] = s;
  }
}

// Vᵀ B (B = V for the panel's Gv, the trailing columns for Wm) over the panel's rows, K split into
// pieces of at least QR_KS rows so a few tiles with a long K still fill the chip: one launch of the
// column-major Gram kernel over a precomputed work list (qr_aux_init) + one combine launch
static hipError_t qr_ksplit(const double* V, int64_t ldv, const double* B, int64_t ldb, int64_t K, int nj,
                            const QRAux* a, int list, double* out, int64_t ldo, hipStream_t st) {
  const QRAux::KList& L = a->klists[(size_t)list];
  if (L.nj != nj) return hipErrorInvalidValue;
  hipError_t e = gram_launch_work_cm(V, ldv, B, ldb, a->ones, K, a->kwork + L.off, L.seglen, L.nsplit, a->kpart, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(qr_combine_kernel, dim3(16, (unsigned)nj), dim3(256), 0, st, a->kpart, L.nsplit, out, ldo);
  return hipGetLastError();
}

// read per call: SCS_QR_COOP=1 the cooperative panel (opt-in: measured slower than the per-column launches --
// n = 8192 89 vs 83 ms, 16384 318 vs 293 ms -- its per-column record sweep reads G x 129 tagged values per
// workgroup, G² x 129 across the chip, and costs 1.7-5.7 µs as G grows; DESIGN §3 QR)
static int qr_coop_mode() {
  const char* e = getenv("SCS_QR_COOP");
  return e && e[0] == '1';
}

static unsigned qr_coop_spin() {   // read per call: SCS_QR_COOP_SPIN (sweeps; 0 = give up at once, tests)
  const char* e = getenv("SCS_QR_COOP_SPIN");
  return e ? (unsigned)strtoul(e, nullptr, 10) : QC_SPIN_MAX;
}

static int qr_device_cus() {
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return ncu;
}

static int qr_coop_nt() {   // read per call (A/B): SCS_QR_COOP_NT = 512 (default) | 1024
  const char* e = getenv("SCS_QR_COOP_NT");
  return (e && atoi(e) == 1024) ? 1024 : 512;
}

// the first panel needs the most workgroups (npad / rows per workgroup); later panels fewer.  One
// workgroup per CU at most (the 512-thread form holds > 128 registers per lane)
bool qr_coop_wanted(int64_t npad) {
  const int64_t G = ceil_div(npad, (int64_t)(qr_coop_nt() / QB) * QC_RPT);
  return qr_coop_mode() && G <= QC_MAXWG && G <= qr_device_cus();
}

// panel p by the cooperative kernel; false when the runtime refused the launch (the caller runs it by
// column steps)
static bool qr_panel_coop(double* A, int64_t ld, int64_t npad, int p, QRAux* a, double* V, double* b, hipStream_t st) {
  const int64_t c0 = (int64_t)p * QB, h = npad - c0;
  const int nt = qr_coop_nt();
  const int G = (int)ceil_div(h, (int64_t)(nt / QB) * QC_RPT);
  double* pA = A;
  int64_t pld = ld, pc0 = c0, ph = h, pldv = npad;
  double* pb = b;
  unsigned long long* pgran = a->gran;
  unsigned ptag = (unsigned)p << 8, pspin = qr_coop_spin();
  double* ptau = a->tau;
  double* pV = V;
  int* pinfo = a->cinfo;
  void* args[] = {&pA, &pld, &pc0, &ph, &pb, &pgran, &ptag, &ptau, &pV, &pldv, &pinfo, &pspin};
  const void* kern = nt == 1024 ? (const void*)qr_panel_coop_kernel<1024> : (const void*)qr_panel_coop_kernel<512>;
  if (hipLaunchCooperativeKernel(kern, dim3((unsigned)G), dim3(nt), args, 0, st) !=
      hipSuccess) {
    (void)hipGetLastError();
    ++a->coop_refused;
    return false;
  }
  return true;
}

// SCS_QR_LA (read per call; default 0): the lookahead trailing update.  After panel p's block
// reflector (V, T) is formed, the next panel's 128 columns take it on the caller's stream and every
// column beyond them on a bulk stream, which runs beside panel p + 1 (its 129 column-step launches);
// V and T alternate between two buffers by panel parity.  Per tile the same kernels, K pieces and
// combine order as the one-stream update: the same factor bit for bit (test_qr_lookahead_bit_identical).
static bool qr_lookahead() {
  const char* e = getenv("SCS_QR_LA");
  return e && e[0] == '1';
}

// A(:, cb .. cb + 128 nj) -= V T (Vᵀ A(:, cb ..)) over the panel's rows (c0 .. npad): Wm = Vᵀ A_t (K split,
// klists[list]), Ym = Tᵀ Wm, Vt = Vᵀ as K-contiguous columns, A_t -= Vt-features x Ym over the panel's
// update rectangle (tiles i < rows / 128, j < nj: j-major, the first nj columns of panel p's rectangle)
static hipError_t qr_apply_block(double* A, int64_t ld, int64_t npad, int p, int64_t cb, int nj, int list,
                                 const double* V, const double* T, double* Wm, double* Ym, double* Vt, double* kpart,
                                 QRAux* a, hipStream_t s) {
  const int64_t c0 = (int64_t)p * QB, rows = npad - c0;
  double* At = A + cb * ld + c0;
  const QRAux::KList& L = a->klists[(size_t)list];
  if (L.nj != nj) return hipErrorInvalidValue;
  hipError_t e = gram_launch_work_cm(V, npad, At, ld, a->ones, rows, a->kwork + L.off, L.seglen, L.nsplit, kpart, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(qr_combine_kernel, dim3(16, (unsigned)nj), dim3(256), 0, s, kpart, L.nsplit, Wm, (int64_t)QB);
  // Ym = Tᵀ Wm: Ym(i, j) = Σ_q T(q, i) Wm(q, j)
  e = gram_launch_gen(T, QB, Wm, QB, a->ones, 0, QB, a->tiles, nj, Ym, QB, 0, s);
  if (e != hipSuccess) return e;
  // A_t -= V Ym: A(r, j) -= Σ_i Vt(i, r) Ym(i, j) (features r of Vt, K = i)
  hipLaunchKernelGGL(qr_transpose_v, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, V, npad, rows, Vt);
  return gram_launch_gen(Vt, QB, Ym, QB, a->ones + npad, 0, QB, a->tiles + a->rect_off[(size_t)p],
                         (int)(rows / QB) * nj, At, ld, /*ACCUMULATE*/ 2, s);
}

hipError_t qr_solve(double* A, int64_t ld, int64_t npad, QRAux* a, double* b, hipStream_t st) {
  hipError_t e = qr_aux_init(a, npad, st);
  if (e != hipSuccess) return e;
  const int nbk = (int)(npad / QB);
  const bool coop = !a->no_coop && qr_coop_wanted(npad);
  const bool la = qr_lookahead() && nbk > 2;
  if (la) {
    if (!a->st2) e = hipStreamCreateWithFlags(&a->st2, hipStreamNonBlocking);
    if (e == hipSuccess && !a->evp) e = hipEventCreateWithFlags(&a->evp, hipEventDisableTiming);
    if (e == hipSuccess && !a->evb) e = hipEventCreateWithFlags(&a->evb, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  e = hipMemsetAsync(a->gran, 0, sizeof(unsigned long long) * (QC_WORDS + 2), st);   // tags, abort word, cinfo
  if (e != hipSuccess) return e;
  bool bulk = false;   // a bulk update is in flight on st2 (evb recorded after it)
  for (int p = 0; p < nbk; ++p) {
    const int64_t c0 = (int64_t)p * QB, c1 = c0 + QB, rows = npad - c0;
    const int nrc = (int)((rows + QR_RC - 1) / QR_RC);
    const int stage = qr_stage() ? 1 : 0;
    // panel p's reflectors (V) and T: the second buffers on odd panels under the lookahead (the bulk
    // update of panel p - 1 may still read the other pair)
    double* V = (la && (p & 1)) ? a->V2 : a->V;
    double* T = (la && (p & 1)) ? a->T2 : a->T;
    if (coop && qr_panel_coop(A, ld, npad, p, a, V, b, st)) {
      // (the panel, its V, tau and R rows as the column steps leave them)
    } else if (qr_step_fused()) {
      const int64_t pslot = (int64_t)(QB + 1) * ((npad + QR_RC - 1) / QR_RC + 1);
      int nrc_prev = 0;
      for (int64_t c = c0; c <= c1; ++c) {
        const int64_t rbeg = c > c0 ? c - 1 : c;
        const int nrc_c = (int)((npad - rbeg + QR_RC - 1) / QR_RC);
        const int ncol = (int)(c1 - c) + 1;   // columns c .. c1-1 and b
        const int cpw = qr_cpw();
        const int rcg = cpw > 1 ? qr_rc() : QR_RC;   // the grouped step's chunk
        const int nrc_g = (int)((npad - rbeg + rcg - 1) / rcg);
        const int64_t pslot_g = (int64_t)(QB + 1) * ((npad + rcg - 1) / rcg + 1);
        const unsigned gy = 1u + (unsigned)((ncol + cpw - 1) / cpw);
#define QR_STEP(CW, R) qr_step_launch<CW, R>(nrc_g, gy, st, A, ld, npad, c, c0, c1, b, a->part, pslot_g, nrc_prev, \
                                            a->rowc, a->xs, a->tau, V)
        if (cpw > 1) {
          if (cpw == 2) { if (rcg == 256) QR_STEP(2, 256); else if (rcg == 512) QR_STEP(2, 512); else QR_STEP(2, 1024); }
          else if (cpw == 4) { if (rcg == 256) QR_STEP(4, 256); else if (rcg == 512) QR_STEP(4, 512); else QR_STEP(4, 1024); }
          else QR_STEP(8, 1024);
          nrc_prev = nrc_g;
          continue;
        }
#undef QR_STEP
        hipLaunchKernelGGL(qr_col_step, dim3((unsigned)nrc_c, (unsigned)(ncol + 1)), dim3(256), 0, st, A, ld, npad,
                             c, c0, c1, b, a->part, pslot, nrc_c, nrc_prev, a->rowc, a->xs, a->tau, V, npad, stage);
        nrc_prev = nrc_c;
      }
    } else
    for (int64_t c = c0; c < c1; ++c) {
      const int ncol = (int)(c1 - c) + 1;
      hipLaunchKernelGGL(qr_col_partials, dim3((unsigned)nrc, (unsigned)ncol), dim3(256), 0, st, A, ld, npad, c, c1, b,
                         a->part, nrc);
      hipLaunchKernelGGL(qr_col_reflect, dim3(1), dim3(256), 0, st, A, ld, c, c1, c0, b, a->part, nrc, a->tw, a->tau,
                         a->scal, V, npad);
      hipLaunchKernelGGL(qr_col_update, dim3((unsigned)((npad - c + 255) / 256), (unsigned)ncol), dim3(256), 0, st, A,
                         ld, npad, c, c1, c0, b, a->tw, a->scal, V, npad);
    }
    const int ntr = nbk - p - 1;   // trailing column blocks
    if (ntr == 0) break;
    // T from Gv = VᵀV over the panel's rows (K split)
    e = qr_ksplit(V, npad, V, npad, rows, 1, a, 2 * p, a->Gv, QB, st);
    if (e != hipSuccess) return e;
    if (qr_step_fused()) {   // T by MFMA doubling (chol.hip wy_t_kernel); SCS_QR_STEP=0: the plain recurrence
      e = wy_t_build(a->Gv, a->tau, T, st);
      if (e != hipSuccess) return e;
    } else {
      hipLaunchKernelGGL(qr_build_t, dim3(1), dim3(QB), 0, st, a->Gv, a->tau, QB, T);
    }
    // the trailing columns.  Lookahead: the previous bulk update wrote the columns this one starts
    // from, so the caller's stream waits for it here -- after this panel, which ran beside it
    if (bulk) {
      e = hipStreamWaitEvent(st, a->evb, 0);
      if (e != hipSuccess) return e;
      bulk = false;
    }
    if (la && ntr > 1) {
      e = hipEventRecord(a->evp, st);
      if (e == hipSuccess) e = hipStreamWaitEvent(a->st2, a->evp, 0);
      if (e == hipSuccess)
        e = qr_apply_block(A, ld, npad, p, c1 + QB, ntr - 1, 2 * nbk + 2 * p + 1, V, T, a->Wm2, a->Ym2, a->Vt2,
                           a->kpart2, a, a->st2);
      if (e == hipSuccess) e = hipEventRecord(a->evb, a->st2);
      if (e != hipSuccess) return e;
      bulk = true;
      // the next panel's columns
      e = qr_apply_block(A, ld, npad, p, c1, 1, 2 * nbk + 2 * p, V, T, a->Wm, a->Ym, a->Vt, a->kpart, a, st);
    } else {
      e = qr_apply_block(A, ld, npad, p, c1, ntr, 2 * p + 1, V, T, a->Wm, a->Ym, a->Vt, a->kpart, a, st);
    }
    if (e != hipSuccess) return e;
  }
  if (bulk) {
    e = hipStreamWaitEvent(st, a->evb, 0);
    if (e != hipSuccess) return e;
  }
  // R x = Qᵀ b: the diagonal blocks' inverses, then the one-launch backward solve (b holds Qᵀ b)
  e = chol_tri_inverse(A, ld, nbk, a->W, st);
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(a->Ym, b, sizeof(double) * npad, hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return e;
  a->gen = ++a->gen == 0 ? ++a->gen : a->gen;
  return chol_back_solve(A, ld, npad, a->W, a->Ym, b, a->flags, a->gen, a->err, st);
}

}  // namespace scs
