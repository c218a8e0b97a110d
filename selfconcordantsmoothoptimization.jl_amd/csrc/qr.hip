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
                                                   double* __restrict__ tau, double* __restrict__ V, int64_t ldv) {
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
  if (tid == 0) {
    double t = 0.0, sc = 0.0, beta = 0.0, twj = 0.0, twc = 0.0;
    if (has_prev) {
      const double* pp = part + (pv & 1) * pslot;
      const double* rp = rowc + (pv & 1) * (QB + 2);
      double xx = 0.0;
      for (int q = 0; q < nrc_prev; ++q) xx += pp[q];
      const double alpha = rp[0];
      beta = alpha;
      if (xx > 0.0) {
        beta = -copysign(sqrt(alpha * alpha + xx), alpha);
        t = (beta - alpha) / beta;
        sc = 1.0 / (alpha - beta);
      }
      auto twf = [&](int64_t j) {   // tau · vᵀ a_j, v(pv) = 1
        double d = 0.0;
        for (int q = 0; q < nrc_prev; ++q) d += pp[(j - pv) * nrc_prev + q];
        return t * (rp[j - pv] + sc * d);
      };
      if (jj >= 0) twj = twf(c + jj);
      if (c < c1) twc = twf(c);
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

static bool qr_step_fused() {   // read per call (A/B)
  const char* e = getenv("SCS_QR_STEP");
  return !(e && e[0] == '0');
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
                     &a->W, &a->rowc, &a->xs, &a->kpart})
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
  a->gen = 0;
  a->npad = 0;
}

hipError_t qr_aux_init(QRAux* a, int64_t npad, hipStream_t st) {
  if (a->npad == npad) return hipSuccess;
  qr_free_bufs(a);
  const int64_t nrc = (npad + QR_RC - 1) / QR_RC;
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
  if (e == hipSuccess) e = hipMalloc(&a->kwork, sizeof(int4) * std::max<size_t>(kw.size(), 1));
  if (e == hipSuccess && !kw.empty())
    e = hipMemcpyAsync(a->kwork, kw.data(), sizeof(int4) * kw.size(), hipMemcpyHostToDevice, st);
  al(&a->kpart, kmax * QB * QB);
  if (e == hipSuccess) e = hipMalloc(&a->tiles, sizeof(int2) * std::max<size_t>(tl.size(), 1));
  if (e == hipSuccess && !tl.empty())
    e = hipMemcpyAsync(a->tiles, tl.data(), sizeof(int2) * tl.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMalloc(&a->flags, sizeof(unsigned) * (size_t)nbk + sizeof(int));
  if (e == hipSuccess) e = hipMemsetAsync(a->flags, 0, sizeof(unsigned) * (size_t)nbk + sizeof(int), st);
  if (e == hipSuccess) a->err = (int*)(a->flags + nbk);
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

hipError_t qr_solve(double* A, int64_t ld, int64_t npad, QRAux* a, double* b, hipStream_t st) {
  hipError_t e = qr_aux_init(a, npad, st);
  if (e != hipSuccess) return e;
  const int nbk = (int)(npad / QB);
  for (int p = 0; p < nbk; ++p) {
    const int64_t c0 = (int64_t)p * QB, c1 = c0 + QB, rows = npad - c0;
    const int nrc = (int)((rows + QR_RC - 1) / QR_RC);
    if (qr_step_fused()) {
      const int64_t pslot = (int64_t)(QB + 1) * ((npad + QR_RC - 1) / QR_RC + 1);
      int nrc_prev = 0;
      for (int64_t c = c0; c <= c1; ++c) {
        const int64_t rbeg = c > c0 ? c - 1 : c;
        const int nrc_c = (int)((npad - rbeg + QR_RC - 1) / QR_RC);
        const int ncol = (int)(c1 - c) + 1;   // columns c .. c1-1 and b
        hipLaunchKernelGGL(qr_col_step, dim3((unsigned)nrc_c, (unsigned)(ncol + 1)), dim3(256), 0, st, A, ld, npad, c,
                           c0, c1, b, a->part, pslot, nrc_c, nrc_prev, a->rowc, a->xs, a->tau, a->V, npad);
        nrc_prev = nrc_c;
      }
    } else
    for (int64_t c = c0; c < c1; ++c) {
      const int ncol = (int)(c1 - c) + 1;
      hipLaunchKernelGGL(qr_col_partials, dim3((unsigned)nrc, (unsigned)ncol), dim3(256), 0, st, A, ld, npad, c, c1, b,
                         a->part, nrc);
      hipLaunchKernelGGL(qr_col_reflect, dim3(1), dim3(256), 0, st, A, ld, c, c1, c0, b, a->part, nrc, a->tw, a->tau,
                         a->scal, a->V, npad);
      hipLaunchKernelGGL(qr_col_update, dim3((unsigned)((npad - c + 255) / 256), (unsigned)ncol), dim3(256), 0, st, A,
                         ld, npad, c, c1, c0, b, a->tw, a->scal, a->V, npad);
    }
    const int ntr = nbk - p - 1;   // trailing column blocks
    if (ntr == 0) break;
    // T from Gv = VᵀV over the panel's rows (K split)
    e = qr_ksplit(a->V, npad, a->V, npad, rows, 1, a, 2 * p, a->Gv, QB, st);
    if (e != hipSuccess) return e;
    if (qr_step_fused()) {   // T by MFMA doubling (chol.hip wy_t_kernel); SCS_QR_STEP=0: the plain recurrence
      e = wy_t_build(a->Gv, a->tau, a->T, st);
      if (e != hipSuccess) return e;
    } else {
      hipLaunchKernelGGL(qr_build_t, dim3(1), dim3(QB), 0, st, a->Gv, a->tau, QB, a->T);
    }
    // Wm (QB x trailing) = Vᵀ A_trail: features = reflectors (A1 = V) x trailing columns (A2), the
    // tiles (0, j < ntr), K split, in one launch
    double* At = A + c1 * ld + c0;
    e = qr_ksplit(a->V, npad, At, ld, rows, ntr, a, 2 * p + 1, a->Wm, QB, st);
    if (e != hipSuccess) return e;
    // Ym = Tᵀ Wm: Ym(i, j) = Σ_q T(q, i) Wm(q, j)
    e = gram_launch_gen(a->T, QB, a->Wm, QB, a->ones, 0, QB, a->tiles, ntr, a->Ym, QB, 0, st);
    if (e != hipSuccess) return e;
    // A_trail -= V Ym: A(r, j) -= Σ_i Vt(i, r) Ym(i, j) (features r of Vt, K = i), panel p's rectangle
    hipLaunchKernelGGL(qr_transpose_v, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, a->V, npad, rows, a->Vt);
    e = gram_launch_gen(a->Vt, QB, a->Ym, QB, a->ones + npad, 0, QB, a->tiles + a->rect_off[(size_t)p],
                        (int)(rows / QB) * ntr, At, ld, /*ACCUMULATE*/ 2, st);
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
