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
    if (t < i) {
      double s = 0.0;
      for (int q = t; q < i; ++q) s += Ts[q * QB + t] * z[q];   // T(0:i,0:i) upper: T(t, q), q >= t
      Ts[i * QB + t] = s;
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
                     &a->W})
    if (*p) {
      (void)hipFree(*p);
      *p = nullptr;
    }
  if (a->tiles) (void)hipFree(a->tiles);
  a->tiles = nullptr;
  a->rect_off.clear();
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
  al(&a->part, (size_t)(QB + 2) * nrc);
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

hipError_t qr_solve(double* A, int64_t ld, int64_t npad, QRAux* a, double* b, hipStream_t st) {
  hipError_t e = qr_aux_init(a, npad, st);
  if (e != hipSuccess) return e;
  const int nbk = (int)(npad / QB);
  for (int p = 0; p < nbk; ++p) {
    const int64_t c0 = (int64_t)p * QB, c1 = c0 + QB, rows = npad - c0;
    const int nrc = (int)((rows + QR_RC - 1) / QR_RC);
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
    // T from Gv = VᵀV over the panel's rows
    e = gram_launch_gen(a->V, npad, a->V, npad, a->ones, 0, rows, a->tiles, 1, a->Gv, QB, 0, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(qr_build_t, dim3(1), dim3(QB), 0, st, a->Gv, a->tau, QB, a->T);
    // Wm (QB x trailing) = Vᵀ A_trail: features = reflectors (A1 = V) x trailing columns (A2), the
    // tiles (0, j < ntr) in one launch
    double* At = A + c1 * ld + c0;
    e = gram_launch_gen(a->V, npad, At, ld, a->ones, 0, rows, a->tiles, ntr, a->Wm, QB, 0, st);
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
