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
#include "common.h"
#include "kernels.h"

namespace scs {

constexpr int CB = 128;          // block size (= Gram tile edge)
constexpr int CLD = CB + 1;      // LDS row pitch (doubles) -> conflict-light column access

// Factor the diagonal block U_kk (upper) of G in place and write W_k = U_kk⁻¹
// (upper, column-major 128 x 128).  info: first non-positive pivot (1-based,
// global) or left untouched.
__global__ __launch_bounds__(1024) void chol_diag_kernel(double* __restrict__ G, int64_t ld, int k,
                                                         double* __restrict__ W, int* __restrict__ info) {
  __shared__ __attribute__((aligned(16))) double sm[CB * CLD];   // column-major: a(r,c) = sm[c*CLD + r]
  double* blk = G + (int64_t)k * CB * ld + (int64_t)k * CB;
  const int tid = threadIdx.x;
  for (int e = tid; e < CB * CB; e += 1024) {
    const int c = e / CB, r = e % CB;
    sm[c * CLD + r] = (r <= c) ? blk[(int64_t)c * ld + r] : 0.0;
  }
  __syncthreads();
  // right-looking upper Cholesky: for j: u_jj = sqrt(a_jj); u_jc = a_jc / u_jj; a_ic -= u_ji u_jc (j < i <= c)
  for (int j = 0; j < CB; ++j) {
    const double ajj = sm[j * CLD + j];
    const double d = sqrt(ajj);
    const bool bad = !(ajj > 0.0);
    __syncthreads();
    if (bad) {
      if (tid == 0 && *info == 0) *info = k * CB + j + 1;
    }
    for (int c = j + 1 + tid; c < CB; c += 1024) sm[c * CLD + j] = sm[c * CLD + j] / d;
    if (tid == 0) sm[j * CLD + j] = d;
    __syncthreads();
    const int n = CB - 1 - j;  // trailing order
    for (int e = tid; e < n * n; e += 1024) {
      const int c = j + 1 + e / n, i = j + 1 + e % n;
      if (i <= c) sm[c * CLD + i] -= sm[i * CLD + j] * sm[c * CLD + j];
    }
    __syncthreads();
  }
  for (int e = tid; e < CB * CB; e += 1024) {
    const int c = e / CB, r = e % CB;
    if (r <= c) blk[(int64_t)c * ld + r] = sm[c * CLD + r];
  }
  // W = U⁻¹ (upper).  Row by row from the bottom: W[i][c] = -(Σ_{i<t<=c} U[i][t] W[t][c]) / U[i][i]
  // for c > i, W[i][i] = 1/U[i][i].  W's strictly-upper entries live transposed in the
  // (unused) strictly-lower half of the LDS tile: W[i][c] -> sm[i*CLD + c]; the diagonal in wd.
  __shared__ double wd[CB];
  if (tid < CB) wd[tid] = 1.0 / sm[tid * CLD + tid];
  __syncthreads();
  {
    const int c = tid >> 3, part = tid & 7;   // 8 threads per column
    for (int i = CB - 2; i >= 0; --i) {
      double s = 0.0;
      if (c > i) {
        for (int t = i + 1 + part; t <= c; t += 8) {
          const double wtc = (t == c) ? wd[c] : sm[t * CLD + c];
          s += sm[t * CLD + i] * wtc;
        }
      }
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      if (c > i && part == 0) sm[i * CLD + c] = -s * wd[i];
      __syncthreads();
    }
  }
  for (int e = tid; e < CB * CB; e += 1024) {
    const int c = e / CB, r = e % CB;
    W[(int64_t)k * CB * CB + (int64_t)c * CB + r] = (r < c) ? sm[r * CLD + c] : (r == c ? wd[c] : 0.0);
  }
}

// Forward solve Uᵀ y = b, block step k (all blocks recompute y_k = W_kᵀ b_k;
// block 0 stores it, the others update b_j -= U_kjᵀ y_k for j > k).
__global__ __launch_bounds__(256) void chol_fwd_step_kernel(const double* __restrict__ G, int64_t ld, int k,
                                                            int nblk, const double* __restrict__ W,
                                                            double* __restrict__ b, double* __restrict__ y) {
  __shared__ double yk[CB];
  __shared__ double bk[CB];
  const int tid = threadIdx.x;
  if (tid < CB) bk[tid] = b[(int64_t)k * CB + tid];
  __syncthreads();
  const double* Wk = W + (int64_t)k * CB * CB;
  if (tid < CB) {  // y_k[t] = Σ_{u<=t} W[u][t] b_k[u]
    double s = 0.0;
    for (int u = 0; u <= tid; ++u) s += Wk[(int64_t)tid * CB + u] * bk[u];
    yk[tid] = s;
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    if (tid < CB) y[(int64_t)k * CB + tid] = yk[tid];
    return;
  }
  // columns of the row panel handled by this block: 64 per block, 16 per wave
  const int lane = tid & 63, wid = tid >> 6;
  const int64_t c0 = (int64_t)(k + 1) * CB + (int64_t)(blockIdx.x - 1) * 64 + wid * 16;
  const double ya = yk[2 * lane], yb = yk[2 * lane + 1];
  for (int q = 0; q < 16; ++q) {
    const int64_t c = c0 + q;
    if (c >= (int64_t)nblk * CB) break;
    const v2d u = *(const v2d*)(G + c * ld + (int64_t)k * CB + 2 * lane);
    const double s = wave_sum(u[0] * ya + u[1] * yb);
    if (lane == 0) b[c] -= s;
  }
}

// Backward solve U x = y, block step k (descending): x_k = W_k y_k; rows above
// the block: y_r -= Σ_t U[r][k*128+t] x_k[t].
__global__ __launch_bounds__(256) void chol_bwd_step_kernel(const double* __restrict__ G, int64_t ld, int k,
                                                            const double* __restrict__ W, double* __restrict__ y,
                                                            double* __restrict__ x) {
  __shared__ double xk[CB];
  __shared__ double ykk[CB];
  const int tid = threadIdx.x;
  if (tid < CB) ykk[tid] = y[(int64_t)k * CB + tid];
  __syncthreads();
  const double* Wk = W + (int64_t)k * CB * CB;
  if (tid < CB) {  // x_k[t] = Σ_{u>=t} W[t][u] y_k[u]
    double s = 0.0;
    for (int u = tid; u < CB; ++u) s += Wk[(int64_t)u * CB + tid] * ykk[u];
    xk[tid] = s;
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    if (tid < CB) x[(int64_t)k * CB + tid] = xk[tid];
    return;
  }
  const int64_t r = (int64_t)(blockIdx.x - 1) * 256 + tid;
  if (r >= (int64_t)k * CB) return;
  double s = 0.0;
  const double* col = G + (int64_t)k * CB * ld + r;
  for (int t = 0; t < CB; ++t) s += col[(int64_t)t * ld] * xk[t];
  y[r] -= s;
}

__global__ void diag_pad_kernel(double* __restrict__ G, int64_t ld, int64_t m, int64_t mpad) {
  const int64_t i = m + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < mpad) G[i * ld + i] = 1.0;
}

hipError_t chol_factor(double* G, int64_t ld, int64_t m, int64_t mpad, double* W, const double* wpm,
                       const int2* rowlist, const int2* trilist, int* info, hipStream_t st) {
  const int nblk = (int)(mpad / CB);
  if (mpad > m) hipLaunchKernelGGL(diag_pad_kernel, dim3((unsigned)ceil_div(mpad - m, 256)), dim3(256), 0, st, G, ld,
                                   m, mpad);
  for (int k = 0; k < nblk; ++k) {
    hipLaunchKernelGGL(chol_diag_kernel, dim3(1), dim3(1024), 0, st, G, ld, k, W, info);
    const int nb = nblk - k - 1;
    if (nb == 0) break;
    double* rowpanel = G + (int64_t)(k + 1) * CB * ld + (int64_t)k * CB;   // U_k,(k+1..) : 128 rows x nb*128 cols
    // panel solve in place: U_kj = W_kᵀ A_kj  (P = W_k, tiles (0, j))
    hipError_t e = gram_launch_gen(W + (int64_t)k * CB * CB, CB, rowpanel, ld, wpm, 0, CB, rowlist, nb, rowpanel,
                                   ld, 0, st);
    if (e != hipSuccess) return e;
    // trailing update (upper): A_(k+1..) -= U_kᵀ U_k
    double* trail = G + (int64_t)(k + 1) * CB * ld + (int64_t)(k + 1) * CB;
    e = gram_launch_gen(rowpanel, ld, rowpanel, ld, wpm + CB, 0, CB, trilist, nb * (nb + 1) / 2, trail, ld,
                        /*GRAM_ACCUMULATE|GRAM_UPPER*/ 2 | 4, st);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

// Solve G x = b given the factor; b (length mpad, zero-padded) is overwritten
// by x; y is scratch (mpad).
hipError_t chol_solve(const double* G, int64_t ld, int64_t mpad, const double* W, double* b, double* y,
                      hipStream_t st) {
  const int nblk = (int)(mpad / CB);
  for (int k = 0; k < nblk; ++k) {
    const int ncols = (nblk - k - 1) * CB;
    const int grid = 1 + (int)ceil_div(ncols, 64);
    hipLaunchKernelGGL(chol_fwd_step_kernel, dim3(grid), dim3(256), 0, st, G, ld, k, nblk, W, b, y);
  }
  for (int k = nblk - 1; k >= 0; --k) {
    const int grid = 1 + (int)ceil_div((int64_t)k * CB, 256);
    hipLaunchKernelGGL(chol_bwd_step_kernel, dim3(grid), dim3(256), 0, st, G, ld, k, W, y, b);
  }
  return hipGetLastError();
}

}  // namespace scs
