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
// global); the caller then takes the LU path.
//
// Inner-blocked (b = 16) right-looking factorization of the LDS copy S:
//   A  wave 0 factors the 16 x 16 diagonal sub-block in registers (lane =
//      column c, rows g + 4q) with shuffles, and inverts it (D⁻¹);
//   B  panel: S(o:o+16, c) = D⁻ᵀ S(o:o+16, c) for the columns to the right;
//   C  trailing update of the upper triangle with 4 x 4 register tiles.
// Then W = U⁻¹ block row by block row from the bottom:
//   W(ii, c) = -D_ii⁻¹ Σ_{t > block ii} U(ii, t) W(t, c),
// overwriting U's rows in LDS as they are consumed.  The reciprocal of each
// pivot is formed once and multiplied in, as LAPACK dpotf2 does.
constexpr int SB = 16;
__global__ __launch_bounds__(256) void chol_diag_kernel(double* __restrict__ G, int64_t ld, int k,
                                                        double* __restrict__ W, int* __restrict__ info) {
  __shared__ double su[CB * CLD];        // S(r, c) = su[c*CLD + r]
  __shared__ double sdinv[SB * SB];      // D⁻¹(r, c) = sdinv[c*SB + r]
  __shared__ double sT[(CB - SB) * SB];  // W phase: T(r, ci) = sT[ci*SB + r]
  double* blk = G + (int64_t)k * CB * ld + (int64_t)k * CB;
  double* Wk = W + (int64_t)k * CB * CB;
  const int tid = threadIdx.x;
  for (int e = tid; e < CB * CB; e += 256) {
    const int c = e >> 7, r = e & 127;
    su[c * CLD + r] = (r <= c) ? blk[(int64_t)c * ld + r] : 0.0;
  }
  __syncthreads();

  for (int kb = 0; kb < CB / SB; ++kb) {
    const int o = kb * SB;
    // ---- A: factor + invert the diagonal sub-block (wave 0)
    if (tid < 64) {
      const int c = tid & 15, g = tid >> 4;
      double a[4], w[4], rinv[SB];
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = su[(o + c) * CLD + o + g + 4 * q];
#pragma unroll
      for (int j = 0; j < SB; ++j) {
        const int gj = j & 3, qj = j >> 2;
        const double ajj = __shfl(a[qj], gj * 16 + j);
        if (tid == 0 && !(ajj > 0.0) && *info == 0) *info = k * CB + o + j + 1;
        const double d = sqrt(ajj);
        const double r = 1.0 / d;
        rinv[j] = r;
        if (g == gj) a[qj] = (c > j) ? a[qj] * r : ((c == j) ? d : a[qj]);
        const double ujc = __shfl(a[qj], gj * 16 + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double uji = __shfl(a[qj], gj * 16 + g + 4 * q);
          if (g + 4 * q > j) a[q] -= uji * ujc;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = (g + 4 * q == c) ? 1.0 : 0.0;
#pragma unroll
      for (int t = SB - 1; t >= 0; --t) {
        const int gt = t & 3, qt = t >> 2;
        if (g == gt) w[qt] *= rinv[t];
        const double wtc = __shfl(w[qt], gt * 16 + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double dit = __shfl(a[q], g * 16 + t);
          if (g + 4 * q < t) w[q] -= dit * wtc;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = g + 4 * q;
        if (r <= c) su[(o + c) * CLD + o + r] = a[q];
        sdinv[c * SB + r] = w[q];
        Wk[(int64_t)(o + c) * CB + o + r] = w[q];
      }
    }
    __syncthreads();
    const int np = CB - o - SB;  // columns right of the sub-block
    if (np == 0) break;
    // ---- B: panel  S(o + t, c) = Σ_{u <= t} D⁻¹(u, t) S(o + u, c)
    {
      const int ci = tid & 127, h = tid >> 7, c = o + SB + ci;
      double X[SB], out[8];
      if (ci < np) {
#pragma unroll
        for (int u = 0; u < SB; ++u) X[u] = su[c * CLD + o + u];
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) {
          const int t = 8 * h + tt;
          double s = 0.0;
#pragma unroll
          for (int u = 0; u < SB; ++u) s += sdinv[t * SB + u] * X[u];
          out[tt] = s;
        }
      }
      __syncthreads();
      if (ci < np) {
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) su[c * CLD + o + 8 * h + tt] = out[tt];
      }
    }
    __syncthreads();
    // ---- C: trailing update  S(i, c) -= Σ_t U(o + t, i) U(o + t, c),  o+16 <= i <= c
    {
      const int nt = np >> 2, ntiles = nt * (nt + 1) / 2;
      for (int id = tid; id < ntiles; id += 256) {
        int C = (int)((sqrtf(8.0f * id + 1.0f) - 1.0f) * 0.5f);
        while (C * (C + 1) / 2 > id) --C;
        while ((C + 1) * (C + 2) / 2 <= id) ++C;
        const int I = id - C * (C + 1) / 2;
        const int i0 = o + SB + 4 * I, c0 = o + SB + 4 * C;
        double acc[4][4] = {};
#pragma unroll
        for (int t = 0; t < SB; ++t) {
          double ui[4], uc[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            ui[q] = su[(i0 + q) * CLD + o + t];
            uc[q] = su[(c0 + q) * CLD + o + t];
          }
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) acc[r][cc] += ui[r] * uc[cc];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int cc = 0; cc < 4; ++cc)
            if (i0 + r <= c0 + cc) su[(c0 + cc) * CLD + i0 + r] -= acc[r][cc];
      }
    }
    __syncthreads();
  }
  // ---- store U
  for (int e = tid; e < CB * CB; e += 256) {
    const int c = e >> 7, r = e & 127;
    if (r <= c) blk[(int64_t)c * ld + r] = su[c * CLD + r];
  }
  __syncthreads();
  // ---- W = U⁻¹, block rows from the bottom (the last diagonal block already is D⁻¹ in Wk)
  for (int ii = CB / SB - 1; ii >= 0; --ii) {
    const int o = ii * SB, np = CB - o - SB;
    sdinv[tid] = Wk[(int64_t)(o + (tid >> 4)) * CB + o + (tid & 15)];
    const int ci = tid & 127, h = tid >> 7, c = o + SB + ci;
    if (ci < np) {
      double T[8] = {};
      for (int t = o + SB; t < CB; ++t) {
        const double wtc = su[c * CLD + t];   // W(t, c) (rows below o+16 already hold W; 0 for t > c)
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) T[tt] += su[t * CLD + o + 8 * h + tt] * wtc;
      }
#pragma unroll
      for (int tt = 0; tt < 8; ++tt) sT[ci * SB + 8 * h + tt] = T[tt];
    }
    __syncthreads();
    if (ci < np) {
#pragma unroll
      for (int tt = 0; tt < 8; ++tt) {
        const int rr = 8 * h + tt;
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < SB; ++u) s += sdinv[u * SB + rr] * sT[ci * SB + u];
        su[c * CLD + o + rr] = -s;
      }
    }
    {
      const int cc = tid >> 4, rr = tid & 15;
      su[(o + cc) * CLD + o + rr] = sdinv[cc * SB + rr];
    }
    __syncthreads();
  }
  for (int e = tid; e < CB * CB; e += 256) {
    const int c = e >> 7, r = e & 127;
    Wk[(int64_t)c * CB + r] = (r <= c) ? su[c * CLD + r] : 0.0;
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
    hipLaunchKernelGGL(chol_diag_kernel, dim3(1), dim3(256), 0, st, G, ld, k, W, info);
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
