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
//   A  wave 0 factors the 16 x 16 diagonal sub-block in registers (lane c =
//      column c; row values broadcast with v_readlane), reciprocal pivots to LDS;
//   B  panel: forward substitution Dᵀ P = S(o:o+16, c), one column per thread;
//   C  trailing update of the upper triangle with 4 x 4 register tiles.
// Then W = U⁻¹: the eight 16 x 16 diagonal inverses (two per wave, in
// registers), and recursive doubling W12 = -W11 · (U12 · W22) at block sizes
// 16 -> 32 -> 64 -> 128, as register-blocked LDS products (4 x S/16 outputs per
// thread); the intermediate T = U12·W22 lives in the (unused) strictly-lower
// triangle of S.  Only the factorization steps are a serial chain.
constexpr int SB = 16;

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

#ifdef CHOL_PROF
// probe_chol -DCHOL_PROF: thread 0 records s_memrealtime (100 MHz) at phase boundaries
__device__ long long chol_prof[64];
#define PROF_MARK(i) \
  if (threadIdx.x == 0 && k == 0) chol_prof[i] = (long long)__builtin_amdgcn_s_memrealtime()
#else
#define PROF_MARK(i)
#endif

// one doubling level: for every pair (i0 = 2pS, j0 = i0 + S):
//   step 1  T(r, c) = Σ_{t <= c} U(i0+r, j0+t) W(j0+t, j0+c)   -> S[j0 + r][i0 + c] (strictly lower)
//   step 2  W(i0+r, j0+c) = -Σ_{t >= r} W(i0+r, i0+t) T(t, c)  -> S[i0 + r][j0 + c]
template <int S>
__device__ __forceinline__ void chol_inv_double(double* su, int tid) {
  constexpr int MC = S / 16;                  // columns per thread (4 rows x MC)
  constexpr int TPP = 256 / (CB / (2 * S));   // threads per pair
  const int pair = tid / TPP, loc = tid % TPP;
  const int rg = loc / 16, cg = loc % 16;
  const int i0 = 2 * S * pair, j0 = i0 + S;
  const int r0 = 4 * rg, c0 = cg * MC;
  double acc[4][MC];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < MC; ++m) acc[q][m] = 0.0;
#pragma unroll 4
  for (int t = 0; t < S; ++t) {
    double u[4], wv[MC];
#pragma unroll
    for (int q = 0; q < 4; ++q) u[q] = su[(j0 + t) * CLD + i0 + r0 + q];
#pragma unroll
    for (int m = 0; m < MC; ++m) wv[m] = (t <= c0 + m) ? su[(j0 + c0 + m) * CLD + j0 + t] : 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int m = 0; m < MC; ++m) acc[q][m] += u[q] * wv[m];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < MC; ++m) su[(i0 + c0 + m) * CLD + j0 + r0 + q] = acc[q][m];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < MC; ++m) acc[q][m] = 0.0;
#pragma unroll 4
  for (int t = 0; t < S; ++t) {
    double wv[4], tv[MC];
#pragma unroll
    for (int q = 0; q < 4; ++q) wv[q] = (t >= r0 + q) ? su[(i0 + t) * CLD + i0 + r0 + q] : 0.0;
#pragma unroll
    for (int m = 0; m < MC; ++m) tv[m] = su[(i0 + c0 + m) * CLD + j0 + t];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int m = 0; m < MC; ++m) acc[q][m] += wv[q] * tv[m];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < MC; ++m) su[(j0 + c0 + m) * CLD + i0 + r0 + q] = -acc[q][m];
  __syncthreads();
}

__global__ __launch_bounds__(256) void chol_diag_kernel(double* __restrict__ G, int64_t ld, int k,
                                                        double* __restrict__ W, int* __restrict__ info) {
  __shared__ double su[CB * CLD];   // S(r, c) = su[c*CLD + r]
  __shared__ double srinv[CB];      // 1 / U(j, j)
  double* blk = G + (int64_t)k * CB * ld + (int64_t)k * CB;
  double* Wk = W + (int64_t)k * CB * CB;
  const int tid = threadIdx.x;
  for (int e = tid; e < CB * CB; e += 256) {
    const int c = e >> 7, r = e & 127;
    su[c * CLD + r] = (r <= c) ? blk[(int64_t)c * ld + r] : 0.0;
  }
  __syncthreads();

  PROF_MARK(0);
  for (int kb = 0; kb < CB / SB; ++kb) {
    const int o = kb * SB;
    PROF_MARK(1 + 4 * kb);
    // ---- A: factor the diagonal sub-block (wave 0; lanes 16..63 mirror lanes 0..15)
    if (tid < 64) {
      const int c = tid & 15;
      double a[SB];
#pragma unroll
      for (int i = 0; i < SB; ++i) a[i] = su[(o + c) * CLD + o + i];   // S(o+i, o+c); zero below the diagonal
#pragma unroll
      for (int j = 0; j < SB; ++j) {
        const double ajj = readlane_d(a[j], j);
        if (tid == 0 && !(ajj > 0.0) && *info == 0) *info = k * CB + o + j + 1;
        const double d = sqrt(ajj);
        const double r = 1.0 / d;
        if (tid == 0) srinv[o + j] = r;
        a[j] = (c > j) ? a[j] * r : ((c == j) ? d : a[j]);    // row j of U: U(j, c)
#pragma unroll
        for (int i = j + 1; i < SB; ++i) a[i] -= readlane_d(a[j], i) * a[j];   // U(j, i) from lane i
      }
      if (tid < SB) {
#pragma unroll
        for (int i = 0; i < SB; ++i)
          if (i <= c) su[(o + c) * CLD + o + i] = a[i];
      }
    }
    __syncthreads();
    PROF_MARK(2 + 4 * kb);
    const int np = CB - o - SB;  // columns right of the sub-block
    if (np == 0) break;
    // ---- B: panel, forward substitution Dᵀ p = x per column (D(u, t) reads are wave-uniform)
    if (tid < np) {
      const int c = o + SB + tid;
      double X[SB];
#pragma unroll
      for (int u = 0; u < SB; ++u) X[u] = su[c * CLD + o + u];
#pragma unroll
      for (int t = 0; t < SB; ++t) {
        double sacc = X[t];
#pragma unroll
        for (int u = 0; u < t; ++u) sacc -= su[(o + t) * CLD + o + u] * X[u];
        X[t] = sacc * srinv[o + t];
      }
#pragma unroll
      for (int u = 0; u < SB; ++u) su[c * CLD + o + u] = X[u];
    }
    __syncthreads();
    PROF_MARK(3 + 4 * kb);
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
  PROF_MARK(33);
  // ---- store U
  for (int e = tid; e < CB * CB; e += 256) {
    const int c = e >> 7, r = e & 127;
    if (r <= c) blk[(int64_t)c * ld + r] = su[c * CLD + r];
  }
  // ---- diagonal 16 x 16 inverses: wave wv inverts blocks wv and wv + 4 (lane c = column c)
  {
    const int wv = tid >> 6, c = tid & 15;
    double w0[SB], w1[SB];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = (wv + 4 * h) * SB;
      double a[SB], w[SB];
#pragma unroll
      for (int i = 0; i < SB; ++i) {
        a[i] = su[(o + c) * CLD + o + i];
        w[i] = (i == c) ? 1.0 : 0.0;
      }
#pragma unroll
      for (int t = SB - 1; t >= 0; --t) {
        w[t] *= srinv[o + t];
#pragma unroll
        for (int i = 0; i < t; ++i) w[i] -= readlane_d(a[i], t) * w[t];
      }
#pragma unroll
      for (int i = 0; i < SB; ++i) {
        if (h == 0) w0[i] = w[i];
        else w1[i] = w[i];
      }
    }
    __syncthreads();   // every wave has read its U blocks
    if ((tid & 63) < SB) {
#pragma unroll
      for (int i = 0; i < SB; ++i) {
        if (i <= c) su[(wv * SB + c) * CLD + wv * SB + i] = w0[i];
        if (i <= c) su[((wv + 4) * SB + c) * CLD + (wv + 4) * SB + i] = w1[i];
      }
    }
    __syncthreads();
  }
  PROF_MARK(34);
  chol_inv_double<16>(su, tid);
  chol_inv_double<32>(su, tid);
  chol_inv_double<64>(su, tid);
  for (int e = tid; e < CB * CB; e += 256) {
    const int c = e >> 7, r = e & 127;
    Wk[(int64_t)c * CB + r] = (r <= c) ? su[c * CLD + r] : 0.0;
  }
  PROF_MARK(35);
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
