// The latency Gram strip (one QC-column strip of a 128 x 128 output tile, one workgroup of 256
// threads), shared by gram_small_kernel (gram.hip) and the Cholesky's dependency-driven chain
// kernel (chol.hip), so both compute every tile with the same MFMA order -- bitwise identical to
// the throughput Gram kernels per tile.
#pragma once
#include "common.h"

namespace scs {

constexpr int GT = 128;   // output tile edge
// GRAM_PRIO (r06): the latency kernel's waves at s_setprio 3 -- the Cholesky chain's launches, which
// share SIMDs with the bulk stream's MFMA waves (chol.hip SCS_CHOL_PRIO)
enum { GRAM_PACKED = 1, GRAM_ACCUMULATE = 2, GRAM_UPPER = 4, GRAM_PRIO = 8 };
constexpr int GBK = 16;   // samples per stage

__device__ __forceinline__ int swz(int f) { return (f >> 1) & 7; }

// Latency variant for the small launches of the Cholesky and the LU (short K or few
// tiles): each 128 x 128 list tile is computed by 128/QC workgroups, one per QC-column
// strip (4 waves of 32 rows x QC along the rows).  A workgroup reads the A2 columns it
// writes and nothing else of the output, so the in-place panel solve (G == A2) stays
// race-free.  The global loads run RING stages (RING x 16 samples) ahead of the MFMAs in a
// register ring: one K = 128 launch pays one memory latency, not one per 16-sample stage.
// Column-major operands (gen form), swizzled LDS stages, and per accumulator the MFMA order of
// gram_f64_kernel / gram_sia_kernel ((p, u) per stage, stages ascending): the tile is bitwise
// the same.  Ai = the tile's A1 columns (feature f at Ai + f·lda1), Aj = the strip's A2
// columns, Gt = the strip's output origin (element (0, 0) in the chosen placement), lds =
// 2 (128 + QC) 16 doubles.
// The strip epilogue: wave wr's 32 x 16 TJ accumulator block into Gt.  With GRAM_ACCUMULATE every old
// value is loaded before the first store (the compiler cannot prove the 2 x TJ x 4 destinations
// distinct and would otherwise pay one memory round trip per element); the sums are the same.
template <int TJ>
__device__ __forceinline__ void gram_strip_store(const v4d (&acc)[2][TJ], double* Gt, int64_t ldg, int wr, int g,
                                                 int fl, int accumulate, int upper) {
  double* dst[2][TJ][4];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t I = wr * 32 + 16 * ti + g + 4 * r;
        const int64_t J = 16 * tj + fl;
        dst[ti][tj][r] = upper ? Gt + I * ldg + J : Gt + J * ldg + I;
      }
  if (accumulate) {
    double old[2][TJ][4];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) old[ti][tj][r] = *dst[ti][tj][r];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) *dst[ti][tj][r] = old[ti][tj][r] + acc[ti][tj][r];
  } else {
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) *dst[ti][tj][r] = acc[ti][tj][r];
  }
}

template <int QC>
__device__ __forceinline__ void gram_small_strip(const double* __restrict__ Ai, int64_t lda1, const double* Aj,
                                                 int64_t lda2, const double* __restrict__ w, int64_t k0, int64_t Nk,
                                                 double* Gt, int64_t ldg, int flags, double* lds) {
  constexpr int RING = 8;                  // stages in flight
  constexpr int NQ = GT / QC;              // workgroups per tile
  constexpr int TJ = QC / 16;              // 16-column MFMA tiles per wave
  constexpr int SBQ = (GT + QC) * GBK;     // doubles per LDS stage (A1 128 x 16 | A2 QC x 16)
  (void)NQ;
  const int accumulate = flags & GRAM_ACCUMULATE, upper = flags & GRAM_UPPER;
  const int tid = threadIdx.x, lane = tid & 63, wr = tid >> 6;
  const int sc = tid & 7, sf0 = tid >> 3;   // staging: feature sf0 + 32 i, 16-B chunk sc
  const bool hasb = QC == 32 || sf0 < QC;   // A2 rows staged by this thread (QC = 16: half the threads)
  const int sfb = sf0 & (QC - 1);           // loads stay unconditional (a branch drains vmcnt)
  v2d ra[RING][4], rb[RING], rw[RING];
  auto gload = [&](int slot, int64_t n0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) ra[slot][i] = *(const v2d*)(Ai + (int64_t)(sf0 + 32 * i) * lda1 + n0 + 2 * sc);
    rb[slot] = *(const v2d*)(Aj + (int64_t)sfb * lda2 + n0 + 2 * sc);
    rw[slot] = *(const v2d*)(w + n0 + 2 * sc);
  };
  auto swrite = [&](int slot, int buf) {
    double* la = lds + buf * SBQ;
    double* lb = la + GT * GBK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = sf0 + 32 * i;
      *(v2d*)(la + f * GBK + 2 * (sc ^ swz(f))) = ra[slot][i];
    }
    if (hasb) *(v2d*)(lb + sf0 * GBK + 2 * (sc ^ swz(sf0))) = rb[slot] * rw[slot];
  };
  v4d acc[2][TJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = (v4d){0.0, 0.0, 0.0, 0.0};
  const int fl = lane & 15, g = lane >> 4, s = swz(fl);
  // nk is a multiple of RING (gram_launch_small); the loads past the end re-read the last stage
  // (branch-free: a conditional load would make the compiler drain vmcnt at every stage)
  const int nk = (int)((Nk - k0) / GBK);
#pragma unroll
  for (int j = 0; j < RING; ++j) gload(j, k0 + (int64_t)j * GBK);
  for (int kk = 0; kk < nk; kk += RING) {
#pragma unroll
    for (int j = 0; j < RING; ++j) {
      const int k = kk + j;
      {
        swrite(j, k & 1);
        gload(j, k0 + (int64_t)min(k + RING, nk - 1) * GBK);
        __syncthreads();
        const double* la = lds + (k & 1) * SBQ;
        const double* lb = la + GT * GBK;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int pc = ((4 * p + g) ^ s) * 2;
          v2d a[2], b[TJ];
#pragma unroll
          for (int t = 0; t < 2; ++t) a[t] = *(const v2d*)(la + (wr * 32 + 16 * t + fl) * GBK + pc);
#pragma unroll
          for (int t = 0; t < TJ; ++t) b[t] = *(const v2d*)(lb + (16 * t + fl) * GBK + pc);
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
              for (int tj = 0; tj < TJ; ++tj)
                acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti][u], b[tj][u], acc[ti][tj], 0, 0, 0);
        }
      }
    }
  }
  gram_strip_store<TJ>(acc, Gt, ldg, wr, g, fl, accumulate, upper);
}

}  // namespace scs
