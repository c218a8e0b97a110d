// Weighted Gram  G = Aᵀ diag(w) A  on fp64 MFMA (v_mfma_f64_16x16x4_f64).
//
// This is the hot spot of ProxGGNSCORE (`(Jt * Q) * Jt'`, prox-GGN-SCORE.jl:129,
// with J = diag(s)·A and Q = diag(q) ⇒ JᵀQJ = Aᵀ diag(s²q) A) and of
// ProxNSCORE's Hessian (hess_fx = Aᵀ diag(h) A, prox-N-SCORE.jl:49-56).
//
// Layout (HBM): A column-major, N_pad x m_pad, lda = N_pad (samples contiguous
// per feature, the Julia Matrix layout); N_pad % 16 == 0 and m_pad % 128 == 0
// with zero padding, so the kernel has no bounds checks.  w has N_pad entries
// (zeros in the padding).
//
// Tiling: one 256-thread workgroup (4 waves, 2 x 2) owns one 128 x 128 output
// tile (bi, bj), bi >= bj (lower triangle; diagonal tiles are computed whole).
// K (= samples) is streamed in 16-sample stages:
//   global -> registers (16 B per lane, 8 lanes per 128-B feature segment,
//   coalesced) -> LDS (XOR-swizzled [feature][16 samples] rows, w folded into
//   the B panel on the way) -> ds_read_b128 fragments -> 64 MFMAs / wave.
// The next stage's global loads are in flight while the current stage's
// MFMAs run; one barrier per stage.  Each wave holds a 64 x 64 sub-tile
// (4 x 4 MFMA tiles, 128 accumulator VGPRs) -> 2 waves / SIMD, 2 WG / CU.
//
// Fragment k-order: lane group g = lane>>4 reads the 16-B chunk c = 4p + g
// (samples 2c, 2c+1) and feeds sample 2c to one MFMA and 2c+1 to the next; A
// and B use the same map, so the contraction is exact (only the summation
// order differs from a textbook loop).
//
// Tile order: tiles are enumerated in 8 x 8 super-blocks of the lower
// triangle and block ids are remapped so that the workgroups sharing one XCD
// (blockIdx % 8, MI355X_MICROARCH.md §Workgroup dispatch) walk a contiguous
// run of that list: the ~64 tiles co-resident on an XCD then read ~16
// distinct column panels, which its 4 MiB L2 serves (speed only; results do
// not depend on placement).
#include "common.h"

namespace scs {

constexpr int GT = 128;   // output tile edge
constexpr int GBK = 16;   // samples per stage

__device__ __forceinline__ int swz(int f) { return (f >> 1) & 7; }

__global__ __launch_bounds__(256, 2) void gram_f64_kernel(
    const double* __restrict__ A, int64_t lda, const double* __restrict__ w, int64_t Nk,
    const int2* __restrict__ tiles, int ntiles, double* __restrict__ G, int64_t ldg, int packed) {
  // All LDS in ONE array (cdna_hip_programming.md §5 item 4a): [buf][panel][128 x 16]
  __shared__ __attribute__((aligned(16))) double lds[2 * 2 * GT * GBK];

  // XCD-aware bijective remap (cdna_hip_programming.md §5 "XCD swizzle")
  const int orig = blockIdx.x;
  const int q8 = ntiles / 8, r8 = ntiles % 8, xcd = orig % 8;
  const int tix = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int2 tl = tiles[tix];
  const int bi = tl.x, bj = tl.y;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const double* __restrict__ Ai = A + (int64_t)bi * GT * lda;
  const double* __restrict__ Aj = A + (int64_t)bj * GT * lda;

  // staging map: chunk q = tid + 256*i  ->  feature f = (tid>>3) + 32 i, chunk c = tid & 7
  const int sc = tid & 7;
  const int sf0 = tid >> 3;
  v2d ra[4], rb[4], rw;

  auto gload = [&](int64_t n0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t f = sf0 + 32 * i;
      ra[i] = *(const v2d*)(Ai + f * lda + n0 + 2 * sc);
      rb[i] = *(const v2d*)(Aj + f * lda + n0 + 2 * sc);
    }
    rw = *(const v2d*)(w + n0 + 2 * sc);
  };
  auto swrite = [&](int buf) {
    double* la = lds + (buf * 2 + 0) * GT * GBK;
    double* lb = lds + (buf * 2 + 1) * GT * GBK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = sf0 + 32 * i;
      const int off = f * GBK + 2 * (sc ^ swz(f));
      *(v2d*)(la + off) = ra[i];
      *(v2d*)(lb + off) = rb[i] * rw;
    }
  };

  v4d acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4d){0.0, 0.0, 0.0, 0.0};

  const int fl = lane & 15, g = lane >> 4, s = swz(fl);
  const int nk = (int)(Nk / GBK);

  gload(0);
  swrite(0);
  __syncthreads();
  for (int k = 0; k < nk; ++k) {
    if (k + 1 < nk) gload((int64_t)(k + 1) * GBK);
    const double* la = lds + ((k & 1) * 2 + 0) * GT * GBK;
    const double* lb = lds + ((k & 1) * 2 + 1) * GT * GBK;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int pc = ((4 * p + g) ^ s) * 2;
      v2d a[4], b[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = *(const v2d*)(la + (wr * 64 + 16 * t + fl) * GBK + pc);
        b[t] = *(const v2d*)(lb + (wc * 64 + 16 * t + fl) * GBK + pc);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ti = 0; ti < 4; ++ti)
#pragma unroll
          for (int tj = 0; tj < 4; ++tj)
            acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti][u], b[tj][u], acc[ti][tj], 0, 0, 0);
    }
    if (k + 1 < nk) swrite((k + 1) & 1);
    __syncthreads();
  }

  // Epilogue.  v_mfma_f64_16x16x4_f64 C/D map: col = lane&15, row = (lane>>4) + 4*r
  // (cdna_hip_programming.md §3; verified by probe_mfma).
  if (packed) {
    double* Gt = G + (int64_t)tix * GT * GT;  // tile-local column-major, packed in list order
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
#pragma unroll
      for (int tj = 0; tj < 4; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wr * 64 + 16 * ti + g + 4 * r;
          const int col = wc * 64 + 16 * tj + fl;
          Gt[col * GT + row] = acc[ti][tj][r];
        }
  } else {
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
#pragma unroll
      for (int tj = 0; tj < 4; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = (int64_t)bi * GT + wr * 64 + 16 * ti + g + 4 * r;
          const int64_t col = (int64_t)bj * GT + wc * 64 + 16 * tj + fl;
          G[col * ldg + row] = acc[ti][tj][r];
        }
  }
}

// Scatter packed tiles (list order) into a column-major m_pad x m_pad matrix.
__global__ void gram_unpack_kernel(const double* __restrict__ P, const int2* __restrict__ tiles,
                                   double* __restrict__ G, int64_t ldg) {
  const int t = blockIdx.y;
  const int2 tl = tiles[t];
  const double* Pt = P + (int64_t)t * GT * GT;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < GT * GT; e += gridDim.x * blockDim.x) {
    const int col = e / GT, row = e % GT;
    G[((int64_t)tl.y * GT + col) * ldg + (int64_t)tl.x * GT + row] = Pt[e];
  }
}

// Host helper: super-blocked lower-triangle tile list.
void gram_tile_list(int nb, int2* out, int* ntiles) {
  const int S = 8;
  const int nsb = (nb + S - 1) / S;
  int t = 0;
  for (int sbi = 0; sbi < nsb; ++sbi)
    for (int sbj = 0; sbj <= sbi; ++sbj)
      for (int i = sbi * S; i < (sbi + 1) * S && i < nb; ++i)
        for (int j = sbj * S; j < (sbj + 1) * S && j < nb; ++j)
          if (i >= j) out[t++] = make_int2(i, j);
  *ntiles = t;
}

hipError_t gram_launch(const double* A, int64_t lda, const double* w, int64_t Nk, const int2* tiles,
                       int ntiles, double* G, int64_t ldg, int packed, hipStream_t st) {
  hipLaunchKernelGGL(gram_f64_kernel, dim3(ntiles), dim3(256), 0, st, A, lda, w, Nk, tiles, ntiles, G, ldg,
                     packed);
  return hipGetLastError();
}

hipError_t gram_unpack_launch(const double* P, const int2* tiles, int ntiles, double* G, int64_t ldg,
                              hipStream_t st) {
  hipLaunchKernelGGL(gram_unpack_kernel, dim3(16, ntiles), dim3(256), 0, st, P, tiles, G, ldg);
  return hipGetLastError();
}

}  // namespace scs
