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
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "common.h"

namespace scs {

}  // namespace scs
#include "gram_strip.h"   // GT, GBK, swz, the GRAM_* flags and the latency strip body
namespace scs {

// Workgroup barrier that orders LDS only: the staged global loads (two stages
// ahead) stay in flight across it (a __syncthreads() here makes hipcc drain
// vmcnt(0) first).  "memory" clobbers keep the compiler from moving LDS
// accesses across.
#define LDS_BARRIER()                                          \
  do {                                                         \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");         \
    __builtin_amdgcn_s_barrier();                              \
    asm volatile("" ::: "memory");                             \
  } while (0)

// TI = 64-row wave groups along i: TI = 2 -> 128 x 128 tiles, 4 waves, 2 WG/CU;
// TI = 4 -> 256 x 128 tiles, 8 waves, 1 WG/CU (25 % less operand traffic per flop).
// TILED: operands are the panel-blocked A (common.h tiled_off), lda1/lda2 = S stages.
// CU-bounded persistent launches (BND instances; the Cholesky's bulk stream, chol.hip): a
// workgroup on a CU whose id within its shader engine (HW_REG_HW_ID bits 11:8) is set in `skip`
// leaves at once -- unless it is the launch's last arrival, so the tiles never depend on where
// the dispatcher puts the workgroups -- and every other workgroup claims tiles until none is left.
// The skipped CUs stay free for the serial chain's launches on the other stream (the effect of a
// CU-masked queue without one).  Claims keep the plain launch's XCD-aware split: the tile list is
// cut into 8 contiguous segments, a workgroup claims from its XCD's segment (HW_REG_XCC_ID) first
// and then from the others in turn.  ctr = {claims per segment [8], arrivals}, zero at launch.
__device__ __forceinline__ int bnd_claim(unsigned* ctr, int ntiles) {
  const int q8 = ntiles / 8, r8 = ntiles % 8;
  const int x0 = (int)((unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20) & 7u);   // HW_REG_XCC_ID
  for (int d = 0; d < 8; ++d) {
    const int x = (x0 + d) & 7, len = q8 + (x < r8 ? 1 : 0);
    if (len == 0) continue;
    const unsigned t = atomicAdd(ctr + x, 1u);
    if ((int)t < len) return x * q8 + (x < r8 ? x : r8) + (int)t;
  }
  return ntiles;
}
// skip: bits 0..15 the CU ids left free, bits 24..31 the XCDs (HW_REG_XCC_ID) where that applies
// (0: every XCD; r06, so that a few CUs of the chip -- not one per shader engine -- can be left free)
__device__ __forceinline__ int bnd_first(unsigned* ctr, unsigned skip, int ntiles, int* s) {
  if (threadIdx.x == 0) {
    const unsigned cu = ((unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 8) & 15u;   // HW_REG_HW_ID
    const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20) & 7u;       // HW_REG_XCC_ID
    const unsigned xm = skip >> 24;
    const bool here = ((skip >> cu) & 1u) && (xm == 0 || ((xm >> xcc) & 1u));
    const unsigned arr = atomicAdd(ctr + 8, 1u);
    *s = (here && arr + 1 < gridDim.x) ? -1 : bnd_claim(ctr, ntiles);
  }
  __syncthreads();
  return *s;
}
__device__ __forceinline__ int bnd_next(unsigned* ctr, int ntiles, int* s) {
  __syncthreads();   // every wave is done with the previous tile's LDS and with *s
  if (threadIdx.x == 0) *s = bnd_claim(ctr, ntiles);
  __syncthreads();
  return *s;
}

// The throughput kernels' epilogue for one 16-row MFMA tile row ti of a wave (4 x 4 accumulator
// registers; the C/D map and placements below).  With GRAM_ACCUMULATE the old values are loaded TJC
// 16-column tiles (4 TJC values) at a time before their stores: the compiler cannot prove the
// destinations distinct, and in the persistent (BND) launches it otherwise paid one memory round trip
// per element (64 per tile).  Same sums.  Only the BND forms use it: in the others the compiler
// already overlaps the loads, and the helper's register use slowed the main Gram (C2 Gram phase
// 92.1 -> 93.0 ms, profiles/r05/epi/).
template <int TJC = 2>
__device__ __forceinline__ void gram_tile_store_row(const v4d (&acc)[4], int ti, int wr, int wc, int g, int fl,
                                                    int part, double* P, int GTI, int packed, int upper,
                                                    int accumulate, double* G, int64_t ldg, int tix, int bi, int bj) {
  auto addr = [&](int tj, int r) -> double* {
    const int il = wr * 64 + 16 * ti + g + 4 * r;
    const int jl = wc * 64 + 16 * tj + fl;
    if (part >= 0) return P + ((int64_t)part * GT + jl) * GTI + il;
    if (packed) return G + ((int64_t)tix * (GTI / GT) + il / GT) * GT * GT + jl * GT + (il % GT);
    if (upper) return G + ((int64_t)bi * GTI + il) * ldg + (int64_t)bj * GT + jl;
    return G + ((int64_t)bj * GT + jl) * ldg + (int64_t)bi * GTI + il;
  };
  if (accumulate && part < 0) {
#pragma unroll
    for (int t0 = 0; t0 < 4; t0 += TJC) {
      double old[TJC][4];
#pragma unroll
      for (int t = 0; t < TJC; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) old[t][r] = *addr(t0 + t, r);
#pragma unroll
      for (int t = 0; t < TJC; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) *addr(t0 + t, r) = old[t][r] + acc[t0 + t][r];
    }
  } else {
#pragma unroll
    for (int tj = 0; tj < 4; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) *addr(tj, r) = acc[tj][r];
  }
}

template <bool NOLOAD, int TI, bool TILED = false, bool BND = false>
__global__ __launch_bounds__(128 * TI, (TI == 2 ? 2 : 1)) void gram_f64_kernel(
    const double* __restrict__ A1, int64_t lda1, const double* __restrict__ A2, int64_t lda2,
    const double* __restrict__ w, int64_t k0, int64_t Nk, const int2* __restrict__ tiles, int ntiles,
    double* __restrict__ G, int64_t ldg, int flags, const int4* __restrict__ work, int seglen, int nsplit,
    double* __restrict__ P) {
  constexpr int GTI = 64 * TI;               // tile rows (A1 panel width)
  constexpr int NT = 128 * TI;               // threads
  constexpr int SB = GTI * GBK + GT * GBK;   // doubles per LDS stage
  const int packed = flags & GRAM_PACKED, accumulate = flags & GRAM_ACCUMULATE, upper = flags & GRAM_UPPER;
  // All LDS in ONE array (cdna_hip_programming.md §5 item 4a): [buf][A1 panel GTI x 16 | A2 panel 128 x 16]
  __shared__ __attribute__((aligned(16))) double lds[2 * SB];

  // XCD-aware bijective remap (cdna_hip_programming.md §5 "XCD swizzle")
  const int orig = blockIdx.x;
  const int xcd = orig % 8;
  int bi, bj, tix, part = -1;
  __shared__ int s_claim;
  if constexpr (BND) {   // counters in P, skip mask in seglen (bnd_first)
    tix = bnd_first(reinterpret_cast<unsigned*>(P), (unsigned)seglen, ntiles, &s_claim);
    if (tix < 0 || tix >= ntiles) return;
    bi = tiles[tix].x;
    bj = tiles[tix].y;
  } else if (work) {
    // scheduled work list (gram_schedule): XCD x runs items [x*seglen, (x+1)*seglen) in order;
    // item = (bi, bj, ks, idx): ks < 0 -> whole K, canonical tile idx; ks >= 0 -> K piece ks of
    // nsplit, partial slot idx; bi < 0 -> padding
    const int4 it = work[xcd * seglen + orig / 8];
    if (it.x < 0) return;
    bi = it.x;
    bj = it.y;
    tix = it.w;
    if (it.z >= 0) {
      const int64_t L = ((Nk - k0 + (int64_t)nsplit * GBK - 1) / ((int64_t)nsplit * GBK)) * GBK;
      part = it.w;
      k0 = k0 + it.z * L;
      Nk = k0 + L < Nk ? k0 + L : Nk;
      if (Nk < k0) Nk = k0;
    }
  } else {
    const int q8 = ntiles / 8, r8 = ntiles % 8;
    tix = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const int2 tl = tiles[tix];
    bi = tl.x;
    bj = tl.y;
  }
bnd_tile:
  int tid_ = threadIdx.x;
  if constexpr (BND) asm volatile("" : "+v"(tid_));   // per tile: nothing derived from it is hoisted out of the loop
  const int tid = tid_, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const double* __restrict__ Ai = A1 + (int64_t)bi * GTI * lda1;
  const double* __restrict__ Aj = A2 + (int64_t)bj * GT * lda2;

  // staging map: chunk q = tid + NT*i  ->  feature f = (tid>>3) + (NT/8) i, chunk c = tid & 7
  constexpr int FS = NT / 8;                 // features per staging sweep
  constexpr int NA = GTI / FS, NB = GT / FS; // sweeps: A1 panel 4, A2 panel 4 (TI=2) or 2 (TI=4)
  const int sc = tid & 7;
  const int sf0 = tid >> 3;
  v2d ra[NA], rb[NB], rw;

  auto gload = [&](int64_t n0) {
    if (NOLOAD && n0 > k0) return;  // timing-only experiment: operands stay in registers
    if (TILED) {
      const int64_t so = (n0 >> 4) * (GT * GBK);
#pragma unroll
      for (int i = 0; i < NA; ++i)
        ra[i] = *(const v2d*)(A1 + tiled_off(lda1, 2 * sc, (int64_t)bi * GTI + sf0 + FS * i) + so);
#pragma unroll
      for (int i = 0; i < NB; ++i)
        rb[i] = *(const v2d*)(A2 + tiled_off(lda2, 2 * sc, (int64_t)bj * GT + sf0 + FS * i) + so);
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) ra[i] = *(const v2d*)(Ai + (int64_t)(sf0 + FS * i) * lda1 + n0 + 2 * sc);
#pragma unroll
      for (int i = 0; i < NB; ++i) rb[i] = *(const v2d*)(Aj + (int64_t)(sf0 + FS * i) * lda2 + n0 + 2 * sc);
    }
    rw = *(const v2d*)(w + n0 + 2 * sc);
  };
  auto swrite = [&](int buf) {
    double* la = lds + buf * SB;
    double* lb = la + GTI * GBK;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int f = sf0 + FS * i;
      *(v2d*)(la + f * GBK + 2 * (sc ^ swz(f))) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int f = sf0 + FS * i;
      *(v2d*)(lb + f * GBK + 2 * (sc ^ swz(f))) = rb[i] * rw;
    }
  };

  v4d acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4d){0.0, 0.0, 0.0, 0.0};

  const int fl = lane & 15, g = lane >> 4, s = swz(fl);
  const int nk = (int)((Nk - k0) / GBK);

  if (nk > 0) {
    gload(k0);
    swrite(0);
  }
  __syncthreads();
  for (int k = 0; k < nk; ++k) {
    if (k + 1 < nk) gload(k0 + (int64_t)(k + 1) * GBK);
    const double* la = lds + (k & 1) * SB;
    const double* lb = la + GTI * GBK;
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
  // (cdna_hip_programming.md §3; verified by probe_mfma).  Element (i, j) of the
  // tile (i in panel bi of A1, j in panel bj of A2) goes to
  //   packed : tile-local column-major slot tix  (row i, col j)
  //   upper  : G[(bi*128+i)*ldg + bj*128+j]       (transposed: row j, col i -- the
  //            upper triangle when bi >= bj; consecutive lanes store consecutive j)
  //   default: G[(bj*128+j)*ldg + bi*128+i]       (lower triangle when bi >= bj)
  if constexpr (BND || !TILED) {   // the persistent and two-operand gen launches: old values loaded first
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
      gram_tile_store_row(acc[ti], ti, wr, wc, g, fl, part, P, GTI, packed, upper, accumulate, G, ldg, tix, bi, bj);
  } else {
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
#pragma unroll
      for (int tj = 0; tj < 4; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int il = wr * 64 + 16 * ti + g + 4 * r;
          const int jl = wc * 64 + 16 * tj + fl;
          double* dst;
          if (part >= 0) {
            P[((int64_t)part * GT + jl) * GTI + il] = acc[ti][tj][r];
            continue;
          }
          if (packed) dst = G + ((int64_t)tix * (GTI / GT) + il / GT) * GT * GT + jl * GT + (il % GT);
          else if (upper) dst = G + ((int64_t)bi * GTI + il) * ldg + (int64_t)bj * GT + jl;
          else dst = G + ((int64_t)bj * GT + jl) * ldg + (int64_t)bi * GTI + il;
          if (accumulate) *dst += acc[ti][tj][r];
          else *dst = acc[ti][tj][r];
        }
  }
  if constexpr (BND) {
    tix = bnd_next(reinterpret_cast<unsigned*>(P), ntiles, &s_claim);
    if (tix >= ntiles) return;
    bi = tiles[tix].x;
    bj = tiles[tix].y;
    goto bnd_tile;
  }
}

// ---------------------------------------------------------------------------
// LDS-DMA variant of the 256 x 128 tile (8 waves, one workgroup per CU).
// Operands go global -> LDS with global_load_lds_dwordx4 (no VGPR staging)
// into a 3-deep ring of 16-sample stages (48 KiB each); per stage every wave
// issues 6 DMA instructions (1 KiB = 8 feature rows each).  The LDS image is
// lane-linear, so the XOR swizzle moves to the per-lane SOURCE address (lane
// L of an instruction fills row 8i + L/8, slot L%8 with global chunk
// slot ^ swz(row); cdna_hip_programming.md §5.4 rule 21) and the fragment
// reads are unchanged.  w is staged by wave 0 in 1 KiB blocks (8 stages) and
// applied to the B fragments in registers (the same products b·w the register
// path stores).  Iteration k: counted s_waitcnt vmcnt(6) (stage k landed, stage
// k+1 stays in flight) + raw s_barrier, then the DMA of stage k+2 into the
// buffer read in iteration k-1, then the MFMAs on stage k.
constexpr int GL_STAGES = 3;
constexpr int GL_SA = 256 * GBK;
constexpr int GL_SS = GL_SA + GT * GBK;
constexpr int GL_W = 128;

__device__ __forceinline__ void glds16(const double* src, double* dst) {
  __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// TILED: A is stored panel-blocked, block (panel p, stage s) = [128 features][16 samples]
// contiguous (16 KiB) at ((p * lda + s) * 128) * 16 doubles, lda = number of 16-sample stages.
// PIPE (1, 2 = no-load timing build): fragment reads software-pipelined across the
// barrier.  Each stage's MFMAs run in two halves (samples 0-7 / 8-15 of the stage);
// iteration k: ds_read F(k,1) | MFMA F(k,0) | wait stage k+1 + barrier | DMA stage
// k+3 into the slot of stage k | ds_read F(k+1,0) | MFMA F(k,1).  No MFMA then
// waits on LDS latency after a barrier (both waves of a SIMD leave it together and
// would otherwise stall on their first fragments at the same time).  Same stages
// in flight (2) as the plain loop; w is applied to B in registers at use.
template <bool TILED, int PIPE = 0>
__global__ __launch_bounds__(512, 1) void gram_glds_kernel(
    const double* __restrict__ A1, int64_t lda1, const double* __restrict__ A2, int64_t lda2,
    const double* __restrict__ w, int64_t k0, int64_t Nk, const int2* __restrict__ tiles, int ntiles,
    double* __restrict__ G, int64_t ldg, int flags, const int4* __restrict__ work, int seglen, int nsplit,
    double* __restrict__ P) {
  constexpr int GTI = 256;
  const int packed = flags & GRAM_PACKED, accumulate = flags & GRAM_ACCUMULATE, upper = flags & GRAM_UPPER;
  __shared__ __attribute__((aligned(16))) double lds[GL_STAGES * GL_SS + 2 * GL_W];

  const int orig = blockIdx.x;
  const int xcd = orig % 8;
  int bi, bj, tix, part = -1;
  if (work) {
    const int4 it = work[xcd * seglen + orig / 8];
    if (it.x < 0) return;
    bi = it.x;
    bj = it.y;
    tix = it.w;
    if (it.z >= 0) {
      const int64_t L = ((Nk - k0 + (int64_t)nsplit * GBK - 1) / ((int64_t)nsplit * GBK)) * GBK;
      part = it.w;
      k0 = k0 + it.z * L;
      Nk = k0 + L < Nk ? k0 + L : Nk;
      if (Nk < k0) Nk = k0;
    }
  } else {
    const int q8 = ntiles / 8, r8 = ntiles % 8;
    tix = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const int2 tl = tiles[tix];
    bi = tl.x;
    bj = tl.y;
  }

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  // this wave's 6 DMA instructions per stage: j = 6 wv + i; j < 32 -> A1 rows 8j.., else A2 rows 8(j-32)..
  const double* src[6];
  int dsto[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int j = 6 * wv + i;
    const bool isA = j < 32;
    const int f = 8 * (isA ? j : j - 32) + (lane >> 3);
    const int slot = lane & 7;
    const int cch = slot ^ swz(f);
    if (TILED) {
      const int64_t pnl = isA ? 2 * (int64_t)bi + (f >> 7) : (int64_t)bj;
      src[i] = (isA ? A1 : A2) + (pnl * (isA ? lda1 : lda2) * GT + (f & 127)) * GBK + 2 * cch;
    } else {
      src[i] = isA ? A1 + ((int64_t)bi * GTI + f) * lda1 + 2 * cch : A2 + ((int64_t)bj * GT + f) * lda2 + 2 * cch;
    }
    dsto[i] = isA ? 8 * j * GBK : GL_SA + 8 * (j - 32) * GBK;
  }
  const int nk = (int)((Nk - k0) / GBK);
  auto issue = [&](int st) {
    const int64_t n0 = k0 + (int64_t)st * GBK;
    double* base = lds + (st % GL_STAGES) * GL_SS;
#pragma unroll
    for (int i = 0; i < 6; ++i) glds16(src[i] + (TILED ? (n0 / GBK) * (GT * GBK) : n0), base + dsto[i]);
    if (__builtin_amdgcn_readfirstlane(wv) == 0 && (st & 7) == 0) {
      const int64_t nw = n0 + 2 * lane < Nk - 1 ? n0 + 2 * lane : Nk - 2;   // clamp past the K range (unused)
      glds16(w + nw, lds + GL_STAGES * GL_SS + ((st >> 3) & 1) * GL_W);
    }
  };

  v4d acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4d){0.0, 0.0, 0.0, 0.0};
  const int fl = lane & 15, g = lane >> 4, sw = swz(fl);

  if (PIPE) {
    // fragment set: A rows (4 v2d), raw B rows (4 v2d), w pair of this lane group
    struct Frag { v2d a[4], b[4], w; };
    auto fread = [&](int st, int p, Frag& F) {
      const double* la = lds + (st % GL_STAGES) * GL_SS;
      const double* lb = la + GL_SA;
      const double* lw = lds + GL_STAGES * GL_SS + ((st >> 3) & 1) * GL_W + (st & 7) * GBK;
      const int c = 4 * p + g;
      const int pc = (c ^ sw) * 2;
      F.w = *(const v2d*)(lw + 2 * c);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        F.a[t] = *(const v2d*)(la + (wr * 64 + 16 * t + fl) * GBK + pc);
        F.b[t] = *(const v2d*)(lb + (wc * 64 + 16 * t + fl) * GBK + pc);
      }
    };
    auto mm = [&](const Frag& F) {
      v2d b[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) b[t] = F.b[t] * F.w;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ti = 0; ti < 4; ++ti)
#pragma unroll
          for (int tj = 0; tj < 4; ++tj)
            acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(F.a[ti][u], b[tj][u], acc[ti][tj], 0, 0, 0);
    };
    const bool live = PIPE == 1;
    // waits are __builtin_amdgcn_s_waitcnt (gfx9 encoding: vmcnt[3:0] | expcnt<<4 | lgkmcnt<<8 |
    // vmcnt[5:4]<<14), visible to the compiler's waitcnt pass, unlike inline asm
    Frag X, Y;
    if (nk > 0) {
      issue(0);
      if (nk > 1) issue(1);
      if (nk > 2) issue(2);
      if (nk > 2) __builtin_amdgcn_s_waitcnt(0x0F7C);   // vmcnt(12)
      else if (nk > 1) __builtin_amdgcn_s_waitcnt(0x0F76);   // vmcnt(6)
      else __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      fread(0, 0, X);
    }
    // one iteration; has1/2/3 = stages k+1/k+2/k+3 exist (compile-time true in the
    // steady-state loop, so its body has no branches for the waitcnt pass to merge over)
    auto body = [&](int k, bool has1, bool has2, bool has3) {
      // X was read during the previous mm(Y) (32 MFMAs ago): retire it explicitly so the Y reads
      // below do not push the LDS queue past lgkmcnt's 4-bit range (which would make the
      // compiler wait for Y too before mm(X))
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
      fread(k, 1, Y);
      __builtin_amdgcn_sched_barrier(0);   // issue all fragment reads before the MFMAs
      mm(X);
      __builtin_amdgcn_sched_barrier(0);   // keep mm(X) above the barrier (MFMAs are not memory ops)
      if (has1) {
        if (has2) __builtin_amdgcn_s_waitcnt(0x0F76);   // vmcnt(6)
        else __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (has3 && live) issue(k + 3);
      if (has1) fread(k + 1, 0, X);
      __builtin_amdgcn_sched_barrier(0);
      mm(Y);
      __builtin_amdgcn_sched_barrier(0);
    };
    int k = 0;
    for (; k + 3 < nk; ++k) body(k, true, true, true);
    for (; k < nk; ++k) body(k, k + 1 < nk, k + 2 < nk, false);
  } else {
  if (nk > 0) issue(0);
  if (nk > 1) issue(1);
  for (int k = 0; k < nk; ++k) {
    if (k + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (k + 2 < nk) issue(k + 2);
    const double* la = lds + (k % GL_STAGES) * GL_SS;
    const double* lb = la + GL_SA;
    const double* lw = lds + GL_STAGES * GL_SS + ((k >> 3) & 1) * GL_W + (k & 7) * GBK;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int c = 4 * p + g;
      const int pc = (c ^ sw) * 2;
      v2d a[4], b[4];
      const v2d wv2 = *(const v2d*)(lw + 2 * c);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = *(const v2d*)(la + (wr * 64 + 16 * t + fl) * GBK + pc);
        b[t] = *(const v2d*)(lb + (wc * 64 + 16 * t + fl) * GBK + pc) * wv2;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ti = 0; ti < 4; ++ti)
#pragma unroll
          for (int tj = 0; tj < 4; ++tj)
            acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti][u], b[tj][u], acc[ti][tj], 0, 0, 0);
    }
  }
  }

#pragma unroll
  for (int ti = 0; ti < 4; ++ti)
#pragma unroll
    for (int tj = 0; tj < 4; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = wr * 64 + 16 * ti + g + 4 * r;
        const int jl = wc * 64 + 16 * tj + fl;
        if (part >= 0) {
          P[((int64_t)part * GT + jl) * GTI + il] = acc[ti][tj][r];
          continue;
        }
        double* dst;
        if (packed) dst = G + ((int64_t)tix * (GTI / GT) + il / GT) * GT * GT + jl * GT + (il % GT);
        else if (upper) dst = G + ((int64_t)bi * GTI + il) * ldg + (int64_t)bj * GT + jl;
        else dst = G + ((int64_t)bj * GT + jl) * ldg + (int64_t)bi * GTI + il;
        if (accumulate) *dst += acc[ti][tj][r];
        else *dst = acc[ti][tj][r];
      }
}

// Scatter packed tiles (list order) into the upper triangle of a column-major m_pad x m_pad matrix
// (same placement as GRAM_UPPER) and the inverse.  A packed slot holds tile element (i, j) at
// i + 128 j, G holds it at (x·128 + i)·ldg + y·128 + j: a transpose, so each workgroup moves one
// 64 x 64 quarter through LDS -- reads and writes both along the contiguous index (r04: the
// element-wise form wrote G with a stride of ldg between lanes; the exchange path's step at C3's
// per-rank shape lost 1.3 ms with this, profiles/r04/unpack/).  Grid (4 quarters, ntiles), 256 threads.
template <bool UNPACK>
__global__ __launch_bounds__(256) void gram_packx_kernel(const double* __restrict__ src, double* __restrict__ dst,
                                                         const int2* __restrict__ tiles, int64_t ldg) {
  __shared__ double q[64][65];
  const int t = blockIdx.y, i0 = 64 * (blockIdx.x & 1), j0 = 64 * (blockIdx.x >> 1);
  const int2 tl = tiles[t];
  const int64_t slot = (int64_t)t * GT * GT;
  const int64_t gbase = ((int64_t)tl.x * GT) * ldg + (int64_t)tl.y * GT;
  const int a = threadIdx.x & 63, b0 = threadIdx.x >> 6;
  if (UNPACK) {   // packed -> LDS along i, LDS -> G along j
    for (int b = b0; b < 64; b += 4) q[b][a] = src[slot + (int64_t)(j0 + b) * GT + i0 + a];   // q[j][i]
    __syncthreads();
    for (int b = b0; b < 64; b += 4) dst[gbase + (int64_t)(i0 + b) * ldg + j0 + a] = q[a][b];
  } else {        // G -> LDS along j, LDS -> packed along i
    for (int b = b0; b < 64; b += 4) q[b][a] = src[gbase + (int64_t)(i0 + b) * ldg + j0 + a];  // q[i][j]
    __syncthreads();
    for (int b = b0; b < 64; b += 4) dst[slot + (int64_t)(j0 + b) * GT + i0 + a] = q[a][b];
  }
}

hipError_t gram_pack_launch(const double* G, int64_t ldg, const int2* tiles, int ntiles, double* P, hipStream_t st) {
  if (ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(gram_packx_kernel<false>, dim3(4, ntiles), dim3(256), 0, st, G, P, tiles, ldg);
  return hipGetLastError();
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

// Super-blocked list of 256 x 128 tiles (BI, bj) for the TI = 4 kernel: row block
// BI covers 128-blocks 2BI, 2BI+1; every tile with bj <= 2BI+1 (the one above the
// diagonal holds the mirror values, stored harmlessly below it).  nb even.
void gram_tile_list_tall(int nb, int2* out, int* ntiles) {
  const int nbi = nb / 2, SI = 4, SJ = 8;
  int t = 0;
  for (int sbi = 0; sbi < (nbi + SI - 1) / SI; ++sbi)
    for (int sbj = 0; sbj <= sbi; ++sbj)
      for (int I = sbi * SI; I < (sbi + 1) * SI && I < nbi; ++I)
        for (int j = sbj * SJ; j < (sbj + 1) * SJ && j < nb; ++j)
          if (j <= 2 * I + 1) out[t++] = make_int2(I, j);
  *ntiles = t;
}

// Row-major lower-triangle order: the first nb'(nb'+1)/2 entries are the list for nb' <= nb.
void gram_tile_list_rowmajor(int nb, int2* out) {
  int t = 0;
  for (int i = 0; i < nb; ++i)
    for (int j = 0; j <= i; ++j) out[t++] = make_int2(i, j);
}

hipError_t gram_launch_gen(const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w,
                           int64_t k0, int64_t k1, const int2* tiles, int ntiles, double* G, int64_t ldg, int flags,
                           hipStream_t st);

// ---------------------------------------------------------------------------
// Interleaved-schedule Gram tiles on the panel-blocked A (4 waves, 2 x 2).
//   TI = 2: 128 x 128 tile, 4 waves, <= 256 VGPRs -> 2 workgroups / CU;
//   TI = 4: 256 x 128 tile, 8 waves, one workgroup per CU, 25 % less operand
//           traffic per flop.  Each wave holds 64 x 64 (16 accumulators).
// One LDS buffer per workgroup (the A1 and A2 stage blocks); the next stage waits
// in registers.  Iteration k (stage k in LDS, its p = 0 fragments F0 already in
// registers, stage k+1 in registers R):
//   phase 1 : the p = 0 MFMAs, the p = 1 fragment reads F1 interleaved;
//             lgkmcnt(0) + barrier (every wave is done reading stage k)
//   phase 2a: R -> LDS (A2 rows scaled by w), the global loads of stage k+2 into
//             R, interleaved with 3/4 of the p = 1 MFMAs; lgkmcnt(0) + barrier
//   phase 2b: the F0 reads of stage k+1 interleaved with the last 1/4.
// No phase waits on LDS latency (measured: the no-load build of this structure
// runs at ~97 % of the fp64 MFMA peak per round, one or two waves per SIMD), the
// global loads have a whole iteration to land, and the MFMA order per
// accumulator is the plain loop's (p, u) order: G is bitwise identical to
// gram_f64_kernel / gram_glds_kernel of the same tile height.
// CM: column-major operands (the Cholesky's trailing updates, gen form with A1 == A2),
// S = leading dimension; stage k of feature f is the 16 samples at f * S + k0 + 16 k.
// AV: the same pass also forms Aᵀv (the Jᵀr / ∇f product of the step, SURVEY §8d "one fused
// Gram + Aᵀv pass"): the tile whose row block holds its column panel (bi = bj GT / GTI, one
// per panel in both tile lists) accumulates its raw A2 registers times v while staging them,
// so Aᵀv costs no HBM pass of its own.  Per thread a running fma over its samples in stage
// order, then a fixed 8-lane butterfly; piece p of a K-split tile writes row p of VP (row
// stride vps, features of panel bj), summed in piece order by gram_vfinal_kernel.  G is
// unchanged bit for bit (the MFMA stream is the same).
template <int PIPE, int TI = 2, bool CM = false, bool AV = false, bool BND = false>
__global__ __launch_bounds__(128 * TI, (TI == 2 ? 2 : 1)) void gram_sia_kernel(
    const double* __restrict__ A, int64_t S, const double* __restrict__ w, int64_t k0, int64_t Nk,
    const int2* __restrict__ tiles, int ntiles, double* __restrict__ G, int64_t ldg, int flags,
    const int4* __restrict__ work, int seglen, int nsplit, double* __restrict__ P,
    const double* __restrict__ v, double* __restrict__ VP, int64_t vps, unsigned* __restrict__ scnt, int sob,
    const double* __restrict__ A2, int64_t S2) {
  static_assert(!(AV && CM), "the fused Aᵀv runs on the panel-blocked A only");
  constexpr int GTI = 64 * TI;        // tile rows (A1 features)
  constexpr int NT = 128 * TI;        // threads
  constexpr int FS = NT / 8;          // features per staging sweep
  constexpr int NTI = 4;              // 16-row MFMA tiles per wave along i
  constexpr int NA = GTI / FS;        // A1 staging chunks per thread per stage (4)
  constexpr int NB = GT / FS;         // A2 staging chunks per thread per stage (4 or 2)
  constexpr int NMM = 2 * NTI * 4;    // MFMAs per fragment set (2 u x NTI x 4)
  constexpr int NRD = NTI + 4;        // ds_read_b128 per fragment set
  constexpr int TAIL = NMM / 4;       // MFMAs left for phase 2b (1/8 and 3/8 measured within noise)
  const int packed = flags & GRAM_PACKED, accumulate = flags & GRAM_ACCUMULATE, upper = flags & GRAM_UPPER;
  __shared__ __attribute__((aligned(16))) double lds[(GTI + GT) * GBK];
  const int orig = blockIdx.x;
  const int xcd = orig % 8;
  int bi, bj, tix, part = -1, piece = 0;
  __shared__ int s_claim;
  if constexpr (BND) {   // counters in scnt, skip mask in sob (bnd_first)
    tix = bnd_first(scnt, (unsigned)sob, ntiles, &s_claim);
    if (tix < 0 || tix >= ntiles) return;
    bi = tiles[tix].x;
    bj = tiles[tix].y;
  } else if (work) {
    const int4 it = work[xcd * seglen + orig / 8];
    if (it.x < 0) return;
    bi = it.x;
    bj = it.y;
    tix = it.w;
    if (it.z >= 0) {
      piece = it.z;
      const int64_t L = ((Nk - k0 + (int64_t)nsplit * GBK - 1) / ((int64_t)nsplit * GBK)) * GBK;
      part = it.w;
      k0 = k0 + it.z * L;
      Nk = k0 + L < Nk ? k0 + L : Nk;
      if (Nk < k0) Nk = k0;
    }
  } else {
    const int q8 = ntiles / 8, r8 = ntiles % 8;
    tix = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const int2 tl = tiles[tix];
    bi = tl.x;
    bj = tl.y;
  }
bnd_tile:
  int tid_ = threadIdx.x;
  if constexpr (BND) asm volatile("" : "+v"(tid_));   // per tile: nothing derived from it is hoisted out of the loop
  const int tid = tid_, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int sc = tid & 7, sf0 = tid >> 3;
  const int64_t st0 = k0 / GBK;
  // this thread's 16-B chunks of a stage: feature sf0 + FS i of the A1 rows (panel
  // (GTI/128) bi + f/128) and of the A2 rows (panel bj), samples 2 sc, 2 sc + 1.
  const double* srcA = CM ? A + ((int64_t)bi * GTI + sf0) * S + k0 + 2 * sc
                          : A + ((int64_t)bi * (GTI / GT) * S + st0) * GT * GBK + sf0 * GBK + 2 * sc;
  // CM with A2: the A2 panels from a second column-major matrix (leading dimension S2; the LU's and
  // the QR's two-operand products, the Cholesky's strip solves), else from A
  const double* B2 = (CM && A2) ? A2 : A;
  const int64_t SB2 = (CM && A2) ? S2 : S;
  const double* srcB = CM ? B2 + ((int64_t)bj * GT + sf0) * SB2 + k0 + 2 * sc
                          : A + ((int64_t)bj * S + st0) * GT * GBK + sf0 * GBK + 2 * sc;
  const double* srcW = w + k0 + 2 * sc;
  const double* srcV = AV ? v + k0 + 2 * sc : nullptr;
  double* la = lds;
  double* lb = lds + GTI * GBK;
  int woff[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int f = sf0 + FS * i;
    woff[i] = f * GBK + 2 * (sc ^ swz(f));
  }
  v2d ra[NA], rb[NB], rw, rv;
  double av[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) av[i] = 0.0;
  // fa: std::bool_constant -- the designated tiles of an AV launch run the loop with the Aᵀv
  // products (FA), every other tile the plain loop (no extra loads or VALU)
  auto gload = [&](int64_t st, auto fa) {
    constexpr bool FA = decltype(fa)::value;
    if (PIPE == 3 && st >= 2) return;   // timing build: no global loads after the prologue
    if (CM) {
#pragma unroll
      for (int i = 0; i < NA; ++i) ra[i] = *(const v2d*)(srcA + st * GBK + (int64_t)FS * i * S);
#pragma unroll
      for (int i = 0; i < NB; ++i) rb[i] = *(const v2d*)(srcB + st * GBK + (int64_t)FS * i * SB2);
    } else {
      const int64_t so = st * GT * GBK;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int f = FS * i;   // + sf0 (in srcA): the panel of f is f / 128 (FS divides 128)
        ra[i] = *(const v2d*)(srcA + so + (f >> 7) * S * GT * GBK + (f & 127) * GBK);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) rb[i] = *(const v2d*)(srcB + so + FS * GBK * i);
    }
    rw = *(const v2d*)(srcW + st * GBK);
    if (FA) rv = *(const v2d*)(srcV + st * GBK);
  };
  auto swrite = [&](auto fa) {
    constexpr bool FA = decltype(fa)::value;
#pragma unroll
    for (int i = 0; i < NA; ++i) *(v2d*)(la + woff[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i) *(v2d*)(lb + woff[i]) = rb[i] * rw;
    if (FA) {
#pragma unroll
      for (int i = 0; i < NB; ++i) av[i] = __builtin_fma(rb[i][1], rv[1], __builtin_fma(rb[i][0], rv[0], av[i]));
    }
  };
  const int fl = lane & 15, g = lane >> 4, s = swz(fl);
  struct Frag {
    v2d a[NTI], b[4];
  };
  auto fread = [&](int p, Frag& F) {
    const int pc = ((4 * p + g) ^ s) * 2;
#pragma unroll
    for (int t = 0; t < NTI; ++t) F.a[t] = *(const v2d*)(la + (wr * 64 + 16 * t + fl) * GBK + pc);
#pragma unroll
    for (int t = 0; t < 4; ++t) F.b[t] = *(const v2d*)(lb + (wc * 64 + 16 * t + fl) * GBK + pc);
  };
  v4d acc[NTI][4];
#pragma unroll
  for (int i = 0; i < NTI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4d){0.0, 0.0, 0.0, 0.0};
  // MFMAs n in [n0, n1) of a fragment set, n = 4 NTI u + 4 ti + tj (the plain loop's order)
  auto mm = [&](const Frag& F, int n0, int n1) {
#pragma unroll
    for (int n = n0; n < n1; ++n) {
      const int u = n / (4 * NTI), ti = (n / 4) % NTI, tj = n & 3;
      acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(F.a[ti][u], F.b[tj][u], acc[ti][tj], 0, 0, 0);
    }
  };
  auto barrier = [&]() {   // also a scheduling fence: nothing (e.g. the w products) crosses a phase
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS traffic is done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  const int nk = (int)((Nk - k0) / GBK);
  Frag F0, F1;
  auto run = [&](auto fa) {
    if (nk > 0) {
      gload(0, fa);
      swrite(fa);
      if (nk > 1) gload(1, fa);
      barrier();
      fread(0, F0);
    }
    auto body = [&](int k, bool has1, bool has2) {
      // phase 1
      __builtin_amdgcn_sched_barrier(0);
      fread(1, F1);
      mm(F0, 0, NMM);
      if (PIPE) {
#pragma unroll
        for (int i = 0; i < NRD; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, NMM / NRD, 0);   // MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);           // DS read
        }
      }
      barrier();
      // phase 2a
      if (has1) swrite(fa);
      if (has2) gload(k + 2, fa);
      mm(F1, 0, NMM - TAIL);
      if (PIPE) {
        if (has1) {
#pragma unroll
          for (int i = 0; i < NA + NB; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, (NMM - TAIL) / (NA + NB), 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                         // DS write
            if (has2) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);               // VMEM read
          }
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NMM, 0);
      }
      // phase 2b
      if (has1) {
        barrier();
        fread(0, F0);
      }
      mm(F1, NMM - TAIL, NMM);
      if (PIPE && has1) {
#pragma unroll
        for (int i = 0; i < NRD; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, TAIL / NRD > 0 ? TAIL / NRD : 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
    };
    int k = 0;
    for (; k + 2 < nk; ++k) body(k, true, true);
    if (k + 1 < nk) {
      body(k, true, false);
      ++k;
    }
    if (k < nk) body(k, false, false);
  };
  const bool dav = AV && (int64_t)bj * GT / GTI == bi;   // this tile owns panel bj's Aᵀv rows
  if constexpr (AV) {
    if (dav) run(std::true_type{});
    else run(std::false_type{});
  } else {
    run(std::false_type{});
  }

  if (dav) {   // lanes 8q .. 8q+7 share a feature
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      double t = av[i];
      t += __shfl_xor(t, 1);
      t += __shfl_xor(t, 2);
      t += __shfl_xor(t, 4);
      if (sc == 0) VP[(int64_t)piece * vps + (int64_t)bj * GT + sf0 + FS * i] = t;
    }
  }

  // epilogue (the C/D map of gram_f64_kernel): element (il, jl) of the GTI x 128 tile
  if constexpr (BND || CM) {   // the persistent and gen-form launches: old values loaded ahead of the stores
#pragma unroll
    for (int ti = 0; ti < NTI; ++ti)
      gram_tile_store_row(acc[ti], ti, wr, wc, g, fl, part, P, GTI, packed, upper, accumulate, G, ldg, tix, bi, bj);
  } else {
#pragma unroll
    for (int ti = 0; ti < NTI; ++ti)
#pragma unroll
      for (int tj = 0; tj < 4; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int il = wr * 64 + 16 * ti + g + 4 * r;
          const int jl = wc * 64 + 16 * tj + fl;
          double* dst;
          if (part >= 0) {
            P[((int64_t)part * GT + jl) * GTI + il] = acc[ti][tj][r];
            continue;
          }
          if (packed) dst = G + ((int64_t)tix * (GTI / GT) + il / GT) * GT * GT + jl * GT + (il % GT);
          else if (upper) dst = G + ((int64_t)bi * GTI + il) * ldg + (int64_t)bj * GT + jl;
          else dst = G + ((int64_t)bj * GT + jl) * ldg + (int64_t)bi * GTI + il;
          if (accumulate) *dst += acc[ti][tj][r];
          else *dst = acc[ti][tj][r];
        }
  }
  // strip completion (scsopt.cpp gram_factor_pipelined, one-launch mode): this tile's rows lie in
  // outer strip bj / sob; each thread's stores are released to device scope before one count
  if (!BND && scnt && part < 0) {
    __threadfence();
    __syncthreads();
    if (tid == 0) atomicAdd(scnt + bj / sob, 1u);
  }
  if constexpr (BND) {
    tix = bnd_next(scnt, ntiles, &s_claim);
    if (tix >= ntiles) return;
    bi = tiles[tix].x;
    bj = tiles[tix].y;
    goto bnd_tile;
  }
}

// Main-Gram kernel selection (A/B switches, read once):
//   SCS_GRAM_SIA  (128 x 128 tiles): unset/1 = interleaved-schedule kernel, 2 = same kernel with
//                 the compiler's schedule, 0 = register-staged gram_f64_kernel;
//   SCS_GRAM_GLDS (256 x 128 tiles): unset/3 = interleaved-schedule kernel, 2 = LDS-DMA ring with
//                 pipelined fragment reads, 1 = LDS-DMA plain loop, 0 = register-staged.
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
int gram_sia_mode() {
  static const int v = env_int("SCS_GRAM_SIA", 1);
  return v;
}
int gram_tall_mode() {
  static const int v = env_int("SCS_GRAM_GLDS", 3);
  return v;
}

// The fused Aᵀv (AV kernels) rides on the default interleaved kernels.  Default: the 256 x 128
// kernel only (C3: the separate 24 ms pass goes, the Gram grows by ~7 ms); on 128 x 128 tiles the
// designated tiles' longer loop costs more than the pass (C2: 111.0 vs 110.4 ms per step), so
// SCS_GRAM_FUSE=2 enables it there too, 0 turns it off (read per call; the tests' references).
int gram_fuse_ok(int tall) {
  const char* e = getenv("SCS_GRAM_FUSE");
  const int mode = e ? atoi(e) : 1;
  if (mode == 0 || (!tall && mode < 2)) return 0;
  return tall ? gram_tall_mode() == 3 : gram_sia_mode() == 1;
}

__global__ void gram_vfinal_kernel(const double* __restrict__ VP, int npiece, int64_t vps, int64_t m,
                                   double* __restrict__ out) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= m) return;
  double s = VP[f];
  for (int p = 1; p < npiece; ++p) s += VP[(int64_t)p * vps + f];
  out[f] = s;
}

hipError_t gram_vfinal_launch(const double* VP, int npiece, int64_t vps, int64_t m, double* out, hipStream_t st) {
  hipLaunchKernelGGL(gram_vfinal_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, VP, npiece, vps, m, out);
  return hipGetLastError();
}

// the kernel of the latest main Gram launch (gram_launch / gram_launch_sched), as rocprofv3 names it
static thread_local const char* g_main_name = "";   // per host thread: a multi-device context drives its devices from one thread each
const char* gram_main_kernel_name() { return g_main_name; }

hipError_t gram_launch(const double* A, int64_t lda, const double* w, int64_t Nk, const int2* tiles,
                       int ntiles, double* G, int64_t ldg, int packed, int tall, hipStream_t st, const double* v,
                       double* VP, int64_t vps) {
  if (ntiles <= 0) return hipSuccess;
  // packed: bit 0 = packed slots (else the upper triangle), bit 1 = accumulate into G
  const int flags = ((packed & 1) ? GRAM_PACKED : GRAM_UPPER) | ((packed & 2) ? GRAM_ACCUMULATE : 0);
  if (v) {
    if (!gram_fuse_ok(tall)) return hipErrorInvalidValue;
    if (tall) {
      g_main_name = "gram_sia_kernel<1, 4, false, true, false>";
      hipLaunchKernelGGL((gram_sia_kernel<1, 4, false, true>), dim3(ntiles), dim3(512), 0, st, A, lda, w, (int64_t)0,
                         Nk, tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, v, VP, vps, nullptr, 0, nullptr, (int64_t)0);
    } else {
      g_main_name = "gram_sia_kernel<1, 2, false, true, false>";
      hipLaunchKernelGGL((gram_sia_kernel<1, 2, false, true>), dim3(ntiles), dim3(256), 0, st, A, lda, w, (int64_t)0,
                         Nk, tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, v, VP, vps, nullptr, 0, nullptr, (int64_t)0);
    }
    return hipGetLastError();
  }
  if (!tall && gram_sia_mode() == 0) {
    g_main_name = "gram_f64_kernel<false, 2, true, false>";
    hipLaunchKernelGGL((gram_f64_kernel<false, 2, true>), dim3(ntiles), dim3(256), 0, st, A, lda, A, lda, w,
                       (int64_t)0, Nk, tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  } else if (!tall) {
    g_main_name = "gram_sia_kernel<1, 2, false, false, false>";
    hipLaunchKernelGGL((gram_sia_kernel<1, 2>), dim3(ntiles), dim3(256), 0, st, A, lda, w, (int64_t)0, Nk, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, nullptr, nullptr, (int64_t)0, nullptr, 0, nullptr, (int64_t)0);
  } else if (gram_tall_mode() == 3) {
    g_main_name = "gram_sia_kernel<1, 4, false, false, false>";
    hipLaunchKernelGGL((gram_sia_kernel<1, 4>), dim3(ntiles), dim3(512), 0, st, A, lda, w, (int64_t)0, Nk, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, nullptr, nullptr, (int64_t)0, nullptr, 0, nullptr, (int64_t)0);
  } else {
    g_main_name = "gram_glds_kernel<true, 1>";
    hipLaunchKernelGGL((gram_glds_kernel<true, 1>), dim3(ntiles), dim3(512), 0, st, A, lda, A, lda, w, (int64_t)0, Nk,
                       tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  }
  return hipGetLastError();
}

// Latency variant for the small launches of the Cholesky and the LU (short K or few
// tiles): each 128 x 128 list tile is computed by 128/QC workgroups, one per QC-column
// strip (4 waves of 32 rows x QC along the rows).  A workgroup reads the A2 columns it
// writes and nothing else of the output, so the in-place panel solve (G == A2) stays
// race-free.  The global loads run RING stages (RING x 16 samples) ahead of the MFMAs in a
// register ring: one K = 128 launch pays one memory latency, not one per 16-sample stage
// (the per-stage double buffer it replaces left each stage's L2/HBM round trip exposed,
// ~1.5 us x 8 stages against ~0.4 us of MFMAs per stage).  Column-major operands (gen
// form), swizzled LDS stages, and per accumulator the MFMA order of gram_f64_kernel /
// gram_sia_kernel ((p, u) per stage, stages ascending): the tile is bitwise the same.
// the strip's output base: element (I0, J0) of the tile in the chosen placement
template <int QC>
__global__ __launch_bounds__(256) void gram_small_kernel(const double* __restrict__ A1, int64_t lda1,
                                                         const double* A2, int64_t lda2,
                                                         const double* __restrict__ w, int64_t k0, int64_t Nk,
                                                         const int2* __restrict__ tiles, double* G, int64_t ldg,
                                                         int flags) {
  constexpr int NQ = GT / QC;
  __shared__ __attribute__((aligned(16))) double lds[2 * (GT + QC) * GBK];
  if (flags & GRAM_PRIO) __builtin_amdgcn_s_setprio(3);
  const int2 tl = tiles[blockIdx.x / NQ];
  const int64_t I0 = (int64_t)tl.x * GT, J0 = (int64_t)tl.y * GT + (blockIdx.x % NQ) * QC;
  double* Gt = (flags & GRAM_UPPER) ? G + I0 * ldg + J0 : G + J0 * ldg + I0;
  gram_small_strip<QC>(A1 + I0 * lda1, lda1, A2 + J0 * lda2, lda2, w, k0, Nk, Gt, ldg, flags, lds);
}

hipError_t gram_launch_small(const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w,
                             int64_t k0, int64_t k1, const int2* tiles, int ntiles, double* G, int64_t ldg, int flags,
                             hipStream_t st) {
  if (ntiles <= 0) return hipSuccess;
  if ((k1 - k0) % (8 * GBK) != 0 || k1 <= k0) return hipErrorInvalidValue;   // whole 8-stage rings
  // 16-column strips (8 workgroups per tile) while the launch would leave most CUs idle
  if (ntiles <= 32)
    hipLaunchKernelGGL(gram_small_kernel<16>, dim3(8 * ntiles), dim3(256), 0, st, A1, lda1, A2, lda2, w, k0, k1, tiles,
                       G, ldg, flags);
  else
    hipLaunchKernelGGL(gram_small_kernel<32>, dim3(4 * ntiles), dim3(256), 0, st, A1, lda1, A2, lda2, w, k0, k1, tiles,
                       G, ldg, flags);
  return hipGetLastError();
}

// Two-operand column-major products (A1 != A2: the LU's TRSM and trailing updates, the QR's Vᵀ
// products, the Cholesky's strip solves) on the interleaved-schedule kernel with its second operand
// (r05; was the register-staged gram_f64_kernel: same MFMA order per tile, the same bits).
// From K = 256 on, and at K = 128 (the Cholesky's strip solves) only in factors with ld >= 32768:
// there the launches are large enough (m = 32768 factor 191.7-194.2 -> 187.7-190.8 ms, the m = 65536
// solve of the C5-shaped GGN step 1420-1426 -> 1414-1420 ms, profiles/r05/sia2k128/), while at
// m = 16384 the interleaved pipeline's prologue did not pay (factor 32.2-32.5 -> 32.6-33.0 ms).  The
// LU's K = 512 updates: n = 16384 212.0 -> 207.8 ms; the QR's Vᵀ products: n = 8192 95.9 -> 93.8 ms
// (profiles/r05/sia2/).  SCS_GRAM_SIA2=0 restores gram_f64_kernel everywhere, 1 takes the
// interleaved kernel for every two-operand launch (read per launch: A/B and the tests).
static bool gram_sia2(int64_t K, int64_t ld) {
  const char* e = getenv("SCS_GRAM_SIA2");
  if (gram_sia_mode() == 0 || (e && e[0] == '0')) return false;
  return K >= 256 || ld >= 32768 || (e && e[0] == '1');
}

// General form: operand panels from two matrices, K range [k0, k1), flags GRAM_*.
hipError_t gram_launch_gen(const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w,
                           int64_t k0, int64_t k1, const int2* tiles, int ntiles, double* G, int64_t ldg, int flags,
                           hipStream_t st) {
  if (ntiles <= 0) return hipSuccess;
  // short contractions with few tiles are latency-bound (one 128 x 128 x 128 tile on one CU is
  // 2048 MFMAs = 13.6 us): spread each tile over 4-8 CUs.  SCS_GRAM_SMALL=<max tiles>, 0 disables.
  // up to 64 tiles (256-512 latency workgroups); beyond, the throughput kernels fill the chip with
  // one 128 x 128 tile per workgroup at 2 per CU (m = 32768: the strip solves of the bulk stream
  // took 26 ms as 397 latency launches, ~8 ms of MFMA work)
  // default 128 since r03 (with the 4-block outer steps): m = 8192 factor 8.07 -> 7.8 ms, m = 16384
  // 34.3 -> 33.6 ms; the m = 32768 cached solve, the LU and the QR at n = 8192 unchanged
  // (profiles/r03/chol/gram_small/)
  const char* se = getenv("SCS_GRAM_SMALL");   // read per launch (tests toggle it in-process)
  const int small_max = se ? atoi(se) : 128;
  if (k1 - k0 <= 512 && (k1 - k0) % (8 * GBK) == 0 && k1 > k0 && ntiles <= small_max) return gram_launch_small(A1, lda1, A2, lda2, w, k0, k1, tiles, ntiles, G, ldg, flags, st);
  if (A1 == A2 && lda1 == lda2 && gram_sia_mode() != 0)   // the Cholesky's trailing updates
    hipLaunchKernelGGL((gram_sia_kernel<1, 2, true>), dim3(ntiles), dim3(256), 0, st, A1, lda1, w, k0, k1, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, nullptr, nullptr, (int64_t)0, nullptr, 0, nullptr, (int64_t)0);
  else if (gram_sia2(k1 - k0, lda2))   // two operands (LU TRSM / updates, strip solves): the interleaved kernel too
    hipLaunchKernelGGL((gram_sia_kernel<1, 2, true>), dim3(ntiles), dim3(256), 0, st, A1, lda1, w, k0, k1, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, nullptr, nullptr, (int64_t)0, nullptr, 0, A2, lda2);
  else
    hipLaunchKernelGGL((gram_f64_kernel<false, 2>), dim3(ntiles), dim3(256), 0, st, A1, lda1, A2, lda2, w, k0, k1,
                       tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  return hipGetLastError();
}

// A K-split work list (bi, bj, piece, partial slot) of two column-major operands over [0, K) (the
// QR's Vᵀ products, qr.hip): every item's partial tile to P, slot-major; the caller combines.
hipError_t gram_launch_work_cm(const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w,
                               int64_t K, const int4* work, int seglen, int nsplit, double* P, hipStream_t st) {
  if (gram_sia2(K, lda2)) {
    hipLaunchKernelGGL((gram_sia_kernel<1, 2, true>), dim3((unsigned)(8 * seglen)), dim3(256), 0, st, A1, lda1, w,
                       (int64_t)0, K, nullptr, 0, nullptr, (int64_t)0, 0, work, seglen, nsplit, P, nullptr, nullptr,
                       (int64_t)0, nullptr, 0, A2, lda2);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((gram_f64_kernel<false, 2>), dim3((unsigned)(8 * seglen)), dim3(256), 0, st, A1, lda1, A2, lda2, w,
                     (int64_t)0, K, nullptr, 0, nullptr, (int64_t)0, 0, work, seglen, nsplit, P);
  return hipGetLastError();
}

// gram_launch_gen's throughput launches as CU-bounded persistent launches (bnd_first): at most
// `slots` workgroups, the CUs of `skip` left free.  Latency-sized launches and skip == 0 take
// gram_launch_gen's path.  Per tile the same kernel body and MFMA order: bitwise the same G.
hipError_t gram_launch_bounded(const double* A1, int64_t lda1, const double* A2, int64_t lda2, const double* w,
                               int64_t k0, int64_t k1, const int2* tiles, int ntiles, double* G, int64_t ldg, int flags,
                               unsigned* ctr, unsigned skip, int slots, hipStream_t st, bool zeroed) {
  if (ntiles <= 0) return hipSuccess;
  const char* se = getenv("SCS_GRAM_SMALL");
  const int small_max = se ? atoi(se) : 128;
  const bool small = k1 - k0 <= 512 && (k1 - k0) % (8 * GBK) == 0 && k1 > k0 && ntiles <= small_max;
  if (!ctr || skip == 0 || slots <= 0 || small)
    return gram_launch_gen(A1, lda1, A2, lda2, w, k0, k1, tiles, ntiles, G, ldg, flags, st);
  if (!zeroed) {   // (the Cholesky's bulk stream hands over counter sets zeroed in advance)
    const hipError_t e = hipMemsetAsync(ctr, 0, 9 * sizeof(unsigned), st);
    if (e != hipSuccess) return e;
  }
  // enough workgroups that the ones left after the skipped CUs' leave take every tile in one round
  // (a launch smaller than the chip), else one per workgroup slot of the device
  const int want = ntiles + (ntiles + 6) / 7 + 8;
  const unsigned grid = (unsigned)(want < slots ? want : slots);
  if (A1 == A2 && lda1 == lda2 && gram_sia_mode() != 0)
    hipLaunchKernelGGL((gram_sia_kernel<1, 2, true, false, true>), dim3(grid), dim3(256), 0, st, A1, lda1, w, k0, k1,
                       tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, nullptr, nullptr, (int64_t)0, ctr,
                       (int)skip, nullptr, (int64_t)0);
  else if (gram_sia2(k1 - k0, lda2))
    hipLaunchKernelGGL((gram_sia_kernel<1, 2, true, false, true>), dim3(grid), dim3(256), 0, st, A1, lda1, w, k0, k1,
                       tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, nullptr, nullptr, (int64_t)0, ctr,
                       (int)skip, A2, lda2);
  else
    hipLaunchKernelGGL((gram_f64_kernel<false, 2, false, true>), dim3(grid), dim3(256), 0, st, A1, lda1, A2, lda2, w,
                       k0, k1, tiles, ntiles, G, ldg, flags, nullptr, (int)skip, 0, reinterpret_cast<double*>(ctr));
  return hipGetLastError();
}

// experiment hook (probe_gram): K range [k0, k1), accumulate into G, optional no-load timing build
hipError_t gram_launch_ex(const double* A, int64_t lda, const double* w, int64_t k0, int64_t k1, const int2* tiles,
                          int ntiles, double* G, int64_t ldg, int accumulate, int noload, hipStream_t st) {
  const int flags = GRAM_UPPER | (accumulate ? GRAM_ACCUMULATE : 0);
  if (noload == 16 || noload == 17)   // 256 x 128 interleaved kernel (tall tile list): loaded / no-load
    hipLaunchKernelGGL((noload == 16 ? gram_sia_kernel<1, 4> : gram_sia_kernel<3, 4>), dim3(ntiles), dim3(512), 0,
                       st, A, (k1 - k0) / GBK, w, k0, k1, tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, nullptr, nullptr, (int64_t)0, nullptr, 0, nullptr, (int64_t)0);
  else if (noload == 12)
    hipLaunchKernelGGL((gram_sia_kernel<3>), dim3(ntiles), dim3(256), 0, st, A, (k1 - k0) / GBK, w, k0, k1, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, nullptr, nullptr, (int64_t)0, nullptr, 0, nullptr, (int64_t)0);
  else if (noload == 9 || noload == 10)
    hipLaunchKernelGGL((noload == 9 ? gram_sia_kernel<1> : gram_sia_kernel<0>), dim3(ntiles), dim3(256), 0, st, A,
                       (k1 - k0) / GBK, w, k0, k1, tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr, nullptr, nullptr, (int64_t)0, nullptr, 0, nullptr, (int64_t)0);
  else if (noload == 11)
    hipLaunchKernelGGL((gram_f64_kernel<false, 2, true>), dim3(ntiles), dim3(256), 0, st, A, (k1 - k0) / GBK, A,
                       (k1 - k0) / GBK, w, k0, k1, tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  else if (noload == 7 || noload == 8)   // pipelined fragment reads (8: no-load ceiling), panel-blocked A
    hipLaunchKernelGGL((noload == 7 ? gram_glds_kernel<true, 1> : gram_glds_kernel<true, 2>), dim3(ntiles), dim3(512),
                       0, st, A, (k1 - k0) / GBK, A, (k1 - k0) / GBK, w, k0, k1, tiles, ntiles, G, ldg, flags, nullptr,
                       0, 0, nullptr);
  else if (noload == 5)   // timing experiment: the same kernel on a panel-blocked (tiled) A, lda = stages
    hipLaunchKernelGGL(gram_glds_kernel<true>, dim3(ntiles), dim3(512), 0, st, A, (k1 - k0) / GBK, A,
                       (k1 - k0) / GBK, w, k0, k1, tiles, ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  else if (noload == 6)
    hipLaunchKernelGGL(gram_glds_kernel<false>, dim3(ntiles), dim3(512), 0, st, A, lda, A, lda, w, k0, k1, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  else if (noload == 4)
    hipLaunchKernelGGL((gram_f64_kernel<true, 4>), dim3(ntiles), dim3(512), 0, st, A, lda, A, lda, w, k0, k1, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  else if (noload == 3)
    hipLaunchKernelGGL((gram_f64_kernel<false, 4>), dim3(ntiles), dim3(512), 0, st, A, lda, A, lda, w, k0, k1, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  else if (noload)
    hipLaunchKernelGGL((gram_f64_kernel<true, 2>), dim3(ntiles), dim3(256), 0, st, A, lda, A, lda, w, k0, k1, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  else
    hipLaunchKernelGGL((gram_f64_kernel<false, 2>), dim3(ntiles), dim3(256), 0, st, A, lda, A, lda, w, k0, k1, tiles,
                       ntiles, G, ldg, flags, nullptr, 0, 0, nullptr);
  return hipGetLastError();
}

// Combine K-split partials of the scheduled tail tiles in piece order and place
// them like the main epilogue (upper triangle, or the packed slot of the
// canonical tile index).  item = (bi, bj, canonical tix, first partial slot).
template <int TI>
__global__ void gram_combine_kernel(const double* __restrict__ P, const int4* __restrict__ items, int nsplit,
                                    double* __restrict__ G, int64_t ldg, int packed) {
  constexpr int GTI = 64 * TI;
  const int4 it = items[blockIdx.y];
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < GTI * GT; e += gridDim.x * blockDim.x) {
    const int jl = e / GTI, il = e % GTI;
    double sum = 0.0;
    for (int sp = 0; sp < nsplit; ++sp) sum += P[(int64_t)(it.w + sp) * GTI * GT + e];
    double* dst = (packed & 1) ? G + ((int64_t)it.z * (GTI / GT) + il / GT) * GT * GT + jl * GT + (il % GT)
                               : G + ((int64_t)it.x * GTI + il) * ldg + (int64_t)it.y * GT + jl;
    if (packed & 2) *dst += sum;
    else *dst = sum;
  }
}

// Scheduled main Gram (gram_schedule's work list + tail combine).
hipError_t gram_launch_sched(const double* A, int64_t lda, const double* w, int64_t Nk, const int4* work, int seglen,
                             int nsplit, const int4* comb, int ncomb, double* P, double* G, int64_t ldg, int packed,
                             int tall, hipStream_t st, const double* v, double* VP, int64_t vps, unsigned* scnt,
                             int sob) {
  if (scnt && !(gram_fuse_ok(tall) || (tall ? gram_tall_mode() == 3 : gram_sia_mode() == 1)))
    return hipErrorInvalidValue;   // strip counts come from the interleaved kernels only
  // packed: bit 0 = packed slots (else the upper triangle), bit 1 = accumulate into G
  const int flags = ((packed & 1) ? GRAM_PACKED : GRAM_UPPER) | ((packed & 2) ? GRAM_ACCUMULATE : 0);
  const int glds = gram_tall_mode();
  if (v && !gram_fuse_ok(tall)) return hipErrorInvalidValue;
  if (v && tall) {
    g_main_name = "gram_sia_kernel<1, 4, false, true, false>";
    hipLaunchKernelGGL((gram_sia_kernel<1, 4, false, true>), dim3(8 * seglen), dim3(512), 0, st, A, lda, w,
                       (int64_t)0, Nk, nullptr, 0, G, ldg, flags, work, seglen, nsplit, P, v, VP, vps, scnt, sob, nullptr, (int64_t)0);
  } else if (v) {
    g_main_name = "gram_sia_kernel<1, 2, false, true, false>";
    hipLaunchKernelGGL((gram_sia_kernel<1, 2, false, true>), dim3(8 * seglen), dim3(256), 0, st, A, lda, w,
                       (int64_t)0, Nk, nullptr, 0, G, ldg, flags, work, seglen, nsplit, P, v, VP, vps, scnt, sob, nullptr, (int64_t)0);
  } else if (tall && glds == 3) {
    g_main_name = "gram_sia_kernel<1, 4, false, false, false>";
    hipLaunchKernelGGL((gram_sia_kernel<1, 4>), dim3(8 * seglen), dim3(512), 0, st, A, lda, w, (int64_t)0, Nk,
                       nullptr, 0, G, ldg, flags, work, seglen, nsplit, P, nullptr, nullptr, (int64_t)0, scnt, sob, nullptr, (int64_t)0);
  } else if (tall && glds == 2) {
    g_main_name = "gram_glds_kernel<true, 1>";
    hipLaunchKernelGGL((gram_glds_kernel<true, 1>), dim3(8 * seglen), dim3(512), 0, st, A, lda, A, lda, w, (int64_t)0,
                       Nk, nullptr, 0, G, ldg, flags, work, seglen, nsplit, P);
  } else if (tall && glds == 1) {
    g_main_name = "gram_glds_kernel<true, 0>";
    hipLaunchKernelGGL(gram_glds_kernel<true>, dim3(8 * seglen), dim3(512), 0, st, A, lda, A, lda, w, (int64_t)0, Nk,
                       nullptr, 0, G, ldg, flags, work, seglen, nsplit, P);
  } else if (tall) {
    g_main_name = "gram_f64_kernel<false, 4, true, false>";
    hipLaunchKernelGGL((gram_f64_kernel<false, 4, true>), dim3(8 * seglen), dim3(512), 0, st, A, lda, A, lda, w,
                       (int64_t)0, Nk, nullptr, 0, G, ldg, flags, work, seglen, nsplit, P);
  } else if (gram_sia_mode() == 1) {
    g_main_name = "gram_sia_kernel<1, 2, false, false, false>";
    hipLaunchKernelGGL((gram_sia_kernel<1, 2>), dim3(8 * seglen), dim3(256), 0, st, A, lda, w, (int64_t)0, Nk, nullptr,
                       0, G, ldg, flags, work, seglen, nsplit, P, nullptr, nullptr, (int64_t)0, scnt, sob, nullptr, (int64_t)0);
  } else if (gram_sia_mode() == 2) {
    g_main_name = "gram_sia_kernel<0, 2, false, false, false>";
    hipLaunchKernelGGL((gram_sia_kernel<0>), dim3(8 * seglen), dim3(256), 0, st, A, lda, w, (int64_t)0, Nk, nullptr, 0,
                       G, ldg, flags, work, seglen, nsplit, P, nullptr, nullptr, (int64_t)0, scnt, sob, nullptr, (int64_t)0);
  } else {
    g_main_name = "gram_f64_kernel<false, 2, true, false>";
    hipLaunchKernelGGL((gram_f64_kernel<false, 2, true>), dim3(8 * seglen), dim3(256), 0, st, A, lda, A, lda, w,
                       (int64_t)0, Nk, nullptr, 0, G, ldg, flags, work, seglen, nsplit, P);
  }
  if (ncomb > 0) {
    if (tall)
      hipLaunchKernelGGL(gram_combine_kernel<4>, dim3(16, ncomb), dim3(256), 0, st, P, comb, nsplit, G, ldg, packed);
    else
      hipLaunchKernelGGL(gram_combine_kernel<2>, dim3(16, ncomb), dim3(256), 0, st, P, comb, nsplit, G, ldg, packed);
  }
  return hipGetLastError();
}

// The factor stream's wait for strip s of a one-launch Gram: one lane polls the strip's count
// (device-scope acquire) until it reaches `target`, sleeping between polls; a wait longer than
// ~30 s (100 MHz s_memrealtime) sets *flag and returns, so the grid always drains (the caller
// then fails the step instead of factoring an incomplete strip).
__global__ void strip_wait_kernel(const unsigned* __restrict__ cnt, unsigned target, int* __restrict__ flag) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(16);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull) {
      __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
}

hipError_t strip_wait_launch(const unsigned* cnt, unsigned target, int* flag, hipStream_t st) {
  hipLaunchKernelGGL(strip_wait_kernel, dim3(1), dim3(64), 0, st, cnt, target, flag);
  return hipGetLastError();
}

// Column-major scheduled form (the Cholesky's left-looking strip updates: long K, few tiles):
// gram_sia_kernel<CM> over the work list, K rows [k0, k1) of X, then the combine.  flags: GRAM_*
// with GRAM_UPPER placement (GRAM_ACCUMULATE adds into G).
hipError_t gram_launch_sched_cm(const double* X, int64_t ld, const double* w, int64_t k0, int64_t k1, const int4* work,
                                int seglen, int nsplit, const int4* comb, int ncomb, double* P, double* G, int64_t ldg,
                                int flags, hipStream_t st) {
  if (seglen <= 0 || k1 <= k0) return hipSuccess;
  hipLaunchKernelGGL((gram_sia_kernel<1, 2, true>), dim3(8 * seglen), dim3(256), 0, st, X, ld, w, k0, k1, nullptr, 0,
                     G, ldg, flags | GRAM_UPPER, work, seglen, nsplit, P, nullptr, nullptr, (int64_t)0, nullptr, 0, nullptr, (int64_t)0);
  if (ncomb > 0)
    hipLaunchKernelGGL(gram_combine_kernel<2>, dim3(16, ncomb), dim3(256), 0, st, P, comb, nsplit, G, ldg,
                       (flags & GRAM_ACCUMULATE) ? 2 : 0);
  return hipGetLastError();
}

// Host: build the scheduled work list from the canonical tile list.  The list is
// cut into 8 contiguous XCD segments (XCD x = blocks orig % 8 == x, run in
// orig order); in each segment the tiles that would form a partial last round
// (fewer than 3/4 of the XCD's `slots` concurrent workgroups) are split into
// nsplit K pieces, so the last round is full; segments are padded to equal
// length with no-op items.  Returns seglen; fills work (8*seglen), comb
// (combine items), *ncomb, *nsplit, *npart (partial slots).
int gram_schedule(const int2* tiles, int ntiles, int slots_per_xcd, std::vector<int4>& work, std::vector<int4>& comb,
                  int* nsplit, int* npart, int diag_first_gti) {
  const int q = ntiles / 8, r = ntiles % 8;
  // per-XCD tail and a common split factor
  int tail_max = 0;
  for (int x = 0; x < 8; ++x) {
    const int n = q + (x < r ? 1 : 0);
    const int t = n % slots_per_xcd;
    tail_max = std::max(tail_max, t);
  }
  int S = 1;
  if (tail_max > 0 && 4 * tail_max < 3 * slots_per_xcd)
    S = std::max(2, std::min(16, slots_per_xcd / tail_max));
  std::vector<std::vector<int4>> seg(8);
  comb.clear();
  int pslot = 0, t0 = 0;
  for (int x = 0; x < 8; ++x) {
    const int n = q + (x < r ? 1 : 0);
    const int tail = (S > 1) ? n % slots_per_xcd : 0;
    for (int i = 0; i < n - tail; ++i) {
      const int2 tl = tiles[t0 + i];
      seg[x].push_back(make_int4(tl.x, tl.y, -1, t0 + i));
    }
    // diag_first_gti (r05): the whole tiles whose row block holds their column panel -- the tiles an
    // AV launch gives the fused Aᵀv, the longer ones -- first in the XCD's order, so they run in its
    // first round instead of lengthening the last (order only: every tile's bits are the same)
    if (diag_first_gti > 0)
      std::stable_partition(seg[x].begin(), seg[x].end(), [&](const int4& it) {
        return it.x == (int)((int64_t)it.y * GT / diag_first_gti);
      });
    for (int i = n - tail; i < n; ++i) {
      const int2 tl = tiles[t0 + i];
      comb.push_back(make_int4(tl.x, tl.y, t0 + i, pslot));
      for (int sp = 0; sp < S; ++sp) seg[x].push_back(make_int4(tl.x, tl.y, sp, pslot + sp));
      pslot += S;
    }
    t0 += n;
  }
  size_t seglen = 0;
  for (auto& v : seg) seglen = std::max(seglen, v.size());
  work.assign(8 * seglen, make_int4(-1, -1, -1, -1));
  for (int x = 0; x < 8; ++x)
    for (size_t i = 0; i < seg[x].size(); ++i) work[x * seglen + i] = seg[x][i];
  *nsplit = S;
  *npart = pslot;
  return (int)seglen;
}

hipError_t gram_unpack_launch(const double* P, const int2* tiles, int ntiles, double* G, int64_t ldg,
                              hipStream_t st) {
  if (ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(gram_packx_kernel<true>, dim3(4, ntiles), dim3(256), 0, st, P, G, tiles, ldg);
  return hipGetLastError();
}

}  // namespace scs
