// Sparse A (BASELINE configs[4]: box-constrained least squares, ρ = 0.01,
// ProxLQNSCORE).  A is held twice: CSR (rows; z = A x) and CSC (columns;
// g = Aᵀ v), the "CSR + CSC copy" layout of SURVEY.md §8d C5.  Values are fp64
// or fp32 (the fp32-vs-fp64 study); accumulation is always fp64.
//
//   spmv_csr : one wave per row, lanes stride the row's nonzeros (coalesced
//              value/index loads, x gathered from L2), fixed-order wave sum.
//   spmv_csc : the same per column.
// Both run on an LDS-blocked copy (below): bytes per pass = nnz * (sizeof(val) + 2) + pointers + vectors.
//
// Synthetic pattern (scs_gen_sparse): k = round(ρ m) "layers"; layer s maps
// row i to column ((a_s i + b_s) mod N) mod m with a_s odd, a bijection of
// [0, N) when N is a power of two and m | N.  Every row then has exactly k
// nonzeros and every column exactly k N / m, so both the CSR and the CSC
// arrays are written in place from closed forms (no sort); the value of
// (i, s) is a counter-RNG normal, identical in both copies.
#include <algorithm>
#include <cstdlib>

#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "common.h"
#include "kernels.h"

namespace scs {

// ---- LDS-blocked layout ------------------------------------------------------
// Gathering x[idx] straight from L2 costs one L2 request per nonzero (the
// indices are scattered), which caps the pass far below HBM rate.  Instead each
// direction is stored "blocked": the index range is cut into blocks of
// BS = 2^shift (<= 16384, 128 KiB of fp64) and block b holds, for every row,
// that row's entries whose index falls in b (16-bit local indices).  A
// workgroup owns (a run of rows, one block): it stages the block's slice of the
// gathered vector in LDS once and streams the rows' (value, local index)
// pairs, so the gathers are LDS reads and HBM sees nnz * (sizeof(val) + 2) B.
// Output: one partial per block, out[b * ldo + r]; the callers sum the blocks
// in fixed order (epilogue z-splits / gemv_t_finalize), so results do not
// depend on scheduling.
constexpr int SPB_MAXSHIFT = 14;
constexpr int SPB_THREADS = 1024;
constexpr int SPB_ROWS = 1024;   // rows per workgroup

// Layout: segments are padded to whole slots -- 4 entries (fp64: one 8-B index load, two 16-B
// value loads per lane) or 8 (fp32: one 16-B index load, two 16-B value loads) -- with index
// SPB_PADIDX = 16384 (the zero slot past the staged x slice, so padding needs no compare) and
// value 0 (blk_pad / hipMemsetD16), and start slot-aligned.
constexpr int SPB_PADIDX = 1 << SPB_MAXSHIFT;

// 64-bit DPP move (two 32-bit halves); lanes the pattern does not reach read 0 (bound_ctrl)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, ROWMASK, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, ROWMASK, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Segmented inclusive prefix sum over lanes [max(rs, 0), lane] of a wave whose lanes' rows are
// nondecreasing (rs = first lane of my row, < 0 if the row began before lane 0): row_shr 1/2/4/8
// inside each 16-lane row, then row_bcast:15 and row_bcast:31 -- the wave prefix-scan pattern
// with each step's add kept only when its source lane lies in my row.  Fixed order.
__device__ __forceinline__ double seg_scan64(double p, int lane, int rs) {
  const int l16 = lane & 15;
  double u;
  u = dpp_f64<0x111, 0xF>(p);
  if (l16 >= 1 && lane - 1 >= rs) p += u;
  u = dpp_f64<0x112, 0xF>(p);
  if (l16 >= 2 && lane - 2 >= rs) p += u;
  u = dpp_f64<0x114, 0xF>(p);
  if (l16 >= 4 && lane - 4 >= rs) p += u;
  u = dpp_f64<0x118, 0xF>(p);
  if (l16 >= 8 && lane - 8 >= rs) p += u;
  u = dpp_f64<0x142, 0xA>(p);   // row_bcast:15 -> rows 1, 3
  if ((lane & 16) && (lane & ~15) - 1 >= rs) p += u;
  u = dpp_f64<0x143, 0xC>(p);   // row_bcast:31 -> rows 2, 3
  if ((lane & 32) && 31 >= rs) p += u;
  return p;
}

// fp64 product ("flat" form, r02).  Each wave owns 64 contiguous rows of block b, whose padded
// segments are one contiguous range of 4-entry slots; it streams that range in windows of 64
// slots -- every lane busy, one window's loads in flight ahead of the compute -- instead of
// per-row rounds (which left ~36 % of the lanes idle on C5's ~41-slot segments and re-read
// clamped slots).  Per window: lane partial over its slot (LDS gathers of the staged x slice),
// the lane's row from the wave's row starts (a wave-uniform walk over the few rows that begin in
// the window), the DPP segmented scan, and each row's register accumulator (lane k = row k)
// pulls its window sum from the row's last lane in the window.  Per row the order is fixed
// (slot partials left to right within a lane's 4 entries, the scan tree, windows in order).
// C5 probe, same box (tools/probes/probe_spmv_flat.hip): 1.318 -> 1.182 ms (A x), 1.326 ->
// 1.185 ms (Aᵀ v) against the per-row pipelined kernel; a plain read of the same bytes takes
// 1.13 ms; the C5 bench 369 -> 397 it/s.  fp32 values on the padded layout through the same
// kernel measured slower than the unpadded one-entry-per-lane kernel below (0.907 vs 0.824 ms).
template <int SLOT>
struct SpmvWin {
  uint64_t id[SLOT / 4];   // SLOT 16-bit local indices
  double v[SLOT];
};
typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int SLOT>
__device__ __forceinline__ void win_load_idx(SpmvWin<SLOT>& w, const uint16_t* __restrict__ lidx, int64_t slot) {
  if (SLOT == 4) {
    w.id[0] = *(const uint64_t*)(lidx + 4 * slot);
  } else {
#pragma unroll
    for (int k = 0; k < SLOT / 8; ++k) {
      const v2u64 t = *(const v2u64*)(lidx + SLOT * slot + 8 * k);
      w.id[2 * k] = t[0];
      w.id[2 * k + 1] = t[1];
    }
  }
}
template <int SLOT>
__device__ __forceinline__ void win_load(SpmvWin<SLOT>& w, const uint16_t* __restrict__ lidx,
                                         const double* __restrict__ val, int64_t slot) {
  win_load_idx(w, lidx, slot);
#pragma unroll
  for (int k = 0; k < SLOT / 2; ++k) {
    const v2d a = *(const v2d*)(val + SLOT * slot + 2 * k);
    w.v[2 * k] = a[0];
    w.v[2 * k + 1] = a[1];
  }
}
template <int SLOT>
__device__ __forceinline__ void win_load(SpmvWin<SLOT>& w, const uint16_t* __restrict__ lidx,
                                         const float* __restrict__ val, int64_t slot) {
  win_load_idx(w, lidx, slot);
#pragma unroll
  for (int k = 0; k < SLOT / 4; ++k) {
    const v4f a = *(const v4f*)(val + SLOT * slot + 4 * k);
#pragma unroll
    for (int q = 0; q < 4; ++q) w.v[4 * k + q] = (double)a[q];
  }
}

template <typename VT, int SLOT>
__global__ __launch_bounds__(SPB_THREADS) void spmv_blk_kernel(const int64_t* __restrict__ ptr,
                                                               const uint16_t* __restrict__ lidx,
                                                               const VT* __restrict__ val,
                                                               const double* __restrict__ x, int64_t nrows,
                                                               int64_t ncols, int shift, double* __restrict__ out,
                                                               int64_t ldo) {
  constexpr int SH = SLOT == 4 ? 2 : SLOT == 8 ? 3 : 4;
  static_assert((1 << SH) == SLOT, "slot width 4, 8 or 16");
  __shared__ double xs[SPB_PADIDX + 1];
  const int b = blockIdx.y;
  const int64_t c0 = (int64_t)b << shift;
  const int nb = (int)min((int64_t)1 << shift, ncols - c0);
  // stage the slice: all loads of a thread in flight before the LDS stores
  {
    constexpr int PER = (1 << SPB_MAXSHIFT) / SPB_THREADS;
    double t[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + k * SPB_THREADS;
      t[k] = (i < nb) ? x[c0 + i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) xs[threadIdx.x + k * SPB_THREADS] = t[k];
    if (threadIdx.x == 0) xs[SPB_PADIDX] = 0.0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t* pb = ptr + (int64_t)b * nrows;
  const int64_t rw0 = (int64_t)blockIdx.x * SPB_ROWS + (int64_t)wv * 64;
  const int nrw = (int)max((int64_t)0, min((int64_t)64, nrows - rw0));
  if (nrw == 0) return;
  const int64_t sb = pb[rw0] >> SH;                     // the wave's first slot
  const int total = (int)((pb[rw0 + nrw] >> SH) - sb);  // its slot count
  // st: slot start of row `lane` relative to sb (lanes past nrw: total); en: its end
  const int st = lane < nrw ? (int)((pb[rw0 + lane] >> SH) - sb) : total;
  const int stn = __shfl(st, min(lane + 1, 63), 64);   // every lane takes part in a shuffle
  const int en = lane + 1 < nrw ? stn : total;
  const int nwin = (total + 63) >> 6;
  SpmvWin<SLOT> nxt;
  win_load(nxt, lidx, val, sb + max(min(lane, total - 1), 0));
  double acc = 0.0;
  int cur = 0;   // row of the window's first slot (wave-uniform)
  for (int t = 0; t < nwin; ++t) {
    const SpmvWin<SLOT> w = nxt;
    if (t + 1 < nwin) win_load(nxt, lidx, val, sb + min(64 * (t + 1) + lane, total - 1));
    const int base = 64 * t, slot = base + lane;
    double p = 0.0;
#pragma unroll
    for (int e = 0; e < SLOT; ++e) p += w.v[e] * xs[(int)((w.id[e / 4] >> (16 * (e & 3))) & 0xFFFF)];
    if (slot >= total) p = 0.0;
    // my row = cur + #{k > cur : st_k <= slot}; the walk stops at the first row starting past
    // the window, and the last row starting at or before base + 64 is the next window's cur
    int r = cur, k = cur + 1;
    while (k < nrw) {
      const int sk = __builtin_amdgcn_readlane(st, k);
      if (sk > base + 64) break;
      r += (slot >= sk) ? 1 : 0;
      ++k;
    }
    cur = k - 1;
    const int rs = __shfl(st, r, 64) - base;
    p = seg_scan64(p, lane, rs);
    const double pt = __shfl(p, max(min(en - base - 1, 63), 0), 64);
    if (st < base + 64 && en > base && st < en) acc += pt;
  }
  if (lane < nrw) out[(int64_t)b * ldo + rw0 + lane] = acc;
}

// fp32-ARITHMETIC product (the compute arm of the C5 tolerance study, BASELINE configs[4];
// scs_set_compute_f32): fp32-stored values, the x slice staged in LDS as fp32, every product, lane
// partial, scan step and row accumulation in fp32 (v_fma_f32 / 32-bit DPP), the row sum widened to
// fp64 on the store.  The window / row bookkeeping is spmv_blk_kernel's, so only the arithmetic type
// differs.  Fixed order per row: bitwise run to run.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWMASK, 0xF, true));
}
__device__ __forceinline__ float seg_scan64_f32(float p, int lane, int rs) {
  const int l16 = lane & 15;
  float u;
  u = dpp_f32<0x111, 0xF>(p);
  if (l16 >= 1 && lane - 1 >= rs) p += u;
  u = dpp_f32<0x112, 0xF>(p);
  if (l16 >= 2 && lane - 2 >= rs) p += u;
  u = dpp_f32<0x114, 0xF>(p);
  if (l16 >= 4 && lane - 4 >= rs) p += u;
  u = dpp_f32<0x118, 0xF>(p);
  if (l16 >= 8 && lane - 8 >= rs) p += u;
  u = dpp_f32<0x142, 0xA>(p);   // row_bcast:15 -> rows 1, 3
  if ((lane & 16) && (lane & ~15) - 1 >= rs) p += u;
  u = dpp_f32<0x143, 0xC>(p);   // row_bcast:31 -> rows 2, 3
  if ((lane & 32) && 31 >= rs) p += u;
  return p;
}

struct SpmvWin32 {
  uint64_t id[2];   // 8 16-bit local indices
  float v[8];
};
__device__ __forceinline__ void win_load32(SpmvWin32& w, const uint16_t* __restrict__ lidx,
                                           const float* __restrict__ val, int64_t slot) {
  const v2u64 t = *(const v2u64*)(lidx + 8 * slot);
  w.id[0] = t[0];
  w.id[1] = t[1];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const v4f a = *(const v4f*)(val + 8 * slot + 4 * k);
#pragma unroll
    for (int q = 0; q < 4; ++q) w.v[4 * k + q] = a[q];
  }
}

__global__ __launch_bounds__(SPB_THREADS) void spmv_blk32_kernel(const int64_t* __restrict__ ptr,
                                                                 const uint16_t* __restrict__ lidx,
                                                                 const float* __restrict__ val,
                                                                 const double* __restrict__ x, int64_t nrows,
                                                                 int64_t ncols, int shift, double* __restrict__ out,
                                                                 int64_t ldo) {
  constexpr int SH = 3;   // 8-entry slots (the fp32 layout)
  __shared__ float xs[SPB_PADIDX + 1];
  const int b = blockIdx.y;
  const int64_t c0 = (int64_t)b << shift;
  const int nb = (int)min((int64_t)1 << shift, ncols - c0);
  {
    constexpr int PER = (1 << SPB_MAXSHIFT) / SPB_THREADS;
    float t[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + k * SPB_THREADS;
      t[k] = (i < nb) ? (float)x[c0 + i] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) xs[threadIdx.x + k * SPB_THREADS] = t[k];
    if (threadIdx.x == 0) xs[SPB_PADIDX] = 0.0f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t* pb = ptr + (int64_t)b * nrows;
  const int64_t rw0 = (int64_t)blockIdx.x * SPB_ROWS + (int64_t)wv * 64;
  const int nrw = (int)max((int64_t)0, min((int64_t)64, nrows - rw0));
  if (nrw == 0) return;
  const int64_t sb = pb[rw0] >> SH;
  const int total = (int)((pb[rw0 + nrw] >> SH) - sb);
  const int st = lane < nrw ? (int)((pb[rw0 + lane] >> SH) - sb) : total;
  const int stn = __shfl(st, min(lane + 1, 63), 64);
  const int en = lane + 1 < nrw ? stn : total;
  const int nwin = (total + 63) >> 6;
  SpmvWin32 nxt;
  win_load32(nxt, lidx, val, sb + max(min(lane, total - 1), 0));
  float acc = 0.0f;
  int cur = 0;
  for (int t = 0; t < nwin; ++t) {
    const SpmvWin32 w = nxt;
    if (t + 1 < nwin) win_load32(nxt, lidx, val, sb + min(64 * (t + 1) + lane, total - 1));
    const int base = 64 * t, slot = base + lane;
    float p = 0.0f;
#pragma unroll
    for (int e = 0; e < 8; ++e) p = fmaf(w.v[e], xs[(int)((w.id[e / 4] >> (16 * (e & 3))) & 0xFFFF)], p);
    if (slot >= total) p = 0.0f;
    int r = cur, k = cur + 1;
    while (k < nrw) {
      const int sk = __builtin_amdgcn_readlane(st, k);
      if (sk > base + 64) break;
      r += (slot >= sk) ? 1 : 0;
      ++k;
    }
    cur = k - 1;
    const int rs = __shfl(st, r, 64) - base;
    p = seg_scan64_f32(p, lane, rs);
    const float pt = __shfl(p, max(min(en - base - 1, 63), 0), 64);
    if (st < base + 64 && en > base && st < en) acc += pt;
  }
  if (lane < nrw) out[(int64_t)b * ldo + rw0 + lane] = (double)acc;
}

int spmv_pad_index() { return SPB_PADIDX; }

int spmv_blk_shift(int64_t ncols) {
  int s = 0;
  while (s < SPB_MAXSHIFT && ((int64_t)1 << s) < ncols) ++s;
  return s;
}

const char* spmv_kernel_name(int f32) {
  return f32 == 2 ? "spmv_blk32_kernel" : f32 ? "spmv_blk_kernel<float, 8>" : "spmv_blk_kernel<double, 4>";
}

hipError_t launch_spmv_blk(const int64_t* ptr, const uint16_t* lidx, const void* val, int f32, const double* x,
                           int64_t nrows, int64_t ncols, int shift, int64_t nnz, double* out, int64_t ldo,
                           hipStream_t st) {
  if (nrows <= 0) return hipSuccess;
  const int nblk = (int)ceil_div(ncols, (int64_t)1 << shift);
  // one 1024-row chunk per workgroup; fp64 in 4-entry slots, fp32 in 8-entry slots
  const dim3 grid((unsigned)ceil_div(nrows, SPB_ROWS), (unsigned)nblk);
  if (f32 == 2)   // fp32-stored values, fp32 arithmetic (the compute arm)
    hipLaunchKernelGGL(spmv_blk32_kernel, grid, dim3(SPB_THREADS), 0, st, ptr, lidx, (const float*)val, x, nrows,
                       ncols, shift, out, ldo);
  else if (f32)
    hipLaunchKernelGGL((spmv_blk_kernel<float, 8>), grid, dim3(SPB_THREADS), 0, st, ptr, lidx, (const float*)val, x,
                       nrows, ncols, shift, out, ldo);
  else
    hipLaunchKernelGGL((spmv_blk_kernel<double, 4>), grid, dim3(SPB_THREADS), 0, st, ptr, lidx, (const double*)val,
                       x, nrows, ncols, shift, out, ldo);
  return hipGetLastError();
}

// ---- building the blocked layout from a row-sorted CSR (indices ascending per row)
// cnt[b*nrows + r] = #entries of row r in block b; first[b*nrows + r] = position of the first one
__global__ void blk_count_kernel(const int64_t* __restrict__ ptr, const int* __restrict__ idx, int64_t nrows,
                                 int shift, int64_t* __restrict__ cnt, int64_t* __restrict__ first) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrows) return;
  const int64_t p0 = ptr[r], p1 = ptr[r + 1];
  for (int64_t p = p0 + lane; p < p1; p += 64) {
    const int b = idx[p] >> shift;
    if (p == p0 || (idx[p - 1] >> shift) != b) first[(int64_t)b * nrows + r] = p;
    if (p == p1 - 1 || (idx[p + 1] >> shift) != b) {
      // last of its block in this row: count = p - first + 1 (first is written by another lane
      // of this wave in the same pass only if p - first < 64; recompute it here instead)
      int64_t q = p;
      while (q > p0 && (idx[q - 1] >> shift) == b) --q;
      cnt[(int64_t)b * nrows + r] = p - q + 1;
    }
  }
}

template <typename VT>
__global__ void blk_scatter_kernel(const int64_t* __restrict__ ptr, const int* __restrict__ idx,
                                   const VT* __restrict__ val, int64_t nrows, int shift,
                                   const int64_t* __restrict__ bptr, const int64_t* __restrict__ first,
                                   uint16_t* __restrict__ lidx, VT* __restrict__ bval) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrows) return;
  const int64_t p0 = ptr[r], p1 = ptr[r + 1];
  const int mask = (1 << shift) - 1;
  for (int64_t p = p0 + lane; p < p1; p += 64) {
    const int c = idx[p];
    const int64_t k = (int64_t)(c >> shift) * nrows + r;
    const int64_t dst = bptr[k] + (p - first[k]);
    lidx[dst] = (uint16_t)(c & mask);
    bval[dst] = val[p];
  }
}

hipError_t blk_count(const int64_t* ptr, const int* idx, int64_t nrows, int shift, int64_t* cnt, int64_t* first,
                     hipStream_t st) {
  hipLaunchKernelGGL(blk_count_kernel, dim3((unsigned)ceil_div(nrows, 4)), dim3(256), 0, st, ptr, idx, nrows, shift,
                     cnt, first);
  return hipGetLastError();
}

// segment counts rounded up to whole slots (the SpMV's per-lane unit: 4 fp64 / 8 fp32 entries)
__global__ void blk_pad_kernel(int64_t* __restrict__ cnt, int64_t n, int64_t w) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) cnt[i] = (cnt[i] + w - 1) & ~(w - 1);
}

int spmv_slot_width(int f32) { return f32 ? 8 : 4; }

hipError_t blk_pad(int64_t* cnt, int64_t n, int f32, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(blk_pad_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, cnt, n,
                     (int64_t)spmv_slot_width(f32));
  return hipGetLastError();
}

hipError_t blk_scan(void* temp, size_t* temp_bytes, const int64_t* cnt, int64_t* bptr, int64_t n, hipStream_t st) {
  return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, cnt, bptr, n, st);
}

hipError_t blk_scatter(const int64_t* ptr, const int* idx, const void* val, int f32, int64_t nrows, int shift,
                       const int64_t* bptr, const int64_t* first, uint16_t* lidx, void* bval, hipStream_t st) {
  const dim3 grid((unsigned)ceil_div(nrows, 4));
  if (f32)
    hipLaunchKernelGGL(blk_scatter_kernel<float>, grid, dim3(256), 0, st, ptr, idx, (const float*)val, nrows, shift,
                       bptr, first, lidx, (float*)bval);
  else
    hipLaunchKernelGGL(blk_scatter_kernel<double>, grid, dim3(256), 0, st, ptr, idx, (const double*)val, nrows,
                       shift, bptr, first, lidx, (double*)bval);
  return hipGetLastError();
}

// ---- sparse Gram G = Aᵀ diag(w) A priced by nnz (Σ_r nnz_r² multiply-adds, not N·m²) ------------
// Jt*Q*Jt' of a SparseMatrixCSC (prox-GGN-SCORE.jl:114,129) and hess_fx = c·Aᵀ diag(h) A
// (prox-N-SCORE.jl:55) on a sparse A.  Gustavson by output column: G(i, j) = Σ_{r ∈ rows(j)}
// (w_r a_rj) a_ri.  A work item is (column j, row block b of G: rows [b·BS, b·BS + BS), BS =
// 2^shift <= 4096); one wave owns it, with the block's slice of column j as an fp64 accumulator in
// LDS (32 KiB).  The wave walks rows(j) (the CSC column, ascending rows) in batches of GB rows:
// lane t < GB loads row t's CSC entry, weight and the row's segment bounds in block b (the
// Gram-blocked CSR copy, unpadded, sorted by column), then every row's first 64 segment entries
// are loaded before any is accumulated (GB rows of memory latency in flight per wave), and the
// rows are accumulated in order -- one ds_add per entry, the entries of a row have distinct
// columns -- so each G(i, j) sums its terms in ascending row order: deterministic run to run.
// Only the upper part is formed (row blocks b with b·BS <= j), and column j is written up to the
// end of its 128-row diagonal tile (what chol_factor and the LU fallback's symmetrize read).
constexpr int SG_ROWS = 8;   // GB: rows per batch
__device__ __forceinline__ int64_t sg_bcast(int64_t v, int lane) {   // lane's value, wave-uniform (SGPRs)
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, lane);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double sg_bcast(double v, int lane) {
  return __builtin_bit_cast(double, sg_bcast(__builtin_bit_cast(int64_t, v), lane));
}
template <typename VT>
__global__ __launch_bounds__(64) void sparse_gram_kernel(const int64_t* __restrict__ colptr,
                                                         const int* __restrict__ rowidx, const VT* __restrict__ valT,
                                                         const int64_t* __restrict__ bptr,
                                                         const uint16_t* __restrict__ lidx,
                                                         const VT* __restrict__ bval, const double* __restrict__ w,
                                                         int64_t nrows, int64_t m, int shift, int64_t j0,
                                                         double* __restrict__ G, int64_t ldg) {
  __shared__ double acc[1 << 12];
  const int lane = threadIdx.x;
  const int BS = 1 << shift;
  // work item -> (column j, block b): column block J = j >> shift has J + 1 items per column, items of
  // column block J start at BS·J(J+1)/2 (relative to column j0, a multiple of BS)
  const int64_t t = (int64_t)blockIdx.x;
  const int64_t J0 = j0 >> shift;
  int64_t J = J0, base = 0;
  while (true) {
    const int64_t n = (int64_t)BS * (J + 1);
    if (t < base + n) break;
    base += n;
    ++J;
  }
  const int64_t loc = t - base;
  const int64_t j = J * BS + loc / (J + 1);
  const int b = (int)(loc % (J + 1));
  if (j >= m) return;
  for (int i = lane; i < BS; i += 64) acc[i] = 0.0;
  __syncthreads();
  const int64_t p0 = colptr[j], p1 = colptr[j + 1];
  for (int64_t p = p0; p < p1; p += SG_ROWS) {
    const int nb = (int)((p1 - p < SG_ROWS) ? (p1 - p) : SG_ROWS);
    double s = 0.0;
    int64_t st = 0, en = 0;
    if (lane < nb) {
      const int r = rowidx[p + lane];
      s = w[r] * (double)valT[p + lane];
      const int64_t k = (int64_t)b * nrows + r;
      st = bptr[k];
      en = bptr[k + 1];
    }
    double v[SG_ROWS];
    int ix[SG_ROWS];
#pragma unroll
    for (int u = 0; u < SG_ROWS; ++u) {
      const int64_t su = sg_bcast(st, u), eu = sg_bcast(en, u);
      const bool on = u < nb && su + lane < eu;
      v[u] = on ? (double)bval[su + lane] : 0.0;
      ix[u] = on ? (int)lidx[su + lane] : -1;
    }
#pragma unroll
    for (int u = 0; u < SG_ROWS; ++u) {
      if (u >= nb) break;
      const double su_s = sg_bcast(s, u);
      if (ix[u] >= 0) atomicAdd(&acc[ix[u]], su_s * v[u]);
      // a segment longer than one wave: the rest of this row before the next row (row order kept)
      const int64_t su = sg_bcast(st, u), eu = sg_bcast(en, u);
      for (int64_t q = su + 64 + lane; q - lane < eu; q += 64)
        if (q < eu) atomicAdd(&acc[lidx[q]], su_s * (double)bval[q]);
    }
  }
  __syncthreads();
  // column j, rows [b·BS, min(b·BS + BS, end of j's diagonal tile))
  const int64_t r0 = (int64_t)b * BS;
  const int64_t rend = ((j >> 7) + 1) << 7;
  const int64_t nr = (rend - r0 < BS) ? rend - r0 : BS;
  double* col = G + j * ldg + r0;
  for (int i = lane; i < nr; i += 64) col[i] = acc[i];
}

// The same walk with its memory latency overlapped (default; SCS_SPARSE_GRAM_KERNEL=1 the kernel
// above): per batch of SG_PR rows the row metadata is a stage ahead -- the row index and CSC value
// (stage 1) two batches ahead, the weight and segment bounds (stage 2) one batch ahead -- so a batch
// is ONE memory round trip (its rows' segment loads, all issued before any is used) instead of
// three per 8 rows.  The accumulation is the same products in the same row order: G is bitwise
// sparse_gram_kernel's.
template <typename VT, int SG_PR, bool BMAJ>   // SG_PR rows per batch; BMAJ: items of a column block b-major
__global__ __launch_bounds__(64) void sparse_gram_pipe_kernel(const int64_t* __restrict__ colptr,
                                                              const int* __restrict__ rowidx,
                                                              const VT* __restrict__ valT,
                                                              const int64_t* __restrict__ bptr,
                                                              const uint16_t* __restrict__ lidx,
                                                              const VT* __restrict__ bval,
                                                              const double* __restrict__ w, int64_t nrows,
                                                              int64_t m, int shift, int64_t j0,
                                                              double* __restrict__ G, int64_t ldg) {
  __shared__ double acc[1 << 12];
  const int lane = threadIdx.x;
  const int BS = 1 << shift;
  const int64_t t = (int64_t)blockIdx.x;
  const int64_t J0 = j0 >> shift;
  int64_t J = J0, base = 0;
  while (true) {
    const int64_t n = (int64_t)BS * (J + 1);
    if (t < base + n) break;
    base += n;
    ++J;
  }
  const int64_t loc = t - base;
  const int64_t j = BMAJ ? J * BS + loc % BS : J * BS + loc / (J + 1);
  const int b = BMAJ ? (int)(loc / BS) : (int)(loc % (J + 1));
  if (j >= m) return;
  for (int i = lane; i < BS; i += 64) acc[i] = 0.0;
  __syncthreads();
  const int64_t p0 = colptr[j], p1 = colptr[j + 1];
  const int64_t boff = (int64_t)b * nrows;
  auto stage1 = [&](int64_t p, int& r, double& a) {   // lane u < SG_PR: row p + u's index and value
    if (lane < SG_PR && p + lane < p1) {
      r = rowidx[p + lane];
      a = (double)valT[p + lane];
    } else {
      r = -1;
      a = 0.0;
    }
  };
  auto stage2 = [&](int r, double a, double& s, int64_t& st, int64_t& en) {
    if (r >= 0) {
      s = w[r] * a;
      st = bptr[boff + r];
      en = bptr[boff + r + 1];
    } else {
      s = 0.0;
      st = en = 0;
    }
  };
  int rc, rn;
  double ac, an;
  double s, sN;
  int64_t st, en, stN, enN;
  stage1(p0, rc, ac);
  stage2(rc, ac, s, st, en);
  stage1(p0 + SG_PR, rn, an);
  for (int64_t p = p0; p < p1; p += SG_PR) {
    // the next batch's stage 2 (its stage 1 landed during the previous batch) and the stage 1 of the
    // one after, issued before this batch's segment loads
    stage2(rn, an, sN, stN, enN);
    stage1(p + 2 * SG_PR, rn, an);
    double v[SG_PR];
    int ix[SG_PR];
#pragma unroll
    for (int u = 0; u < SG_PR; ++u) {
      const int64_t su = sg_bcast(st, u), eu = sg_bcast(en, u);
      const bool on = su + lane < eu;
      v[u] = on ? (double)bval[su + lane] : 0.0;
      ix[u] = on ? (int)lidx[su + lane] : -1;
    }
#pragma unroll
    for (int u = 0; u < SG_PR; ++u) {   // rows past the column's end: no segment (st = en = 0)
      const double su_s = sg_bcast(s, u);
      if (ix[u] >= 0) atomicAdd(&acc[ix[u]], su_s * v[u]);
      // a segment longer than one wave: the rest of this row before the next row (row order kept)
      const int64_t su = sg_bcast(st, u), eu = sg_bcast(en, u);
      for (int64_t q = su + 64 + lane; q - lane < eu; q += 64)
        if (q < eu) atomicAdd(&acc[lidx[q]], su_s * (double)bval[q]);
    }
    s = sN;
    st = stN;
    en = enN;
  }
  __syncthreads();
  const int64_t r0 = (int64_t)b * BS;
  const int64_t rend = ((j >> 7) + 1) << 7;
  const int64_t nr = (rend - r0 < BS) ? rend - r0 : BS;
  double* col = G + j * ldg + r0;
  for (int i = lane; i < nr; i += 64) col[i] = acc[i];
}

// r04 (variant 6, default when the Gram-blocked copy has < 2^31 entries): the pipelined walk with
// the per-row instruction count cut.  The r03 kernel was issue-bound, not byte-bound: ~30
// instructions per (column, row, block) triple -- 64-bit segment bounds broadcast by four
// v_readlane, an exec-masked load branch per row, and the long-segment check (four more readlanes)
// per row -- at ~0.13 ns per triple chip-wide whatever the block width (shift 12: 5.8e9 triples in
// 773 ms; shift 11: twice the triples, 1463 ms).  Here the bounds are 32-bit (start, length) pairs
// (one readlane each), every lane loads unconditionally (lanes past the segment read entry 0 and add
// -0.0: no exec branches), and the long-segment pass runs only in batches
// that hold a segment longer than one wave (a ballot per batch).  The same products accumulate in
// the same row order into every G entry: bitwise variant 5's G.
template <typename VT>
__global__ __launch_bounds__(64) void sparse_gram_flat_kernel(const int64_t* __restrict__ colptr,
                                                              const int* __restrict__ rowidx,
                                                              const VT* __restrict__ valT,
                                                              const int64_t* __restrict__ bptr,
                                                              const uint16_t* __restrict__ lidx,
                                                              const VT* __restrict__ bval,
                                                              const double* __restrict__ w, int64_t nrows,
                                                              int64_t m, int shift, int64_t j0,
                                                              double* __restrict__ G, int64_t ldg) {
  constexpr int PR = 64;                  // rows per batch
  __shared__ double acc[1 << 12];   // 32 KiB: five waves per CU, as variant 5
  const int lane = threadIdx.x;
  const int BS = 1 << shift;
  const int64_t t = (int64_t)blockIdx.x;
  const int64_t J0 = j0 >> shift;
  int64_t J = J0, base = 0;
  while (true) {
    const int64_t n = (int64_t)BS * (J + 1);
    if (t < base + n) break;
    base += n;
    ++J;
  }
  const int64_t loc = t - base;
  const int64_t j = J * BS + loc % BS;   // items b-major within a column block
  const int b = (int)(loc / BS);
  if (j >= m) return;
  for (int i = lane; i < BS; i += 64) acc[i] = 0.0;
  __syncthreads();
  const int64_t p0 = colptr[j], p1 = colptr[j + 1];
  const int64_t boff = (int64_t)b * nrows;
  auto stage1 = [&](int64_t p, int& r, double& a) {   // lane u: row p + u's index and CSC value
    if (p + lane < p1) {
      r = rowidx[p + lane];
      a = (double)valT[p + lane];
    } else {
      r = -1;
      a = 0.0;
    }
  };
  auto stage2 = [&](int r, double a, double& s, int& st, int& ln) {   // its weight x value, segment
    if (r >= 0) {
      s = w[r] * a;
      const int64_t s0 = bptr[boff + r], s1 = bptr[boff + r + 1];
      st = (int)s0;
      ln = (int)(s1 - s0);
    } else {
      s = 0.0;
      st = ln = 0;
    }
  };
  int rc, rn;
  double ac, an, s, sN;
  int st, ln, stN, lnN;
  stage1(p0, rc, ac);
  stage2(rc, ac, s, st, ln);
  stage1(p0 + PR, rn, an);
  for (int64_t p = p0; p < p1; p += PR) {
    stage2(rn, an, sN, stN, lnN);
    stage1(p + 2 * PR, rn, an);
    const bool longseg = __builtin_amdgcn_ballot_w64(ln > 64) != 0;   // wave-uniform
    double v[PR];
    int ix[PR];
#pragma unroll
    for (int u = 0; u < PR; ++u) {   // every row's first 64 entries in flight before any is used
      const int su = __builtin_amdgcn_readlane(st, u), lu = __builtin_amdgcn_readlane(ln, u);
      const int q = lane < lu ? su + lane : 0;
      v[u] = (double)bval[q];
      ix[u] = lidx[q];
    }
    // rows in order (rows past the column's end: length 0).  A lane past the segment adds -0.0 into
    // slot `lane`: x + (-0.0) == x for every x (signed zeros included), so no exec branch and no
    // extra LDS (a dummy slot would cost the fifth wave per CU)
    auto row = [&](int u) {
      const double su_s = sg_bcast(s, u);
      const int lu = __builtin_amdgcn_readlane(ln, u);
      const bool on = lane < lu;
      atomicAdd(&acc[on ? ix[u] : lane], on ? su_s * v[u] : -0.0);
    };
    if (!longseg) {
#pragma unroll
      for (int u = 0; u < PR; ++u) row(u);
    } else {
#pragma unroll
      for (int u = 0; u < PR; ++u) {
        row(u);
        const int lu = __builtin_amdgcn_readlane(ln, u);
        if (lu > 64) {   // the rest of this row before the next row (row order kept)
          const double su_s = sg_bcast(s, u);
          const int su = __builtin_amdgcn_readlane(st, u);
          for (int q = 64 + lane; q - lane < lu; q += 64)
            if (q < lu) atomicAdd(&acc[lidx[su + q]], su_s * (double)bval[su + q]);
        }
      }
    }
    s = sN;
    st = stN;
    ln = lnN;
  }
  __syncthreads();
  const int64_t r0 = (int64_t)b * BS;
  const int64_t rend = ((j >> 7) + 1) << 7;
  const int64_t nr = (rend - r0 < BS) ? rend - r0 : BS;
  double* col = G + j * ldg + r0;
  for (int i = lane; i < nr; i += 64) col[i] = acc[i];
}

// ---- variant 8 (r04): the walk on a per-triple table and interleaved segments ----------------------
// The PMC passes of variant 6 (profiles/r04/pmc_sgram/) put its fabric reads at 5.1e12 B per Gram
// (2 x FETCH_SIZE, the gfx950 rule) in 695 ms -- ~7.4 TB/s, i.e. the walk is bandwidth-bound -- about
// 930 B per (column, row, block) triple against ~410 B of segment payload: a 128-B line for the
// weight w[r], one for the segment bounds bptr[b][r], and partial lines at both ends of the two
// separate value / index ranges.  Here
//   * the segment of (block b, row r) is ONE record: its n values, then its n 16-bit local indices,
//     each part rounded up to 8 B, at 8-B unit uptr[b][r] of `seg` (seg_units: vunits(n) + ceil(n/4));
//   * a table T lists, per column j, per upper block b <= j >> shift and per row k of column j (CSC
//     order), the packed (n << 40 | unit) of that row's segment in b, so an item reads its rows'
//     segment positions as one coalesced 8-B stream instead of gathering bptr;
//   * sw[p] = w[rowidx[p]] * valT[p] is formed per Gram as one streaming pass over the CSC, so the
//     walk reads the scaled column entry instead of gathering w.
// The structure (seg, T) is built once per sparsity pattern.  Same products (w[r]·a_rj computed the
// same way) added in the same row order: G bitwise variant 5's.
__host__ __device__ inline int64_t seg_vunits(int64_t n, int vb) { return (n * vb + 7) >> 3; }
__host__ __device__ inline int64_t seg_units(int64_t n, int vb) { return seg_vunits(n, vb) + ((n + 3) >> 2); }
int64_t seg_units_host(int64_t n, int f32) { return seg_units(n, f32 ? 4 : 8); }

__global__ void seg_units_kernel(const int64_t* __restrict__ cnt, int64_t n, int vb, int64_t* __restrict__ ucnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ucnt[i] = seg_units(cnt[i], vb);
}

template <typename VT>
__global__ void seg_scatter_kernel(const int64_t* __restrict__ ptr, const int* __restrict__ idx,
                                   const VT* __restrict__ val, int64_t nrows, int shift,
                                   const int64_t* __restrict__ cnt, const int64_t* __restrict__ first,
                                   const int64_t* __restrict__ uptr, uint64_t* __restrict__ seg) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrows) return;
  const int64_t p0 = ptr[r], p1 = ptr[r + 1];
  const int mask = (1 << shift) - 1;
  for (int64_t p = p0 + lane; p < p1; p += 64) {
    const int c = idx[p];
    const int64_t k = (int64_t)(c >> shift) * nrows + r;
    const int64_t n = cnt[k], off = p - first[k];
    char* base = reinterpret_cast<char*>(seg + uptr[k]);
    reinterpret_cast<VT*>(base)[off] = val[p];
    reinterpret_cast<uint16_t*>(base + 8 * seg_vunits(n, (int)sizeof(VT)))[off] = (uint16_t)(c & mask);
  }
}

// T[tptr[j] + b·n_j + k] = cnt[b][r] << 40 | uptr[b][r] for r = rowidx[colptr[j] + k], b <= j >> shift
__global__ void seg_table_kernel(const int64_t* __restrict__ colptr, const int* __restrict__ rowidx,
                                 const int64_t* __restrict__ cnt, const int64_t* __restrict__ uptr, int64_t nrows,
                                 int shift, int64_t j0, const int64_t* __restrict__ tptr, uint64_t* __restrict__ T) {
  const int64_t j = j0 + blockIdx.x;
  const int64_t p0 = colptr[j], n = colptr[j + 1] - p0;
  uint64_t* Tj = T + tptr[j];
  const int J = (int)(j >> shift);
  for (int b = 0; b <= J; ++b)
    for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
      const int64_t q = (int64_t)b * nrows + rowidx[p0 + k];
      Tj[(int64_t)b * n + k] = ((uint64_t)cnt[q] << 40) | (uint64_t)uptr[q];
    }
}

template <typename VT>
__global__ void csc_weight_kernel(const int* __restrict__ rowidx, const VT* __restrict__ valT,
                                  const double* __restrict__ w, int64_t nnz, double* __restrict__ sw) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x)
    sw[p] = w[rowidx[p]] * (double)valT[p];
}

// DIAG (timing builds, SCS_SPARSE_GRAM_DIAG; G is WRONG): 1 = every atomic to slot `lane` (the same
// ds_add_f64 count, no bank conflicts), 2 = no LDS accumulation (a register sum per lane) -- to split
// the walk's time between its loads and its LDS atomics (tools/sgram_diag.py: C5 shape 533 / 538 /
// 502 ms, profiles/r04/sgdiag/: the loads bound it, not the atomics); 3 = as 2 with two rows per load
// instruction (lanes 0-31 row u, 32-63 row u+1, one 16-B value and one 4-B index load per lane): 425-433
// ms.  Real walks on that load structure, kept in row order (three LDS atomic instructions per row
// pair; or the rows put back on whole waves by v_permlane32_swap, one atomic per row), measured 646 and
// 570 ms (profiles/r04/v9/, v9b/): the load-only gain does not survive the accumulation
template <typename VT, int DIAG = 0>
__global__ __launch_bounds__(64) void sparse_gram_seg_kernel(const int64_t* __restrict__ colptr,
                                                             const double* __restrict__ sw,
                                                             const int64_t* __restrict__ tptr,
                                                             const uint64_t* __restrict__ T,
                                                             const uint64_t* __restrict__ seg, int64_t m,
                                                             int shift, int64_t j0, double* __restrict__ G,
                                                             int64_t ldg) {
  constexpr int PR = 64;
  constexpr int VB = (int)sizeof(VT);
  __shared__ double acc[1 << 12];
  const int lane = threadIdx.x;
  const int BS = 1 << shift;
  const int64_t t = (int64_t)blockIdx.x;
  const int64_t J0 = j0 >> shift;
  int64_t J = J0, base = 0;
  while (true) {
    const int64_t n = (int64_t)BS * (J + 1);
    if (t < base + n) break;
    base += n;
    ++J;
  }
  const int64_t loc = t - base;
  const int64_t j = J * BS + loc % BS;   // items b-major within a column block
  const int b = (int)(loc / BS);
  if (j >= m) return;
  for (int i = lane; i < BS; i += 64) acc[i] = 0.0;
  __syncthreads();
  const int64_t p0 = colptr[j], nj = colptr[j + 1] - p0;
  const uint64_t* Tb = T + tptr[j] + (int64_t)b * nj;
  const double* swj = sw + p0;
  auto stage = [&](int64_t k, double& sv, int& st, int& ln) {   // lane u: row k + u of the column
    if (k + lane < nj) {
      sv = swj[k + lane];
      const uint64_t tv = Tb[k + lane];
      st = (int)(uint32_t)tv;
      ln = (int)(tv >> 40);
    } else {
      sv = 0.0;
      st = ln = 0;
    }
  };
  double s, sN;
  int st, ln, stN, lnN;
  double rsum = 0.0;   // DIAG 2
  stage(0, s, st, ln);
  for (int64_t k = 0; k < nj; k += PR) {
    stage(k + PR, sN, stN, lnN);   // the next batch's scaled entries and segment positions
    const bool longseg = __builtin_amdgcn_ballot_w64(ln > 64) != 0;
    if constexpr (DIAG == 3) {   // two rows per load instruction, two entries per lane (no LDS)
      const int h = lane >> 5, q2 = 2 * (lane & 31);
#pragma unroll
      for (int u = 0; u < PR; u += 2) {
        const int su0 = __builtin_amdgcn_readlane(st, u), su1 = __builtin_amdgcn_readlane(st, u + 1);
        const int lu0 = __builtin_amdgcn_readlane(ln, u), lu1 = __builtin_amdgcn_readlane(ln, u + 1);
        const int su = h ? su1 : su0, lu = h ? lu1 : lu0;
        const char* rec = reinterpret_cast<const char*>(seg + su);
        const int q = q2 < lu ? q2 : 0;
        const v2d a = *reinterpret_cast<const v2d*>(reinterpret_cast<const double*>(rec) + q);
        const uint32_t i2 = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint16_t*>(rec + 8 * seg_vunits(lu, 8)) + q);
        rsum += a[0] + a[1] + (double)i2;
      }
      s = sN;
      st = stN;
      ln = lnN;
      continue;
    }
    double v[PR];
    int ix[PR];
#pragma unroll
    for (int u = 0; u < PR; ++u) {   // every row's first 64 entries in flight before any is used
      const int su = __builtin_amdgcn_readlane(st, u), lu = __builtin_amdgcn_readlane(ln, u);
      const char* rec = reinterpret_cast<const char*>(seg + su);   // wave-uniform record address
      const int q = lane < lu ? lane : 0;
      v[u] = (double)reinterpret_cast<const VT*>(rec)[q];
      ix[u] = reinterpret_cast<const uint16_t*>(rec + 8 * seg_vunits(lu, VB))[q];
    }
    auto row = [&](int u) {   // a lane past its segment adds -0.0 into slot `lane` (x + (-0.0) == x)
      const double su_s = sg_bcast(s, u);
      const int lu = __builtin_amdgcn_readlane(ln, u);
      const bool on = lane < lu;
      if constexpr (DIAG == 2) rsum += on ? su_s * v[u] + (double)ix[u] : 0.0;
      else if constexpr (DIAG == 1) atomicAdd(&acc[lane], on ? su_s * v[u] + (double)ix[u] : -0.0);
      else atomicAdd(&acc[on ? ix[u] : lane], on ? su_s * v[u] : -0.0);
    };
    if (!longseg) {
#pragma unroll
      for (int u = 0; u < PR; ++u) row(u);
    } else {
#pragma unroll
      for (int u = 0; u < PR; ++u) {
        row(u);
        const int lu = __builtin_amdgcn_readlane(ln, u);
        if (lu > 64) {   // the rest of this row before the next row (row order kept)
          const double su_s = sg_bcast(s, u);
          const char* rec = reinterpret_cast<const char*>(seg + __builtin_amdgcn_readlane(st, u));
          const VT* rv = reinterpret_cast<const VT*>(rec);
          const uint16_t* ri = reinterpret_cast<const uint16_t*>(rec + 8 * seg_vunits(lu, VB));
          for (int q = 64 + lane; q - lane < lu; q += 64)
            if (q < lu) atomicAdd(&acc[ri[q]], su_s * (double)rv[q]);
        }
      }
    }
    s = sN;
    st = stN;
    ln = lnN;
  }
  if constexpr (DIAG >= 2) acc[lane] = rsum;
  __syncthreads();
  const int64_t r0 = (int64_t)b * BS;
  const int64_t rend = ((j >> 7) + 1) << 7;
  const int64_t nr = (rend - r0 < BS) ? rend - r0 : BS;
  double* col = G + j * ldg + r0;
  for (int i = lane; i < nr; i += 64) col[i] = acc[i];
}

hipError_t seg_units(const int64_t* cnt, int64_t n, int f32, int64_t* ucnt, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(seg_units_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, cnt, n, f32 ? 4 : 8, ucnt);
  return hipGetLastError();
}

hipError_t seg_scatter(const int64_t* ptr, const int* idx, const void* val, int f32, int64_t nrows, int shift,
                       const int64_t* cnt, const int64_t* first, const int64_t* uptr, uint64_t* seg, hipStream_t st) {
  if (nrows <= 0) return hipSuccess;
  const dim3 grid((unsigned)ceil_div(nrows, 4));
  if (f32)
    hipLaunchKernelGGL(seg_scatter_kernel<float>, grid, dim3(256), 0, st, ptr, idx, (const float*)val, nrows, shift,
                       cnt, first, uptr, seg);
  else
    hipLaunchKernelGGL(seg_scatter_kernel<double>, grid, dim3(256), 0, st, ptr, idx, (const double*)val, nrows,
                       shift, cnt, first, uptr, seg);
  return hipGetLastError();
}

hipError_t seg_table(const int64_t* colptr, const int* rowidx, const int64_t* cnt, const int64_t* uptr, int64_t nrows,
                     int64_t m, int shift, const int64_t* tptr, uint64_t* T, hipStream_t st) {
  for (int64_t j0 = 0; j0 < m; j0 += 1 << 20) {   // launches of at most 2^20 columns
    const int64_t nj = std::min<int64_t>(m - j0, 1 << 20);
    hipLaunchKernelGGL(seg_table_kernel, dim3((unsigned)nj), dim3(256), 0, st, colptr, rowidx, cnt, uptr, nrows, shift,
                       j0, tptr, T);
  }
  return hipGetLastError();
}

hipError_t csc_weight(const int* rowidx, const void* valT, int f32, const double* w, int64_t nnz, double* sw,
                      hipStream_t st) {
  if (nnz <= 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(nnz, 256), 65536);
  if (f32)
    hipLaunchKernelGGL(csc_weight_kernel<float>, dim3(grid), dim3(256), 0, st, rowidx, (const float*)valT, w, nnz, sw);
  else
    hipLaunchKernelGGL(csc_weight_kernel<double>, dim3(grid), dim3(256), 0, st, rowidx, (const double*)valT, w, nnz,
                       sw);
  return hipGetLastError();
}

hipError_t launch_sparse_gram_seg(const int64_t* colptr, const double* sw, const int64_t* tptr, const uint64_t* T,
                                  const uint64_t* seg, int f32, int64_t m, int shift, double* G, int64_t ldg,
                                  hipStream_t st) {
  if (m <= 0) return hipSuccess;
  if (shift > 12 || shift < 7) return hipErrorInvalidValue;
  const int64_t BS = (int64_t)1 << shift;
  int64_t j0 = 0;
  while (j0 < m) {
    int64_t j1 = j0;
    while (j1 < m && sparse_gram_items(j0, j1 + BS, shift) < ((int64_t)1 << 30)) j1 += BS;
    if (j1 == j0) j1 = j0 + BS;
    const int64_t items = sparse_gram_items(j0, j1, shift);
    const char* dg = getenv("SCS_SPARSE_GRAM_DIAG");   // timing builds only (wrong G)
    const int diag = dg ? atoi(dg) : 0;
    if (f32)
      hipLaunchKernelGGL(sparse_gram_seg_kernel<float>, dim3((unsigned)items), dim3(64), 0, st, colptr, sw, tptr, T,
                         seg, m, shift, j0, G, ldg);
    else if (diag == 1)
      hipLaunchKernelGGL((sparse_gram_seg_kernel<double, 1>), dim3((unsigned)items), dim3(64), 0, st, colptr, sw, tptr,
                         T, seg, m, shift, j0, G, ldg);
    else if (diag == 2)
      hipLaunchKernelGGL((sparse_gram_seg_kernel<double, 2>), dim3((unsigned)items), dim3(64), 0, st, colptr, sw, tptr,
                         T, seg, m, shift, j0, G, ldg);
    else if (diag == 3)
      hipLaunchKernelGGL((sparse_gram_seg_kernel<double, 3>), dim3((unsigned)items), dim3(64), 0, st, colptr, sw, tptr,
                         T, seg, m, shift, j0, G, ldg);
    else
      hipLaunchKernelGGL(sparse_gram_seg_kernel<double>, dim3((unsigned)items), dim3(64), 0, st, colptr, sw, tptr, T,
                         seg, m, shift, j0, G, ldg);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    j0 = j1;
  }
  return hipSuccess;
}

// SCS_SPARSE_GRAM_KERNEL (read per call: A/B and the bit-identity test): 1 the one-round-trip-per-8-
// rows kernel; 2 / 3: the pipelined kernel, 32 / 64 rows per batch, items j-major; 4 / 5: the same,
// items b-major (concurrent waves share a 4096-row block of the Gram-blocked CSR copy); 6: the
// flat-issue walk above (r04 default; 5 where the copy has 2^31 entries or more).  C5-shaped Gram
// 1733 (1) -> 934 (2) / 794 (3) / 901 (4) / 766 ms (5), profiles/r03/sparse_gram/.
int sparse_gram_requested() {   // SCS_SPARSE_GRAM_KERNEL, default 8 (the host builds its structure)
  const char* e = getenv("SCS_SPARSE_GRAM_KERNEL");
  return e ? atoi(e) : 8;
}
// the variant launch_sparse_gram (the Gram-blocked copy's walks) runs: 8 falls back to 6 there
static int sparse_gram_variant(int64_t entries) {
  int v = sparse_gram_requested();
  if (v >= 6) v = 6;   // 8 (and the dropped 7) fall back to 6 on the Gram-blocked copy
  return (v == 6 && entries >= ((int64_t)1 << 31)) ? 5 : v;   // variant 6: 32-bit segment positions
}

const char* sparse_gram_kernel_name(int f32, int64_t entries) {
  const int var = sparse_gram_variant(entries);
  if (var == 1) return f32 ? "sparse_gram_kernel<float>" : "sparse_gram_kernel<double>";
  if (var == 6) return f32 ? "sparse_gram_flat_kernel<float>" : "sparse_gram_flat_kernel<double>";
  static const char* names[2][4] = {
      {"sparse_gram_pipe_kernel<double, 32, false>", "sparse_gram_pipe_kernel<double, 64, false>",
       "sparse_gram_pipe_kernel<double, 32, true>", "sparse_gram_pipe_kernel<double, 64, true>"},
      {"sparse_gram_pipe_kernel<float, 32, false>", "sparse_gram_pipe_kernel<float, 64, false>",
       "sparse_gram_pipe_kernel<float, 32, true>", "sparse_gram_pipe_kernel<float, 64, true>"}};
  return names[f32 ? 1 : 0][(var >= 3 && var <= 5) ? var - 2 : 0];
}

// the row-block width of G items / of the Gram-blocked CSR copy: 2^12 (default); SCS_SPARSE_GRAM_SHIFT
// (7..12) for A/B -- a narrower block makes each block's slice of the copy smaller (C5: 430 MB at 12,
// 215 MB at 11, i.e. within the 256 MB MALL) at twice the items and half the segment per row
int sparse_gram_shift() {
  const char* e = getenv("SCS_SPARSE_GRAM_SHIFT");
  const int v = e ? atoi(e) : 12;
  return v < 7 ? 7 : (v > 12 ? 12 : v);
}

int64_t sparse_gram_items(int64_t j0, int64_t j1, int shift) {
  // items of columns [j0, j1) (j0, j1 multiples of 2^shift, j1 may be the padded end)
  const int64_t BS = (int64_t)1 << shift;
  int64_t n = 0;
  for (int64_t J = j0 >> shift; J < (j1 + BS - 1) >> shift; ++J) n += BS * (J + 1);
  return n;
}

hipError_t launch_sparse_gram(const int64_t* colptr, const int* rowidx, const void* valT, const int64_t* bptr,
                              const uint16_t* lidx, const void* bval, int64_t entries, int f32, const double* w,
                              int64_t nrows, int64_t m, int shift, double* G, int64_t ldg, hipStream_t st) {
  if (m <= 0) return hipSuccess;
  if (shift > 12 || shift < 7) return hipErrorInvalidValue;
  const int64_t BS = (int64_t)1 << shift;
  // launches of at most 2^30 items: one per run of column blocks
  int64_t j0 = 0;
  while (j0 < m) {
    int64_t j1 = j0;
    while (j1 < m && sparse_gram_items(j0, j1 + BS, shift) < ((int64_t)1 << 30)) j1 += BS;
    if (j1 == j0) j1 = j0 + BS;
    const int64_t items = sparse_gram_items(j0, j1, shift);
    const int var = sparse_gram_variant(entries);
    if (var == 6) {
      if (f32)
        hipLaunchKernelGGL(sparse_gram_flat_kernel<float>, dim3((unsigned)items), dim3(64), 0, st, colptr, rowidx,
                           (const float*)valT, bptr, lidx, (const float*)bval, w, nrows, m, shift, j0, G, ldg);
      else
        hipLaunchKernelGGL(sparse_gram_flat_kernel<double>, dim3((unsigned)items), dim3(64), 0, st, colptr, rowidx,
                           (const double*)valT, bptr, lidx, (const double*)bval, w, nrows, m, shift, j0, G, ldg);
    } else if (var != 1) {
      // 2: 32 rows per batch, 3: 64 rows, 4 / 5: the same with b-major items (5: default)
      auto go = [&](auto kf, auto kd) {
        if (f32)
          hipLaunchKernelGGL(kf, dim3((unsigned)items), dim3(64), 0, st, colptr, rowidx, (const float*)valT, bptr, lidx,
                             (const float*)bval, w, nrows, m, shift, j0, G, ldg);
        else
          hipLaunchKernelGGL(kd, dim3((unsigned)items), dim3(64), 0, st, colptr, rowidx, (const double*)valT, bptr,
                             lidx, (const double*)bval, w, nrows, m, shift, j0, G, ldg);
      };
      if (var == 3) go(sparse_gram_pipe_kernel<float, 64, false>, sparse_gram_pipe_kernel<double, 64, false>);
      else if (var == 4) go(sparse_gram_pipe_kernel<float, 32, true>, sparse_gram_pipe_kernel<double, 32, true>);
      else if (var == 5) go(sparse_gram_pipe_kernel<float, 64, true>, sparse_gram_pipe_kernel<double, 64, true>);
      else go(sparse_gram_pipe_kernel<float, 32, false>, sparse_gram_pipe_kernel<double, 32, false>);
    } else if (f32)
      hipLaunchKernelGGL(sparse_gram_kernel<float>, dim3((unsigned)items), dim3(64), 0, st, colptr, rowidx,
                         (const float*)valT, bptr, lidx, (const float*)bval, w, nrows, m, shift, j0, G, ldg);
    else
      hipLaunchKernelGGL(sparse_gram_kernel<double>, dim3((unsigned)items), dim3(64), 0, st, colptr, rowidx,
                         (const double*)valT, bptr, lidx, (const double*)bval, w, nrows, m, shift, j0, G, ldg);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    j0 = j1;
  }
  return hipSuccess;
}

// ---- synthetic generator ---------------------------------------------------
__device__ __forceinline__ uint64_t smix_s(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double uni_s(uint64_t seed, uint64_t idx) {
  const uint64_t h = smix_s(smix_s(seed) ^ idx);
  return ((double)(h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ double gauss_s(uint64_t seed, uint64_t idx) {
  const double u1 = uni_s(seed, 2 * idx), u2 = uni_s(seed, 2 * idx + 1);
  return sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
}
struct LayerMap {
  uint64_t a, ainv, b;
};
__host__ __device__ inline uint64_t inv_pow2(uint64_t a) {  // a odd -> a⁻¹ mod 2^64
  uint64_t x = a;
  for (int i = 0; i < 6; ++i) x *= 2 - a * x;
  return x;
}

template <typename VT>
__global__ void gen_csr_kernel(int64_t N, int64_t m, int k, uint64_t seed, const LayerMap* __restrict__ L,
                               double scale, int64_t* __restrict__ rowptr, int* __restrict__ col,
                               VT* __restrict__ val) {
  const uint64_t Nm = (uint64_t)N - 1;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < N * k; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / k;
    const int s = (int)(e - i * k);
    const uint64_t u = (L[s].a * (uint64_t)i + L[s].b) & Nm;
    col[e] = (int)(u % (uint64_t)m);
    val[e] = (VT)(scale * gauss_s(seed, (uint64_t)i * k + s));
    if (s == 0) rowptr[i] = e;
    if (e == N * k - 1) rowptr[N] = N * k;
  }
}

template <typename VT>
__global__ void gen_csc_kernel(int64_t N, int64_t m, int k, uint64_t seed, const LayerMap* __restrict__ L,
                               double scale, int64_t* __restrict__ colptr, int* __restrict__ row,
                               VT* __restrict__ val) {
  const uint64_t Nm = (uint64_t)N - 1;
  const int64_t r = N / m;          // entries per column per layer
  const int64_t per_col = (int64_t)k * r;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < m * per_col;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e / per_col;
    const int64_t q = e - c * per_col;
    const int s = (int)(q / r);
    const int64_t t = q - (int64_t)s * r;
    const uint64_t u = (uint64_t)c + (uint64_t)t * (uint64_t)m;
    const uint64_t i = (L[s].ainv * (u - L[s].b)) & Nm;
    row[e] = (int)i;
    val[e] = (VT)(scale * gauss_s(seed, i * k + s));
    if (q == 0) colptr[c] = e;
    if (e == m * per_col - 1) colptr[m] = m * per_col;
  }
}

void sparse_layer_maps(uint64_t seed, int k, int64_t N, void* out_host) {
  LayerMap* L = (LayerMap*)out_host;
  for (int s = 0; s < k; ++s) {
    uint64_t z = seed * 0x2545F4914F6CDD1Dull + (uint64_t)s * 0x9E3779B97F4A7C15ull;
    auto mix = [](uint64_t v) {
      v ^= v >> 33; v *= 0xff51afd7ed558ccdull; v ^= v >> 33; v *= 0xc4ceb9fe1a85ec53ull; v ^= v >> 33;
      return v;
    };
    const uint64_t a = (mix(z) | 1ull) & ((uint64_t)N - 1);
    const uint64_t b = mix(z + 1) & ((uint64_t)N - 1);
    L[s].a = a | 1ull;
    L[s].ainv = inv_pow2(L[s].a);
    L[s].b = b;
  }
}

size_t sparse_layer_map_bytes(int k) { return sizeof(LayerMap) * (size_t)k; }

hipError_t launch_gen_sparse(int64_t N, int64_t m, int k, uint64_t seed, const void* Ldev, int f32, double scale,
                             int64_t* rowptr, int* col, void* val, int64_t* colptr, int* row, void* valT,
                             hipStream_t st) {
  const LayerMap* L = (const LayerMap*)Ldev;
  if (f32) {
    hipLaunchKernelGGL(gen_csr_kernel<float>, dim3(8192), dim3(256), 0, st, N, m, k, seed, L, scale, rowptr, col,
                       (float*)val);
    hipLaunchKernelGGL(gen_csc_kernel<float>, dim3(8192), dim3(256), 0, st, N, m, k, seed, L, scale, colptr, row,
                       (float*)valT);
  } else {
    hipLaunchKernelGGL(gen_csr_kernel<double>, dim3(8192), dim3(256), 0, st, N, m, k, seed, L, scale, rowptr, col,
                       (double*)val);
    hipLaunchKernelGGL(gen_csc_kernel<double>, dim3(8192), dim3(256), 0, st, N, m, k, seed, L, scale, colptr, row,
                       (double*)valT);
  }
  return hipGetLastError();
}

// Sort each segment's (index, value) pairs by index (segments = CSC columns).
// With temp == nullptr only *temp_bytes is set.  Ascending row order per
// column makes the concurrently running column waves sweep the gathered vector
// in the same direction, so its lines are reused in L2 instead of re-fetched.
hipError_t sort_segments(void* temp, size_t* temp_bytes, const int* kin, int* kout, const void* vin, void* vout,
                         int f32, int64_t nnz, int64_t nseg, const int64_t* off, int end_bit, hipStream_t st) {
  if (f32)
    return hipcub::DeviceSegmentedRadixSort::SortPairs(temp, *temp_bytes, kin, kout, (const float*)vin, (float*)vout,
                                                       (int)nnz, (int)nseg, off, off + 1, 0, end_bit, st);
  return hipcub::DeviceSegmentedRadixSort::SortPairs(temp, *temp_bytes, kin, kout, (const double*)vin, (double*)vout,
                                                     (int)nnz, (int)nseg, off, off + 1, 0, end_bit, st);
}

// Dense panel-blocked mirror of a CSR A (common.h tiled_off; Ad zeroed by the caller) for the
// Gram-based methods (Jt*Q*Jt' of a SparseMatrixCSC, prox-GGN-SCORE.jl:129).  One thread per
// row walks its entries in CSR order, so duplicates are summed race-free.
template <typename V>
__global__ void densify_kernel(const int64_t* __restrict__ rowptr, const int* __restrict__ col,
                               const V* __restrict__ val, int64_t N, int64_t S, double* __restrict__ Ad) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x)
    for (int64_t p = rowptr[r]; p < rowptr[r + 1]; ++p) Ad[tiled_off(S, r, col[p])] += (double)val[p];
}

hipError_t launch_densify(const int64_t* rowptr, const int* col, const void* val, int f32, int64_t N, int64_t Npad,
                          double* Ad, hipStream_t st) {
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(std::max<int64_t>(N, 1), 256), 16384);
  if (f32)
    hipLaunchKernelGGL(densify_kernel<float>, dim3(grid), dim3(256), 0, st, rowptr, col, (const float*)val, N,
                       Npad / 16, Ad);
  else
    hipLaunchKernelGGL(densify_kernel<double>, dim3(grid), dim3(256), 0, st, rowptr, col, (const double*)val, N,
                       Npad / 16, Ad);
  return hipGetLastError();
}

// Streaming sparse Gram (scsopt.cpp gram_main): CSR rows [r0, r0 + n) -> the panel-blocked slot Ab
// (S stages), entries summed in CSR order (duplicates race-free); zero = 1 writes zeros at the
// same positions instead, which clears a slot for its next chunk (the slot is otherwise zero).
template <typename V>
__global__ void densify_range_kernel(const int64_t* __restrict__ rowptr, const int* __restrict__ col,
                                     const V* __restrict__ val, int64_t r0, int64_t n, int64_t S, int zero,
                                     double* __restrict__ Ab) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    for (int64_t p = rowptr[r0 + r]; p < rowptr[r0 + r + 1]; ++p) {
      double* dst = Ab + tiled_off(S, r, col[p]);
      if (zero) *dst = 0.0;
      else *dst += (double)val[p];
    }
}

hipError_t launch_densify_range(const int64_t* rowptr, const int* col, const void* val, int f32, int64_t r0,
                                int64_t n, int64_t Npad_b, int zero, double* Ab, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n, 256), 16384);
  if (f32)
    hipLaunchKernelGGL(densify_range_kernel<float>, dim3(grid), dim3(256), 0, st, rowptr, col, (const float*)val, r0,
                       n, Npad_b / 16, zero, Ab);
  else
    hipLaunchKernelGGL(densify_range_kernel<double>, dim3(grid), dim3(256), 0, st, rowptr, col, (const double*)val,
                       r0, n, Npad_b / 16, zero, Ab);
  return hipGetLastError();
}

// Minibatch of a sparse A: CSR rows rows[0..n) -> dense panel-blocked batch Ab (Npad_b rows,
// zeroed by the caller), y -> yb.  One thread per batch row, entries in CSR order.
template <typename V>
__global__ void densify_rows_kernel(const int64_t* __restrict__ rowptr, const int* __restrict__ col,
                                    const V* __restrict__ val, const int64_t* __restrict__ rows, int64_t n,
                                    int64_t Npad_b, const double* __restrict__ y, double* __restrict__ Ab,
                                    double* __restrict__ yb) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < Npad_b; r += (int64_t)gridDim.x * blockDim.x) {
    if (r >= n) {
      yb[r] = 0.0;
      continue;
    }
    const int64_t src = rows[r];
    yb[r] = y[src];
    for (int64_t p = rowptr[src]; p < rowptr[src + 1]; ++p) Ab[tiled_off(Npad_b / 16, r, col[p])] += (double)val[p];
  }
}

hipError_t launch_densify_rows(const int64_t* rowptr, const int* col, const void* val, int f32, const int64_t* rows,
                               int64_t n, int64_t Npad_b, const double* y, double* Ab, double* yb, hipStream_t st) {
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(std::max<int64_t>(Npad_b, 1), 256), 16384);
  if (f32)
    hipLaunchKernelGGL(densify_rows_kernel<float>, dim3(grid), dim3(256), 0, st, rowptr, col, (const float*)val, rows,
                       n, Npad_b, y, Ab, yb);
  else
    hipLaunchKernelGGL(densify_rows_kernel<double>, dim3(grid), dim3(256), 0, st, rowptr, col, (const double*)val,
                       rows, n, Npad_b, y, Ab, yb);
  return hipGetLastError();
}

// x_true ~ U(-1.5, 1.5); y = A x_true + 0.1 ε computed by the caller
__global__ void gen_uniform_kernel(double* __restrict__ x, int64_t m, uint64_t seed, double lo, double hi) {
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j < m) x[j] = lo + (hi - lo) * uni_s(seed + 5, j);
}
hipError_t launch_gen_uniform(double* x, int64_t m, uint64_t seed, double lo, double hi, hipStream_t st) {
  hipLaunchKernelGGL(gen_uniform_kernel, dim3((unsigned)ceil_div(m, 256)), dim3(256), 0, st, x, m, seed, lo, hi);
  return hipGetLastError();
}

}  // namespace scs
