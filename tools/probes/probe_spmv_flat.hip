// Experiment harness (not part of libscsopt): C5-shaped LDS-blocked fp64 SpMV.
//   product : launch_spmv_blk (sparse.hip): per-row rounds, 2 rows per wave round
//   stream  : read-only ceiling over the same padded (index, value) bytes, no gather
//   flat<W> : each wave streams its 64 rows' slots as one contiguous range, 64 slots per
//             window (fully active lanes), row of each slot from the wave's row starts,
//             segmented prefix sum inside the window, per-row LDS accumulator; W windows
//             of loads in flight ahead of the compute
// usage: probe_spmv_flat [dir]   dir 0: 2^20 rows x 4 blocks (A x), 1: 2^16 rows x 64 blocks (Aᵀ v)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "common.h"
#include "kernels.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

using namespace scs;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename VT>
__global__ void fill_kernel(const int64_t* pb, int64_t nseg, const int64_t* pa, uint16_t* ib, VT* vb, int padi) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nseg) return;
  const int lane = threadIdx.x & 63;
  const int64_t L = pa[s + 1] - pa[s], b0 = pb[s], b1 = pb[s + 1];
  for (int64_t e = lane; e < b1 - b0; e += 64) {
    if (e < L) {
      const uint64_t h = mix64((uint64_t)s * 1000003ull + e);
      ib[b0 + e] = (uint16_t)(h & 16383);
      vb[b0 + e] = (VT)(((double)(h >> 20) * (1.0 / 17592186044416.0)) - 0.5);
    } else {
      ib[b0 + e] = (uint16_t)padi;
      vb[b0 + e] = (VT)0;
    }
  }
}

// read-only ceiling: every lane streams 16-B value loads + 8-B index loads of consecutive slots
template <int LDSKB>
__global__ __launch_bounds__(1024) void stream_kernel(const uint64_t* __restrict__ id, const v2d* __restrict__ v,
                                                      int64_t nslot, double* out) {
  __shared__ double pad[LDSKB * 128 + 1];
  double acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nslot; s += 2 * stride) {
    const int64_t s2 = min(s + stride, nslot - 1);
    const uint64_t i0 = id[s], i1 = id[s2];
    const v2d a0 = v[2 * s], b0 = v[2 * s + 1], a1 = v[2 * s2], b1 = v[2 * s2 + 1];
    acc += a0[0] + a0[1] + b0[0] + b0[1] + (double)(i0 & 7) + a1[0] + a1[1] + b1[0] + b1[1] + (double)(i1 & 7);
  }
  if (LDSKB) {
    pad[threadIdx.x] = acc;
    __syncthreads();
    acc = pad[(threadIdx.x + 1) & 1023];
  }
  if (acc == 12345.678) out[0] = acc;
}

struct Win {
  uint64_t id;
  double v[4];
};

__device__ __forceinline__ void win_load(Win& w, const uint64_t* __restrict__ id4, const double* __restrict__ val,
                                         int64_t sb, int q) {
  w.id = id4[sb + q];
  const v2d a = *(const v2d*)(val + 4 * (sb + q)), b = *(const v2d*)(val + 4 * (sb + q) + 2);
  w.v[0] = a[0];
  w.v[1] = a[1];
  w.v[2] = b[0];
  w.v[3] = b[1];
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, ROWMASK, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, ROWMASK, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// segmented inclusive prefix sum over lanes [max(rs, 0), lane] (rows of lanes nondecreasing)
template <int SCAN>
__device__ __forceinline__ double seg_scan(double p, int lane, int rs) {
  if (SCAN == 0) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double u = __shfl_up(p, off, 64);
      if (lane - off >= rs && lane >= off) p += u;
    }
    return p;
  }
  const int l16 = lane & 15;
  double u;
  u = dpp_d<0x111, 0xF>(p); if (l16 >= 1 && lane - 1 >= rs) p += u;
  u = dpp_d<0x112, 0xF>(p); if (l16 >= 2 && lane - 2 >= rs) p += u;
  u = dpp_d<0x114, 0xF>(p); if (l16 >= 4 && lane - 4 >= rs) p += u;
  u = dpp_d<0x118, 0xF>(p); if (l16 >= 8 && lane - 8 >= rs) p += u;
  u = dpp_d<0x142, 0xA>(p); if ((lane & 16) && (lane & ~15) - 1 >= rs) p += u;   // row_bcast:15
  u = dpp_d<0x143, 0xC>(p); if ((lane & 32) && 31 >= rs) p += u;                  // row_bcast:31
  return p;
}

template <int W, int SCAN = 0>
__global__ __launch_bounds__(1024) void flat_kernel(const int64_t* __restrict__ ptr, const uint16_t* __restrict__ lidx,
                                                    const double* __restrict__ val, const double* __restrict__ x,
                                                    int64_t nrows, int64_t ncols, int shift, double* __restrict__ out,
                                                    int64_t ldo) {
  __shared__ double xs[1 << 14];
  const int b = blockIdx.y;
  const int64_t c0 = (int64_t)b << shift;
  const int nb = (int)min((int64_t)1 << shift, ncols - c0);
  {
    constexpr int PER = (1 << 14) / 1024;
    double t[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + k * 1024;
      t[k] = (i < nb) ? x[c0 + i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) xs[threadIdx.x + k * 1024] = t[k];
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  const int64_t* pb = ptr + (int64_t)b * nrows;
  const int64_t rw0 = (int64_t)blockIdx.x * 1024 + (int64_t)wv * 64;
  const int nrw = (int)max((int64_t)0, min((int64_t)64, nrows - rw0));
  if (nrw == 0) return;
  const int64_t sb = pb[rw0] >> 2;                    // wave's first slot
  const int total = (int)((pb[rw0 + nrw] >> 2) - sb);  // wave's slot count
  // st: relative slot start of row `lane` (rows past nrw: total)
  const int st = lane < nrw ? (int)((pb[rw0 + lane] >> 2) - sb) : total;
  const uint64_t* id4 = (const uint64_t*)lidx;
  const int nwin = (total + 63) >> 6;
  Win buf[W];
#pragma unroll
  for (int j = 0; j < W; ++j) win_load(buf[j], id4, val, sb, max(min(64 * j + lane, total - 1), 0));
  const int stn = __shfl(st, min(lane + 1, 63), 64);
  const int en = lane + 1 < nrw ? stn : total;   // end slot of row `lane`
  double acc = 0.0;
  int cur = 0;   // row of slot `base` (wave-uniform)
  for (int t0 = 0; t0 < nwin; t0 += W) {
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const int t = t0 + j;
      if (t >= nwin) break;
      const Win w = buf[j];
      const int tn = t + W;
      if (tn < nwin) win_load(buf[j], id4, val, sb, min(64 * tn + lane, total - 1));
      const int base = 64 * t, slot = base + lane;
      double p = 0.0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = (int)((w.id >> (16 * e)) & 0xFFFF);
        if (c != 0xFFFF) p += w.v[e] * xs[c];
      }
      if (slot >= total) p = 0.0;
      // row of my slot: cur + #{k > cur : st_k <= slot}
      int r = cur, k = cur + 1;
      while (k < nrw) {
        const int sk = __builtin_amdgcn_readlane(st, k);
        if (sk > base + 64) break;
        r += (slot >= sk) ? 1 : 0;
        ++k;
      }
      cur = k - 1;
      // segment start lane of my row inside the window
      const int rs = __shfl(st, r, 64) - base;   // may be < 0 (row began in an earlier window)
      p = seg_scan<SCAN>(p, lane, rs);
      // row `lane` pulls its window sum from its tail lane (last slot of the row in the window)
      // (every lane takes part in the shuffle: a bpermute from a lane masked off by a branch reads garbage)
      const double pt = __shfl(p, max(min(en - base - 1, 63), 0), 64);
      if (st < base + 64 && en > base && st < en) acc += pt;
    }
  }
  if (lane < nrw) out[(int64_t)b * ldo + rw0 + lane] = acc;
}

typedef unsigned long long v2u __attribute__((ext_vector_type(2)));
template <int SLOT>
struct WinS {
  uint64_t id[SLOT / 4];
  double v[SLOT];
};
typedef float v4f __attribute__((ext_vector_type(4)));
template <int SLOT>
__device__ __forceinline__ void wins_load(WinS<SLOT>& w, const uint16_t* __restrict__ lidx,
                                          const float* __restrict__ val, int64_t slot) {
  if (SLOT == 4) {
    w.id[0] = *(const uint64_t*)(lidx + 4 * slot);
  } else {
#pragma unroll
    for (int k = 0; k < SLOT / 8; ++k) {
      const v2u t = *(const v2u*)(lidx + SLOT * slot + 8 * k);
      w.id[2 * k] = t[0];
      w.id[2 * k + 1] = t[1];
    }
  }
#pragma unroll
  for (int k = 0; k < SLOT / 4; ++k) {
    const v4f a = *(const v4f*)(val + SLOT * slot + 4 * k);
#pragma unroll
    for (int q = 0; q < 4; ++q) w.v[4 * k + q] = a[q];
  }
}
template <int SLOT>
__device__ __forceinline__ void wins_load(WinS<SLOT>& w, const uint16_t* __restrict__ lidx,
                                          const double* __restrict__ val, int64_t slot) {
  if (SLOT == 4) {
    w.id[0] = *(const uint64_t*)(lidx + 4 * slot);
  } else {
    const v2u t = *(const v2u*)(lidx + 8 * slot);
    w.id[0] = t[0];
    w.id[SLOT / 4 - 1] = t[1];
  }
#pragma unroll
  for (int k = 0; k < SLOT / 2; ++k) {
    const v2d a = *(const v2d*)(val + SLOT * slot + 2 * k);
    w.v[2 * k] = a[0];
    w.v[2 * k + 1] = a[1];
  }
}

// flat2: DPP segmented scan, one window of loads ahead, SLOT entries per lane (segments padded to
// SLOT), PADZ: padding index = 16384 with xs[16384] = 0 (no per-entry compare)
template <int SLOT, bool PADZ, typename VT = double>
__global__ __launch_bounds__(1024) void flat2_kernel(const int64_t* __restrict__ ptr, const uint16_t* __restrict__ lidx,
                                                     const VT* __restrict__ val, const double* __restrict__ x,
                                                     int64_t nrows, int64_t ncols, int shift, double* __restrict__ out,
                                                     int64_t ldo) {
  constexpr int SH = SLOT == 4 ? 2 : SLOT == 8 ? 3 : 4;
  __shared__ double xs[(1 << 14) + 2];
  const int b = blockIdx.y;
  const int64_t c0 = (int64_t)b << shift;
  const int nb = (int)min((int64_t)1 << shift, ncols - c0);
  {
    constexpr int PER = (1 << 14) / 1024;
    double t[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + k * 1024;
      t[k] = (i < nb) ? x[c0 + i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) xs[threadIdx.x + k * 1024] = t[k];
    if (threadIdx.x == 0) xs[1 << 14] = 0.0;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  const int64_t* pb = ptr + (int64_t)b * nrows;
  const int64_t rw0 = (int64_t)blockIdx.x * 1024 + (int64_t)wv * 64;
  const int nrw = (int)max((int64_t)0, min((int64_t)64, nrows - rw0));
  if (nrw == 0) return;
  const int64_t sb = pb[rw0] >> SH;
  const int total = (int)((pb[rw0 + nrw] >> SH) - sb);
  const int st = lane < nrw ? (int)((pb[rw0 + lane] >> SH) - sb) : total;
  const int stn = __shfl(st, min(lane + 1, 63), 64);
  const int en = lane + 1 < nrw ? stn : total;
  const int nwin = (total + 63) >> 6;
  WinS<SLOT> buf;
  wins_load<SLOT>(buf, lidx, val, sb + max(min(lane, total - 1), 0));
  double acc = 0.0;
  int cur = 0;
  for (int t = 0; t < nwin; ++t) {
    const WinS<SLOT> w = buf;
    if (t + 1 < nwin) wins_load<SLOT>(buf, lidx, val, sb + min(64 * (t + 1) + lane, total - 1));
    const int base = 64 * t, slot = base + lane;
    double p = 0.0;
#pragma unroll
    for (int e = 0; e < SLOT; ++e) {
      const int c = (int)((w.id[e / 4] >> (16 * (e & 3))) & 0xFFFF);
      if (PADZ) p += w.v[e] * xs[c];
      else if (c != 0xFFFF) p += w.v[e] * xs[c];
    }
    if (slot >= total) p = 0.0;
    int r = cur, k = cur + 1;
    while (k < nrw) {
      const int sk = __builtin_amdgcn_readlane(st, k);
      if (sk > base + 64) break;
      r += (slot >= sk) ? 1 : 0;
      ++k;
    }
    cur = k - 1;
    const int rs = __shfl(st, r, 64) - base;
    p = seg_scan<1>(p, lane, rs);
    const double pt = __shfl(p, max(min(en - base - 1, 63), 0), 64);
    if (st < base + 64 && en > base && st < en) acc += pt;
  }
  if (lane < nrw) out[(int64_t)b * ldo + rw0 + lane] = acc;
}

static void run(int dir) {
  const int64_t nrows = dir == 0 ? (1 << 20) : (1 << 16);
  const int64_t ncols = dir == 0 ? (1 << 16) : (1 << 20);
  const int shift = 14;
  const int nblk = (int)(ncols >> shift);
  const int64_t nseg = nrows * nblk;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd(164.0, 11.0);
  std::vector<int64_t> pa(nseg + 1), pb(nseg + 1), p8(nseg + 1), p16(nseg + 1);
  pa[0] = pb[0] = p8[0] = p16[0] = 0;
  for (int64_t s = 0; s < nseg; ++s) {
    int64_t L = std::max<int64_t>(0, (int64_t)std::llround(nd(rng)));
    if (s % 97 == 5) L = 0;          // some empty segments
    if (s % 1013 == 7) L = 700;      // some long ones
    pa[s + 1] = pa[s] + L;
    pb[s + 1] = pb[s] + ((L + 3) & ~3LL);
    p8[s + 1] = p8[s] + ((L + 7) & ~7LL);
    p16[s + 1] = p16[s] + ((L + 15) & ~15LL);
  }
  const int64_t nnz = pa[nseg], nnzb = pb[nseg];
  printf("dir %d nrows %lld nblk %d nnz %lld padded %lld\n", dir, (long long)nrows, nblk, (long long)nnz,
         (long long)nnzb);
  int64_t *dpa, *dpb;
  uint16_t* ib;
  double *vb, *x, *oa, *ob;
  CK(hipMalloc(&dpa, 8 * (nseg + 1)));
  CK(hipMalloc(&dpb, 8 * (nseg + 1)));
  CK(hipMalloc(&ib, 2 * nnzb + 64));
  CK(hipMalloc(&vb, 8 * nnzb + 64));
  CK(hipMalloc(&x, 8 * ncols));
  CK(hipMalloc(&oa, 8 * nseg));
  CK(hipMalloc(&ob, 8 * nseg));
  CK(hipMemcpy(dpa, pa.data(), 8 * (nseg + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(dpb, pb.data(), 8 * (nseg + 1), hipMemcpyHostToDevice));
  std::vector<double> hx(ncols);
  for (auto& t : hx) t = std::uniform_real_distribution<double>(-1, 1)(rng);
  CK(hipMemcpy(x, hx.data(), 8 * ncols, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill_kernel<double>, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, 0, dpb, nseg, dpa, ib, vb, 0xFFFF);
  const int64_t nnz8 = p8[nseg];
  int64_t *dp8;
  uint16_t *ibz, *ib8;
  double *vbz, *vb8;
  CK(hipMalloc(&dp8, 8 * (nseg + 1)));
  CK(hipMalloc(&ibz, 2 * nnzb + 64));
  CK(hipMalloc(&vbz, 8 * nnzb + 64));
  CK(hipMalloc(&ib8, 2 * nnz8 + 64));
  CK(hipMalloc(&vb8, 8 * nnz8 + 64));
  CK(hipMemcpy(dp8, p8.data(), 8 * (nseg + 1), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill_kernel<double>, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, 0, dpb, nseg, dpa, ibz, vbz, 16384);
  hipLaunchKernelGGL(fill_kernel<double>, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, 0, dp8, nseg, dpa, ib8, vb8, 16384);
  printf("8-padded nnz %lld (+%.2f%%)\n", (long long)nnz8, 100.0 * (nnz8 - nnz) / nnz);
  CK(hipDeviceSynchronize());
  // the product layout: ptr is nblk x (nrows + 1), segment (row r, block b) at pb[b * nrows + r]
  // -- the probe's segment order is block-major too (s = b * nrows + r), so pb serves directly
  // with the per-block pointer arrays overlapping by one (pb[b*nrows + nrows] = next block start)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)nnz * 10;
  auto timeit = [&](const char* name, auto&& launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("  %-26s %.4f ms  %.0f GB/s (nnz*10 B)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  timeit("product", [&] { CK(launch_spmv_blk(dpb, ib, vb, 0, x, nrows, ncols, shift, nnzb, oa, nrows, 0)); });
  const int64_t nslot = nnzb / 4;
  for (int g : {256, 512, 1024, 2048}) {
    char nm[64];
    snprintf(nm, sizeof nm, "stream lds128 grid %d", g);
    timeit(nm, [&] {
      hipLaunchKernelGGL(stream_kernel<128>, dim3(g), dim3(1024), 0, 0, (const uint64_t*)ib, (const v2d*)vb, nslot, ob);
    });
    snprintf(nm, sizeof nm, "stream nolds grid %d", g);
    timeit(nm, [&] {
      hipLaunchKernelGGL(stream_kernel<0>, dim3(g), dim3(1024), 0, 0, (const uint64_t*)ib, (const v2d*)vb, nslot, ob);
    });
  }
  const dim3 grid((unsigned)((nrows + 1023) / 1024), (unsigned)nblk);
  std::vector<double> ha(nseg), hb(nseg);
  CK(hipMemcpy(ha.data(), oa, 8 * nseg, hipMemcpyDeviceToHost));
  std::vector<uint16_t> hib(nnzb);
  std::vector<double> hvb(nnzb);
  CK(hipMemcpy(hib.data(), ib, 2 * nnzb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hvb.data(), vb, 8 * nnzb, hipMemcpyDeviceToHost));
  auto host_check = [&](const char* name, const std::vector<double>& o) {
    double md = 0;
    int64_t worst = -1;
    for (int64_t s = 0; s < nseg; s += (s % 1013 == 7 || s % 97 == 5) ? 1 : 7) {
      const int64_t bb = s / nrows;
      double acc = 0;
      for (int64_t e = pb[s]; e < pb[s + 1]; ++e)
        if (hib[e] != 0xFFFF) acc += hvb[e] * hx[(bb << shift) + hib[e]];
      const double d = std::fabs(acc - o[s]);
      if (d > md) { md = d; worst = s; }
    }
    if (md > 1e-10) {   // wave of the worst segment: rows, exp vs got
      const int64_t w0 = worst - (worst % nrows) % 64;
      int nbad = 0;
      for (int64_t q = w0; q < w0 + 64; ++q) {
        const int64_t bb = q / nrows;
        double acc = 0;
        for (int64_t e = pb[q]; e < pb[q + 1]; ++e)
          if (hib[e] != 0xFFFF) acc += hvb[e] * hx[(bb << shift) + hib[e]];
        if (std::fabs(acc - o[q]) > 1e-10) {
          ++nbad;
          printf("    row %lld slot0 %lld len %lld exp %.6f got %.6f\n", (long long)(q - w0),
                 (long long)((pb[q] - pb[w0]) / 4), (long long)(pb[q + 1] - pb[q]), acc, o[q]);
        }
      }
      printf("    bad rows in wave: %d\n", nbad);
    }
    printf("  %s vs host: max diff %.3e at seg %lld (len %lld)\n", name, md, (long long)worst,
           worst >= 0 ? (long long)(pb[worst + 1] - pb[worst]) : -1LL);
  };
  host_check("product", ha);
  auto check = [&](const char* name) {
    CK(hipMemcpy(hb.data(), ob, 8 * nseg, hipMemcpyDeviceToHost));
    host_check(name, hb);
    double md = 0, mx = 0;
    for (int64_t s = 0; s < nseg; ++s) {
      md = std::max(md, std::fabs(ha[s] - hb[s]));
      mx = std::max(mx, std::fabs(ha[s]));
    }
    printf("  %s max |product - it| = %.3e (max %.3e)\n", name, md, mx);
  };
  timeit("flat W=1", [&] {
    hipLaunchKernelGGL(flat_kernel<1>, grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows);
  });
  check("flat W=1");
  timeit("flat W=2", [&] {
    hipLaunchKernelGGL(flat_kernel<2>, grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows);
  });
  check("flat W=2");
  timeit("flat W=1 dpp", [&] {
    hipLaunchKernelGGL((flat_kernel<1, 1>), grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows);
  });
  check("flat W=1 dpp");
  timeit("flat W=2 dpp", [&] {
    hipLaunchKernelGGL((flat_kernel<2, 1>), grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows);
  });
  check("flat W=2 dpp");
  timeit("flat2 S4 padz", [&] {
    hipLaunchKernelGGL((flat2_kernel<4, true>), grid, dim3(1024), 0, 0, dpb, ibz, vbz, x, nrows, ncols, shift, ob, nrows);
  });
  check("flat2 S4 padz");
  timeit("flat2 S4", [&] {
    hipLaunchKernelGGL((flat2_kernel<4, false>), grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows);
  });
  check("flat2 S4");
  timeit("flat2 S8 padz", [&] {
    hipLaunchKernelGGL((flat2_kernel<8, true>), grid, dim3(1024), 0, 0, dp8, ib8, vb8, x, nrows, ncols, shift, ob, nrows);
  });
  check("flat2 S8 padz");
  {
    uint16_t *fia, *fib, *fi8, *fi16;
    float *fva, *fvb, *fv8, *fv16;
    int64_t* dp16;
    const int64_t nnz16 = p16[nseg];
    CK(hipMalloc(&dp16, 8 * (nseg + 1)));
    CK(hipMemcpy(dp16, p16.data(), 8 * (nseg + 1), hipMemcpyHostToDevice));
    CK(hipMalloc(&fi16, 2 * nnz16 + 64));
    CK(hipMalloc(&fv16, 4 * nnz16 + 64));
    hipLaunchKernelGGL(fill_kernel<float>, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, 0, dp16, nseg, dpa, fi16, fv16, 16384);
    printf("16-padded +%.2f%%\n", 100.0 * (nnz16 - nnz) / nnz);
    CK(hipMalloc(&fia, 2 * nnz + 64));
    CK(hipMalloc(&fva, 4 * nnz + 64));
    CK(hipMalloc(&fib, 2 * nnzb + 64));
    CK(hipMalloc(&fvb, 4 * nnzb + 64));
    CK(hipMalloc(&fi8, 2 * nnz8 + 64));
    CK(hipMalloc(&fv8, 4 * nnz8 + 64));
    hipLaunchKernelGGL(fill_kernel<float>, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, 0, dpa, nseg, dpa, fia, fva, 0xFFFF);
    hipLaunchKernelGGL(fill_kernel<float>, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, 0, dpb, nseg, dpa, fib, fvb, 16384);
    hipLaunchKernelGGL(fill_kernel<float>, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, 0, dp8, nseg, dpa, fi8, fv8, 16384);
    CK(hipDeviceSynchronize());
    const double fbytes = (double)nnz * 6;
    auto ftime = [&](const char* name, auto&& launch) {
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 20;
      printf("  %-26s %.4f ms  %.0f GB/s (nnz*6 B)\n", name, ms, fbytes / (ms * 1e-3) / 1e9);
    };
    ftime("f32 product", [&] { CK(launch_spmv_blk(dpa, fia, fva, 1, x, nrows, ncols, shift, nnz, oa, nrows, 0)); });
    ftime("f32 flat2 S4", [&] {
      hipLaunchKernelGGL((flat2_kernel<4, true, float>), grid, dim3(1024), 0, 0, dpb, fib, fvb, x, nrows, ncols, shift, ob, nrows);
    });
    {
      std::vector<double> fa(nseg), fb(nseg);
      CK(hipMemcpy(fa.data(), oa, 8 * nseg, hipMemcpyDeviceToHost));
      CK(hipMemcpy(fb.data(), ob, 8 * nseg, hipMemcpyDeviceToHost));
      double md = 0;
      for (int64_t q = 0; q < nseg; ++q) md = std::max(md, std::fabs(fa[q] - fb[q]));
      printf("  f32 S4 max |product - it| = %.3e\n", md);
    }
    ftime("f32 flat2 S8", [&] {
      hipLaunchKernelGGL((flat2_kernel<8, true, float>), grid, dim3(1024), 0, 0, dp8, fi8, fv8, x, nrows, ncols, shift, ob, nrows);
    });
    {
      std::vector<double> fa(nseg), fb(nseg);
      CK(hipMemcpy(fa.data(), oa, 8 * nseg, hipMemcpyDeviceToHost));
      CK(hipMemcpy(fb.data(), ob, 8 * nseg, hipMemcpyDeviceToHost));
      double md = 0;
      for (int64_t q = 0; q < nseg; ++q) md = std::max(md, std::fabs(fa[q] - fb[q]));
      printf("  f32 S8 max |product - it| = %.3e\n", md);
    }
    ftime("f32 flat2 S16", [&] {
      hipLaunchKernelGGL((flat2_kernel<16, true, float>), grid, dim3(1024), 0, 0, dp16, fi16, fv16, x, nrows, ncols, shift, ob, nrows);
    });
    {
      std::vector<double> fa(nseg), fb(nseg);
      CK(hipMemcpy(fa.data(), oa, 8 * nseg, hipMemcpyDeviceToHost));
      CK(hipMemcpy(fb.data(), ob, 8 * nseg, hipMemcpyDeviceToHost));
      double md = 0;
      for (int64_t q = 0; q < nseg; ++q) md = std::max(md, std::fabs(fa[q] - fb[q]));
      printf("  f32 S16 max |product - it| = %.3e\n", md);
    }
  }
  if (getenv("PROBE_FULL")) timeit("flat W=3", [&] {
    hipLaunchKernelGGL(flat_kernel<3>, grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows);
  });
  check("flat W=3");
  timeit("flat W=4", [&] {
    hipLaunchKernelGGL(flat_kernel<4>, grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows);
  });
  check("flat W=4");
  timeit("product", [&] { CK(launch_spmv_blk(dpb, ib, vb, 0, x, nrows, ncols, shift, nnzb, oa, nrows, 0)); });
}

int main(int argc, char** argv) {
  run(argc > 1 ? atoi(argv[1]) : 0);
  return 0;
}
