// Experiment harness (not part of libscsopt): the LDS-blocked SpMV (sparse.hip) at C5's shape
// against candidate variants.  Segment lengths ~ 164 +- 11 per (row, block), as C5 has them.
//   A  : the product kernel (launch_spmv_blk): fp64 on the padded layout, fp32 unpadded
//   B  : this file's copy of the padded-segment kernel (one lane = 4 consecutive entries, 8-B
//        index load + 16/32-B value loads, transposed multi-row wave reduction) at other RW /
//        chunk settings.  (The unpadded one-entry-per-lane form it replaced ran fp64 1.380 ms,
//        fp32 0.943 ms at dir 0.)
// usage: probe_spmv [f32] [dir]   dir 0: 2^20 rows x 4 blocks (A x), 1: 2^16 rows x 64 blocks (Aᵀ v)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "common.h"
#include "kernels.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

using namespace scs;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// one wave per segment: entry e of segment s -> idx, value; written to the unpadded (pa) and the
// padded (pb) layouts; padding of pb: index 0xFFFF, value 0
template <typename VT>
__global__ void fill_kernel(const int64_t* pa, const int64_t* pb, int64_t nseg, uint16_t* ia, VT* va, uint16_t* ib,
                            VT* vb) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nseg) return;
  const int lane = threadIdx.x & 63;
  const int64_t a0 = pa[s], a1 = pa[s + 1], b0 = pb[s], b1 = pb[s + 1];
  for (int64_t e = lane; e < b1 - b0; e += 64) {
    if (e < a1 - a0) {
      const uint64_t h = mix64((uint64_t)s * 1000003ull + e);
      const uint16_t id = (uint16_t)(h & 16383);
      const VT v = (VT)(((double)(h >> 20) * (1.0 / 17592186044416.0)) - 0.5);
      ia[a0 + e] = id;
      va[a0 + e] = v;
      ib[b0 + e] = id;
      vb[b0 + e] = v;
    } else {
      ib[b0 + e] = 0xFFFF;
      vb[b0 + e] = (VT)0;
    }
  }
}

template <typename VT>
struct V4;
template <>
struct V4<double> {
  double v[4];
};
template <>
struct V4<float> {
  float v[4];
};

__device__ __forceinline__ void load4(const double* p, double (&o)[4]) {
  const v2d a = *(const v2d*)p, b = *(const v2d*)(p + 2);
  o[0] = a[0];
  o[1] = a[1];
  o[2] = b[0];
  o[3] = b[1];
}
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void load4(const float* p, double (&o)[4]) {
  const v4f a = *(const v4f*)p;
  o[0] = a[0];
  o[1] = a[1];
  o[2] = a[2];
  o[3] = a[3];
}

// RW rows' lane partials -> lane l holds the sum of row rowof(l) over its group of 64/RW lanes
template <int RW>
__device__ __forceinline__ double multi_row_sum(double (&acc)[RW], int lane, int& row) {
  row = 0;
  int off = 32;
#pragma unroll
  for (int half = RW / 2; half >= 1; half >>= 1) {
    const bool hi = (lane & off) != 0;
#pragma unroll
    for (int j = 0; j < half; ++j) {
      const double keep = hi ? acc[j + half] : acc[j];
      const double send = hi ? acc[j] : acc[j + half];
      acc[j] = keep + __shfl_xor(send, off, 64);
    }
    if (hi) row += half;
    off >>= 1;
  }
  double v = acc[0];
  for (int o = off; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename VT, int RW>
__global__ __launch_bounds__(1024) void spmv_b_kernel(const int64_t* __restrict__ ptr, const uint16_t* __restrict__ lidx,
                                                      const VT* __restrict__ val, const double* __restrict__ x,
                                                      int64_t nrows, int64_t ncols, int shift, double* __restrict__ out,
                                                      int64_t ldo, int chunks) {
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
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t* pb = ptr + (int64_t)b * nrows;
  for (int ch = 0; ch < chunks; ++ch) {
    const int64_t cb = (int64_t)blockIdx.x * chunks + ch;
    if (cb * 1024 >= nrows) break;
    const int64_t r1 = min(nrows, (cb + 1) * 1024);
    const int64_t rw0 = cb * 1024 + (int64_t)wv * 64;
    const int64_t myr = rw0 + lane;
    const int64_t mp0 = (myr < r1) ? pb[myr] : 0, mp1 = (myr < r1) ? pb[myr + 1] : 0;
    const int nrw = (int)max((int64_t)0, min((int64_t)64, r1 - rw0));
    for (int k0 = 0; k0 < nrw; k0 += RW) {
      const uint16_t* li[RW];
      const VT* va[RW];
      int n4[RW];
      double acc[RW];
      int rem = 0;
#pragma unroll
      for (int j = 0; j < RW; ++j) {
        const int k = k0 + j;
        const int64_t a0 = ((int64_t)__builtin_amdgcn_readlane((int)(mp0 >> 32), k) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)mp0, k);
        const int64_t a1 = ((int64_t)__builtin_amdgcn_readlane((int)(mp1 >> 32), k) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)mp1, k);
        n4[j] = (int)((a1 - a0) >> 2);
        li[j] = lidx + a0;
        va[j] = val + a0;
        acc[j] = 0.0;
        rem = max(rem, n4[j]);
      }
      for (int o = lane; o - lane < rem; o += 64) {
        uint64_t id[RW];
        double v[RW][4];
#pragma unroll
        for (int j = 0; j < RW; ++j) {
          const int q = max(min(o, n4[j] - 1), 0);
          id[j] = *(const uint64_t*)(li[j] + 4 * q);
          load4(va[j] + 4 * q, v[j]);
        }
#pragma unroll
        for (int j = 0; j < RW; ++j)
          if (o < n4[j]) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int c = (int)((id[j] >> (16 * e)) & 0xFFFF);
              if (c != 0xFFFF) acc[j] += v[j][e] * xs[c];
            }
          }
      }
      int row;
      const double s = multi_row_sum<RW>(acc, lane, row);
      if ((lane & (64 / RW - 1)) == 0 && k0 + row < nrw) out[(int64_t)b * ldo + rw0 + k0 + row] = s;
    }
  }
}

// C: B with the next round's loads issued before the current round's LDS gathers, FMAs and
// reduction (software pipelining across rounds; each wave keeps its loads in flight while it
// computes).  Segments longer than 256 entries take extra unpipelined passes.
template <typename VT, int RW>
struct Round {
  const uint16_t* li[RW];
  const VT* va[RW];
  int n4[RW];
  int rem;
  uint64_t id[RW];
  double v[RW][4];
};

template <typename VT, int RW>
__device__ __forceinline__ void round_setup(Round<VT, RW>& R, const uint16_t* lidx, const VT* val, int64_t mp0,
                                            int64_t mp1, int k0) {
  R.rem = 0;
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    const int k = k0 + j;
    const int64_t a0 = ((int64_t)__builtin_amdgcn_readlane((int)(mp0 >> 32), k) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)mp0, k);
    const int64_t a1 = ((int64_t)__builtin_amdgcn_readlane((int)(mp1 >> 32), k) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)mp1, k);
    R.n4[j] = (int)((a1 - a0) >> 2);
    R.li[j] = lidx + a0;
    R.va[j] = val + a0;
    R.rem = max(R.rem, R.n4[j]);
  }
}

template <typename VT, int RW>
__device__ __forceinline__ void round_load(Round<VT, RW>& R, int o) {
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    const int q = max(min(o, R.n4[j] - 1), 0);
    R.id[j] = *(const uint64_t*)(R.li[j] + 4 * q);
    load4(R.va[j] + 4 * q, R.v[j]);
  }
}

template <typename VT, int RW>
__device__ __forceinline__ void round_fma(const Round<VT, RW>& R, int o, const double* xs, double (&acc)[RW]) {
#pragma unroll
  for (int j = 0; j < RW; ++j)
    if (o < R.n4[j]) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = (int)((R.id[j] >> (16 * e)) & 0xFFFF);
        if (c != 0xFFFF) acc[j] += R.v[j][e] * xs[c];
      }
    }
}

template <typename VT, int RW>
__global__ __launch_bounds__(1024) void spmv_c_kernel(const int64_t* __restrict__ ptr, const uint16_t* __restrict__ lidx,
                                                      const VT* __restrict__ val, const double* __restrict__ x,
                                                      int64_t nrows, int64_t ncols, int shift, double* __restrict__ out,
                                                      int64_t ldo, int chunks) {
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
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t* pb = ptr + (int64_t)b * nrows;
  for (int ch = 0; ch < chunks; ++ch) {
    const int64_t cb = (int64_t)blockIdx.x * chunks + ch;
    if (cb * 1024 >= nrows) break;
    const int64_t r1 = min(nrows, (cb + 1) * 1024);
    const int64_t rw0 = cb * 1024 + (int64_t)wv * 64;
    const int64_t myr = rw0 + lane;
    const int64_t mp0 = (myr < r1) ? pb[myr] : 0, mp1 = (myr < r1) ? pb[myr + 1] : 0;
    const int nrw = (int)max((int64_t)0, min((int64_t)64, r1 - rw0));
    if (nrw == 0) continue;
    Round<VT, RW> R0, R1;   // named (a dynamically indexed pair would live in scratch)
    auto step = [&](Round<VT, RW>& A, Round<VT, RW>& B, int k0) {
      if (k0 + RW < nrw) {   // uniform: the next round's loads go out before this round's work
        round_setup(B, lidx, val, mp0, mp1, k0 + RW);
        round_load(B, lane);
      }
      double acc[RW];
#pragma unroll
      for (int j = 0; j < RW; ++j) acc[j] = 0.0;
      round_fma(A, lane, xs, acc);
      for (int o = lane + 64; o - lane < A.rem; o += 64) {   // segments past 256 entries
        round_load(A, o);
        round_fma(A, o, xs, acc);
      }
      int row;
      const double sm = multi_row_sum<RW>(acc, lane, row);
      if ((lane & (64 / RW - 1)) == 0 && k0 + row < nrw) out[(int64_t)b * ldo + rw0 + k0 + row] = sm;
    };
    round_setup(R0, lidx, val, mp0, mp1, 0);
    round_load(R0, lane);
    for (int k0 = 0; k0 < nrw; k0 += 2 * RW) {
      step(R0, R1, k0);
      if (k0 + RW >= nrw) break;
      step(R1, R0, k0 + RW);
    }
  }
}

template <typename VT>
static void run(int dir) {
  const int64_t nrows = dir == 0 ? (1 << 20) : (1 << 16);
  const int64_t ncols = dir == 0 ? (1 << 16) : (1 << 20);
  const int shift = 14;
  const int nblk = (int)(ncols >> shift);
  const int64_t nseg = nrows * nblk;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd(164.0, 11.0);
  std::vector<int64_t> pa(nseg + 1), pb(nseg + 1);
  pa[0] = pb[0] = 0;
  for (int64_t s = 0; s < nseg; ++s) {
    const int64_t L = std::max<int64_t>(0, (int64_t)std::llround(nd(rng)));
    pa[s + 1] = pa[s] + L;
    pb[s + 1] = pb[s] + ((L + 3) & ~3LL);
  }
  const int64_t nnz = pa[nseg], nnzb = pb[nseg];
  printf("dir %d %s nrows %lld nblk %d nnz %lld padded %lld (+%.2f%%)\n", dir, sizeof(VT) == 4 ? "f32" : "f64",
         (long long)nrows, nblk, (long long)nnz, (long long)nnzb, 100.0 * (nnzb - nnz) / nnz);
  int64_t *dpa, *dpb;
  uint16_t *ia, *ib;
  VT *va, *vb;
  double *x, *oa, *ob;
  CK(hipMalloc(&dpa, 8 * (nseg + 1)));
  CK(hipMalloc(&dpb, 8 * (nseg + 1)));
  CK(hipMalloc(&ia, 2 * nnz + 64));
  CK(hipMalloc(&ib, 2 * nnzb + 64));
  CK(hipMalloc(&va, sizeof(VT) * nnz + 64));
  CK(hipMalloc(&vb, sizeof(VT) * nnzb + 64));
  CK(hipMalloc(&x, 8 * ncols));
  CK(hipMalloc(&oa, 8 * nseg));
  CK(hipMalloc(&ob, 8 * nseg));
  CK(hipMemcpy(dpa, pa.data(), 8 * (nseg + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(dpb, pb.data(), 8 * (nseg + 1), hipMemcpyHostToDevice));
  std::vector<double> hx(ncols);
  for (auto& t : hx) t = std::uniform_real_distribution<double>(-1, 1)(rng);
  CK(hipMemcpy(x, hx.data(), 8 * ncols, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill_kernel<VT>, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, 0, dpa, dpb, nseg, ia, va, ib, vb);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)nnz * (sizeof(VT) + 2);
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
    printf("  %-28s %.4f ms  %.0f GB/s (nnz*(val+2) B)\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const int f32 = sizeof(VT) == 4;
  timeit("A product", [&] {
    if (f32) CK(launch_spmv_blk(dpa, ia, va, f32, x, nrows, ncols, shift, nnz, oa, nrows, 0));
    else CK(launch_spmv_blk(dpb, ib, vb, f32, x, nrows, ncols, shift, nnz, oa, nrows, 0));
  });
  for (int chunks : {1, 2, 4}) {
    const dim3 grid((unsigned)((nrows / 1024 + chunks - 1) / chunks), (unsigned)nblk);
    char nm[64];
    snprintf(nm, sizeof nm, "B RW=4 chunks=%d", chunks);
    timeit(nm, [&] {
      hipLaunchKernelGGL((spmv_b_kernel<VT, 4>), grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows,
                         chunks);
    });
    snprintf(nm, sizeof nm, "C RW=4 chunks=%d", chunks);
    timeit(nm, [&] {
      hipLaunchKernelGGL((spmv_c_kernel<VT, 4>), grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows,
                         chunks);
    });
    snprintf(nm, sizeof nm, "C RW=2 chunks=%d", chunks);
    timeit(nm, [&] {
      hipLaunchKernelGGL((spmv_c_kernel<VT, 2>), grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows,
                         chunks);
    });
    snprintf(nm, sizeof nm, "B RW=8 chunks=%d", chunks);
    timeit(nm, [&] {
      hipLaunchKernelGGL((spmv_b_kernel<VT, 8>), grid, dim3(1024), 0, 0, dpb, ib, vb, x, nrows, ncols, shift, ob, nrows,
                         chunks);
    });
  }
  std::vector<double> ha(nseg), hb(nseg);
  CK(hipMemcpy(ha.data(), oa, 8 * nseg, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), ob, 8 * nseg, hipMemcpyDeviceToHost));
  double md = 0, mx = 0;
  for (int64_t s = 0; s < nseg; ++s) {
    md = std::max(md, std::fabs(ha[s] - hb[s]));
    mx = std::max(mx, std::fabs(ha[s]));
  }
  printf("  max |A - B| = %.3e (max |A| %.3e)\n", md, mx);
  (void)hipFree(dpa);
  (void)hipFree(dpb);
  (void)hipFree(ia);
  (void)hipFree(ib);
  (void)hipFree(va);
  (void)hipFree(vb);
  (void)hipFree(x);
  (void)hipFree(oa);
  (void)hipFree(ob);
}

int main(int argc, char** argv) {
  const bool f32 = argc > 1 && !strcmp(argv[1], "f32");
  const int dir = argc > 2 ? atoi(argv[2]) : 0;
  if (f32)
    run<float>(dir);
  else
    run<double>(dir);
  return 0;
}
