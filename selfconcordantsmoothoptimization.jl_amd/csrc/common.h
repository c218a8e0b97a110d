// Shared device helpers for libscsopt (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Several kernels size static LDS for gfx950's 160 KiB per CU (lu_swap_cols_kernel 128 KiB,
// lu_diag_inv_kernel ~134 KiB, spmv_blk_kernel 131 KiB): the library is built for gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "libscsopt targets gfx950 (MI355X) only: kernels here use more than 64 KiB of static LDS"
#endif

namespace scs {

constexpr int WAVE = 64;
constexpr double JL_EPS = 2.220446049250313e-16;  // Julia eps()

typedef double v2d __attribute__((ext_vector_type(2)));
typedef double v4d __attribute__((ext_vector_type(4)));

// ---- Julia scalar semantics ------------------------
// Base._isless(x, y) = (x < y) || (signbit(x) > signbit(y))
__device__ __forceinline__ bool jl_isless(double x, double y) {
  return (x < y) || (__builtin_signbit(x) && !__builtin_signbit(y));
}
// max/min(x::Float64, y::Float64): NaN propagates, -0.0 < +0.0.  IEEE
// fmax/fmin (maxNum) drop NaN and leave the zero sign unspecified, so they
// are NOT used anywhere on the parity path.
__device__ __forceinline__ double jl_max(double x, double y) {
  return (__builtin_isnan(x) || (!__builtin_isnan(y) && jl_isless(y, x))) ? x : y;
}
__device__ __forceinline__ double jl_min(double x, double y) {
  return (__builtin_isnan(x) || (!__builtin_isnan(y) && jl_isless(x, y))) ? x : y;
}
// sign(x::Float64): ±1.0, or x itself for ±0.0 and NaN.
__device__ __forceinline__ double jl_sign(double x) {
  return x < 0.0 ? -1.0 : (x > 0.0 ? 1.0 : x);
}

// ---- deterministic reductions ---------------------------------------------
// Butterfly over the 64 lanes; every lane ends with the same fixed-order sum.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum in a fixed order (wave partials summed by thread 0 in wave
// order).  `sh` must hold NT/64 doubles.  Result broadcast to all threads.
// T = float: the same fixed order in fp32 arithmetic (the partials kept in the double scratch,
// exactly representable).
template <int NT, typename T = double>
__device__ __forceinline__ T block_sum(T v, double* sh) {
  v = wave_sum<T>(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = (double)v;
  __syncthreads();
  if (threadIdx.x == 0) {
    T r = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) r += (T)sh[i];
    sh[0] = (double)r;
  }
  __syncthreads();
  const T r = (T)sh[0];
  __syncthreads();
  return r;
}

__host__ __device__ __forceinline__ int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- device layout of A: panel-blocked ("tiled") ------------------------------
// Block (panel p = j / 128, stage s = n / 16) holds [128 features][16 samples]
// contiguously (16 KiB); blocks of one panel follow each other in stage order.
// S = N_pad / 16 stages.  Every 16-sample K step of the Gram then reads two
// contiguous 16 KiB blocks instead of 256 scattered 128-B column pieces.
__host__ __device__ __forceinline__ int64_t tiled_off(int64_t S, int64_t n, int64_t j) {
  return (((j >> 7) * S + (n >> 4)) * 128 + (j & 127)) * 16 + (n & 15);
}
__host__ __device__ __forceinline__ int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

}  // namespace scs
