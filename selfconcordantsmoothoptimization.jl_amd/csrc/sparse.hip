// Sparse A (BASELINE configs[4]: box-constrained least squares, ρ = 0.01,
// ProxLQNSCORE).  A is held twice: CSR (rows; z = A x) and CSC (columns;
// g = Aᵀ v), the "CSR + CSC copy" layout of SURVEY.md §8d C5.  Values are fp64
// or fp32 (the fp32-vs-fp64 study); accumulation is always fp64.
//
//   spmv_csr : one wave per row, lanes stride the row's nonzeros (coalesced
//              value/index loads, x gathered from L2), fixed-order wave sum.
//   spmv_csc : the same per column.
// Both are HBM-bound: bytes per pass = nnz * (sizeof(val) + 4) + vectors.
//
// Synthetic pattern (scs_gen_sparse): k = round(ρ m) "layers"; layer s maps
// row i to column ((a_s i + b_s) mod N) mod m with a_s odd, a bijection of
// [0, N) when N is a power of two and m | N.  Every row then has exactly k
// nonzeros and every column exactly k N / m, so both the CSR and the CSC
// arrays are written in place from closed forms (no sort); the value of
// (i, s) is a counter-RNG normal, identical in both copies.
#include "common.h"
#include "kernels.h"

namespace scs {

template <typename VT>
__global__ __launch_bounds__(256) void spmv_kernel(const int64_t* __restrict__ ptr, const int* __restrict__ idx,
                                                   const VT* __restrict__ val, const double* __restrict__ x,
                                                   int64_t nrows, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const int64_t p0 = ptr[row], p1 = ptr[row + 1];
  double acc = 0.0;
  for (int64_t p = p0 + lane; p < p1; p += 64) acc += (double)val[p] * x[idx[p]];
  acc = wave_sum(acc);
  if (lane == 0) out[row] = acc;
}

hipError_t launch_spmv(const int64_t* ptr, const int* idx, const void* val, int f32, const double* x, int64_t nrows,
                       double* out, hipStream_t st) {
  const unsigned grid = (unsigned)ceil_div(nrows, 4);
  if (f32)
    hipLaunchKernelGGL(spmv_kernel<float>, dim3(grid), dim3(256), 0, st, ptr, idx, (const float*)val, x, nrows, out);
  else
    hipLaunchKernelGGL(spmv_kernel<double>, dim3(grid), dim3(256), 0, st, ptr, idx, (const double*)val, x, nrows,
                       out);
  return hipGetLastError();
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
