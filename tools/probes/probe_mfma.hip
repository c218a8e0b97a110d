// probe_mfma: measures the facts the Gram kernel is designed around.
//  (1) the C/D lane->element map of v_mfma_f64_16x16x4_f64 (asymmetric
//      integer operands, checked against the map used in gram.hip);
//  (2) back-to-back v_mfma_f64_16x16x4_f64 throughput per SIMD and the
//      chip-wide fp64 MFMA peak (random operands, all CUs busy);
//  (3) the v_fma_f64 VALU peak for comparison;
//  (4) a streaming-copy HBM bandwidth reference.
// Built as a standalone executable (make probe); not part of libscsopt.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

typedef double v4d __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__global__ void layout_kernel(const double* a, const double* b, double* out) {
  const int l = threadIdx.x;
  v4d acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[l], b[l], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

template <int NACC>
__global__ __launch_bounds__(256) void mfma_rate_kernel(const double* seed, double* out, int iters) {
  const int l = threadIdx.x;
  double a = seed[l & 63] + blockIdx.x * 1e-9, b = seed[(l + 7) & 63] - blockIdx.x * 1e-9;
  v4d acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (v4d){a, b, a * b, a + b};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + l] = s;
}

__global__ __launch_bounds__(256) void valu_rate_kernel(const double* seed, double* out, int iters) {
  const int l = threadIdx.x;
  double a = seed[l & 63], b = seed[(l + 3) & 63];
  double c0 = a, c1 = b, c2 = a + 1, c3 = b + 1, c4 = a * 2, c5 = b * 2, c6 = a - 1, c7 = b - 1;
  for (int it = 0; it < iters; ++it) {
    c0 = fma(c0, a, b); c1 = fma(c1, a, b); c2 = fma(c2, a, b); c3 = fma(c3, a, b);
    c4 = fma(c4, a, b); c5 = fma(c5, a, b); c6 = fma(c6, a, b); c7 = fma(c7, a, b);
  }
  out[blockIdx.x * blockDim.x + l] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

__global__ void copy_kernel(const double4* __restrict__ in, double4* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = in[i];
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  printf("device %s  CUs %d  clock %d kHz  arch %s\n", prop.name, prop.multiProcessorCount, prop.clockRate,
         prop.gcnArchName);
  // ---- (1) layout
  std::vector<double> ha(64), hb(64), hout(256);
  // A[i][k] = i + 100 k (lane l: i = l&15, k = l>>4); B[k][j] = 1000*k + 10000*j ... use exact ints
  for (int l = 0; l < 64; ++l) {
    int i = l & 15, k = l >> 4;
    ha[l] = (k == 0) ? (double)(i + 1) : 0.0;        // A[:,0] = i+1, other k zero
    hb[l] = (k == 0) ? (double)(100 * (i + 1)) : 0.0;  // B[0][j] = 100 (j+1)
  }
  double *da, *db, *dout;
  CK(hipMalloc(&da, 64 * 8)); CK(hipMalloc(&db, 64 * 8)); CK(hipMalloc(&dout, 256 * 8));
  CK(hipMemcpy(da, ha.data(), 64 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hb.data(), 64 * 8, hipMemcpyHostToDevice));
  layout_kernel<<<1, 64>>>(da, db, dout);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hout.data(), dout, 256 * 8, hipMemcpyDeviceToHost));
  // D[i][j] = (i+1)*100*(j+1)
  int ok_map_a = 1, ok_map_b = 1;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      double v = hout[l * 4 + r];
      int col = l & 15;
      int rowA = (l >> 4) + 4 * r;   // map used by gram.hip
      int rowB = 4 * (l >> 4) + r;   // the f32 16x16 map
      if (v != (double)(rowA + 1) * 100.0 * (col + 1)) ok_map_a = 0;
      if (v != (double)(rowB + 1) * 100.0 * (col + 1)) ok_map_b = 0;
    }
  printf("LAYOUT f64 16x16x4: row=(lane>>4)+4*r %s ; row=4*(lane>>4)+r %s\n", ok_map_a ? "MATCH" : "no",
         ok_map_b ? "MATCH" : "no");

  // ---- (2) MFMA rate
  std::vector<double> seed(64);
  for (int i = 0; i < 64; ++i) seed[i] = 0.5 + 0.001 * i;
  double* dseed; CK(hipMalloc(&dseed, 64 * 8));
  CK(hipMemcpy(dseed, seed.data(), 64 * 8, hipMemcpyHostToDevice));
  const int nblk = prop.multiProcessorCount * 4;  // 4 x 256-thread blocks per CU = 4 waves/SIMD
  double* dbig; CK(hipMalloc(&dbig, (size_t)nblk * 256 * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; ++rep) {
    const int iters = 4000;
    mfma_rate_kernel<8><<<nblk, 256>>>(dseed, dbig, 100);
    CK(hipEventRecord(e0));
    mfma_rate_kernel<8><<<nblk, 256>>>(dseed, dbig, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double flops = (double)nblk * 4 /*waves*/ * iters * 8 * (16.0 * 16 * 4 * 2);
    printf("MFMA f64 16x16x4 (8 acc, 4 waves/SIMD): %.2f ms  %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  {
    // one wave per SIMD, 1 block of 256 per CU
    const int iters = 4000;
    const int nb1 = prop.multiProcessorCount;
    mfma_rate_kernel<8><<<nb1, 256>>>(dseed, dbig, 100);
    CK(hipEventRecord(e0));
    mfma_rate_kernel<8><<<nb1, 256>>>(dseed, dbig, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double flops = (double)nb1 * 4 * iters * 8 * (16.0 * 16 * 4 * 2);
    double cyc_per = (ms * 1e-3) * (prop.clockRate * 1e3) / ((double)iters * 8);
    printf("MFMA f64 1 wave/SIMD: %.2f TFLOP/s  ~%.1f cycles/MFMA at nominal clock\n", flops / ms / 1e9, cyc_per);
  }
  {
    const int iters = 4000;
    const int nb1 = prop.multiProcessorCount;
    mfma_rate_kernel<1><<<nb1, 256>>>(dseed, dbig, 100);
    CK(hipEventRecord(e0));
    mfma_rate_kernel<1><<<nb1, 256>>>(dseed, dbig, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double cyc_per = (ms * 1e-3) * (prop.clockRate * 1e3) / ((double)iters);
    printf("MFMA f64 dependent chain: ~%.1f cycles/MFMA latency at nominal clock\n", cyc_per);
  }
  // ---- (3) VALU fp64
  {
    const int iters = 20000;
    valu_rate_kernel<<<nblk, 256>>>(dseed, dbig, 100);
    CK(hipEventRecord(e0));
    valu_rate_kernel<<<nblk, 256>>>(dseed, dbig, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double flops = (double)nblk * 256 * iters * 8 * 2.0;
    printf("VALU v_fma_f64: %.2f TFLOP/s\n", flops / ms / 1e9);
  }
  // ---- (4) copy bandwidth
  {
    size_t bytes = (size_t)4 << 30;
    size_t n4 = bytes / 32;
    double4 *s, *d;
    CK(hipMalloc(&s, bytes)); CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 0, bytes));
    copy_kernel<<<4096, 256>>>(s, d, n4);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) copy_kernel<<<4096, 256>>>(s, d, n4);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("copy 4 GiB: %.2f TB/s (read+write)\n", 5.0 * 2 * bytes / (ms * 1e-3) / 1e12);
    CK(hipFree(s)); CK(hipFree(d));
  }
  return 0;
}
