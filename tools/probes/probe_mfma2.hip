// probe_mfma2: fp64 MFMA issue-rate calibration (no memory traffic).
//   For NACC independent 16x16 accumulators per wave and W waves per SIMD (1..4, set by the
//   grid: 256 threads = 4 waves per workgroup, one per SIMD; W workgroups per CU), run
//   ITERS x NACC v_mfma_f64_16x16x4_f64 and report TF/s.  BAR = 1 adds one s_barrier per
//   NACC MFMAs (the Gram kernels' per-stage barrier), LDS = 1 adds 8 ds_read_b128 per 64
//   MFMAs (the Gram's fragment reads).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double v4d __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);    \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

template <int NACC, int BAR, int LDS>
__global__ __launch_bounds__(256) void mfma_kernel(double* out, int iters, double seed) {
  __shared__ double lds[4096];
  v4d acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
  const int lane = threadIdx.x & 63;
  if (LDS) {
    for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = seed * i;
    __syncthreads();
  }
  v2d a = {seed + lane, seed - lane}, b = {seed * 0.5, seed * 0.25};
  for (int it = 0; it < iters; ++it) {
    if (LDS) {
      v2d r[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) r[q] = *(const v2d*)(lds + ((q * 64 + lane) * 2 + (it & 7)) % 4096);
#pragma unroll
      for (int q = 0; q < 8; ++q) a += r[q] * 1e-300;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc[i], 0, 0, 0);
    if (BAR) __builtin_amdgcn_s_barrier();
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[threadIdx.x] = s;
}

template <int NACC, int BAR, int LDS>
static void run(int wps, int cus, double* out) {
  const int iters = 4096;
  dim3 grid(cus * wps), block(256);
  hipLaunchKernelGGL((mfma_kernel<NACC, BAR, LDS>), grid, block, 0, 0, out, 16, 1.0);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((mfma_kernel<NACC, BAR, LDS>), grid, block, 0, 0, out, iters, 1.0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double flops = 2.0 * 16 * 16 * 4 * (double)NACC * 2 * iters * 4 /*waves per WG*/ * grid.x;
  printf("NACC %2d BAR %d LDS %d waves/SIMD %d: %8.3f ms  %6.2f TF/s\n", NACC, BAR, LDS, wps, ms,
         flops / (ms * 1e-3) / 1e12);
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  printf("CUs %d clock %d kHz\n", cus, p.clockRate);
  double* out;
  CK(hipMalloc(&out, 4096 * sizeof(double)));
  for (int wps = 1; wps <= 4; wps *= 2) {
    run<4, 0, 0>(wps, cus, out);
    run<8, 0, 0>(wps, cus, out);
    run<16, 0, 0>(wps, cus, out);
    run<16, 1, 0>(wps, cus, out);
    run<16, 0, 1>(wps, cus, out);
    run<16, 1, 1>(wps, cus, out);
  }
  run<32, 0, 0>(1, cus, out);
  run<32, 1, 0>(1, cus, out);
  run<32, 0, 0>(2, cus, out);
  return 0;
}
