// probe_mfma_valu: do the fp64 matrix pipe and the fp64 VALU run concurrently on gfx950?
//   One 512-thread workgroup per CU (8 waves: two per SIMD).  Waves 0-3 (one per SIMD) issue back-to-back
//   v_mfma_f64_16x16x4_f64 on NACC independent accumulators, waves 4-7 independent v_fma_f64 chains
//   (NV per lane); MODE 1 = MFMA waves only, 2 = VALU waves only, 3 = both.  No memory traffic.
//   Prints each mode's time and TF/s: if "both" takes ~max(mfma, valu) rather than the sum, the two
//   pipes overlap and a Gram could split its tiles between them.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double v4d __attribute__((ext_vector_type(4)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int NACC = 8, NV = 16;

__global__ __launch_bounds__(512) void mix_kernel(double* out, int mode, int it_m, int it_v, double seed) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w < 4) {
    if (!(mode & 1)) return;
    v4d acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
    const double a = seed + lane * 1e-3, b = seed - lane * 1e-3;
    for (int it = 0; it < it_m; ++it) {
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[(blockIdx.x * 512 + threadIdx.x)] = s;
  } else {
    if (!(mode & 2)) return;
    double x[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) x[i] = seed + i + lane * 1e-3;
    const double a = 0.999999, b = 1e-7 * seed;
    for (int it = 0; it < it_v; ++it) {
#pragma unroll
      for (int i = 0; i < NV; ++i) x[i] = __builtin_fma(x[i], a, b);
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += x[i];
    out[(blockIdx.x * 512 + threadIdx.x)] = s;
  }
}

int main(int argc, char** argv) {
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int it_m = argc > 1 ? atoi(argv[1]) : 100000;
  const int it_v = argc > 2 ? atoi(argv[2]) : 800000;
  const int grid = ncu;
  double* out;
  CK(hipMalloc(&out, sizeof(double) * grid * 512));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double fm = (double)grid * 4 * it_m * NACC * 2048.0;      // MFMA flops
  const double fv = (double)grid * 4 * 64 * (double)it_v * NV * 2.0;   // VALU flops
  for (int rep = 0; rep < 2; ++rep)
    for (int mode : {1, 2, 3}) {
      hipLaunchKernelGGL(mix_kernel, dim3(grid), dim3(512), 0, 0, out, mode, it_m / 10, it_v / 10, 1.0);   // warm
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(mix_kernel, dim3(grid), dim3(512), 0, 0, out, mode, it_m, it_v, 1.0);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double f = (mode & 1 ? fm : 0.0) + (mode & 2 ? fv : 0.0);
      printf("mode %d (%s): %.2f ms, %.1f TF/s (mfma part %.1f, valu part %.1f)\n", mode,
             mode == 1 ? "mfma" : mode == 2 ? "valu" : "both", ms, f / (ms * 1e-3) / 1e12,
             mode & 1 ? fm / (ms * 1e-3) / 1e12 : 0.0, mode & 2 ? fv / (ms * 1e-3) / 1e12 : 0.0);
    }
  return 0;
}
