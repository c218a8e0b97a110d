// probe_lu: the blocked LU (lu.hip) factor in isolation, with -DLU_PROF the cooperative panel's per-column
// phases (workgroup 0: sweep | pick + stage | barrier | update | publish), summed over every column.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "common.h"
#include "kernels.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

namespace scs {
#ifdef LU_PROF
extern __device__ unsigned long long lu_prof[8];
#endif
}

__global__ void rnd_fill(double* A, int64_t n, int64_t ld) {   // uniform(-0.5, 0.5) by a counter hash
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n * n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / n, j = e % n;
    const uint64_t h = (uint64_t)(e + 1) * 0x9E3779B97F4A7C15ull;
    A[i * ld + j] = (double)((h >> 11) & 0xFFFFF) / 1048576.0 - 0.5;
  }
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const char* ps = getenv("PROBE_SIZES");
  std::vector<int64_t> sizes;
  for (const char* q = ps ? ps : "8192"; *q;) {
    char* end;
    const long v = strtol(q, &end, 10);
    if (end == q) break;
    sizes.push_back(v);
    q = *end ? end + 1 : end;
  }
  for (int64_t n : sizes) {
    const int64_t np = (n + 127) / 128 * 128;
    double *A, *A0;
    int* info;
    CK(hipMalloc(&A, np * np * 8)); CK(hipMalloc(&A0, np * np * 8)); CK(hipMalloc(&info, 4));
    CK(hipMemset(A0, 0, np * np * 8));
    rnd_fill<<<4096, 256>>>(A0, n, np);
    scs::LUAux aux;
    CK(scs::lu_aux_init(&aux, np, st));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemcpy(A, A0, np * np * 8, hipMemcpyDeviceToDevice));
      CK(hipMemset(info, 0, 4));
      CK(hipDeviceSynchronize());
#ifdef LU_PROF
      unsigned long long z[8] = {0};
      CK(hipMemcpyToSymbol(HIP_SYMBOL(scs::lu_prof), z, sizeof(z)));
#endif
      CK(hipEventRecord(e0, st));
      CK(scs::lu_factor(A, np, n, np, &aux, info, st));
      CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      int hinfo; CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
      printf("n=%ld lu_factor: %.2f ms (info %d)\n", (long)n, ms, hinfo);
#ifdef LU_PROF
      unsigned long long p[8];
      CK(hipMemcpyFromSymbol(p, HIP_SYMBOL(scs::lu_prof), sizeof(p)));
      const double nc = (double)p[5];
      printf("  per column (us, %ld columns): sweep %.2f  pick+stage %.2f  barrier %.2f  update %.2f  publish %.2f\n",
             (long)p[5], p[0] / nc / 100.0, p[1] / nc / 100.0, p[2] / nc / 100.0, p[3] / nc / 100.0, p[4] / nc / 100.0);
#endif
    }
    CK(hipFree(A)); CK(hipFree(A0)); CK(hipFree(info));
    scs::lu_aux_free(&aux);
  }
  return 0;
}
