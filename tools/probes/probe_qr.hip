// probe_qr: the reference-solver Householder QR solve (qr.hip) in isolation, with -DQR_PROF the
// cooperative panel's per-column phases (workgroup 0: sweep | reflector + v | rows | B2 | publish),
// summed over every column.  PROBE_SIZES=2048,8192 (orders); SCS_QR_COOP=0 the per-column launches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "common.h"
#include "kernels.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

#ifdef QR_PROF
#include "qr.hip"   // (the profiled build: qr_prof is a device variable of this translation unit)
#endif

__global__ void rnd_fill(double* A, int64_t n, int64_t ld) {   // uniform(-0.5, 0.5) by a counter hash, + n on the diagonal
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n * n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / n, j = e % n;
    const uint64_t h = (uint64_t)(e + 1) * 0x9E3779B97F4A7C15ull;
    A[j * ld + i] = (double)((h >> 11) & 0xFFFFF) / 1048576.0 - 0.5 + (i == j ? 4.0 : 0.0);
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
    double *A, *A0, *b, *b0;
    CK(hipMalloc(&A, np * np * 8)); CK(hipMalloc(&A0, np * np * 8));
    CK(hipMalloc(&b, np * 8)); CK(hipMalloc(&b0, np * 8));
    CK(hipMemset(A0, 0, np * np * 8));
    rnd_fill<<<4096, 256>>>(A0, n, np);
    std::vector<double> hb(np, 0.0);
    for (int64_t i = 0; i < n; ++i) hb[i] = 1.0 + 0.001 * (double)(i % 97);
    CK(hipMemcpy(b0, hb.data(), np * 8, hipMemcpyHostToDevice));
    CK(scs::qr_prepare(A0, np, n, np, st));
    scs::QRAux aux;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemcpyAsync(A, A0, np * np * 8, hipMemcpyDeviceToDevice, st));
      CK(hipMemcpyAsync(b, b0, np * 8, hipMemcpyDeviceToDevice, st));
      CK(scs::qr_aux_init(&aux, np, st));
      CK(hipStreamSynchronize(st));
#ifdef QR_PROF
      unsigned long long z[32] = {0};
      CK(hipMemcpyToSymbol(HIP_SYMBOL(scs::qr_prof), z, sizeof(z)));
#endif
      CK(hipEventRecord(e0, st));
      CK(scs::qr_solve(A, np, np, &aux, b, st));
      CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      int ci = 0; CK(hipMemcpy(&ci, aux.cinfo, 4, hipMemcpyDeviceToHost));
      std::vector<double> x(np);
      CK(hipMemcpy(x.data(), b, np * 8, hipMemcpyDeviceToHost));
      double cs = 0; for (double v : x) cs += v;
      printf("n=%ld qr_solve: %.2f ms (coop info %d, refused %ld) sum(x) %.17g\n", (long)n, ms, ci, (long)aux.coop_refused, cs);
#ifdef QR_PROF
      unsigned long long p[32];
      CK(hipMemcpyFromSymbol(p, HIP_SYMBOL(scs::qr_prof), sizeof(p)));
      const double nc = (double)p[5];
      if (nc > 0)
        printf("  per column (us, %ld columns): sweep %.2f  reflector+v %.2f  rows %.2f  B2 %.2f  publish %.2f  "
               "(last wave's rows %.2f)\n",
               (long)p[5], p[0] / nc / 100.0, p[1] / nc / 100.0, p[2] / nc / 100.0, p[3] / nc / 100.0, p[4] / nc / 100.0,
               p[6] / nc / 100.0);
      if (nc > 0) {
        printf("  per wave (us): column pass");
        for (int w = 0; w < 16; ++w) if (p[8 + w]) printf(" %.2f", p[8 + w] / nc / 100.0);
        printf(" | owner writes");
        for (int w = 0; w < 16; ++w) if (p[16 + w]) printf(" %.2f", p[16 + w] / nc / 100.0);
        printf("\n");
      }
#endif
    }
    CK(hipFree(A)); CK(hipFree(A0)); CK(hipFree(b)); CK(hipFree(b0));
    scs::qr_aux_free(&aux);
  }
  return 0;
}
