// probe_chol: timing of the blocked Cholesky pieces (chol.hip) in isolation.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "common.h"
#include "kernels.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

namespace scs {
hipError_t launch_chol_diag(double* G, int64_t ld, int k, double* W, int* info, hipStream_t st);
#ifdef CHOL_PROF
extern __device__ long long chol_prof[128];
#endif
#ifdef CHOL_DTIME
extern __device__ long long chol_dtime[2 * 1024];
#endif
}

__global__ void spd_fill(double* G, int64_t n) {   // G = I*n + small symmetric noise (upper valid)
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n * n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e / n, r = e % n;
    const uint64_t h = (uint64_t)(r < c ? r * 1315423911ull + c : c * 1315423911ull + r) * 0x9E3779B97F4A7C15ull;
    G[e] = (r == c) ? (double)n : ((double)((h >> 11) & 0xFFFF) / 65536.0 - 0.5);
  }
}

__global__ void rowsum(const double* G, int64_t n, double* b) {   // b = G * ones (G symmetric, full)
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int64_t j = 0; j < n; ++j) s += G[j * n + i];
  b[i] = s;
}

// order-independent checksum of the bits of the upper triangle of G (n x n) and of W (n x 128): a
// wrapping sum of the 64-bit patterns, to compare factor variants bit for bit
__global__ void bitsum(const double* G, int64_t n, const double* W, unsigned long long* out) {
  unsigned long long s = 0, t = 0;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n * n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e / n, r = e % n;
    if (r <= c) s += __double_as_longlong(G[e]) * (unsigned long long)(e + 1);
    if (e < n * 128) t += __double_as_longlong(W[e]) * (unsigned long long)(e + 1);
  }
  atomicAdd(out, s);
  atomicAdd(out + 1, t);
}

int main(int argc, char** argv) {
  // the library's context stream is non-blocking: the factor's (CU-masked, blocking) bulk stream
  // would serialize with the legacy null stream
  hipStream_t sq;
  CK(hipStreamCreateWithFlags(&sq, hipStreamNonBlocking));
  // PROBE_SIZES: comma-separated m values (multiples of 128), default 8192,16384
  std::vector<int64_t> sizes;
  {
    const char* ps = getenv("PROBE_SIZES");
    const char* q = ps ? ps : "8192,16384";
    while (*q) {
      char* end;
      const long v = strtol(q, &end, 10);
      if (end == q) break;
      sizes.push_back(v);
      q = *end ? end + 1 : end;
    }
  }
  for (int64_t n : sizes) {
    double *G, *G0, *W, *b, *y;
    int* info;
    CK(hipMalloc(&G, n * n * 8)); CK(hipMalloc(&G0, n * n * 8)); CK(hipMalloc(&W, n * 128 * 8));
    CK(hipMalloc(&b, n * 8)); CK(hipMalloc(&y, n * 8)); CK(hipMalloc(&info, 4));
    spd_fill<<<4096, 256>>>(G0, n);
    const int nb = (int)(n / 128);
    std::vector<int2> rl(nb), tr((size_t)nb * (nb + 1) / 2);
    for (int j = 0; j < nb; ++j) rl[j] = make_int2(0, j);
    scs::gram_tile_list_rowmajor(nb, tr.data());
    int2 *drl, *dtr; double* wpm;
    CK(hipMalloc(&drl, nb * 8)); CK(hipMalloc(&dtr, tr.size() * 8)); CK(hipMalloc(&wpm, 256 * 8));
    CK(hipMemcpy(drl, rl.data(), nb * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtr, tr.data(), tr.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> hw(256); for (int i = 0; i < 256; ++i) hw[i] = i < 128 ? 1.0 : -1.0;
    CK(hipMemcpy(wpm, hw.data(), 256 * 8, hipMemcpyHostToDevice));
    scs::CholAux aux;
    CK(scs::chol_aux_init(&aux, n, sq));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); float ms;
    // diag kernel alone, 64 launches on distinct blocks of a fresh copy
    CK(hipMemcpy(G, G0, n * n * 8, hipMemcpyDeviceToDevice));
    CK(hipMemset(info, 0, 4));
    CK(hipEventRecord(e0));
    for (int k = 0; k < 64; ++k) CK(scs::launch_chol_diag(G, n, k, W, info, 0));
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("n=%ld diag kernel: %.1f us/launch\n", (long)n, ms * 1000 / 64);
#ifdef CHOL_PROF
    {
      long long hp[128];
      CK(hipMemcpyFromSymbol(hp, HIP_SYMBOL(scs::chol_prof), sizeof(hp)));
      // s_memtime runs at the 100 MHz constant clock on gfx950
      printf("phase times (k=0 launch, us): ");
      for (int kb = 0; kb < 8; ++kb) {
        const long long a0 = hp[1 + 4 * kb], a1 = hp[2 + 4 * kb], a2 = hp[3 + 4 * kb];
        const long long a3 = (kb < 7) ? hp[1 + 4 * (kb + 1)] : hp[33];
        printf("[kb%d A %.2f B %.2f C %.2f] ", kb, (a1 - a0) / 100.0, kb < 7 ? (a2 - a1) / 100.0 : 0.0,
               kb < 7 ? (a3 - a2) / 100.0 : 0.0);
      }
      printf("\n  C detail (us from C start): ");
      for (int kb = 0; kb < 7; ++kb) {
        const long long c0 = hp[3 + 4 * kb];
        printf("[kb%d w0 tile %.2f fac %.2f | inv %.2f | w1 %.2f w2 %.2f w3 %.2f] ", kb, (hp[36 + kb] - c0) / 100.0,
               (hp[43 + kb] - c0) / 100.0, (hp[50 + kb] - c0) / 100.0, (hp[57 + 3 * kb] - c0) / 100.0,
               (hp[58 + 3 * kb] - c0) / 100.0, (hp[59 + 3 * kb] - c0) / 100.0);
      }
      printf("\n  load %.2f  factor %.2f  storeU+diaginv %.2f  doubling+storeW %.2f  total %.2f\n", (hp[1] - hp[0]) / 100.0,
             (hp[33] - hp[1]) / 100.0, (hp[34] - hp[33]) / 100.0, (hp[35] - hp[34]) / 100.0,
             (hp[35] - hp[0]) / 100.0);
    }
#endif
    // full factorization + solve
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemcpy(G, G0, n * n * 8, hipMemcpyDeviceToDevice));
      CK(hipMemset(info, 0, 4));
      // a device-to-device hipMemcpy may return before it completes, and sq is non-blocking: without
      // this the factor's launches overtook the copy's tail at n = 16384 (stale trailing columns)
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, sq));
      CK(scs::chol_factor(G, n, n, n, W, &aux, dtr, info, sq));
      CK(hipEventRecord(e1, sq)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      int hinfo; CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
      printf("n=%ld factor: %.2f ms (info %d)\n", (long)n, ms, hinfo);
#ifdef CHOL_DTIME
      {   // the diagonal kernels' in-kernel time (entry -> exit of wave 0), and the gap from one's exit
          // to the next one's entry (the rest of the chain between them)
        std::vector<long long> dt(2 * 1024);
        CK(hipMemcpyFromSymbol(dt.data(), HIP_SYMBOL(scs::chol_dtime), sizeof(long long) * 2 * 1024));
        double run = 0, gap = 0, rmax = 0;
        for (int k = 0; k < nb; ++k) {
          const double r = (dt[2 * k + 1] - dt[2 * k]) / 100.0;
          run += r;
          rmax = r > rmax ? r : rmax;
          if (k > 0) gap += (dt[2 * k] - dt[2 * k - 1]) / 100.0;
        }
        printf("n=%ld diag in-kernel: avg %.1f us, max %.1f us; exit->next entry avg %.1f us (%d blocks)\n", (long)n,
               run / nb, rmax, gap / (nb - 1), nb);
      }
#endif
      if (rep == 0) {
        unsigned long long* dsum;
        unsigned long long hs[2];
        CK(hipMalloc(&dsum, 16));
        CK(hipMemsetAsync(dsum, 0, 16, sq));
        hipLaunchKernelGGL(bitsum, dim3(2048), dim3(256), 0, sq, G, n, W, dsum);
        CK(hipMemcpyAsync(hs, dsum, 16, hipMemcpyDeviceToHost, sq));
        CK(hipStreamSynchronize(sq));
        CK(hipFree(dsum));
        printf("n=%ld bits U %016llx W %016llx\n", (long)n, hs[0], hs[1]);
      }
      hipLaunchKernelGGL(rowsum, dim3((unsigned)(n / 256)), dim3(256), 0, sq, G0, n, b);
      CK(hipEventRecord(e0, sq));
      CK(scs::chol_solve(G, n, n, W, b, y, &aux, sq));
      CK(hipEventRecord(e1, sq)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<double> hx(n);
      CK(hipMemcpy(hx.data(), b, n * 8, hipMemcpyDeviceToHost));
      double err = 0.0;
      for (int64_t i = 0; i < n; ++i) err = fmax(err, fabs(hx[i] - 1.0));
      printf("n=%ld solve: %.2f ms  max|x-1| = %.3e\n", (long)n, ms, err);
    }
    CK(hipFree(G)); CK(hipFree(G0)); CK(hipFree(W)); CK(hipFree(b)); CK(hipFree(y)); CK(hipFree(info));
    CK(hipFree(drl)); CK(hipFree(dtr)); CK(hipFree(wpm));
    scs::chol_aux_free(&aux);
  }
  return 0;
}
