// probe_gram: standalone correctness + speed check of gram.hip (no library).
//   probe_gram            -> small-size exactness check vs a CPU fp64 loop, then timing
//   probe_gram N m reps   -> timing only at N x m
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include "common.h"

namespace scs {
void gram_tile_list(int nb, int2* out, int* ntiles);
void gram_tile_list_tall(int nb, int2* out, int* ntiles);
hipError_t gram_launch(const double* A, int64_t S, const double* w, int64_t Nk, const int2* tiles, int ntiles,
                       double* G, int64_t ldg, int packed, int tall, hipStream_t st, const double* v = nullptr,
                       double* VP = nullptr, int64_t vps = 0);
hipError_t gram_launch_ex(const double* A, int64_t lda, const double* w, int64_t k0, int64_t k1, const int2* tiles,
                          int ntiles, double* G, int64_t ldg, int accumulate, int noload, hipStream_t st);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__device__ inline uint64_t smix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void fill_kernel(double* p, size_t n, uint64_t seed, double scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t h = smix(seed ^ (i * 0x632BE59BD9B4E019ull));
    p[i] = scale * (((double)(h >> 11) + 0.5) * (1.0 / 9007199254740992.0) - 0.5);
  }
}

static int run(int64_t N, int64_t m, int reps, bool check, int tall) {
  const int64_t lda = N;
  double *A, *w, *G;
  CK(hipMalloc(&A, (size_t)lda * m * 8));
  CK(hipMalloc(&w, (size_t)N * 8));
  CK(hipMalloc(&G, (size_t)m * m * 8));
  fill_kernel<<<4096, 256>>>(A, (size_t)lda * m, 1234, 2.0);
  fill_kernel<<<256, 256>>>(w, (size_t)N, 99, 1.0);
  CK(hipMemset(G, 0, (size_t)m * m * 8));
  const int nb = (int)(m / 128);
  std::vector<int2> tl((size_t)nb * (nb + 1) / 2 + nb);
  int nt = 0;
  if (tall) scs::gram_tile_list_tall(nb, tl.data(), &nt);
  else scs::gram_tile_list(nb, tl.data(), &nt);
  int2* dtl;
  CK(hipMalloc(&dtl, nt * sizeof(int2)));
  CK(hipMemcpy(dtl, tl.data(), nt * sizeof(int2), hipMemcpyHostToDevice));
  // gram_launch reads the panel-blocked layout (S = N/16 stages); the fill is layout-agnostic
  CK(scs::gram_launch(A, N / 16, w, N, dtl, nt, G, m, 0, tall, 0));
  CK(hipDeviceSynchronize());
  if (check) {
    std::vector<double> hA((size_t)lda * m), hw(N), hG((size_t)m * m);
    CK(hipMemcpy(hA.data(), A, hA.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hw.data(), w, hw.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hG.data(), G, hG.size() * 8, hipMemcpyDeviceToHost));
    double maxrel = 0;
    for (int64_t j = 0; j < m; ++j)
      for (int64_t i = j; i < m; ++i) {
        double s = 0, sa = 0;
        for (int64_t n = 0; n < N; ++n) {
          double t = hA[scs::tiled_off(N / 16, n, i)] * hw[n] * hA[scs::tiled_off(N / 16, n, j)];
          s += t; sa += fabs(t);
        }
        double e = fabs(hG[i * m + j] - s) / (sa > 0 ? sa : 1);  // upper triangle: (row j, col i)
        if (e > maxrel) maxrel = e;
      }
    printf("CHECK tall=%d N=%ld m=%ld max |G-ref|/sum|terms| = %.3e  %s\n", tall, (long)N, (long)m, maxrel,
           maxrel < 1e-14 ? "PASS" : "FAIL");
    if (tall) {   // gram_launch runs the pipelined variant: same MFMA order as the plain loop -> bitwise identical
      double* G2;
      CK(hipMalloc(&G2, (size_t)m * m * 8));
      CK(hipMemcpy(G2, G, (size_t)m * m * 8, hipMemcpyDeviceToDevice));
      CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G2, m, 0, 5, 0));   // plain LDS-DMA loop
      std::vector<double> hG2((size_t)m * m);
      CK(hipMemcpy(hG2.data(), G2, hG2.size() * 8, hipMemcpyDeviceToHost));
      size_t ndiff = 0;
      for (size_t e = 0; e < hG2.size(); ++e) ndiff += hG2[e] != hG[e];
      printf("CHECK pipe N=%ld m=%ld bitwise diffs vs plain: %zu  %s\n", (long)N, (long)m, ndiff, ndiff ? "FAIL" : "PASS");
      CK(hipFree(G2));
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  if (getenv("GRAM_ONLY")) {   // one launch of one experiment kernel (for rocprofv3 --pmc passes)
    if (tall) return 0;
    CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, atoi(getenv("GRAM_ONLY")), 0));
    CK(hipDeviceSynchronize());
    return 0;
  }
  if (getenv("GRAM_SIA") && tall) {
    // 256 x 128 interleaved kernel (16; 17 = no-load build) vs the LDS-DMA pipelined kernel (7)
    const double alg0 = (double)N * m * (m + 1);
    std::vector<double> ref((size_t)m * m), got((size_t)m * m);
    CK(hipMemset(G, 0, (size_t)m * m * 8));
    CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, 7, 0));
    CK(hipMemcpy(ref.data(), G, ref.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemset(G, 0, (size_t)m * m * 8));
    CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, 16, 0));
    CK(hipMemcpy(got.data(), G, got.size() * 8, hipMemcpyDeviceToHost));
    size_t nd = 0;
    for (size_t e = 0; e < got.size(); ++e) nd += got[e] != ref[e];
    printf("CHECK sia-tall N=%ld m=%ld bitwise diffs vs glds pipe: %zu  %s\n", (long)N, (long)m, nd, nd ? "FAIL" : "PASS");
    for (int v : {7, 16, 17}) {
      float t;
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, v, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t, e0, e1));
      t /= reps;
      printf("SIA-TALL kernel %d N=%ld m=%ld: %.3f ms  %.2f TF/s\n", v, (long)N, (long)m, t, alg0 / t / 1e9);
    }
  }
  if (getenv("GRAM_SIA") && !tall) {
    // interleaved-schedule kernel (9: sched_group_barrier patterns, 10: compiler schedule) vs the
    // register-staged 128 x 128 kernel on the same panel-blocked A (11): bitwise, then timing
    const double alg0 = (double)N * m * (m + 1);
    std::vector<double> ref((size_t)m * m), got((size_t)m * m);
    CK(hipMemset(G, 0, (size_t)m * m * 8));
    CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, 11, 0));
    CK(hipMemcpy(ref.data(), G, ref.size() * 8, hipMemcpyDeviceToHost));
    for (int v : {9, 10}) {
      CK(hipMemset(G, 0, (size_t)m * m * 8));
      CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, v, 0));
      CK(hipMemcpy(got.data(), G, got.size() * 8, hipMemcpyDeviceToHost));
      size_t nd = 0;
      for (size_t e = 0; e < got.size(); ++e) nd += got[e] != ref[e];
      printf("CHECK sia%d N=%ld m=%ld bitwise diffs vs register kernel: %zu  %s\n", v, (long)N, (long)m, nd,
             nd ? "FAIL" : "PASS");
    }
    for (int v : {9, 12}) {
      float t;
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, v, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t, e0, e1));
      t /= reps;
      printf("SIA kernel %d N=%ld m=%ld: %.3f ms  %.2f TF/s\n", v, (long)N, (long)m, t, alg0 / t / 1e9);
    }
  }
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) CK(scs::gram_launch(A, N / 16, w, N, dtl, nt, G, m, 0, tall, 0));
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double alg = (double)N * m * (m + 1);   // symmetric Gram, algorithmic
  if (getenv("GRAM_EXPERIMENTS") && tall) {
    CK(hipEventRecord(e0));
    CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, 4, 0));
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float t; CK(hipEventElapsedTime(&t, e0, e1));
    printf("EXP tall noload: %.3f ms  %.2f TF/s\n", t, alg / t / 1e9);
    for (int v : {5, 7, 8, 5, 7}) {   // glds panel-blocked: plain loop / pipelined fragments / pipelined no-load
      CK(hipEventRecord(e0));
      CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, v, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t, e0, e1));
      printf("EXP %s: %.3f ms  %.2f TF/s\n", v == 5 ? "glds tiled-A" : v == 7 ? "glds pipe" : "glds pipe noload", t,
             alg / t / 1e9);
    }
  } else if (getenv("GRAM_EXPERIMENTS")) {
    // (a) operands held in registers after the first stage: compute + LDS + barrier ceiling
    CK(hipEventRecord(e0));
    CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, nt, G, m, 0, 1, 0));
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float t; CK(hipEventElapsedTime(&t, e0, e1));
    printf("EXP noload: %.3f ms  %.2f TF/s\n", t, alg / t / 1e9);
    // (c) only the first 512*floor(nt/512) tiles: whole rounds, no partial tail round
    {
      const int ntr = (nt / 512) * 512;
      CK(hipEventRecord(e0));
      CK(scs::gram_launch_ex(A, lda, w, 0, N, dtl, ntr, G, m, 0, 0, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t, e0, e1));
      printf("EXP whole-rounds %d tiles: %.3f ms  %.2f TF/s (per-tile rate)\n", ntr, t,
             alg * ntr / nt / t / 1e9);
    }
    // (b) K split into chunks of 2^k samples, one launch per chunk, accumulating
    for (int64_t kc : {(int64_t)1 << 17, (int64_t)1 << 15, (int64_t)1 << 13}) {
      if (kc >= N) continue;
      CK(hipEventRecord(e0));
      for (int64_t k0 = 0; k0 < N; k0 += kc)
        CK(scs::gram_launch_ex(A, lda, w, k0, k0 + kc < N ? k0 + kc : N, dtl, nt, G, m, k0 > 0, 0, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t, e0, e1));
      printf("EXP kchunk %ld: %.3f ms  %.2f TF/s\n", (long)kc, t, alg / t / 1e9);
    }
  }
  double exe = 2.0 * N * (tall ? 256.0 : 128.0) * 128.0 * nt;  // executed incl. full diagonal tiles
  printf("GRAM tall=%d N=%ld m=%ld tiles=%d: %.3f ms/launch  alg %.2f TF/s  exec %.2f TF/s\n", tall, (long)N, (long)m,
         nt, ms,
         alg / ms / 1e9, exe / ms / 1e9);
  CK(hipFree(A)); CK(hipFree(w)); CK(hipFree(G)); CK(hipFree(dtl));
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3) {
    run(atoll(argv[1]), atoll(argv[2]), argc > 3 ? atoi(argv[3]) : 3, false, 0);
    return run(atoll(argv[1]), atoll(argv[2]), argc > 3 ? atoi(argv[3]) : 3, false, 1);
  }
  for (int tall = 0; tall < 2; ++tall) {
    run(48, 256, 1, true, tall);
    if (!tall) run(1024, 384, 1, true, tall);
    run(4096, 1024, 1, true, tall);
    run(1 << 17, 8192, 3, false, tall);
    run(1 << 17, 16384, 2, false, tall);
  }
  return 0;
}
