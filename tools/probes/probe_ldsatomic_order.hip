// probe_ldsatomic_order: in which order does ONE ds_add_f64 instruction apply the lanes that hit the
// same LDS address?  Lane l adds x_l chosen so that the rounded fp64 sum depends on the order
// (a big value, then small ones that vanish or survive depending on when the big one cancels).
// Compares the result against host sums in ascending and descending lane order, for several
// active-lane patterns (the lower half / upper half split a paired walk would rely on).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__global__ void order_kernel(const double* __restrict__ x, const unsigned long long* __restrict__ mask, int ncase,
                             double* __restrict__ out) {
  __shared__ double acc[64];
  const int lane = threadIdx.x;
  for (int c = 0; c < ncase; ++c) {
    acc[lane] = 0.0;
    __syncthreads();
    const bool on = (mask[c] >> lane) & 1ull;
    if (on) atomicAdd(&acc[0], x[c * 64 + lane]);
    __syncthreads();
    if (lane == 0) out[c] = acc[0];
    __syncthreads();
  }
}

int main() {
  const int ncase = 64;
  std::vector<double> hx(ncase * 64);
  std::vector<unsigned long long> hm(ncase);
  srand(7);
  for (int c = 0; c < ncase; ++c) {
    // active lanes: two random lanes per half at least, the rest random
    unsigned long long m = 0;
    for (int l = 0; l < 64; ++l)
      if (rand() % 3 == 0) m |= 1ull << l;
    m |= 1ull << (rand() % 32);
    m |= 1ull << (32 + rand() % 32);
    hm[c] = m;
    for (int l = 0; l < 64; ++l) {
      const int r = rand() % 4;
      hx[c * 64 + l] = r == 0 ? 1e16 : r == 1 ? -1e16 : (rand() % 7 + 1) * 0.75;
    }
  }
  double *dx, *dout;
  unsigned long long* dm;
  CK(hipMalloc(&dx, hx.size() * 8));
  CK(hipMalloc(&dm, hm.size() * 8));
  CK(hipMalloc(&dout, ncase * 8));
  CK(hipMemcpy(dx, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dm, hm.data(), hm.size() * 8, hipMemcpyHostToDevice));
  int asc = 0, desc = 0, both = 0, neither = 0;
  for (int rep = 0; rep < 20; ++rep) {
    hipLaunchKernelGGL(order_kernel, dim3(1), dim3(64), 0, 0, dx, dm, ncase, dout);
    std::vector<double> ho(ncase);
    CK(hipMemcpy(ho.data(), dout, ncase * 8, hipMemcpyDeviceToHost));
    for (int c = 0; c < ncase; ++c) {
      double sa = 0.0, sd = 0.0;
      for (int l = 0; l < 64; ++l)
        if ((hm[c] >> l) & 1ull) sa += hx[c * 64 + l];
      for (int l = 63; l >= 0; --l)
        if ((hm[c] >> l) & 1ull) sd += hx[c * 64 + l];
      const bool a = ho[c] == sa, d = ho[c] == sd;
      if (a && d) ++both;
      else if (a) ++asc;
      else if (d) ++desc;
      else ++neither;
    }
  }
  printf("cases x reps: ascending-lane order only %d, descending only %d, either (order-free) %d, neither %d\n", asc,
         desc, both, neither);
  return 0;
}
