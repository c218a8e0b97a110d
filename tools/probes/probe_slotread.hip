// probe_slotread: read bandwidth of the SpMV's value stream in two orders, on a 4 GiB array.
//   slot   : lane l of a wave reads its 32-B slot (sb + l) as two 16-B loads (the current layout:
//            each instruction touches every 128-B line of the wave's 2 KiB, half of it)
//   group  : the same 64 slots stored in 8-slot groups [8 first halves | 8 second halves], so each
//            instruction reads whole 128-B lines
//   flat   : a plain float4 stream (lane l, instruction k: 16 B at 16 (l + 64 k)) -- the ceiling
// Each wave walks its range in windows of 64 slots with one window in flight (as the SpMV).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

template <int MODE>
__device__ __forceinline__ void load2(const double* __restrict__ v, long slot, v2d& a, v2d& b) {
  if (MODE == 0) {
    a = *(const v2d*)(v + 4 * slot);
    b = *(const v2d*)(v + 4 * slot + 2);
  } else {
    const double* g = v + 32 * (slot >> 3) + 2 * (slot & 7);
    a = *(const v2d*)g;
    b = *(const v2d*)(g + 16);
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void slot_read(const double* __restrict__ v, long slots_per_wave, double* out) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long sb = wave * slots_per_wave;
  const int nwin = (int)(slots_per_wave / 64);
  v2d a, b;
  load2<MODE>(v, sb + lane, a, b);
  double acc = 0.0;
  for (int t = 0; t < nwin; ++t) {
    const v2d ca = a, cb = b;
    if (t + 1 < nwin) load2<MODE>(v, sb + 64 * (t + 1) + lane, a, b);
    acc += ca[0] + ca[1] + cb[0] + cb[1];
  }
  if (acc == 1234.5) out[0] = acc;   // keeps the loads
}

__global__ __launch_bounds__(256) void flat_read(const double* __restrict__ v, long n2, double* out) {
  double acc = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) {
    const v2d a = *(const v2d*)(v + 2 * i);
    acc += a[0] + a[1];
  }
  if (acc == 1234.5) out[0] = acc;
}

int main() {
  const long bytes = 4L << 30, nd = bytes / 8, slots = nd / 4;
  const long spw = 704;   // ~ one SpMV wave's slots on C5 (64 rows x ~11 slots)
  const long waves = slots / spw;
  double *v, *out;
  CK(hipMalloc(&v, bytes));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(v, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned grid = (unsigned)(waves / 4);
  const double used = (double)grid * 4 * spw * 32;
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 3; ++mode) {
      float ms;
      CK(hipEventRecord(e0));
      for (int it = 0; it < 5; ++it) {
        if (mode == 0) hipLaunchKernelGGL(slot_read<0>, dim3(grid), dim3(256), 0, 0, v, spw, out);
        else if (mode == 1) hipLaunchKernelGGL(slot_read<1>, dim3(grid), dim3(256), 0, 0, v, spw, out);
        else hipLaunchKernelGGL(flat_read, dim3(4096), dim3(256), 0, 0, v, (long)(used / 16), out);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%s: %.3f ms per pass, %.2f TB/s\n", mode == 0 ? "slot " : mode == 1 ? "group" : "flat ", ms / 5,
             used / (ms / 5 * 1e-3) / 1e12);
    }
  }
  return 0;
}
