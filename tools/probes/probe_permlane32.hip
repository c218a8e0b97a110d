// probe_permlane32: what __builtin_amdgcn_permlane32_swap(x, y, false, false) returns on gfx950
// (x = lane, y = 100 + lane): prints both results for lanes 0, 1, 31, 32, 33, 63.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(int* out) {
  const int l = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
}

int main() {
  int* d;
  int h[128];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %2d: r0 = %3d  r1 = %3d\n", l, h[l], h[64 + l]);
  return 0;
}
