// Which hardware ids do workgroups report (HW_REG_HW_ID: wave/simd/pipe/cu/sh/se fields, and
// HW_REG_XCC_ID)?  Used to pick a CU subset a bulk launch leaves to the Cholesky's chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <set>
#include <vector>
__global__ void hwid_kernel(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID, 32 bits
    unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID, 16 bits
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    __builtin_amdgcn_s_sleep(100);
  }
}
int main() {
  const int n = 8192;
  unsigned* d;
  (void)hipMalloc(&d, sizeof(unsigned) * 2 * n);
  hipLaunchKernelGGL(hwid_kernel, dim3(n), dim3(64), 0, 0, d);
  std::vector<unsigned> h(2 * n);
  (void)hipMemcpy(h.data(), d, sizeof(unsigned) * 2 * n, hipMemcpyDeviceToHost);
  std::set<unsigned> units;
  std::map<unsigned, std::set<unsigned>> cu_per_xcc;
  for (int i = 0; i < n; ++i) {
    const unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xF;
    const unsigned cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    units.insert((xcc << 12) | (se << 8) | (sh << 4) | cu);
    cu_per_xcc[xcc].insert((se << 8) | (sh << 4) | cu);
    if (i < 24) printf("blk %d hw 0x%08x xcc 0x%x -> se %u sh %u cu %u\n", i, hw, h[2 * i + 1], se, sh, cu);
  }
  printf("distinct (xcc,se,sh,cu): %zu\n", units.size());
  for (auto& kv : cu_per_xcc) {
    printf("xcc %u: %zu units:", kv.first, kv.second.size());
    for (unsigned u : kv.second) printf(" %u.%u.%u", u >> 8, (u >> 4) & 15, u & 15);
    printf("\n");
  }
  return 0;
}
