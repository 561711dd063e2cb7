// Semantics check of gfx950 v_permlane32_swap (__builtin_amdgcn_permlane32_swap):
// x = 1000 + lane, y = 2000 + lane; prints what each lane gets back in r[0], r[1].
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  const unsigned lane = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(1000u + lane, 2000u + lane, false, false);
  o[lane] = r[0];
  o[64 + lane] = r[1];
}
int main() {
  unsigned* d;
  unsigned h[128];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %2d: r0 %u r1 %u\n", l, h[l], h[64 + l]);
  hipFree(d);
  return 0;
}
