// Semantics check of v_permlane16_swap / v_permlane32_swap with both operands
// equal (lane l reads lane l^16 / l^32): prints the source lane each lane gets.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/permlane_probe tools/probe/permlane_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(int* out) {
  const unsigned x = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  out[threadIdx.x] = (threadIdx.x & 16) ? (int)r[0] : (int)r[1];
  const auto s = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  out[64 + threadIdx.x] = (threadIdx.x & 32) ? (int)s[0] : (int)s[1];
}
int main() {
  int* d; int h[128];
  if (hipMalloc(&d, 512) != hipSuccess) return 1;
  k<<<1, 64>>>(d);
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int ok16 = 1, ok32 = 1;
  for (int l = 0; l < 64; ++l) { ok16 &= h[l] == (l ^ 16); ok32 &= h[64 + l] == (l ^ 32); }
  printf("xor16 via permlane16_swap: %s  xor32 via permlane32_swap: %s\n", ok16 ? "ok" : "WRONG", ok32 ? "ok" : "WRONG");
  for (int l = 0; l < 64; ++l) printf("%d ", h[l]);
  printf("\n");
  return ok16 && ok32 ? 0 : 2;
}
