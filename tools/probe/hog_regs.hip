// Probe kernels: hold one CU's worth of 1024-thread workgroup (a pass-A
// footprint: `lds` bytes of LDS and NV VGPRs per lane, forced by a clobber of
// v(NV-1)) for a while, sleeping, so the streaming passes beside it get only
// the registers and LDS the hog leaves.  hog_regs_launch(nv = 64 / 96 / 128).
#include <hip/hip_runtime.h>

template <int NV>
__global__ __launch_bounds__(1024) void hog_regs_kernel(long long cycles, int* sink) {
  extern __shared__ int lds[];
  if constexpr (NV == 128) asm volatile("" ::: "v127");
  else if constexpr (NV == 96) asm volatile("" ::: "v95");
  else asm volatile("" ::: "v63");
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(127);
  if (threadIdx.x == 0 && cycles < 0) { lds[0] = 1; sink[blockIdx.x] = lds[0]; }
}

extern "C" int hog_regs_launch(int nwg, int nv, int lds, long long cycles, int* sink, hipStream_t s) {
  const void* f = nv == 128 ? (const void*)hog_regs_kernel<128>
                  : nv == 96 ? (const void*)hog_regs_kernel<96> : (const void*)hog_regs_kernel<64>;
  hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return (int)e;
  if (nv == 128) hipLaunchKernelGGL(hog_regs_kernel<128>, dim3(nwg), dim3(1024), lds, s, cycles, sink);
  else if (nv == 96) hipLaunchKernelGGL(hog_regs_kernel<96>, dim3(nwg), dim3(1024), lds, s, cycles, sink);
  else hipLaunchKernelGGL(hog_regs_kernel<64>, dim3(nwg), dim3(1024), lds, s, cycles, sink);
  return (int)hipGetLastError();
}
