// Probe kernel: occupy whole CUs (all 160 KB of LDS) for a while, sleeping,
// so concurrent kernels that need LDS cannot be placed on them.
#include <hip/hip_runtime.h>
extern "C" __global__ __launch_bounds__(1024) void hog_kernel(long long cycles, int* sink) {
  extern __shared__ int lds[];
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(127);
  if (threadIdx.x == 0 && cycles < 0) { lds[0] = 1; sink[blockIdx.x] = lds[0]; }
}
extern "C" int hog_launch(int nwg, long long cycles, int* sink, hipStream_t s) {
  static int set = 0;
  if (!set) {
    hipError_t e = hipFuncSetAttribute((const void*)hog_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    set = 1;
  }
  hipLaunchKernelGGL(hog_kernel, dim3(nwg), dim3(1024), 160 * 1024, s, cycles, sink);
  return (int)hipGetLastError();
}
