// Probe: calibration of rocprofv3 FETCH_SIZE for pass 1's load widths.
// Reads a known byte count (4 buffers of 96 MiB cycled: 384 MiB > the 256 MiB
// Infinity Cache) with coalesced 16-, 8- and 4-byte-per-lane rows, the widths
// pass 1 uses for C3 / C4 / C5 (PPL 4 / 2 / 1), each kernel 4 launches.
// Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace`: FETCH_SIZE x 1024 /
// 100663296 = the counter's reading per byte for that width.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/pmc_control tools/probe/pmc_control.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

template <typename T>
__global__ __launch_bounds__(256) void read_w(const T* __restrict__ x, size_t n, float* out) {
  float s = 0.0f;
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const T v = __builtin_nontemporal_load(x + i);
    if constexpr (sizeof(T) == 16) s += (v.x + v.y) + (v.z + v.w);
    else if constexpr (sizeof(T) == 8) s += v.x + v.y;
    else s += v;
  }
  if (s == 12345.678f) out[0] = s;   // keep the loads
}

int main() {
  const size_t bytes = (size_t)96 << 20;
  float* buf[4];
  float* out;
  for (int i = 0; i < 4; ++i) { CK(hipMalloc(&buf[i], bytes)); CK(hipMemset(buf[i], 0, bytes)); }
  CK(hipMalloc(&out, 4));
  CK(hipDeviceSynchronize());
  for (int r = 0; r < 4; ++r) {
    hipLaunchKernelGGL(read_w<f4v>, dim3(8192), dim3(256), 0, 0, (const f4v*)buf[r], bytes / 16, out);
    hipLaunchKernelGGL(read_w<f2v>, dim3(8192), dim3(256), 0, 0, (const f2v*)buf[(r + 1) % 4], bytes / 8, out);
    hipLaunchKernelGGL(read_w<float>, dim3(8192), dim3(256), 0, 0, (const float*)buf[(r + 2) % 4], bytes / 4, out);
  }
  CK(hipDeviceSynchronize());
  printf("read %zu bytes per launch with 16 / 8 / 4-byte lanes, 4 launches each\n", bytes);
  return 0;
}
