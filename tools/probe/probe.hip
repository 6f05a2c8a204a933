#include <hip/hip_runtime.h>
extern "C" __global__ void add_one(float* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = rintf(p[i] + 1.0f);
}
extern "C" int probe_launch(float* p, int n, hipStream_t s) {
  hipLaunchKernelGGL(add_one, dim3((n + 255) / 256), dim3(256), 0, s, p, n);
  return (int)hipGetLastError();
}
