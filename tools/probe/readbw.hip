// Diagnostic: HBM read patterns of pass 1 (standalone; hipcc -O3 --offload-arch=gfx950 readbw.hip -o readbw)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

// rows-per-wave pattern: a workgroup of 4 waves reads 256 px x (4 * R) rows of
// one image (C rows of HW floats); wave w rows w*R .. w*R+R-1.
template <int R>
__global__ __launch_bounds__(256) void rows_kernel(const float* x, float* out, int C, int HW, int upi) {
  const int u = blockIdx.x, b = u / upi, chunk = u % upi;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ngrp = C / (4 * R);
  const float* xb = x + (size_t)b * C * HW;
  float acc = 0.f;
  for (int g = 0; g < ngrp; ++g) {
    float4 v[R];
#pragma unroll
    for (int i = 0; i < R; ++i) v[i] = *reinterpret_cast<const float4*>(xb + (size_t)(g * 4 * R + w * R + i) * HW + chunk * 256 + lane * 4);
#pragma unroll
    for (int i = 0; i < R; ++i) acc += v[i].x + v[i].y + v[i].z + v[i].w;
  }
  if (acc == 12345.f) out[threadIdx.x] = acc;
}

// contiguous streaming read, grid-stride float4
__global__ __launch_bounds__(256) void stream_kernel(const float4* x, float* out, size_t n4) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = x[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void copy_kernel(const float4* x, float4* y, size_t n4) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) y[i] = x[i];
}

template <typename F>
float timeit(F f, int reps = 20) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f(); hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const int B = 32, C = 64, HW = 6400;
  const size_t n = (size_t)B * C * HW;
  float *x, *y, *out;
  hipMalloc(&x, n * 4); hipMalloc(&y, n * 4); hipMalloc(&out, 4096);
  hipMemset(x, 0, n * 4);
  const int upi = HW / 256;
  const double mb = n * 4.0;
  float t;
  t = timeit([&] { rows_kernel<16><<<B * upi, 256>>>(x, out, C, HW, upi); });
  printf("rows R=16 (1 grp)     %7.1f us %7.1f GB/s\n", t, mb / t / 1e3);
  t = timeit([&] { rows_kernel<8><<<B * upi, 256>>>(x, out, C, HW, upi); });
  printf("rows R=8  (2 grp)     %7.1f us %7.1f GB/s\n", t, mb / t / 1e3);
  t = timeit([&] { rows_kernel<4><<<B * upi, 256>>>(x, out, C, HW, upi); });
  printf("rows R=4  (4 grp)     %7.1f us %7.1f GB/s\n", t, mb / t / 1e3);
  for (int g : {1024, 2048, 4096, 8192}) {
    t = timeit([&] { stream_kernel<<<g, 256>>>((const float4*)x, out, n / 4); });
    printf("stream grid %5d     %7.1f us %7.1f GB/s\n", g, t, mb / t / 1e3);
  }
  for (int g : {2048, 8192}) {
    t = timeit([&] { copy_kernel<<<g, 256>>>((const float4*)x, (float4*)y, n / 4); });
    printf("copy grid %5d       %7.1f us %7.1f GB/s\n", g, t, 2 * mb / t / 1e3);
  }
  // bigger: 1 GiB stream
  const size_t nb = (size_t)256 << 20;
  float* z; hipMalloc(&z, nb * 4); hipMemset(z, 0, nb * 4);
  t = timeit([&] { stream_kernel<<<8192, 256>>>((const float4*)z, out, nb / 4); });
  printf("stream 1GiB          %7.1f us %7.1f GB/s\n", t, nb * 4.0 / t / 1e3);
  return 0;
}
