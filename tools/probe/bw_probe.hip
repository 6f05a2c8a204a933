// HBM ceiling probe for the hook path's two streaming passes (config 2 sizes):
// a read-only pass over x (pass 1's traffic, 4 B/element) and a read + write
// pass (pass 2's traffic, 8 B/element), as plain grid-stride float4 kernels
// at several grid sizes, timed per launch with HIP events.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/bw_probe tools/probe/bw_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void read_sum(const float4* __restrict__ x, size_t n4, float* out) {
  float s = 0.0f;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const float4 a = x[i], b = x[i + stride], c = x[i + 2 * stride], d = x[i + 3 * stride];
    s += (a.x + a.y + a.z + a.w) + (b.x + b.y + b.z + b.w) + (c.x + c.y + c.z + c.w) + (d.x + d.y + d.z + d.w);
  }
  for (; i < n4; i += stride) { const float4 a = x[i]; s += a.x + a.y + a.z + a.w; }
  if (s == 12345.678f) out[0] = s;   // keep the loads
}

__global__ __launch_bounds__(256) void copy4(const float4* __restrict__ x, float4* __restrict__ y, size_t n4) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const float4 a = x[i], b = x[i + stride], c = x[i + 2 * stride], d = x[i + 3 * stride];
    y[i] = a; y[i + stride] = b; y[i + 2 * stride] = c; y[i + 3 * stride] = d;
  }
  for (; i < n4; i += stride) y[i] = x[i];
}


// pass-1-shaped read: unit = 256 pixels x C channels of one image (C3 shape:
// 64 x 80 x 80), wave w loads rows w, w+4, ... (ROWS per wave) as float4 per
// lane, 1 KB per row; NWG_MIN = workgroups per CU requested
template <int ROWS, int MINW>
__global__ __launch_bounds__(256, MINW) void shape_read(const float* __restrict__ x, int C, int HW, float* out) {
  const int upi = HW / 256;
  const int b = blockIdx.x / upi, chunk = blockIdx.x - b * upi;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float* xb = x + (size_t)b * C * HW + chunk * 256 + lane * 4;
  float s = 0.0f;
  float4 v[ROWS];
#pragma unroll
  for (int i = 0; i < ROWS; ++i) v[i] = *reinterpret_cast<const float4*>(xb + (size_t)(wv * ROWS + i) * HW);
#pragma unroll
  for (int i = 0; i < ROWS; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  if (s == 12345.678f) out[0] = s;
}

int main() {
  // config 2: 32 x (64*6400 + 128*1600 + 256*400) floats; 3 input batches cycled
  const size_t n = (size_t)32 * (64 * 6400 + 128 * 1600 + 256 * 400);
  const size_t n4 = n / 4;
  const int nb = 3;
  float4 *x[nb], *y[nb];
  float* out;
  for (int k = 0; k < nb; ++k) { CK(hipMalloc(&x[k], n * 4)); CK(hipMalloc(&y[k], n * 4)); CK(hipMemset(x[k], 0, n * 4)); }
  CK(hipMalloc(&out, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int grids[] = {1024, 2048, 4096, 8192, 16384};
  for (int gi = 0; gi < 5; ++gi) {
    const int g = grids[gi];
    for (int mode = 0; mode < 2; ++mode) {
      for (int w = 0; w < 3; ++w) {
        if (mode == 0) read_sum<<<g, 256>>>(x[w % nb], n4, out); else copy4<<<g, 256>>>(x[w % nb], y[w % nb], n4);
      }
      CK(hipDeviceSynchronize());
      const int reps = 30;
      float tot = 0.0f;
      for (int r = 0; r < reps; ++r) {
        // the dispatch's own start / end (hipExtLaunchKernel events)
        if (mode == 0)
          hipExtLaunchKernelGGL(read_sum, dim3(g), dim3(256), 0, 0, e0, e1, 0, (const float4*)x[r % nb], n4, out);
        else
          hipExtLaunchKernelGGL(copy4, dim3(g), dim3(256), 0, 0, e0, e1, 0, (const float4*)x[r % nb], y[r % nb], n4);
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        tot += ms;
      }
      const double us = tot * 1e3 / reps;
      const double bytes = (mode == 0 ? 4.0 : 8.0) * n;
      printf("%-8s grid %6d  %7.2f us  %7.1f GB/s\n", mode == 0 ? "read" : "copy", g, us, bytes / (us * 1e-6) / 1e9);
    }
  }

  {
    // C3 shape of config 2: B 32, C 64, 80 x 80 (52 MB)
    const int B = 32, C = 64, HW = 6400;
    const size_t bytes = (size_t)B * C * HW * 4;
    const int grid = B * HW / 256;
    for (int v = 0; v < 3; ++v) {
      float tot = 0.0f;
      const int reps = 30;
      for (int r = 0; r < reps + 3; ++r) {
        const float* xp = (const float*)x[r % nb];
        if (v == 0) hipExtLaunchKernelGGL((shape_read<16, 4>), dim3(grid), dim3(256), 0, 0, e0, e1, 0, xp, C, HW, out);
        if (v == 1) hipExtLaunchKernelGGL((shape_read<16, 2>), dim3(grid), dim3(256), 0, 0, e0, e1, 0, xp, C, HW, out);
        if (v == 2) hipExtLaunchKernelGGL(read_sum, dim3(8192), dim3(256), 0, 0, e0, e1, 0, (const float4*)xp, bytes / 16, out);
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) tot += ms;
      }
      const double us = tot * 1e3 / reps;
      printf("C3 %-22s %7.2f us  %7.1f GB/s\n", v == 0 ? "shape_read<16,4>" : (v == 1 ? "shape_read<16,2>" : "read_sum grid 8192"),
             us, bytes / (us * 1e-6) / 1e9);
    }
  }
  return 0;
}
