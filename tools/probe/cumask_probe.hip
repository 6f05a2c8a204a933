// Probe: (1) do CU-masked streams (hipExtStreamCreateWithCUMask) restrict a
// kernel's workgroups, and how much HBM bandwidth do N CUs sustain for the
// hook path's read-only (pass 1) and read+write (pass 2) traffic; (2) does a
// HIP graph with two independent branches run them concurrently; (3) host
// cost of event record / stream wait / launch.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/cumask_probe tools/probe/cumask_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void read_sum(const f4v* __restrict__ x, size_t n4, float* out) {
  float s = 0.0f;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const f4v a = x[i], b = x[i + stride], c = x[i + 2 * stride], d = x[i + 3 * stride];
    s += (a.x + a.y + a.z + a.w) + (b.x + b.y + b.z + b.w) + (c.x + c.y + c.z + c.w) + (d.x + d.y + d.z + d.w);
  }
  for (; i < n4; i += stride) { const f4v a = x[i]; s += a.x + a.y + a.z + a.w; }
  if (s == 12345.678f) out[0] = s;
}
__global__ __launch_bounds__(256) void copy4(const f4v* __restrict__ x, f4v* __restrict__ y, size_t n4) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    f4v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = x[i + k * stride];
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v[k] * 0.5f, y + i + k * stride);
  }
  for (; i < n4; i += stride) y[i] = x[i] * 0.5f;
}
// records the hardware CU id of each workgroup (HW_REG_HW_ID: CU_ID bits 8..11, SH 12, SE 13..15)
__global__ void cu_census(unsigned* ids) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, all 32 bits
    unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
    ids[2 * blockIdx.x] = hw;
    ids[2 * blockIdx.x + 1] = xcc;
  }
  // keep the workgroup resident a while so others spread
  long long t0 = clock64();
  while (clock64() - t0 < 200000) {}
}
__global__ void spin(long long cycles, float* out) {
  long long t0 = clock64();
  float v = threadIdx.x;
  while (clock64() - t0 < cycles) v = v * 1.0000001f + 1e-7f;
  if (v == 1234.5f) out[0] = v;
}

static hipEvent_t e0, e1;
static float* outp;
static float timed_read(hipStream_t s, const float* x, size_t n, int grid) {
  std::vector<float> t;
  for (int r = 0; r < 14; ++r) {
    hipExtLaunchKernelGGL(read_sum, dim3(grid), dim3(256), 0, s, e0, e1, 0, (const f4v*)(x + (size_t)(r % 4) * n), n / 4, outp);
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 4) t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}
static float timed_copy(hipStream_t s, const float* x, float* y, size_t n, int grid) {
  std::vector<float> t;
  for (int r = 0; r < 14; ++r) {
    hipExtLaunchKernelGGL(copy4, dim3(grid), dim3(256), 0, s, e0, e1, 0, (const f4v*)(x + (size_t)(r % 4) * n), (f4v*)(y + (size_t)(r % 4) * n), n / 4);
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 4) t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  printf("CUs %d\n", ncu);
  const size_t n = (size_t)32 * (64 * 6400 + 128 * 1600 + 256 * 400);
  float *x, *y;
  CK(hipMalloc(&x, 4 * n * 4)); CK(hipMalloc(&y, 4 * n * 4));
  CK(hipMemset(x, 0, 4 * n * 4)); CK(hipMemset(y, 0, 4 * n * 4));
  CK(hipMalloc(&outp, 4));
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int words = (ncu + 31) / 32;
  auto make_mask = [&](int ncus, bool spread, int offset) {
    std::vector<uint32_t> m(words, 0);
    for (int k = 0; k < ncus; ++k) {
      const int c = spread ? (offset + (int)((long long)k * ncu / ncus)) % ncu : (offset + k) % ncu;
      m[c / 32] |= 1u << (c % 32);
    }
    return m;
  };
  // 1. does a masked stream run at all (watchdog: 2 s)
  for (int cfg = 0; cfg < 3; ++cfg) {
    hipStream_t s;
    std::vector<uint32_t> m = cfg == 0 ? make_mask(ncu, false, 0) : (cfg == 1 ? make_mask(32, false, 0) : make_mask(32, true, 0));
    CK(hipExtStreamCreateWithCUMask(&s, words, m.data()));
    std::vector<uint32_t> back(words);
    CK(hipExtStreamGetCUMask(s, words, back.data()));
    printf("mask cfg %d: readback w0 %08x w1 %08x w7 %08x\n", cfg, back[0], back[1], back[words - 1]);
    fflush(stdout);
    spin<<<64, 64, 0, s>>>(1000, outp);
    auto t0 = std::chrono::high_resolution_clock::now();
    bool done = false;
    while (std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count() < 2.0) {
      if (hipStreamQuery(s) == hipSuccess) { done = true; break; }
    }
    printf("  masked stream %s\n", done ? "ran" : "DID NOT RUN within 2 s");
    fflush(stdout);
    if (!done) return 2;
    CK(hipStreamDestroy(s));
  }
  // 2. bandwidth vs CUs
  printf("read 91.75 MB (4 buffers cycled), grid 8192 / copy grid 16384:\n");
  {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    printf("  unmasked stream       read %7.2f us   copy %7.2f us\n", timed_read(s, x, n, 8192), timed_copy(s, x, y, n, 16384));
    CK(hipStreamDestroy(s));
  }
  const int counts[] = {32, 64, 128, 160, 192, 224, 240, 256};
  for (int spread = 0; spread < 2; ++spread)
    for (int ci = 0; ci < 8; ++ci) {
      const int c = counts[ci];
      if (c > ncu) continue;
      hipStream_t s;
      std::vector<uint32_t> m = make_mask(c, spread != 0, 0);
      CK(hipExtStreamCreateWithCUMask(&s, words, m.data()));
      const float r = timed_read(s, x, n, 8192), cp = timed_copy(s, x, y, n, 16384);
      printf("  %3d CUs %-7s read %7.2f us (%6.0f GB/s)  copy %7.2f us (%6.0f GB/s)\n", c, spread ? "spread" : "first",
             r, n * 4.0 / (r * 1e3), cp, n * 8.0 / (cp * 1e3));
      CK(hipStreamDestroy(s));
    }
  // 3. graph with two independent branches: concurrent?
  {
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t f, j;
    CK(hipEventCreateWithFlags(&f, hipEventDisableTiming)); CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
    const long long cyc = 100000;   // ~50 us at ~2 GHz
    spin<<<8, 64, 0, s0>>>(cyc, outp);
    CK(hipStreamSynchronize(s0));
    CK(hipEventRecord(e0, s0));
    spin<<<8, 64, 0, s0>>>(cyc, outp);
    CK(hipEventRecord(e1, s0));
    CK(hipEventSynchronize(e1));
    float one; CK(hipEventElapsedTime(&one, e0, e1));
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(f, s0));
    CK(hipStreamWaitEvent(s1, f, 0));
    spin<<<8, 64, 0, s0>>>(cyc, outp);
    spin<<<8, 64, 0, s1>>>(cyc, outp);
    CK(hipEventRecord(j, s1));
    CK(hipStreamWaitEvent(s0, j, 0));
    CK(hipStreamEndCapture(s0, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s0));
    CK(hipStreamSynchronize(s0));
    CK(hipEventRecord(e0, s0));
    for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, s0));
    CK(hipEventRecord(e1, s0));
    CK(hipEventSynchronize(e1));
    float two; CK(hipEventElapsedTime(&two, e0, e1));
    printf("graph branches: one spin kernel %.1f us; graph of two parallel spins %.1f us per replay (%s)\n",
           one * 1e3, two * 1e3 / 10, two * 1e3 / 10 < 1.5 * one * 1e3 ? "concurrent" : "serialised");
    // 4. host costs
    const int N = 2000;
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int r = 0; r < N; ++r) CK(hipEventRecord(f, s0));
    auto t1 = std::chrono::high_resolution_clock::now();
    for (int r = 0; r < N; ++r) CK(hipStreamWaitEvent(s1, f, 0));
    auto t2 = std::chrono::high_resolution_clock::now();
    for (int r = 0; r < N; ++r) spin<<<1, 64, 0, s0>>>(0, outp);
    auto t3 = std::chrono::high_resolution_clock::now();
    CK(hipDeviceSynchronize());
    for (int r = 0; r < N / 10; ++r) CK(hipGraphLaunch(ge, s0));
    auto t4 = std::chrono::high_resolution_clock::now();
    CK(hipDeviceSynchronize());
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    printf("host: hipEventRecord %.2f us, hipStreamWaitEvent %.2f us, launch %.2f us, graph launch %.2f us\n",
           us(t0, t1) / N, us(t1, t2) / N, us(t2, t3) / N, us(t3, t4) / (N / 10));
  }
  return 0;
}
