// Infinity-Cache (MALL) probe for the hook path's two streaming passes at
// config-2 size (91.75 MB of x per batch): does pass 2's re-read of x come
// from the 256 MiB Infinity Cache when only pass 1 (and little else) ran
// between the two reads, and how fast is that read?
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/mall_probe tools/probe/mall_probe.hip
// Every dispatch is timed by its own start/stop events (hipExtLaunchKernel);
// medians over the repetitions.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void read_sum(const f4v* __restrict__ x, size_t n4, float* out) {
  float s = 0.0f;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    f4v a, b, c, d;
    if (NT) {
      a = __builtin_nontemporal_load(x + i); b = __builtin_nontemporal_load(x + i + stride);
      c = __builtin_nontemporal_load(x + i + 2 * stride); d = __builtin_nontemporal_load(x + i + 3 * stride);
    } else {
      a = x[i]; b = x[i + stride]; c = x[i + 2 * stride]; d = x[i + 3 * stride];
    }
    s += (a.x + a.y + a.z + a.w) + (b.x + b.y + b.z + b.w) + (c.x + c.y + c.z + c.w) + (d.x + d.y + d.z + d.w);
  }
  for (; i < n4; i += stride) { const f4v a = x[i]; s += a.x + a.y + a.z + a.w; }
  if (s == 12345.678f) out[0] = s;
}

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy4(const f4v* __restrict__ x, f4v* __restrict__ y, size_t n4) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    f4v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = NTL ? __builtin_nontemporal_load(x + i + k * stride) : x[i + k * stride];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f4v o = v[k] * 0.5f;
      if (NTS) __builtin_nontemporal_store(o, y + i + k * stride); else y[i + k * stride] = o;
    }
  }
  for (; i < n4; i += stride) y[i] = x[i] * 0.5f;
}

__global__ void fill(float* p, size_t n, unsigned seed) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (float)(h & 0xffff) * (1.0f / 65536.0f) - 0.25f;
  }
}

static hipEvent_t e0, e1;
static float* outp;
enum Kind { RD, RD_NT, CP, CP_NTS, CP_NTL_NTS };
static const int RG = 8192, CG = 16384;

static void launch(Kind k, const float* x, float* y, size_t n, bool timed) {
  const size_t n4 = n / 4;
  hipEvent_t a = timed ? e0 : nullptr, b = timed ? e1 : nullptr;
  switch (k) {
    case RD: hipExtLaunchKernelGGL(read_sum<false>, dim3(RG), dim3(256), 0, 0, a, b, 0, (const f4v*)x, n4, outp); break;
    case RD_NT: hipExtLaunchKernelGGL(read_sum<true>, dim3(RG), dim3(256), 0, 0, a, b, 0, (const f4v*)x, n4, outp); break;
    case CP: hipExtLaunchKernelGGL((copy4<false, false>), dim3(CG), dim3(256), 0, 0, a, b, 0, (const f4v*)x, (f4v*)y, n4); break;
    case CP_NTS: hipExtLaunchKernelGGL((copy4<false, true>), dim3(CG), dim3(256), 0, 0, a, b, 0, (const f4v*)x, (f4v*)y, n4); break;
    case CP_NTL_NTS: hipExtLaunchKernelGGL((copy4<true, true>), dim3(CG), dim3(256), 0, 0, a, b, 0, (const f4v*)x, (f4v*)y, n4); break;
  }
}
static float elapsed_us() {
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f;
}
static float median(std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main() {
  const size_t n = (size_t)32 * (64 * 6400 + 128 * 1600 + 256 * 400);   // config 2 x: 22.94 M floats
  const double MB = n * 4.0 / 1e6;
  const int NB = 8;
  float *X[NB], *Y[NB], *Z;
  const size_t nz = (size_t)512 << 20 >> 2;   // 512 MiB eviction sweep
  for (int k = 0; k < NB; ++k) {
    CK(hipMalloc(&X[k], n * 4)); CK(hipMalloc(&Y[k], n * 4));
    fill<<<4096, 256>>>(X[k], n, 17u * k + 1);
    fill<<<4096, 256>>>(Y[k], n, 91u * k + 3);
  }
  CK(hipMalloc(&Z, nz * 4));
  fill<<<4096, 256>>>(Z, nz, 7u);
  CK(hipMalloc(&outp, 4));
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipDeviceSynchronize());
  printf("x per batch %.2f MB; read = %.2f MB per launch, copy = %.2f MB\n", MB, MB, 2 * MB);
  const int reps = 24;
  auto rep = [&](const char* name, double bytes, auto body) {
    std::vector<float> t;
    for (int r = 0; r < reps + 4; ++r) { float us = body(r); if (r >= 4) t.push_back(us); }
    const float m = median(t);
    printf("%-60s %8.2f us  %7.1f GB/s\n", name, m, bytes / (m * 1e-6) / 1e9);
  };
  // 1. read, same buffer every time (resident after the first) vs 8 buffers cycled (736 MB: HBM)
  rep("read same x (resident)", MB * 1e6, [&](int) { launch(RD, X[0], 0, n, true); return elapsed_us(); });
  rep("read nt same x", MB * 1e6, [&](int) { launch(RD_NT, X[0], 0, n, true); return elapsed_us(); });
  rep("read x cycled over 8 (HBM)", MB * 1e6, [&](int r) { launch(RD, X[r % NB], 0, n, true); return elapsed_us(); });
  rep("read nt x cycled over 8 (HBM)", MB * 1e6, [&](int r) { launch(RD_NT, X[r % NB], 0, n, true); return elapsed_us(); });
  // 2. copy
  rep("copy same x->y (resident)", 2 * MB * 1e6, [&](int) { launch(CP, X[0], Y[0], n, true); return elapsed_us(); });
  rep("copy x->y cycled over 8 (HBM)", 2 * MB * 1e6, [&](int r) { launch(CP, X[r % NB], Y[r % NB], n, true); return elapsed_us(); });
  rep("copy nts x->y cycled over 8 (HBM)", 2 * MB * 1e6, [&](int r) { launch(CP_NTS, X[r % NB], Y[r % NB], n, true); return elapsed_us(); });
  rep("copy ntl+nts x->y cycled over 8 (HBM)", 2 * MB * 1e6, [&](int r) { launch(CP_NTL_NTS, X[r % NB], Y[r % NB], n, true); return elapsed_us(); });
  // 3. pass-1 read of x_k, then pass-2 copy of x_k (cycled over 8): is the copy's read served on-die?
  const Kind p1[2] = {RD, RD_NT};
  const Kind p2[3] = {CP, CP_NTS, CP_NTL_NTS};
  const char* p1n[2] = {"plain", "nt"};
  const char* p2n[3] = {"plain", "nts", "ntl+nts"};
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 3; ++b) {
      char nm[128];
      snprintf(nm, sizeof nm, "copy right after read of same x (p1 %s, p2 %s)", p1n[a], p2n[b]);
      rep(nm, 2 * MB * 1e6, [&](int r) { launch(p1[a], X[r % NB], 0, n, false); launch(p2[b], X[r % NB], Y[r % NB], n, true); return elapsed_us(); });
      snprintf(nm, sizeof nm, "  same, 512 MiB sweep between (evicted)");
      rep(nm, 2 * MB * 1e6, [&](int r) {
        launch(p1[a], X[r % NB], 0, n, false); launch(RD_NT, Z, 0, nz, false);
        launch(p2[b], X[r % NB], Y[r % NB], n, true); return elapsed_us(); });
      snprintf(nm, sizeof nm, "  pipelined order read(k+1) then copy(k)");
      rep(nm, 2 * MB * 1e6, [&](int r) {
        launch(p1[a], X[(r + 1) % NB], 0, n, false);
        launch(p2[b], X[r % NB], Y[r % NB], n, true); return elapsed_us(); });
    }
  // 4. whole-step proxies, wall time per step over 40 steps
  for (int order = 0; order < 2; ++order)
    for (int b = 0; b < 3; ++b) {
      const int steps = 40;
      for (int w = 0; w < 4; ++w) { launch(RD_NT, X[w % NB], 0, n, false); launch(p2[b], X[w % NB], Y[w % NB], n, false); }
      CK(hipDeviceSynchronize());
      hipEvent_t s0, s1;
      CK(hipEventCreate(&s0)); CK(hipEventCreate(&s1));
      CK(hipEventRecord(s0, 0));
      for (int r = 0; r < steps; ++r) {
        if (order == 0) { launch(RD_NT, X[r % NB], 0, n, false); launch(p2[b], X[r % NB], Y[r % NB], n, false); }
        else { launch(RD_NT, X[(r + 1) % NB], 0, n, false); launch(p2[b], X[r % NB], Y[r % NB], n, false); }
      }
      CK(hipEventRecord(s1, 0));
      CK(hipEventSynchronize(s1));
      float ms;
      CK(hipEventElapsedTime(&ms, s0, s1));
      const double us = ms * 1e3 / steps;
      printf("step proxy %s read(nt) + copy(%s): %7.2f us/step = %7.1f GB/s of 12 B/elem (%.3f of 8 TB/s)\n",
             order ? "pipelined" : "same-batch", p2n[b], us, 3 * MB * 1e6 / (us * 1e-6) / 1e9,
             3 * MB * 1e6 / (us * 1e-6) / 8e12);
    }
  return 0;
}
