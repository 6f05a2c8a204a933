// How much of the chip do the streaming passes need?  Pass-2-shaped copies
// (unit = T/64 waves x 8 rows x 1 KB, lane l owns 16 bytes of every row;
// plain loads, nontemporal stores) and pass-1-shaped reads as PERSISTENT
// kernels on G workgroups held to one per CU by a dynamic LDS allocation,
// units looped with a register pipeline D units deep.  If a narrow grid
// already reaches the ~6 TB/s the one-unit-per-workgroup kernels reach on the
// whole chip, the streaming passes and the morphology could run on disjoint
// CU sets; if not, the CU-time budget stands.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/narrow_probe tools/probe/narrow_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <int T>
__device__ __forceinline__ void ld_unit(f4v (&r)[8], const f4v* __restrict__ x, int u) {
  constexpr int UF4 = (T / 64) * 8 * 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const f4v* p = x + (size_t)u * UF4 + wv * 512 + lane;
#pragma unroll
  for (int c = 0; c < 8; ++c) r[c] = p[c * 64];
}

template <int T>
__device__ __forceinline__ void st_unit(const f4v (&r)[8], f4v* __restrict__ y, int u) {
  constexpr int UF4 = (T / 64) * 8 * 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  f4v* p = y + (size_t)u * UF4 + wv * 512 + lane;
#pragma unroll
  for (int c = 0; c < 8; ++c) __builtin_nontemporal_store(r[c] * 1.5f, p + c * 64);
}

// kWrite: copy (pass 2 traffic) or read-only (pass 1 traffic)
template <int T, int D, bool kWrite>
__global__ __launch_bounds__(T) void stream_units(const f4v* __restrict__ x, f4v* __restrict__ y, int units,
                                                  float* sink) {
  extern __shared__ float occ[];   // occupancy only
  const int G = gridDim.x;
  f4v r[D][8];
  f4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int s = 0; s < D - 1; ++s) ld_unit<T>(r[s], x, min((int)blockIdx.x + s * G, units - 1));
  for (int u0 = blockIdx.x; u0 < units; u0 += D * G) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      const int u = u0 + s * G;
      ld_unit<T>(r[(s + D - 1) % D], x, min(u + (D - 1) * G, units - 1));
      if (kWrite) {
        st_unit<T>(r[s], y, min(u, units - 1));   // a clamped repeat rewrites the same values
      } else {
#pragma unroll
        for (int c = 0; c < 8; ++c) acc += r[s][c];
      }
    }
  }
  if (!kWrite && acc.x + acc.y + acc.z + acc.w == 12345.678f) sink[0] = acc.x;
  if (threadIdx.x == 0 && G < 0) occ[0] = 0.0f;
}

typedef void (*kfn)(const f4v*, f4v*, int, float*);

struct Variant {
  const char* name;
  kfn k;
  int T, D;
  bool write;
};

int main(int argc, char** argv) {
  // config-2 bytes: 91.75 MB of x per batch (22.94 M floats), 5 batch buffers cycled (more than the 256 MB Infinity Cache between reuses)
  const size_t nf = (size_t)32 * (64 * 6400 + 128 * 1600 + 256 * 400);
  const int nb = 5;
  f4v *x[nb], *y[nb];
  float* sink;
  const size_t bytes = nf * 4 + (1 << 20);
  for (int i = 0; i < nb; ++i) {
    CK(hipMalloc(&x[i], bytes));
    CK(hipMalloc(&y[i], bytes));
    CK(hipMemset(x[i], 0, bytes));
    CK(hipMemset(y[i], 0, bytes));
  }
  CK(hipMalloc(&sink, 64));
  const Variant vs[] = {
      {"copy T256 D1", stream_units<256, 1, true>, 256, 1, true},
      {"copy T256 D2", stream_units<256, 2, true>, 256, 2, true},
      {"copy T256 D3", stream_units<256, 3, true>, 256, 3, true},
      {"copy T512 D2", stream_units<512, 2, true>, 512, 2, true},
      {"copy T1024 D2", stream_units<1024, 2, true>, 1024, 2, true},
      {"read T256 D2", stream_units<256, 2, false>, 256, 2, false},
      {"read T512 D2", stream_units<512, 2, false>, 512, 2, false},
      {"read T1024 D3", stream_units<1024, 3, false>, 1024, 3, false},
  };
  const int grids[] = {32, 64, 96, 128, 160, 192, 224, 256, 0};   // 0: one unit per workgroup, no LDS pin
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 12;
  printf("%-14s %6s %9s %9s %s\n", "variant", "grid", "us", "TB/s", "(1 WG per CU via 96 KB LDS; grid 0 = one unit per WG)");
  for (const Variant& v : vs) {
    const size_t ubytes = (size_t)(v.T / 64) * 8 * 1024;
    const int units = (int)((nf * 4) / ubytes);
    const double moved = (double)units * ubytes * (v.write ? 2.0 : 1.0);
    for (int g : grids) {
      const int G = g ? g : units;
      const size_t lds = g ? 96 * 1024 : 0;
      if (lds) CK(hipFuncSetAttribute((const void*)v.k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(v.k, dim3(G), dim3(v.T), lds, 0, x[w], y[w], units, sink);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(v.k, dim3(G), dim3(v.T), lds, 0, x[r % nb], y[r % nb], units, sink);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float ms = 0.0f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1000.0 / reps;
      printf("%-14s %6d %9.2f %9.3f\n", v.name, g, us, moved / us * 1e-6);
      fflush(stdout);
    }
  }
  return 0;
}
