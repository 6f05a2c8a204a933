// Access-shape probe for the hook path's two HBM passes at config-2 sizes
// (yolov8n bs32: C3 64x80x80, C4 128x40x40, C5 256x20x20; 91.75 MB of x per
// batch), x cold (4 batches cycled: every dispatch's batch was last touched
// 3 dispatches earlier, > 256 MiB of traffic ago).
//
//   copy  (pass-2 shape): read x, write y = 0.5 x.  A unit = P pixels x S
//         channels of one image; the 4 waves split the channels; lane l owns
//         pixels 4l..4l+3 of each 256-pixel row segment (16-byte accesses);
//         every load of the unit is issued before the first store.
//   read  (pass-1 shape): unit = P pixels x all C channels, waves split the
//         16-row channel blocks, 16 rows loaded at once.
// Unit order: "cs" = (image, chunk, slice) with the slice fastest (the
// current pass 2), "sc" = slice slowest.  Each dispatch is timed by its own
// start/stop events (hipExtLaunchKernel); medians over the repetitions.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/shape_probe tools/probe/shape_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef float f4v __attribute__((ext_vector_type(4)));

struct Scale { const float* x; float* y; int C, HW, units, begin; };
struct Args { Scale s[3]; int P, S, order, nscales, units; float* sink; };

__device__ __forceinline__ int scale_of(const Args& a, int u) {
  return u >= a.s[2].begin ? 2 : (u >= a.s[1].begin ? 1 : 0);
}

// pass-2 shaped copy; RPW = row segments (of 256 px) per wave = (P/256) * (S/4)
template <int RPW>
__global__ __launch_bounds__(256, 6) void copy_units(Args a) {
  const int u = blockIdx.x;
  const int si = scale_of(a, u);
  const Scale& S = a.s[si];
  int lu = u - S.begin;
  const int segs = a.P / 256;                       // 256-px segments per unit
  const int upi = (S.HW + a.P - 1) / a.P;
  const int nsl = (S.C + a.S - 1) / a.S;
  int slice, chunk, b;
  if (a.order == 0) { slice = lu % nsl; lu /= nsl; chunk = lu % upi; b = lu / upi; }
  else { chunk = lu % upi; lu /= upi; b = lu % (a.s[si].units / (upi * nsl)); slice = lu / (a.s[si].units / (upi * nsl)); }
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cpw = a.S / 4;                          // channels per wave
  f4v v[RPW];
  size_t off[RPW];
  bool ok[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int c = slice * a.S + wv * cpw + r / segs;
    const int p = chunk * a.P + (r % segs) * 256 + lane * 4;
    ok[r] = c < S.C && p < S.HW;
    off[r] = ((size_t)b * S.C + (c < S.C ? c : 0)) * S.HW + (p < S.HW ? p : 0);
    v[r] = *reinterpret_cast<const f4v*>(S.x + off[r]);
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r)
    if (ok[r]) __builtin_nontemporal_store(v[r] * 0.5f, reinterpret_cast<f4v*>(S.y + off[r]));
}

// pass-1 shaped read: P pixels (256 * segs) x all channels, 16-row blocks
__global__ __launch_bounds__(256, 4) void read_units(Args a) {
  const int u = blockIdx.x;
  const int si = scale_of(a, u);
  const Scale& S = a.s[si];
  const int lu = u - S.begin;
  const int upi = (S.HW + a.P - 1) / a.P;
  const int chunk = lu % upi, b = lu / upi;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nblk = S.C / 16;
  const int segs = a.P / 256;
  float acc = 0.0f;
  for (int blk = wv; blk < nblk; blk += 4) {
    for (int sg = 0; sg < segs; ++sg) {
      const int p = chunk * a.P + sg * 256 + lane * 4;
      const int pc = p < S.HW ? p : 0;
      f4v v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        v[i] = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(S.x + ((size_t)b * S.C + blk * 16 + i) * S.HW + pc));
#pragma unroll
      for (int i = 0; i < 16; ++i) acc += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
  }
  if (acc == 12345.678f) a.sink[0] = acc;
}

// pass-1 shape, channel-split: unit = (image, 256-px chunk, group of 64
// channels); wave w reads the 16-row block 4 * group + w (one round)
__global__ __launch_bounds__(256, 4) void read_units_split(Args a) {
  const int u = blockIdx.x;
  const int si = scale_of(a, u);
  const Scale& S = a.s[si];
  const int lu = u - S.begin;
  const int upi = (S.HW + 255) / 256;
  const int ngr = S.C / 64;
  const int grp = lu % ngr, chunk = (lu / ngr) % upi, b = lu / (ngr * upi);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int blk = grp * 4 + wv;
  const int p = chunk * 256 + lane * 4;
  const int pc = p < S.HW ? p : 0;
  f4v v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    v[i] = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(S.x + ((size_t)b * S.C + blk * 16 + i) * S.HW + pc));
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  if (acc == 12345.678f) a.sink[0] = acc;
}

__global__ void fill(float* p, size_t n, unsigned seed) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (float)(h & 0xffff) * (1.0f / 65536.0f) - 0.25f;
  }
}
__global__ __launch_bounds__(256) void copy_flat(const f4v* __restrict__ x, f4v* __restrict__ y, size_t n4) {
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
__global__ __launch_bounds__(256) void read_flat(const f4v* __restrict__ x, size_t n4, float* out) {
  float s = 0.0f;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const f4v a = __builtin_nontemporal_load(x + i), b = __builtin_nontemporal_load(x + i + stride);
    const f4v c = __builtin_nontemporal_load(x + i + 2 * stride), d = __builtin_nontemporal_load(x + i + 3 * stride);
    s += (a.x + a.y + a.z + a.w) + (b.x + b.y + b.z + b.w) + (c.x + c.y + c.z + c.w) + (d.x + d.y + d.z + d.w);
  }
  for (; i < n4; i += stride) { const f4v a = x[i]; s += a.x + a.y + a.z + a.w; }
  if (s == 12345.678f) out[0] = s;
}

static hipEvent_t e0, e1;
static float med(std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }
static float el() { float ms; CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1)); return ms * 1e3f; }

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int B = 32, NB = 4;
  const int Cs[3] = {64, 128, 256}, HWs[3] = {6400, 1600, 400};
  size_t per = 0;
  for (int i = 0; i < 3; ++i) per += (size_t)B * Cs[i] * HWs[i];
  float *X[NB], *Y[NB], *sink;
  for (int k = 0; k < NB; ++k) {
    CK(hipMalloc(&X[k], per * 4)); CK(hipMalloc(&Y[k], per * 4));
    fill<<<4096, 256>>>(X[k], per, 11u * k + 1); fill<<<4096, 256>>>(Y[k], per, 7u * k + 5);
  }
  CK(hipMalloc(&sink, 64));
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipDeviceSynchronize());
  const double MB = per * 4.0 / 1e6;
  printf("x per batch %.2f MB\n", MB);
  const int reps = 40;
  auto run = [&](const char* name, double bytes, auto launch) {
    std::vector<float> t;
    for (int r = 0; r < reps + 4; ++r) { launch(r % NB); const float us = el(); if (r >= 4) t.push_back(us); }
    const float m = med(t);
    printf("%-52s %7.2f us  %7.1f GB/s\n", name, m, bytes / (m * 1e-6) / 1e9);
  };
  run("copy flat grid-stride (16384 wg)", 2 * MB * 1e6, [&](int k) {
    hipExtLaunchKernelGGL(copy_flat, dim3(16384), dim3(256), 0, 0, e0, e1, 0, (const f4v*)X[k], (f4v*)Y[k], per / 4); });
  run("read flat grid-stride nt (8192 wg)", MB * 1e6, [&](int k) {
    hipExtLaunchKernelGGL(read_flat, dim3(8192), dim3(256), 0, 0, e0, e1, 0, (const f4v*)X[k], per / 4, sink); });
  auto mkargs = [&](int k, int P, int S, int order, bool read) {
    Args a{};
    size_t off = 0;
    int units = 0;
    for (int i = 0; i < 3; ++i) {
      a.s[i].x = X[k] + off; a.s[i].y = Y[k] + off; a.s[i].C = Cs[i]; a.s[i].HW = HWs[i];
      const int upi = (HWs[i] + P - 1) / P;
      const int nsl = read ? 1 : (Cs[i] + S - 1) / S;
      a.s[i].units = B * upi * nsl; a.s[i].begin = units; units += a.s[i].units;
      off += (size_t)B * Cs[i] * HWs[i];
    }
    a.P = P; a.S = S; a.order = order; a.nscales = 3; a.units = units; a.sink = sink;
    return a;
  };
  const int PS[4][2] = {{256, 32}, {512, 16}, {1024, 8}, {256, 16}};
  for (int order = 0; order < 2; ++order)
    for (int q = 0; q < 4; ++q) {
      const int P = PS[q][0], S = PS[q][1];
      char nm[96];
      snprintf(nm, sizeof nm, "copy units P=%d S=%d order %s", P, S, order ? "sc" : "cs");
      run(nm, 2 * MB * 1e6, [&](int k) {
        Args a = mkargs(k, P, S, order, false);
        const int rpw = (P / 256) * (S / 4);
        if (rpw == 8) hipExtLaunchKernelGGL(copy_units<8>, dim3(a.units), dim3(256), 0, 0, e0, e1, 0, a);
        else hipExtLaunchKernelGGL(copy_units<4>, dim3(a.units), dim3(256), 0, 0, e0, e1, 0, a);
      });
    }
  for (int P : {256, 512, 1024}) {
    char nm[96];
    snprintf(nm, sizeof nm, "read units P=%d (16-row blocks)", P);
    run(nm, MB * 1e6, [&](int k) {
      Args a = mkargs(k, P, 0, 0, true);
      hipExtLaunchKernelGGL(read_units, dim3(a.units), dim3(256), 0, 0, e0, e1, 0, a);
    });
  }
  run("read units split (256 px x 64 ch, 1 round)", MB * 1e6, [&](int k) {
    Args a = mkargs(k, 256, 0, 0, true);
    int units = 0;
    for (int i = 0; i < 3; ++i) { a.s[i].units = B * ((HWs[i] + 255) / 256) * (Cs[i] / 64); a.s[i].begin = units; units += a.s[i].units; }
    a.units = units;
    hipExtLaunchKernelGGL(read_units_split, dim3(units), dim3(256), 0, 0, e0, e1, 0, a);
  });
  return 0;
}
