// mcaq_dp.h - the data-parallel QAT step's all-gather unpack (dist.shard_hooks).
//
// Batch-sharded training runs the bit mapper's train-mode BatchNorm layers
// (bit_allocation.py:126) over the GLOBAL batch of tiles: every rank
// all-gathers the mapper's inputs (and, riding along, its quantizers' batch
// channel min / max, quantization.py:319-353) ONCE, runs the mapper on the
// global batch - so its bits, batch statistics and running statistics are the
// single-process values bit for bit - and keeps its own slice.  The backward
// all-gathers the bits' gradients the same way.  all_gather_into_tensor
// leaves [rank][send buffer]; a hook scale's global batch is [scale][rank]
// (rank order = image order of the global batch).  This kernel does the
// transposition and the min / max over ranks in ONE launch.
#pragma once

namespace mcaq {

struct DpArgs {
  mcaq_dp_seg s[MCAQ_DP_MAXSEG];
  long long first[MCAQ_DP_MAXSEG + 1];   // first item of each segment (exclusive scan)
  int nseg, world, stride;
};

constexpr int DP_TH = 256;

__global__ __launch_bounds__(DP_TH) void mcaq_dp_unpack_kernel(const float* __restrict__ g, DpArgs a) {
  const long long total = a.first[a.nseg];
  for (long long i = (long long)blockIdx.x * DP_TH + threadIdx.x; i < total; i += (long long)gridDim.x * DP_TH) {
    int k = 0;
    while (k + 1 < a.nseg && i >= a.first[k + 1]) ++k;
    const mcaq_dp_seg& S = a.s[k];
    const long long j = i - a.first[k];
    if (S.mode == 0) {
      // item j = (rank r, element e) of this scale's global buffer
      const long long r = j / S.n, e = j - r * S.n;
      S.out[j] = g[r * a.stride + S.off + e];
    } else {
      float v = g[S.off + j];
      for (int r = 1; r < a.world; ++r) {
        const float u = g[(long long)r * a.stride + S.off + j];
        // NaN propagates, as the single-process amin / amax over the batch
        v = (u != u || v != v) ? __builtin_nanf("") : (S.mode == 1 ? fminf(v, u) : fmaxf(v, u));
      }
      S.out[j] = v;
    }
  }
}

}  // namespace mcaq

extern "C" {

int mcaq_dp_unpack(const float* g, int world, int stride, const mcaq_dp_seg* segs, int nseg, hipStream_t stream) {
  using namespace mcaq;
  if (!g || !segs || world < 1 || stride < 1 || nseg < 1 || nseg > MCAQ_DP_MAXSEG) return (int)hipErrorInvalidValue;
  DpArgs a{};
  a.nseg = nseg;
  a.world = world;
  a.stride = stride;
  long long t = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_dp_seg& s = segs[k];
    if (!s.out || s.n < 1 || s.off < 0 || (long long)s.off + s.n > stride || s.mode < 0 || s.mode > 2)
      return (int)hipErrorInvalidValue;
    a.s[k] = s;
    a.first[k] = t;
    t += s.mode == 0 ? (long long)world * s.n : (long long)s.n;
  }
  a.first[nseg] = t;
  const long long blocks = (t + DP_TH - 1) / DP_TH;
  hipLaunchKernelGGL(mcaq_dp_unpack_kernel, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(DP_TH), 0, stream,
                     g, a);
  return (int)hipGetLastError();
}

}  // extern "C"
