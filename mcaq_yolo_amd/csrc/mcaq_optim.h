// mcaq_optim.h - the optimizer end of the QAT training step in TWO launches:
// global gradient-norm clip (torch.nn.utils.clip_grad_norm_), AdamW with
// decoupled weight decay (torch.optim.AdamW) and the |W| projection of the
// bit mapper (bit_allocation.py:186-197, Eq. 18) - train.py:626-641 issues
// them as ~14 small ATen / multi-tensor kernels per step on ~8 k floats of
// hook parameters.
//
// Both launches cut the flat concatenation of the segments (parameter
// tensors) into 1,024-element chunks, one 256-thread workgroup each, 4
// consecutive elements a thread.  Launch 1: every chunk's squared gradients
// staged in LDS, each segment's part summed by one wave in element order ->
// work[chunk][segment].  Launch 2: every workgroup folds those partials in
// chunk order into the per-tensor squared norms, combines them in tensor
// order into the total norm (the norm of the per-tensor norms, as
// clip_grad_norm_ computes it) and the clip coefficient, then updates its
// chunk: torch's fused AdamW arithmetic (double hyper-parameters) and |W|.
// The norm reduces in another order than ATen's, so the values agree with
// torch's clip + fused AdamW within fp32 rounding (tests/test_optim_gpu.py),
// not bit for bit.  (Round 5 first ran both phases in ONE 1,024-thread
// workgroup: 25 us in the graph; two launches over ~9 workgroups each take
// less: the per-chunk work is one load round trip, not eight.)
#pragma once

namespace mcaq {

static_assert(sizeof(mcaq_adamw_seg) * MCAQ_OPT_MAXSEG + 64 <= 4096, "optimizer kernel arguments exceed 4 KiB");

struct AdamwArgs {
  mcaq_adamw_seg s[MCAQ_OPT_MAXSEG];
  const mcaq_adamw_group* g;   // device table, read at run time (a captured step follows lr changes)
  int nseg, ngroups;
  float* steps;        // device per-parameter step counters (float, like torch's capturable AdamW)
  float max_norm;      // <= 0: no clipping
  float* total_norm;   // or nullptr
};

constexpr int OPT_TH = 256;
constexpr int OPT_E = 4;                    // consecutive elements per thread
constexpr int OPT_CH = OPT_TH * OPT_E;      // elements per chunk (one workgroup)
constexpr int OPT_WORK0 = MCAQ_OPT_MAXSEG;  // work[k < nseg]: segment k's step after this one; partials from here

// beta^step for an integer-valued step by binary exponentiation in double (a
// few multiplies instead of the library pow; within an ulp or two of pow)
__device__ __forceinline__ double pow_int(double b, float step) {
  long long e = (long long)step;
  double r = 1.0;
  while (e > 0) {
    if (e & 1) r *= b;
    b *= b;
    e >>= 1;
  }
  return r;
}

// the segment table into LDS (a dword per thread, from the kernel argument
// through a pointer: no per-lane indexing of the argument) and the segments'
// first flat elements (exclusive scan of the sizes over wave 0)
__device__ __forceinline__ void opt_table(const AdamwArgs& a, mcaq_adamw_seg* sg, int* st) {
  const int tid = (int)threadIdx.x, nseg = a.nseg;
  constexpr int SW = (int)(sizeof(mcaq_adamw_seg) / 4);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&a.s[0]);
  for (int i = tid; i < nseg * SW; i += OPT_TH) reinterpret_cast<uint32_t*>(sg)[i] = src[i];
  __syncthreads();
  if (tid < 64) {
    int carry = 0;
    for (int k0 = 0; k0 < nseg; k0 += 64) {
      const int k = k0 + tid;
      const int nk = k < nseg ? sg[k].n : 0;
      int incl = nk;
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (tid >= o) incl += t;
      }
      if (k < nseg) st[k] = carry + incl - nk;
      carry += __shfl(incl, 63, 64);
    }
    if (tid == 0) st[nseg] = carry;
  }
  __syncthreads();
}

// the segment holding flat element j (binary search over the starts)
__device__ __forceinline__ int opt_seg_of(const int* st, int nseg, int j) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (st[mid] <= j) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// launch 1: this chunk's squared-gradient sum of every segment (0 where the
// segment does not overlap the chunk) -> work[OPT_WORK0 + chunk * nseg + k]
__global__ __launch_bounds__(OPT_TH) void mcaq_adamw_norm_kernel(AdamwArgs a, float* work) {
  __shared__ mcaq_adamw_seg sg[MCAQ_OPT_MAXSEG];
  __shared__ int st[MCAQ_OPT_MAXSEG + 1];
  __shared__ float sq[OPT_CH];
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nseg = a.nseg;
  opt_table(a, sg, st);
  const int total = st[nseg];
  const int base = (int)blockIdx.x * OPT_CH, e0 = base + tid * OPT_E;
  int k = opt_seg_of(st, nseg, imin_(e0, total - 1));
  float v[OPT_E];
#pragma unroll
  for (int q = 0; q < OPT_E; ++q) {
    const int j = imin_(e0 + q, total - 1);
    while (k + 1 < nseg && j >= st[k + 1]) ++k;
    v[q] = sg[k].grad[j - st[k]];
  }
#pragma unroll
  for (int q = 0; q < OPT_E; ++q) sq[tid * OPT_E + q] = e0 + q < total ? v[q] * v[q] : 0.0f;
  __syncthreads();
  float* out = work + OPT_WORK0 + (size_t)blockIdx.x * nseg;
  for (int kk = wv; kk < nseg; kk += OPT_TH / 64) {
    const int lo = imax_(st[kk], base), hi = imin_(st[kk + 1], base + OPT_CH);
    float acc = 0.0f;
    if (lo < hi) {
      // four independent partial sums per lane (fixed order), then the wave
      float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
      int i = lo + lane;
      for (; i + 192 < hi; i += 256) {
        a0 += sq[i - base]; a1 += sq[i + 64 - base]; a2 += sq[i + 128 - base]; a3 += sq[i + 192 - base];
      }
      for (; i < hi; i += 64) a0 += sq[i - base];
      acc = (a0 + a1) + (a2 + a3);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    }
    if (lane == 0) out[kk] = acc;
  }
  if (blockIdx.x == 0 && tid < nseg) work[tid] = a.steps[sg[tid].step_idx] + 1.0f;
}

// launch 2: the clip coefficient from launch 1's partials (every workgroup
// the same, in the same order), then AdamW and |W| on this chunk
__global__ __launch_bounds__(OPT_TH) void mcaq_adamw_update_kernel(AdamwArgs a, const float* work, int nchunk) {
  __shared__ mcaq_adamw_seg sg[MCAQ_OPT_MAXSEG];
  __shared__ int st[MCAQ_OPT_MAXSEG + 1];
  __shared__ float seg_acc[MCAQ_OPT_MAXSEG];
  __shared__ float coef_s;
  __shared__ float s_bc2s[MCAQ_OPT_MAXSEG], s_ss[MCAQ_OPT_MAXSEG];
  __shared__ double g_hp[MCAQ_OPT_MAXGROUPS][7];   // lr * wd, beta1, 1 - beta1, beta2, 1 - beta2, eps, lr
  const int tid = (int)threadIdx.x;
  const int nseg = a.nseg;
  const bool clip = a.max_norm > 0.0f;
  // per-tensor squared norms: the chunks' partials in chunk order, 8 loads
  // of a thread in flight (clamped index)
  if (clip && tid < nseg) {
    const float* pk = work + OPT_WORK0 + tid;
    float s = 0.0f;
    for (int w0 = 0; w0 < nchunk; w0 += 8) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = pk[(size_t)imin_(w0 + r, nchunk - 1) * nseg];
#pragma unroll
      for (int r = 0; r < 8; ++r) s = w0 + r < nchunk ? s + v[r] : s;
    }
    seg_acc[tid] = s;
  }
  if (tid < a.ngroups) {
    // the hyper-parameter table as the host last wrote it
    const mcaq_adamw_group G = a.g[tid];
    g_hp[tid][0] = G.lr * G.weight_decay;
    g_hp[tid][1] = G.beta1; g_hp[tid][2] = 1.0 - G.beta1;
    g_hp[tid][3] = G.beta2; g_hp[tid][4] = 1.0 - G.beta2;
    g_hp[tid][5] = G.eps; g_hp[tid][6] = G.lr;
  }
  opt_table(a, sg, st);    // (its barriers also publish seg_acc and the group table)
  if (tid >= 64 && tid < 64 + nseg) {
    // bias corrections of each parameter at its own step (fused AdamW: fp32
    // values of the double expressions; torch keeps a step per parameter)
    const int k = tid - 64;
    const float step = work[k];
    const double* hp = g_hp[sg[k].group];
    const float bc1 = (float)(1.0 - pow_int(hp[1], step));
    s_bc2s[k] = sqrtf((float)(1.0 - pow_int(hp[3], step)));
    s_ss[k] = (float)(hp[6] / (double)bc1);
    if (blockIdx.x == 0) a.steps[sg[k].step_idx] = step;   // every workgroup reads the steps from work
  }
  if (clip) {
    if (tid < 64) {
      // the norm of the per-tensor norms (clip_grad_norm_): squares of the
      // tensor norms summed over the wave (fixed tree)
      float t2 = 0.0f;
      for (int k = tid; k < nseg; k += 64) {
        const float nk = sqrtf(seg_acc[k]);
        t2 = fmaf(nk, nk, t2);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) t2 += __shfl_xor(t2, o, 64);
      const float tot = sqrtf(t2);
      if (tid == 0) {
        if (a.total_norm && blockIdx.x == 0) a.total_norm[0] = tot;
        const float c = a.max_norm / (tot + 1e-6f);
        coef_s = c < 1.0f ? c : 1.0f;   // clamp(max=1.0); NaN propagates as in torch
        if (!(c == c)) coef_s = c;
      }
    }
  } else if (tid == 0) {
    coef_s = 1.0f;
  }
  __syncthreads();
  const float coef = coef_s;
  const int total = st[nseg];
  // ---- AdamW per element, then |W|.  The arithmetic of torch's
  // _fused_adamw_ (adam_math, fused_adam_utils.cuh): hyper-parameters are
  // doubles, so the weight decay and both moment updates are evaluated in
  // double and rounded once to fp32 (an fp32 1 - beta2 alone is 1.3e-5 off);
  // step size and denominator are fp32 values, the final update fp32.
  // A thread loads its 4 elements' gradient, parameter and moments first.
  const int e0 = (int)blockIdx.x * OPT_CH + tid * OPT_E;
  if (e0 < total) {
    int k = opt_seg_of(st, nseg, e0);
    int ks[OPT_E];
    float gv[OPT_E], pv[OPT_E], mv[OPT_E], vv[OPT_E];
#pragma unroll
    for (int q = 0; q < OPT_E; ++q) {
      const int j = e0 + q < total ? e0 + q : total - 1;
      while (k + 1 < nseg && j >= st[k + 1]) ++k;
      ks[q] = k;
      const mcaq_adamw_seg& S = sg[k];
      const int e = j - st[k];
      gv[q] = S.grad[e]; pv[q] = S.param[e]; mv[q] = S.exp_avg[e]; vv[q] = S.exp_avg_sq[e];
    }
#pragma unroll
    for (int q = 0; q < OPT_E; ++q) {
      const int j = e0 + q;
      if (j >= total) break;
      const mcaq_adamw_seg& S = sg[ks[q]];
      const int e = j - st[ks[q]];
      const int gi = S.group;
      const double* hp = g_hp[gi];
      float g = gv[q];
      if (clip) {
        g = g * coef;
        S.grad[e] = g;             // clip_grad_norm_ scales .grad in place
      }
      float p = pv[q];
      p = (float)((double)p - hp[0] * (double)p);
      const float m = (float)(hp[1] * (double)mv[q] + hp[2] * (double)g);
      const float v = (float)(hp[3] * (double)vv[q] + hp[4] * (double)g * (double)g);
      const float denom = (float)((double)(sqrtf(v) / s_bc2s[ks[q]]) + hp[5]);
      p = p - s_ss[ks[q]] * m / denom;
      if (S.project_abs) p = fabsf(p);
      S.exp_avg[e] = m;
      S.exp_avg_sq[e] = v;
      S.param[e] = p;
    }
  }
}

// ---- ONE launch (round 6): the same two phases, the chunks' squared-norm
// partials exchanged inside the launch as write-through granules (the data is
// the flag: mcaq_train.h mapx_*, cdna_hip_programming.md s.6 Guideline 16
// R2) instead of through a launch boundary; each thread keeps its elements'
// gradient, parameter and moments in registers from the first phase to the
// update.  The arithmetic and its order are the two launches', so the
// results are bit-identical.  Sync buffer: word 0 the epoch, word 1 the
// status (nonzero after a timed-out exchange), granules from byte 256
// (chunk-major, nseg per chunk).  Every workgroup must be resident at once:
// at most OPT_FUSED_MAX_CHUNKS chunks.
constexpr int OPT_FUSED_MAX_CHUNKS = 256;
constexpr int OPT_SYNC_HDR = 64;   // header words

__global__ __launch_bounds__(OPT_TH) void mcaq_adamw_fused_kernel(AdamwArgs a, unsigned* sync, int nchunk) {
  __shared__ mcaq_adamw_seg sg[MCAQ_OPT_MAXSEG];
  __shared__ int st[MCAQ_OPT_MAXSEG + 1];
  __shared__ float sq[OPT_CH];
  __shared__ float seg_acc[MCAQ_OPT_MAXSEG];
  __shared__ float s_step[MCAQ_OPT_MAXSEG];
  __shared__ float coef_s;
  __shared__ float s_bc2s[MCAQ_OPT_MAXSEG], s_ss[MCAQ_OPT_MAXSEG];
  __shared__ double g_hp[MCAQ_OPT_MAXGROUPS][7];
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nseg = a.nseg;
  mapx_t* const gran = reinterpret_cast<mapx_t*>(sync + OPT_SYNC_HDR);
  const unsigned tag = __builtin_amdgcn_readfirstlane(
                           __hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  if (tid < a.ngroups) {
    const mcaq_adamw_group G = a.g[tid];
    g_hp[tid][0] = G.lr * G.weight_decay;
    g_hp[tid][1] = G.beta1; g_hp[tid][2] = 1.0 - G.beta1;
    g_hp[tid][3] = G.beta2; g_hp[tid][4] = 1.0 - G.beta2;
    g_hp[tid][5] = G.eps; g_hp[tid][6] = G.lr;
  }
  opt_table(a, sg, st);
  const int total = st[nseg];
  const int base = (int)blockIdx.x * OPT_CH, e0 = base + tid * OPT_E;
  // this thread's elements, loaded once for both phases
  int k = opt_seg_of(st, nseg, imin_(e0, total - 1));
  int ks[OPT_E];
  float gv[OPT_E], pv[OPT_E], mv[OPT_E], vv[OPT_E];
#pragma unroll
  for (int q = 0; q < OPT_E; ++q) {
    const int j = imin_(e0 + q, total - 1);
    while (k + 1 < nseg && j >= st[k + 1]) ++k;
    ks[q] = k;
    const mcaq_adamw_seg& S = sg[k];
    const int e = j - st[k];
    gv[q] = S.grad[e]; pv[q] = S.param[e]; mv[q] = S.exp_avg[e]; vv[q] = S.exp_avg_sq[e];
  }
  if (tid >= 64 && tid < 64 + nseg) {
    // this step's count and bias corrections (read before this workgroup
    // publishes: workgroup 0 writes the counts back after its sweep)
    const int kk = tid - 64;
    const float step = a.steps[sg[kk].step_idx] + 1.0f;
    const double* hp = g_hp[sg[kk].group];
    const float bc1 = (float)(1.0 - pow_int(hp[1], step));
    s_bc2s[kk] = sqrtf((float)(1.0 - pow_int(hp[3], step)));
    s_ss[kk] = (float)(hp[6] / (double)bc1);
    s_step[kk] = step;
  }
#pragma unroll
  for (int q = 0; q < OPT_E; ++q) sq[tid * OPT_E + q] = e0 + q < total ? gv[q] * gv[q] : 0.0f;
  __syncthreads();
  // phase 1: this chunk's squared sum of every segment, published
  for (int kk = wv; kk < nseg; kk += OPT_TH / 64) {
    const int lo = imax_(st[kk], base), hi = imin_(st[kk + 1], base + OPT_CH);
    float acc = 0.0f;
    if (lo < hi) {
      float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
      int i = lo + lane;
      for (; i + 192 < hi; i += 256) {
        a0 += sq[i - base]; a1 += sq[i + 64 - base]; a2 += sq[i + 128 - base]; a3 += sq[i + 192 - base];
      }
      for (; i < hi; i += 64) a0 += sq[i - base];
      acc = (a0 + a1) + (a2 + a3);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    }
    if (lane == 0) mapx_put(gran + (size_t)blockIdx.x * nseg + kk, tag, acc);
  }
  // phase 2: per-tensor squared norms, every chunk's partial in chunk order
  if (tid < nseg) {
    float s = 0.0f;
    for (int w0 = 0; w0 < nchunk; w0 += 8) {
      mapx_t* gp[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) gp[r] = gran + (size_t)imin_(w0 + r, nchunk - 1) * nseg + tid;
      float v[8];
      mapx_get<8>(gp, tag, v, sync + 1);
#pragma unroll
      for (int r = 0; r < 8; ++r) s = w0 + r < nchunk ? s + v[r] : s;
    }
    seg_acc[tid] = s;
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    // every workgroup has published, so every workgroup has read the counts
    // and the epoch: the counts advance, the next launch takes the next epoch
    if (tid < nseg) a.steps[sg[tid].step_idx] = s_step[tid];
    if (tid == 0) __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid < 64) {
    float t2 = 0.0f;
    for (int kk = tid; kk < nseg; kk += 64) {
      const float nk = sqrtf(seg_acc[kk]);
      t2 = fmaf(nk, nk, t2);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t2 += __shfl_xor(t2, o, 64);
    const float tot = sqrtf(t2);
    if (tid == 0) {
      if (a.total_norm && blockIdx.x == 0) a.total_norm[0] = tot;
      const float c = a.max_norm / (tot + 1e-6f);
      coef_s = c < 1.0f ? c : 1.0f;
      if (!(c == c)) coef_s = c;
    }
  }
  __syncthreads();
  const float coef = coef_s;
  if (e0 < total) {
#pragma unroll
    for (int q = 0; q < OPT_E; ++q) {
      const int j = e0 + q;
      if (j >= total) break;
      const mcaq_adamw_seg& S = sg[ks[q]];
      const int e = j - st[ks[q]];
      const double* hp = g_hp[S.group];
      float g = gv[q] * coef;
      S.grad[e] = g;
      float p = pv[q];
      p = (float)((double)p - hp[0] * (double)p);
      const float m = (float)(hp[1] * (double)mv[q] + hp[2] * (double)g);
      const float v = (float)(hp[3] * (double)vv[q] + hp[4] * (double)g * (double)g);
      const float denom = (float)((double)(sqrtf(v) / s_bc2s[ks[q]]) + hp[5]);
      p = p - s_ss[ks[q]] * m / denom;
      if (S.project_abs) p = fabsf(p);
      S.exp_avg[e] = m;
      S.exp_avg_sq[e] = v;
      S.param[e] = p;
    }
  }
}

}  // namespace mcaq

extern "C" {

size_t mcaq_clip_adamw_sync_bytes(int total, int nseg) {
  using namespace mcaq;
  if (total < 1 || nseg < 1) return 0;
  return (size_t)OPT_SYNC_HDR * 4 + (size_t)((total + OPT_CH - 1) / OPT_CH) * nseg * 8;
}

int mcaq_clip_adamw_fused(const mcaq_adamw_seg* segs, int nseg, const mcaq_adamw_group* groups, int ngroups,
                          float* steps, float max_norm, float* total_norm, void* sync, size_t sync_bytes,
                          hipStream_t stream) {
  using namespace mcaq;
  if (!segs || !groups || !steps || !sync || nseg < 1 || nseg > MCAQ_OPT_MAXSEG || ngroups < 1 ||
      ngroups > MCAQ_OPT_MAXGROUPS || !(max_norm > 0.0f) || ((uintptr_t)sync & 7) != 0)
    return (int)hipErrorInvalidValue;
  AdamwArgs a{};
  long long total = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_adamw_seg& g = segs[k];
    if (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq || g.n < 1 || g.group < 0 || g.group >= ngroups ||
        g.step_idx < 0)
      return (int)hipErrorInvalidValue;
    for (int j = 0; j < k; ++j)
      if (segs[j].step_idx == g.step_idx) return (int)hipErrorInvalidValue;
    a.s[k] = g;
    total += g.n;
  }
  const long long nchunk = (total + OPT_CH - 1) / OPT_CH;
  if (nchunk > OPT_FUSED_MAX_CHUNKS || sync_bytes < mcaq_clip_adamw_sync_bytes((int)total, nseg))
    return (int)hipErrorInvalidValue;
  a.g = groups;
  a.ngroups = ngroups;
  a.nseg = nseg;
  a.steps = steps;
  a.max_norm = max_norm;
  a.total_norm = total_norm;
  hipLaunchKernelGGL(mcaq_adamw_fused_kernel, dim3((int)nchunk), dim3(OPT_TH), 0, stream, a,
                     static_cast<unsigned*>(sync), (int)nchunk);
  return (int)hipGetLastError();
}

size_t mcaq_clip_adamw_work_floats(int total) {
  return (size_t)mcaq::OPT_WORK0 + (size_t)((total + mcaq::OPT_CH - 1) / mcaq::OPT_CH) * MCAQ_OPT_MAXSEG;
}

int mcaq_clip_adamw(const mcaq_adamw_seg* segs, int nseg, const mcaq_adamw_group* groups, int ngroups,
                    float* steps, float max_norm, float* total_norm, float* work, hipStream_t stream) {
  using namespace mcaq;
  if (!segs || !groups || !steps || !work || nseg < 1 || nseg > MCAQ_OPT_MAXSEG || ngroups < 1 ||
      ngroups > MCAQ_OPT_MAXGROUPS)
    return (int)hipErrorInvalidValue;
  AdamwArgs a{};
  long long total = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_adamw_seg& g = segs[k];
    if (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq || g.n < 1 || g.group < 0 || g.group >= ngroups ||
        g.step_idx < 0)
      return (int)hipErrorInvalidValue;
    for (int j = 0; j < k; ++j)
      if (segs[j].step_idx == g.step_idx) return (int)hipErrorInvalidValue;   // one step counter per parameter
    a.s[k] = g;
    total += g.n;
  }
  if (total > (1LL << 30)) return (int)hipErrorInvalidValue;
  a.g = groups;
  a.ngroups = ngroups;
  a.nseg = nseg;
  a.steps = steps;
  a.max_norm = max_norm;
  a.total_norm = total_norm;
  const int nchunk = (int)((total + OPT_CH - 1) / OPT_CH);
  // launch 1 also writes work[0 .. nseg) (the next step counts) for launch 2
  hipLaunchKernelGGL(mcaq_adamw_norm_kernel, dim3(nchunk), dim3(OPT_TH), 0, stream, a, work);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(mcaq_adamw_update_kernel, dim3(nchunk), dim3(OPT_TH), 0, stream, a, (const float*)work, nchunk);
  return (int)hipGetLastError();
}

}  // extern "C"
