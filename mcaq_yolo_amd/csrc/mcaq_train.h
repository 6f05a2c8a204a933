// mcaq_train.h - train-mode (QAT, BASELINE config 5) tile networks of the
// hook as fused kernels, replacing ~700 small ATen kernels of autograd glue
// per step (r02 DESIGN s.8) (included by mcaq_kernels.hip; C ABI in
// include/mcaq_hip.h):
//
//   bit mapper, train mode (bit_allocation.py:218-280, 120-130):
//     z = [C, C^2, log1p C] -> 3 x (Linear, BatchNorm1d over the batch's
//     tiles, ReLU) -> Linear -> sigmoid -> b_min + (b_max - b_min) h, x T,
//     straight-through clamp (and round);  forward = 4 launches (one per
//     batch-statistics barrier), backward = 4 + 1 (parameter reduction)
//   analyzer head backward (morphology.py:81-97, 309-354, 959-968):
//     bilateral adjoint per image, then the complexity MLP (Linear-LN-ReLU x2,
//     Linear, sigmoid) recomputed and differentiated per tile
//   soft mask backward (quantization.py:213-239): 5x5 smoothing and nearest
//     upsample adjoints, softmax, 1x1 conv, ReLU, 3x3 conv (zero pad)
//
// Forward values of the analyzer and the soft mask stay those of the morph
// kernel (bit-exact with the reference); these kernels are fp32 with their
// own summation orders (train-mode gradients are tolerance-checked, DESIGN
// s.4).  Parameter gradients: every workgroup writes partial sums of its
// tiles; one reduction launch sums them in workgroup order (deterministic).
#pragma once

namespace mcaq {

// ---- shared helpers --------------------------------------------------------
constexpr int TR_TPB = 64;          // tiles per workgroup (one per lane of a wave)

__device__ __forceinline__ float tr_sigmoid(float a) { return 1.0f / (1.0f + expf(-a)); }

// sum over the 64 lanes of a wave (every lane gets the total)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Chan / Welford combination of per-workgroup (count, mean, M2) partials in
// workgroup order -> batch mean and biased variance
__device__ __forceinline__ void chan_combine(const float* part, int nwg, int stride, int j, int nfeat,
                                             const float* cnt, float& mean, float& var) {
  float n = 0.0f, m = 0.0f, M2 = 0.0f;
  for (int w = 0; w < nwg; ++w) {
    const float nb = cnt[w];
    if (nb <= 0.0f) continue;
    const float mb = part[(size_t)w * stride + j], M2b = part[(size_t)w * stride + nfeat + j];
    const float nn = n + nb;
    const float d = mb - m;
    m = m + d * (nb / nn);
    M2 = M2 + M2b + d * d * (n * nb / nn);
    n = nn;
  }
  mean = m;
  var = n > 0.0f ? M2 / n : 0.0f;
}

// ---- parameter-gradient reduction ------------------------------------------
// out[e] (+)= sum_w part[w * stride + e], e < count, w in order
__global__ __launch_bounds__(256) void mcaq_tr_reduce_kernel(const float* __restrict__ part, int nwg, int stride,
                                                             int count, float* __restrict__ out, int accumulate) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= count) return;
  float s = 0.0f;
  for (int w = 0; w < nwg; ++w) s += part[(size_t)w * stride + e];
  out[e] = accumulate ? out[e] + s : s;
}

// ============================================================================
// bit mapper, train mode
// ============================================================================
// gradient layout (flat, floats): the torch parameter order of mapping_network
enum : int {
  MG_W1 = 0, MG_B1 = 96, MG_G1 = 128, MG_BE1 = 160, MG_W2 = 192, MG_B2 = 2240, MG_G2 = 2304, MG_BE2 = 2368,
  MG_W3 = 2432, MG_B3 = 4480, MG_G3 = 4512, MG_BE3 = 4544, MG_W4 = 4576, MG_B4 = 4608, MG_SIZE = 4609
};

struct MapperTrainArgs {
  mcaq_mapper_params P;
  const float* c;       // (n) complexity
  const float* gbits;   // (n) upstream gradient of the bit map (backward)
  float* bits;          // (n) forward output
  float* gc;            // (n) gradient of c (backward)
  float* work;          // mcaq_mapper_work_floats(n)
  float* gpart;         // backward parameter partials [nwg][MG_SIZE]
  int n, nwg;
  float min_bits, max_bits, temperature, momentum;   // temperature <= 0: none
  int round_bits, update_stats;
};

// work layout (floats)
struct MapperWork {
  float *a1, *a2, *a3, *o, *gy;   // pre-BN activations (n x 32 / 64 / 32), sigmoid out, gradient scratch (n x 64)
  float *part, *cnt;              // per-workgroup (mean[64], M2[64]) and counts
  float *stat;                    // 3 layers x (mean[64], rstd[64])
  float *bpart;                   // backward BN partials [2][nwg][2 x 64]
  int nwg;
  __host__ __device__ float* fpart(int layer) const { return part + (size_t)(layer & 1) * nwg * 128; }
  __host__ __device__ float* bpart_of(int stage) const { return bpart + (size_t)(stage & 1) * nwg * 128; }
};
// part / bpart are double-buffered by layer parity: a launch reads the
// partials the previous launch wrote while writing its own
__host__ __device__ inline size_t mapper_work_floats(int n) {
  const int nwg = (n + TR_TPB - 1) / TR_TPB;
  return (size_t)n * (32 + 64 + 32 + 1 + 64) + (size_t)2 * nwg * 128 + nwg + 3 * 128 + (size_t)2 * nwg * 128 + 64;
}
__host__ __device__ inline MapperWork mapper_work(float* w, int n) {
  const int nwg = (n + TR_TPB - 1) / TR_TPB;
  MapperWork m;
  m.a1 = w; m.a2 = m.a1 + (size_t)n * 32; m.a3 = m.a2 + (size_t)n * 64; m.o = m.a3 + (size_t)n * 32;
  m.gy = m.o + n; m.part = m.gy + (size_t)n * 64; m.cnt = m.part + (size_t)2 * nwg * 128; m.stat = m.cnt + nwg;
  m.bpart = m.stat + 3 * 128;
  m.nwg = nwg;
  return m;
}

// layer input dims / output dims: L1 3->32, L2 32->64, L3 64->32, L4 32->1
template <int L> struct MapL;
template <> struct MapL<1> { enum { K = 3, N = 32 }; };
template <> struct MapL<2> { enum { K = 32, N = 64 }; };
template <> struct MapL<3> { enum { K = 64, N = 32 }; };
template <> struct MapL<4> { enum { K = 32, N = 1 }; };
template <> struct MapL<0> { enum { K = 1, N = 1 }; };

// BN layer parameters of layer L (1..3)
__device__ __forceinline__ void map_bn(const mcaq_mapper_params& P, int L, const float*& g, const float*& be, float*& rm,
                                       float*& rv, long long*& nbt) {
  g = L == 1 ? P.g1 : (L == 2 ? P.g2 : P.g3);
  be = L == 1 ? P.be1 : (L == 2 ? P.be2 : P.be3);
  rm = L == 1 ? P.rm1 : (L == 2 ? P.rm2 : P.rm3);
  rv = L == 1 ? P.rv1 : (L == 2 ? P.rv2 : P.rv3);
  nbt = L == 1 ? P.nbt1 : (L == 2 ? P.nbt2 : P.nbt3);
}

// per-workgroup (mean, M2) of feature j over this workgroup's valid tiles;
// 256 threads = 4 waves x 64 tiles, each wave one quarter of the features.
// v[f]: this lane's tile's value of feature f0 + f (f < NQ)
template <int NQ>
__device__ __forceinline__ void wg_moments(const float (&v)[NQ], bool valid, float nvalid, int f0, float* part, int nfeat) {
#pragma unroll
  for (int f = 0; f < NQ; ++f) {
    const float s = wave_sum(valid ? v[f] : 0.0f);
    const float mean = s / nvalid;
    const float d = valid ? v[f] - mean : 0.0f;
    const float M2 = wave_sum(d * d);
    if ((threadIdx.x & 63) == 0) { part[f0 + f] = mean; part[nfeat + f0 + f] = M2; }
  }
}

// batch statistics of layer L from the forward partials: mean, rstd for the
// thread's quarter of features (and, once per launch, the running-stats update)
template <int L>
__device__ void map_stats(const MapperTrainArgs& A, const MapperWork& W, float* s_mean, float* s_rstd) {
  constexpr int N = MapL<L>::N;
  const int tid = threadIdx.x;
  if (tid < N) {
    float mean, var;
    chan_combine(W.fpart(L), A.nwg, 128, tid, N, W.cnt, mean, var);
    const float rstd = 1.0f / sqrtf(var + 1e-5f);
    s_mean[tid] = mean; s_rstd[tid] = rstd;
    if (blockIdx.x == 0) {
      W.stat[(L - 1) * 128 + tid] = mean;
      W.stat[(L - 1) * 128 + 64 + tid] = rstd;
      if (A.update_stats) {
        const float* g; const float* be; float* rm; float* rv; long long* nbt;
        map_bn(A.P, L, g, be, rm, rv, nbt);
        const float nf = (float)A.n;
        const float unb = A.n > 1 ? var * (nf / (nf - 1.0f)) : var;
        rm[tid] = (1.0f - A.momentum) * rm[tid] + A.momentum * mean;
        rv[tid] = (1.0f - A.momentum) * rv[tid] + A.momentum * unb;
        if (tid == 0 && nbt) nbt[0] += 1;
      }
    }
  }
}

// stage S (1..4) of the train-mode forward
template <int S>
__global__ __launch_bounds__(256) void mcaq_mapper_fwd_kernel(MapperTrainArgs A) {
  __shared__ float s_in[TR_TPB][65];     // this workgroup's tiles' layer inputs
  __shared__ float s_mean[64], s_rstd[64];
  const MapperWork W = mapper_work(A.work, A.n);
  const mcaq_mapper_params& P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
  const int t = blockIdx.x * TR_TPB + lane;
  const bool valid = t < A.n;
  const int tc = valid ? t : A.n - 1;
  const float nvalid = (float)imin_(TR_TPB, A.n - (int)blockIdx.x * TR_TPB);
  if constexpr (S >= 2) map_stats<S - 1>(A, W, s_mean, s_rstd);
  // ---- layer inputs of this workgroup's tiles -> s_in
  if constexpr (S == 1) {
    if (q == 0) {
      const float c = clampf_(A.c[tc], 0.0f, 1.0f);
      s_in[lane][0] = c; s_in[lane][1] = c * c; s_in[lane][2] = log1pf(c);
    }
  }
  __syncthreads();
  if constexpr (S >= 2) {
    // h = relu(gamma (a - mean) rstd + beta) of the previous layer
    constexpr int KP = S == 2 ? 32 : (S == 3 ? 64 : 32);
    const float* aprev = S == 2 ? W.a1 : (S == 3 ? W.a2 : W.a3);
    const float* g = S == 2 ? P.g1 : (S == 3 ? P.g2 : P.g3);
    const float* be = S == 2 ? P.be1 : (S == 3 ? P.be2 : P.be3);
    for (int k = q; k < KP; k += 4) {
      const float a = aprev[(size_t)tc * KP + k];
      const float y = g[k] * ((a - s_mean[k]) * s_rstd[k]) + be[k];
      s_in[lane][k] = y > 0.0f ? y : 0.0f;
    }
    __syncthreads();
  }
  if constexpr (S <= 3) {
    constexpr int K = MapL<S>::K, N = MapL<S>::N, NQ = N / 4;
    const float* w = S == 1 ? P.w1 : (S == 2 ? P.w2 : P.w3);
    const float* bb = S == 1 ? P.b1 : (S == 2 ? P.b2 : P.b3);
    float* aout = S == 1 ? W.a1 : (S == 2 ? W.a2 : W.a3);
    float x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = s_in[lane][k];
    float o[NQ];
#pragma unroll
    for (int f = 0; f < NQ; ++f) {
      const int j = q * NQ + f;
      float acc = bb[j];
#pragma unroll
      for (int k = 0; k < K; ++k) acc = fmaf(w[j * K + k], x[k], acc);
      o[f] = acc;
      if (valid) aout[(size_t)t * N + j] = acc;
    }
    wg_moments<NQ>(o, valid, nvalid, q * NQ, W.fpart(S) + (size_t)blockIdx.x * 128, N);
    if (tid == 0) W.cnt[blockIdx.x] = nvalid;
  } else {
    // last layer + sigmoid + bit range, temperature, clamp (+ round)
    if (q == 0 && valid) {
      float acc = P.b4[0];
#pragma unroll 8
      for (int k = 0; k < 32; ++k) acc = fmaf(P.w4[k], s_in[lane][k], acc);
      const float o = tr_sigmoid(acc);
      W.o[t] = o;
      float bv = A.min_bits + (A.max_bits - A.min_bits) * o;
      if (A.temperature > 0.0f) bv = bv * A.temperature;
      bv = clampf_(bv, A.min_bits, A.max_bits);
      if (A.round_bits) bv = rintf(bv);
      A.bits[t] = bv;
    }
  }
}

// backward stage S (4, 3, 2, 1): gradient of layer S's output activation ->
// (BN S-1 backward inputs, weight partials of layer S)
//   S = 4: g_bits -> g_a4 -> g_h3 -> g_y3 (through ReLU), partials of W4 / b4
//          and of BN3 (sum g_y3, sum g_y3 xhat3)
//   S = 3, 2: g_y(S) + BN(S) sums -> g_a(S) -> W(S) / b(S) / BN(S) gamma-beta
//          partials, g_h(S-1) -> g_y(S-1), BN(S-1) partials
//   S = 1: g_y1 + BN1 sums -> g_a1 -> W1 / b1 partials, g_z -> g_c
template <int S>
__global__ __launch_bounds__(256) void mcaq_mapper_bwd_kernel(MapperTrainArgs A) {
  __shared__ float s_h[TR_TPB][65];     // this layer's input activations h(S-1)
  __shared__ float s_g[TR_TPB][65];     // gradient of this layer's pre-activation a(S)
  __shared__ float s_mean[64], s_rstd[64], s_sg[64], s_sgx[64];
  const MapperWork W = mapper_work(A.work, A.n);
  const mcaq_mapper_params& P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
  const int t = blockIdx.x * TR_TPB + lane;
  const bool valid = t < A.n;
  const int tc = valid ? t : A.n - 1;
  float* gp = A.gpart + (size_t)blockIdx.x * MG_SIZE;
  float* bp = W.bpart_of(S) + (size_t)blockIdx.x * 128;   // BN(S-1) partials written here
  // ---- 1. gradient of a(S) for this workgroup's tiles -> s_g
  if constexpr (S == 4) {
    if (q == 0) {
      float g = valid ? A.gbits[t] : 0.0f;   // straight-through round / clamp
      if (A.temperature > 0.0f) g = g * A.temperature;
      const float o = W.o[tc];
      s_g[lane][0] = valid ? (A.max_bits - A.min_bits) * g * (o * (1.0f - o)) : 0.0f;
    }
  } else {
    // BN(S) backward: g_a = gamma rstd (g_y - S1/n - xhat S2/n)
    constexpr int N = MapL<S>::N;
    const float* g = S == 1 ? P.g1 : (S == 2 ? P.g2 : P.g3);
    const float* aS = S == 1 ? W.a1 : (S == 2 ? W.a2 : W.a3);
    if (tid < N) {
      float s1 = 0.0f, s2 = 0.0f;
      const float* bq = W.bpart_of(S + 1);   // written by the previous launch (stage S + 1)
      for (int w = 0; w < A.nwg; ++w) { s1 += bq[(size_t)w * 128 + tid]; s2 += bq[(size_t)w * 128 + 64 + tid]; }
      s_sg[tid] = s1; s_sgx[tid] = s2;
      s_mean[tid] = W.stat[(S - 1) * 128 + tid]; s_rstd[tid] = W.stat[(S - 1) * 128 + 64 + tid];
      // gamma / beta gradients are the BN sums themselves: workgroup 0's
      // partial slot holds them, the others zero
      const int og = S == 1 ? MG_G1 : (S == 2 ? MG_G2 : MG_G3), ob = S == 1 ? MG_BE1 : (S == 2 ? MG_BE2 : MG_BE3);
      gp[og + tid] = blockIdx.x == 0 ? s2 : 0.0f;
      gp[ob + tid] = blockIdx.x == 0 ? s1 : 0.0f;
    }
    __syncthreads();
    const float inv_n = 1.0f / (float)A.n;
    for (int j = q; j < N; j += 4) {
      const float gy = W.gy[(size_t)tc * 64 + j];
      const float xh = (aS[(size_t)tc * N + j] - s_mean[j]) * s_rstd[j];
      s_g[lane][j] = valid ? g[j] * s_rstd[j] * (gy - s_sg[j] * inv_n - xh * (s_sgx[j] * inv_n)) : 0.0f;
    }
  }
  // ---- 2. this layer's input activations h(S-1) -> s_h
  constexpr int K = S == 4 ? 32 : (S == 1 ? 3 : MapL<S>::K);
  if constexpr (S == 1) {
    if (q == 0) {
      const float c = clampf_(A.c[tc], 0.0f, 1.0f);
      s_h[lane][0] = valid ? c : 0.0f; s_h[lane][1] = valid ? c * c : 0.0f; s_h[lane][2] = valid ? log1pf(c) : 0.0f;
    }
  } else {
    const float* ap = S == 4 ? W.a3 : (S == 3 ? W.a2 : W.a1);
    const float* g = S == 4 ? P.g3 : (S == 3 ? P.g2 : P.g1);
    const float* be = S == 4 ? P.be3 : (S == 3 ? P.be2 : P.be1);
    const int L = S - 1;
    for (int k = q; k < K; k += 4) {
      const float mean = W.stat[(L - 1) * 128 + k], rstd = W.stat[(L - 1) * 128 + 64 + k];
      const float y = g[k] * ((ap[(size_t)tc * K + k] - mean) * rstd) + be[k];
      s_h[lane][k] = valid && y > 0.0f ? y : 0.0f;
    }
  }
  __syncthreads();
  // ---- 3. weight / bias partials of layer S: sum over the tiles of g_a (x) h
  {
    constexpr int NO = S == 4 ? 1 : MapL<S>::N;
    const int ow = S == 4 ? MG_W4 : (S == 3 ? MG_W3 : (S == 2 ? MG_W2 : MG_W1));
    const int ob = S == 4 ? MG_B4 : (S == 3 ? MG_B3 : (S == 2 ? MG_B2 : MG_B1));
    for (int e = tid; e < NO * K; e += 256) {
      const int j = e / K, k = e - (e / K) * K;
      float s = 0.0f;
      for (int u = 0; u < TR_TPB; ++u) s = fmaf(s_g[u][j], s_h[u][k], s);
      gp[ow + e] = s;
    }
    for (int j = tid; j < NO; j += 256) {
      float s = 0.0f;
      for (int u = 0; u < TR_TPB; ++u) s += s_g[u][j];
      gp[ob + j] = s;
    }
  }
  // ---- 4. gradient of the layer input: g_h = W^T g_a, through ReLU / BN(S-1)
  if constexpr (S >= 2) {
    constexpr int NO = S == 4 ? 1 : MapL<S>::N;
    const float* w = S == 4 ? P.w4 : (S == 3 ? P.w3 : P.w2);
    const int L = S - 1;
    constexpr int NQ = K / 4;
    float gyv[NQ], xhv[NQ];
    const float* ap = S == 4 ? W.a3 : (S == 3 ? W.a2 : W.a1);
    const float* g = S == 4 ? P.g3 : (S == 3 ? P.g2 : P.g1);
    const float* be = S == 4 ? P.be3 : (S == 3 ? P.be2 : P.be1);
#pragma unroll
    for (int f = 0; f < NQ; ++f) {
      const int k = q * NQ + f;
      float acc = 0.0f;
      for (int j = 0; j < NO; ++j) acc = fmaf(w[j * K + k], s_g[lane][j], acc);
      const float mean = W.stat[(L - 1) * 128 + k], rstd = W.stat[(L - 1) * 128 + 64 + k];
      const float xh = (ap[(size_t)tc * K + k] - mean) * rstd;
      const float y = g[k] * xh + be[k];
      const float gy = (valid && y > 0.0f) ? acc : 0.0f;
      gyv[f] = gy; xhv[f] = xh;
      if (valid) W.gy[(size_t)t * 64 + k] = gy;
    }
    __syncthreads();   // every lane has read its W.gy row of this launch's input (S < 4) before it is overwritten
    // BN(S-1) partial sums: sum g_y, sum g_y xhat
#pragma unroll
    for (int f = 0; f < NQ; ++f) {
      const float s1 = wave_sum(gyv[f]), s2 = wave_sum(gyv[f] * xhv[f]);
      if (lane == 0) { bp[q * NQ + f] = s1; bp[64 + q * NQ + f] = s2; }
    }
  } else {
    // g_z = W1^T g_a1 -> g_c (through the clamp: torch passes the gradient on [0, 1])
    if (q == 0 && valid) {
      float g0 = 0.0f, g1 = 0.0f, g2 = 0.0f;
      for (int j = 0; j < 32; ++j) {
        const float ga = s_g[lane][j];
        g0 = fmaf(P.w1[j * 3 + 0], ga, g0); g1 = fmaf(P.w1[j * 3 + 1], ga, g1); g2 = fmaf(P.w1[j * 3 + 2], ga, g2);
      }
      const float craw = A.c[t];
      const float c = clampf_(craw, 0.0f, 1.0f);
      const float gcv = g0 + 2.0f * c * g1 + g2 / (1.0f + c);
      A.gc[t] = (craw >= 0.0f && craw <= 1.0f) ? gcv : 0.0f;
    }
  }
}

// ============================================================================
// analyzer head backward: clamp + bilateral adjoint (per image), complexity
// MLP backward (per tile)
// ============================================================================
// gradient layout: torch parameter order of complexity_mlp
enum : int {
  CG_W1 = 0, CG_B1 = 512, CG_G1 = 576, CG_BE1 = 640, CG_W2 = 704, CG_B2 = 2752, CG_G2 = 2784, CG_BE2 = 2816,
  CG_W3 = 2848, CG_B3 = 2880, CG_SIZE = 2881
};

struct HeadTrainArgs {
  mcaq_cmlp_params P;
  const float* phi;     // (n, 8)
  const float* craw;    // (n) complexity MLP output (before the bilateral)
  const float* gC;      // (n) gradient of C = clamp(bilateral(craw), 0, 1)
  float* gcraw;         // (n) work: gradient of craw
  float* gpart;         // [nwg][CG_SIZE]
  int B, ht, wt, n, nwg;
};

// bilateral (morphology.py:309-354, sigma_s 2, sigma_r 0.1, 5x5, replicate):
// C_t = N_t / D_t, N = sum_k w_k p_k, D = sum_k w_k + 1e-8,
// w_k = sp_k exp(-(p_k - c_t)^2 / 0.02), p_k = craw[clamp(t + o_k)].
// One workgroup per image: forward quantities per tile, then the adjoint
// gathered per tile u over every (t, k) with clamp(t + o_k) == u.
__global__ __launch_bounds__(256) void mcaq_bilateral_bwd_kernel(HeadTrainArgs A) {
  extern __shared__ float smem_tr[];
  const int b = blockIdx.x, ht = A.ht, wt = A.wt, NT = ht * wt;
  float* cr = smem_tr;            // craw of the image
  float* gd = cr + NT;            // per tile: g_C / D  (0 outside the clamp)
  float* gcen = gd + NT;          // per tile: sum_k gd (p_k - C) w_k (p_k - c)/0.01  (-> own craw)
  float* cc = gcen + NT;          // C before the clamp
  const float* crg = A.craw + (size_t)b * NT;
  for (int t = threadIdx.x; t < NT; t += 256) cr[t] = crg[t];
  __syncthreads();
  for (int t = threadIdx.x; t < NT; t += 256) {
    const int th = t / wt, tw = t - th * wt;
    const float c = cr[t];
    float num = 0.0f, den = 0.0f;
    for (int k = 0; k < 25; ++k) {
      const int hh = imin_(imax_(th + k / 5 - 2, 0), ht - 1), ww = imin_(imax_(tw + k % 5 - 2, 0), wt - 1);
      const float p = cr[hh * wt + ww];
      const float d = p - c;
      const float w = bits_as_float(k_bilat_sp_bits[k]) * expf(-(d * d) / 0.02f);
      num = fmaf(w, p, num);
      den += w;
    }
    den += 1e-8f;
    const float Cv = num / den;
    cc[t] = Cv;
    const float g = A.gC[(size_t)b * NT + t];
    gd[t] = (Cv >= 0.0f && Cv <= 1.0f) ? g / den : 0.0f;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < NT; t += 256) {
    const int th = t / wt, tw = t - th * wt;
    const float c = cr[t], Cv = cc[t], g = gd[t];
    float s = 0.0f;
    for (int k = 0; k < 25; ++k) {
      const int hh = imin_(imax_(th + k / 5 - 2, 0), ht - 1), ww = imin_(imax_(tw + k % 5 - 2, 0), wt - 1);
      const float p = cr[hh * wt + ww];
      const float d = p - c;
      const float w = bits_as_float(k_bilat_sp_bits[k]) * expf(-(d * d) / 0.02f);
      s = fmaf((p - Cv) * w, d / 0.01f, s);   // d C / d c_t through the range weights
    }
    gcen[t] = g * s;
  }
  __syncthreads();
  // adjoint gather: g_craw[u] = gcen[u] + sum over (t, k), clamp(t + o_k) = u, of
  //   gd_t (w_k + (p_k - C_t) w_k (-(p_k - c_t) / 0.01))
  for (int u = threadIdx.x; u < NT; u += 256) {
    const int uh = u / wt, uw = u - uh * wt;
    float s = gcen[u];
    for (int th = imax_(uh - 2, 0); th <= imin_(uh + 2, ht - 1); ++th) {
      for (int i = 0; i < 5; ++i) {
        if (imin_(imax_(th + i - 2, 0), ht - 1) != uh) continue;
        for (int tw = imax_(uw - 2, 0); tw <= imin_(uw + 2, wt - 1); ++tw) {
          const int t = th * wt + tw;
          const float c = cr[t], Cv = cc[t], g = gd[t];
          for (int j = 0; j < 5; ++j) {
            if (imin_(imax_(tw + j - 2, 0), wt - 1) != uw) continue;
            const float p = cr[u];
            const float d = p - c;
            const float w = bits_as_float(k_bilat_sp_bits[i * 5 + j]) * expf(-(d * d) / 0.02f);
            s = fmaf(g, w - (p - Cv) * w * (d / 0.01f), s);
          }
        }
      }
    }
    A.gcraw[(size_t)b * NT + u] = s;
  }
}

// complexity MLP backward, one tile per lane, 64 tiles per workgroup (one
// wave); the per-tile vectors meet in LDS and the weight partials are sums
// over the workgroup's tiles in tile order
__global__ __launch_bounds__(64) void mcaq_cmlp_bwd_kernel(HeadTrainArgs A) {
  extern __shared__ float smem_tr[];
  constexpr int ST = 8 + 64 + 64 + 32 + 32 + 64 + 64 + 32 + 32 + 1;   // per-tile vector floats
  float* sv = smem_tr;                       // [TR_TPB][ST + 1]
  const mcaq_cmlp_params& P = A.P;
  const int lane = threadIdx.x;
  const int t = blockIdx.x * TR_TPB + lane;
  const bool valid = t < A.n;
  const int tc = valid ? t : A.n - 1;
  float* v = sv + lane * (ST + 1);
  float* phi = v;                 // 8
  float* r1 = phi + 8;            // 64
  float* ga1 = r1 + 64;           // 64
  float* r2 = ga1 + 64;           // 32
  float* ga2 = r2 + 32;           // 32
  float* gyx1 = ga2 + 32;         // 64
  float* gy1 = gyx1 + 64;         // 64
  float* gyx2 = gy1 + 64;         // 32
  float* gy2 = gyx2 + 32;         // 32
  float* ga3 = gy2 + 32;          // 1
  {
    float ph[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { ph[k] = A.phi[(size_t)tc * 8 + k]; phi[k] = ph[k]; }
    // ---- forward recompute
    float a1[64];
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      float acc = P.b1[j];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = fmaf(P.w1[j * 8 + k], ph[k], acc);
      a1[j] = acc;
      s += acc;
    }
    const float mu1 = s / 64.0f;
    float vs = 0.0f;
#pragma unroll
    for (int j = 0; j < 64; ++j) { const float d = a1[j] - mu1; vs = fmaf(d, d, vs); }
    const float rs1 = 1.0f / sqrtf(vs / 64.0f + 1e-5f);
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      a1[j] = (a1[j] - mu1) * rs1;                      // xhat1
      const float y = P.g1[j] * a1[j] + P.be1[j];
      r1[j] = y > 0.0f ? y : 0.0f;
    }
    float a2[32];
    s = 0.0f;
    for (int j = 0; j < 32; ++j) {
      float acc = P.b2[j];
      for (int k = 0; k < 64; ++k) acc = fmaf(P.w2[j * 64 + k], r1[k], acc);
      a2[j] = acc;
      s += acc;
    }
    const float mu2 = s / 32.0f;
    vs = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) { const float d = a2[j] - mu2; vs = fmaf(d, d, vs); }
    const float rs2 = 1.0f / sqrtf(vs / 32.0f + 1e-5f);
    float a3 = P.b3[0];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      a2[j] = (a2[j] - mu2) * rs2;                      // xhat2
      const float y = P.g2[j] * a2[j] + P.be2[j];
      r2[j] = y > 0.0f ? y : 0.0f;
      a3 = fmaf(P.w3[j], r2[j], a3);
    }
    const float cv = tr_sigmoid(a3);
    // ---- backward
    const float g3 = valid ? A.gcraw[t] * (cv * (1.0f - cv)) : 0.0f;
    ga3[0] = g3;
    float gx2[32];
    float m1 = 0.0f, m2 = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const float y = P.g2[j] * a2[j] + P.be2[j];
      const float gy = y > 0.0f ? P.w3[j] * g3 : 0.0f;
      gy2[j] = gy; gyx2[j] = gy * a2[j];
      gx2[j] = gy * P.g2[j];
      m1 += gx2[j]; m2 = fmaf(gx2[j], a2[j], m2);
    }
    m1 /= 32.0f; m2 /= 32.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) ga2[j] = rs2 * (gx2[j] - m1 - a2[j] * m2);
    float gx1[64];
    m1 = 0.0f; m2 = 0.0f;
    for (int k = 0; k < 64; ++k) {
      float acc = 0.0f;
      for (int j = 0; j < 32; ++j) acc = fmaf(P.w2[j * 64 + k], ga2[j], acc);
      const float y = P.g1[k] * a1[k] + P.be1[k];
      const float gy = y > 0.0f ? acc : 0.0f;
      gy1[k] = gy; gyx1[k] = gy * a1[k];
      gx1[k] = gy * P.g1[k];
      m1 += gx1[k]; m2 = fmaf(gx1[k], a1[k], m2);
    }
    m1 /= 64.0f; m2 /= 64.0f;
    for (int k = 0; k < 64; ++k) ga1[k] = rs1 * (gx1[k] - m1 - a1[k] * m2);
  }
  __syncthreads();
  // ---- weight partials: sums over the workgroup's tiles (invalid lanes hold zeros
  // in ga*, gy*, gyx* because their upstream gradient is zero)
  float* gp = A.gpart + (size_t)blockIdx.x * CG_SIZE;
  const int nt = TR_TPB;
  auto tv = [&](int u) { return sv + u * (ST + 1); };
  for (int e = lane; e < CG_SIZE; e += 64) {
    float s = 0.0f;
    if (e < CG_B1) {                       // W1 (64 x 8): ga1 (x) phi
      const int j = e >> 3, k = e & 7;
      for (int u = 0; u < nt; ++u) s = fmaf(tv(u)[72 + j], tv(u)[k], s);
    } else if (e < CG_G1) {                // b1
      const int j = e - CG_B1;
      for (int u = 0; u < nt; ++u) s += tv(u)[72 + j];
    } else if (e < CG_BE1) {               // LN1 gamma
      const int j = e - CG_G1;
      for (int u = 0; u < nt; ++u) s += tv(u)[200 + j];
    } else if (e < CG_W2) {                // LN1 beta
      const int j = e - CG_BE1;
      for (int u = 0; u < nt; ++u) s += tv(u)[264 + j];
    } else if (e < CG_B2) {                // W2 (32 x 64): ga2 (x) r1
      const int jj = e - CG_W2, j = jj >> 6, k = jj & 63;
      for (int u = 0; u < nt; ++u) s = fmaf(tv(u)[168 + j], tv(u)[8 + k], s);
    } else if (e < CG_G2) {                // b2
      const int j = e - CG_B2;
      for (int u = 0; u < nt; ++u) s += tv(u)[168 + j];
    } else if (e < CG_BE2) {               // LN2 gamma
      const int j = e - CG_G2;
      for (int u = 0; u < nt; ++u) s += tv(u)[328 + j];
    } else if (e < CG_W3) {                // LN2 beta
      const int j = e - CG_BE2;
      for (int u = 0; u < nt; ++u) s += tv(u)[360 + j];
    } else if (e < CG_B3) {                // W3 (1 x 32): ga3 * r2
      const int k = e - CG_W3;
      for (int u = 0; u < nt; ++u) s = fmaf(tv(u)[392], tv(u)[136 + k], s);
    } else {                               // b3
      for (int u = 0; u < nt; ++u) s += tv(u)[392];
    }
    gp[e] = s;
  }
}

// ============================================================================
// soft mask backward (one workgroup per image)
// ============================================================================
// gradient layout: net.0.weight (8,2,3,3), net.0.bias, net.2.weight (2,8,1,1), net.2.bias
enum : int { SG_W1 = 0, SG_B1 = 144, SG_W2 = 152, SG_B2 = 168, SG_SIZE = 170 };

struct MaskTrainArgs {
  mcaq_smask_params P;
  const float* bits;     // (B, ht, wt)
  const float* absmean;  // (B, H, W)
  const float* gm;       // (B, H, W) gradient of m(p)
  float* gbits;          // (B, ht, wt) gradient of the bit map (accumulated if accumulate)
  float* gpart;          // [B][SG_SIZE]
  int B, H, W, ht, wt, accumulate;
};

__global__ __launch_bounds__(256) void mcaq_smask_bwd_kernel(MaskTrainArgs A) {
  extern __shared__ float smem_tr[];
  const int b = blockIdx.x, H = A.H, W = A.W, ht = A.ht, wt = A.wt, NT = ht * wt;
  const int tid = threadIdx.x;
  float* f0 = smem_tr;               // bits feature, clamp((b - 2) / 6, 0, 1)
  float* f1 = f0 + NT;               // activation feature
  float* gl = f1 + NT;               // per tile: gradient of logit 0 (logit 1 gets -gl)
  float* gpre = gl + NT;             // per tile x 8: gradient of the hidden pre-activation
  float* rel = gpre + 8 * NT;        // per tile x 8: relu(hidden)
  float* red = rel + 8 * NT;         // 64 reduction slots
  const float* am = A.absmean + (size_t)b * H * W;
  const float* gm = A.gm + (size_t)b * H * W;
  const float sch = (float)ht / (float)H, scw = (float)wt / (float)W;
  // ---- forward recompute: per-tile activation (adaptive_avg_pool2d), amax
  float lmx = -3.402823466e38f;
  for (int t = tid; t < NT; t += 256) {
    const int i = t / wt, j = t - i * wt;
    const int ha = (i * H) / ht, hb = ((i + 1) * H + ht - 1) / ht;
    const int wa = (j * W) / wt, wb = ((j + 1) * W + wt - 1) / wt;
    float s = 0.0f;
    for (int h = ha; h < hb; ++h)
      for (int w = wa; w < wb; ++w) s += am[h * W + w];
    const float a = (s / (float)(hb - ha)) / (float)(wb - wa);
    f1[t] = a;
    lmx = fmax_(lmx, a);
    const float bv = A.bits[(size_t)b * NT + t];
    f0[t] = clampf_((bv - 2.0f) / 6.0f, 0.0f, 1.0f);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lmx = fmax_(lmx, __shfl_xor(lmx, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = lmx;
  __syncthreads();
  const float amax = fmax_(fmax_(red[0], red[1]), fmax_(red[2], red[3]));
  const float den = amax + 1e-8f;
  for (int t = tid; t < NT; t += 256) f1[t] = f1[t] / den;
  __syncthreads();
  // ---- per tile: hidden layer, logits, m(tile); gradient of m(tile) from
  // the m(p) gradient through the 5x5 smoothing (replicate pad) and the
  // nearest upsample: g_mt(t) = sum_p g_m(p) sum_{i,j: src(clamp(p + o_ij)) = t} k_ij
  for (int t = tid; t < NT; t += 256) {
    const int i = t / wt, j = t - i * wt;
    float hid[8];
#pragma unroll
    for (int oc = 0; oc < 8; ++oc) {
      float acc = A.P.b1[oc];
#pragma unroll
      for (int qq = 0; qq < 9; ++qq) {
        const int ii = i + qq / 3 - 1, jj = j + qq % 3 - 1;
        if (ii < 0 || ii >= ht || jj < 0 || jj >= wt) continue;
        const int s = ii * wt + jj;
        acc = fmaf(A.P.w1[(oc * 2 + 0) * 9 + qq], f0[s], acc);
        acc = fmaf(A.P.w1[(oc * 2 + 1) * 9 + qq], f1[s], acc);
      }
      hid[oc] = acc;
      rel[t * 8 + oc] = acc > 0.0f ? acc : 0.0f;
    }
    float l0 = A.P.b2[0], l1 = A.P.b2[1];
#pragma unroll
    for (int ic = 0; ic < 8; ++ic) { l0 = fmaf(A.P.w2[ic], rel[t * 8 + ic], l0); l1 = fmaf(A.P.w2[8 + ic], rel[t * 8 + ic], l1); }
    const float mt = 1.0f / (1.0f + expf(l1 - l0));
    // pixels whose 5x5 window reaches this tile's nearest-upsample block
    int h0 = H, h1 = -1, w0 = W, w1 = -1;
    for (int h = 0; h < H; ++h) if (imin_((int)floorf((float)h * sch), ht - 1) == i) { h0 = imin_(h0, h); h1 = h; }
    for (int w = 0; w < W; ++w) if (imin_((int)floorf((float)w * scw), wt - 1) == j) { w0 = imin_(w0, w); w1 = w; }
    float gmt = 0.0f;
    for (int h = imax_(h0 - 2, 0); h <= imin_(h1 + 2, H - 1); ++h) {
      float rw[5];
#pragma unroll
      for (int ii = 0; ii < 5; ++ii) {
        const int hs = imin_(imax_(h + ii - 2, 0), H - 1);
        rw[ii] = (hs >= h0 && hs <= h1) ? 1.0f : 0.0f;
      }
      for (int w = imax_(w0 - 2, 0); w <= imin_(w1 + 2, W - 1); ++w) {
        float kw = 0.0f;
#pragma unroll
        for (int jj = 0; jj < 5; ++jj) {
          const int ws = imin_(imax_(w + jj - 2, 0), W - 1);
          if (ws < w0 || ws > w1) continue;
#pragma unroll
          for (int ii = 0; ii < 5; ++ii) kw = fmaf(bits_as_float(k_smooth5_bits[ii * 5 + jj]), rw[ii], kw);
        }
        gmt = fmaf(gm[h * W + w], kw, gmt);
      }
    }
    // softmax (2 classes): d m / d l0 = m (1 - m) = -d m / d l1
    const float g0 = gmt * (mt * (1.0f - mt));
    gl[t] = g0;
#pragma unroll
    for (int ic = 0; ic < 8; ++ic) {
      const float gr = A.P.w2[ic] * g0 - A.P.w2[8 + ic] * g0;
      gpre[t * 8 + ic] = hid[ic] > 0.0f ? gr : 0.0f;
    }
  }
  __syncthreads();
  // ---- gradient of the bits feature: 3x3 transposed conv of gpre, then
  // through the clamp and the affine map
  for (int u = tid; u < NT; u += 256) {
    const int i = u / wt, j = u - i * wt;
    float s = 0.0f;
#pragma unroll
    for (int qq = 0; qq < 9; ++qq) {
      const int ti = i - (qq / 3 - 1), tj = j - (qq % 3 - 1);   // tile whose tap qq lands on u
      if (ti < 0 || ti >= ht || tj < 0 || tj >= wt) continue;
      const int t = ti * wt + tj;
#pragma unroll
      for (int oc = 0; oc < 8; ++oc) s = fmaf(A.P.w1[(oc * 2 + 0) * 9 + qq], gpre[t * 8 + oc], s);
    }
    const float bv = A.bits[(size_t)b * NT + u];
    const float f = (bv - 2.0f) / 6.0f;
    const float gb = (f >= 0.0f && f <= 1.0f) ? s / 6.0f : 0.0f;
    float* dst = A.gbits + (size_t)b * NT + u;
    *dst = A.accumulate ? *dst + gb : gb;
  }
  // ---- parameter partials of this image
  float* gp = A.gpart + (size_t)b * SG_SIZE;
  for (int e = tid; e < SG_SIZE; e += 256) {
    float s = 0.0f;
    if (e < SG_B1) {                  // W1[oc][ic][qq]
      const int oc = e / 18, ic = (e / 9) & 1, qq = e % 9;
      const float* f = ic == 0 ? f0 : f1;
      for (int t = 0; t < NT; ++t) {
        const int i = t / wt, j = t - i * wt;
        const int ii = i + qq / 3 - 1, jj = j + qq % 3 - 1;
        if (ii < 0 || ii >= ht || jj < 0 || jj >= wt) continue;
        s = fmaf(gpre[t * 8 + oc], f[ii * wt + jj], s);
      }
    } else if (e < SG_W2) {           // b1
      const int oc = e - SG_B1;
      for (int t = 0; t < NT; ++t) s += gpre[t * 8 + oc];
    } else if (e < SG_B2) {           // W2[o][ic]: g_l(o) relu_ic, g_l1 = -g_l0
      const int o = (e - SG_W2) >> 3, ic = (e - SG_W2) & 7;
      for (int t = 0; t < NT; ++t) s = fmaf(o == 0 ? gl[t] : -gl[t], rel[t * 8 + ic], s);
    } else {                          // b2
      const int o = e - SG_B2;
      for (int t = 0; t < NT; ++t) s += o == 0 ? gl[t] : -gl[t];
    }
    gp[e] = s;
  }
}

}  // namespace mcaq

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

size_t mcaq_mapper_work_floats(int n) { return mcaq::mapper_work_floats(n); }

int mcaq_mapper_train_forward(const mcaq_mapper_params* P, const float* c, int n, float min_bits, float max_bits,
                              float temperature, float momentum, int round_bits, int update_stats, float* bits,
                              float* work, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !c || !bits || !work || n < 1) return (int)hipErrorInvalidValue;
  MapperTrainArgs A{};
  A.P = *P; A.c = c; A.bits = bits; A.work = work; A.n = n; A.nwg = (n + TR_TPB - 1) / TR_TPB;
  A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature; A.momentum = momentum;
  A.round_bits = round_bits; A.update_stats = update_stats;
  const dim3 g(A.nwg), t(256);
  hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<1>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<2>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<3>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<4>, g, t, 0, stream, A);
  return (int)hipGetLastError();
}

int mcaq_mapper_train_backward(const mcaq_mapper_params* P, const float* c, int n, const float* gbits,
                               float min_bits, float max_bits, float temperature, float* work, float* gc,
                               float* gparams, float* gpart, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !c || !gbits || !gc || !gparams || !gpart || !work || n < 1) return (int)hipErrorInvalidValue;
  MapperTrainArgs A{};
  A.P = *P; A.c = c; A.gbits = gbits; A.gc = gc; A.work = work; A.gpart = gpart; A.n = n;
  A.nwg = (n + TR_TPB - 1) / TR_TPB;
  A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature;
  const dim3 g(A.nwg), t(256);
  hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<4>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<3>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<2>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<1>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_tr_reduce_kernel, dim3((MG_SIZE + 255) / 256), dim3(256), 0, stream, (const float*)gpart,
                     A.nwg, (int)MG_SIZE, (int)MG_SIZE, gparams, 0);
  return (int)hipGetLastError();
}

size_t mcaq_mapper_gpart_floats(int n) { return (size_t)((n + mcaq::TR_TPB - 1) / mcaq::TR_TPB) * mcaq::MG_SIZE; }

size_t mcaq_head_gpart_floats(int n) { return (size_t)((n + mcaq::TR_TPB - 1) / mcaq::TR_TPB) * mcaq::CG_SIZE; }

int mcaq_head_train_backward(const mcaq_cmlp_params* P, const float* phi, const float* craw, const float* gC, int B,
                             int ht, int wt, float* gcraw, float* gparams, float* gpart, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !phi || !craw || !gC || !gcraw || !gparams || !gpart || B < 1 || ht < 1 || wt < 1)
    return (int)hipErrorInvalidValue;
  HeadTrainArgs A{};
  A.P = *P; A.phi = phi; A.craw = craw; A.gC = gC; A.gcraw = gcraw; A.gpart = gpart;
  A.B = B; A.ht = ht; A.wt = wt; A.n = B * ht * wt; A.nwg = (A.n + TR_TPB - 1) / TR_TPB;
  const size_t lb = (size_t)4 * ht * wt * sizeof(float);
  if (lb > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mcaq_bilateral_bwd_kernel, dim3(B), dim3(256), lb, stream, A);
  constexpr int ST = 8 + 64 + 64 + 32 + 32 + 64 + 64 + 32 + 32 + 1;
  const size_t lc = (size_t)TR_TPB * (ST + 1) * sizeof(float);
  static bool set = false;
  if (!set) {
    const hipError_t e = hipFuncSetAttribute((const void*)mcaq_cmlp_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lc);
    if (e != hipSuccess) return (int)e;
    set = true;
  }
  hipLaunchKernelGGL(mcaq_cmlp_bwd_kernel, dim3(A.nwg), dim3(64), lc, stream, A);
  hipLaunchKernelGGL(mcaq_tr_reduce_kernel, dim3((CG_SIZE + 255) / 256), dim3(256), 0, stream, (const float*)gpart,
                     A.nwg, (int)CG_SIZE, (int)CG_SIZE, gparams, 0);
  return (int)hipGetLastError();
}

size_t mcaq_smask_gpart_floats(int B) { return (size_t)B * mcaq::SG_SIZE; }

int mcaq_smask_train_backward(const mcaq_smask_params* P, const float* bits, const float* absmean, const float* gm,
                              int B, int H, int W, int ht, int wt, float* gbits, int accumulate, float* gparams,
                              float* gpart, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !bits || !absmean || !gm || !gbits || !gparams || !gpart || B < 1 || ht < 1 || wt < 1 || H < ht || W < wt)
    return (int)hipErrorInvalidValue;
  MaskTrainArgs A{};
  A.P = *P; A.bits = bits; A.absmean = absmean; A.gm = gm; A.gbits = gbits; A.gpart = gpart;
  A.B = B; A.H = H; A.W = W; A.ht = ht; A.wt = wt; A.accumulate = accumulate;
  const int NT = ht * wt;
  const size_t lb = ((size_t)19 * NT + 64) * sizeof(float);
  if (lb > 160 * 1024 - 1024) return (int)hipErrorInvalidValue;
  static int set = 0;
  if ((int)lb > set) {
    const hipError_t e = hipFuncSetAttribute((const void*)mcaq_smask_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             160 * 1024 - 1024);
    if (e != hipSuccess) return (int)e;
    set = 160 * 1024 - 1024;
  }
  hipLaunchKernelGGL(mcaq_smask_bwd_kernel, dim3(B), dim3(256), lb, stream, A);
  hipLaunchKernelGGL(mcaq_tr_reduce_kernel, dim3(1), dim3(256), 0, stream, (const float*)gpart, B, (int)SG_SIZE,
                     (int)SG_SIZE, gparams, 0);
  return (int)hipGetLastError();
}

}  // extern "C"
