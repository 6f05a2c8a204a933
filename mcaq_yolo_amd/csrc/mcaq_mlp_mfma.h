// mcaq_mlp_mfma.h - the two tile MLPs on fp32 MFMA (gfx950 device code only).
//
// v_mfma_f32_16x16x4_f32 computes D = fma(a_k3, b_k3, ... fma(a_k0, b_k0, C)),
// a k-ordered fp32 FMA chain (cdna_hip_programming.md "FP32-input MFMA"), so
// chaining K/4 of them from C = 0 reproduces the oracle's Linear exactly:
// sequential FMA over k = 0..K-1 from 0, then + bias.
//
// One wave owns a block of 16*NH tiles = NH 16-tile halves h (NH = 1 with
// 512-thread pass B workgroups, 2 with 256).  Layout
// (transposed product, M = neurons, N = tiles):
//   A (16 neurons x 4 k): lane l holds W[16*mb + (l&15)][4s + (l>>4)]
//   B (4 k x 16 tiles)  : lane l holds X[tile 16h + (l&15)][4s + (l>>4)]
//   D (16 x 16)         : lane l, register r -> neuron 16*mb + 4*(l>>4) + r,
//                         tile 16h + (l&15)
// A layer's activations go to a per-wave LDS scratch X[32 tiles][XS] and the
// next layer reads its B operands from there (one ds_read per k-step, all
// issued before the chain).  Every layer runs 2·NB independent accumulator
// chains of K/4 steps (the 16x16x4 form's dependent latency is ~40 cycles),
// where the 32x32x2 form needed one chain of K/2 dependent steps.  LayerNorm
// statistics use the pairwise tree of the oracle's tree_sum: register pairs,
// quads, then lane xor 16 / xor 32, then neuron blocks.
#pragma once
#include <hip/hip_runtime.h>
#include "mcaq_math.h"
// included by mcaq_morph.h after the layout enums / helpers it uses

namespace mcaq {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// host-permuted weight layouts appended after the plain blobs (params.py)
enum : int {
  // complexity MLP (plain block CM_SIZE floats first)
  CMQ_W1 = CM_SIZE,                 // 4 blocks x 2 steps x 64   = 512
  CMQ_W2 = CMQ_W1 + 512,            // 2 blocks x 16 steps x 64  = 2048
  CMQ_SIZE = CMQ_W2 + 2048,
  // mapper MLP (plain block MM_SIZE floats first)
  MMQ_W1 = MM_SIZE,                 // 2 blocks x 1 step x 64 (K padded 3->4) = 128
  MMQ_W2 = MMQ_W1 + 128,            // 4 blocks x 8 steps x 64   = 2048
  MMQ_W3 = MMQ_W2 + 2048,           // 2 blocks x 16 steps x 64  = 2048
  MMQ_SIZE = MMQ_W3 + 2048,
};

// weight / folded-BN pointers of the tile MLPs: LDS-typed when the weights are
// staged in the workgroup's LDS (ds_read; a generic pointer compiles to flat loads)
typedef const __attribute__((address_space(3))) float* lds_cf;
typedef __attribute__((address_space(3))) float* lds_f;

// diagnostic build only (-DMCAQ_STAMPS): wave-level cycle stamps (no barrier)
#if defined(MCAQ_STAMPS) && !defined(MCAQ_STAMPS_ACC) && defined(__HIP_DEVICE_COMPILE__)
#define WSTAMP(on, k) do { if ((on) && (threadIdx.x & 63) == 0) g_mcaq_stamps[(k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define WSTAMP(on, k) do {} while (0)
#endif

// the scratch is private to the wave: LDS requests of one wave are served in
// order, so a compiler barrier is the only fence a write->read hand-off needs
#define MLP_WAVE_FENCE() do { __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory"); } while (0)

__device__ __forceinline__ f32x4 zero4() {
  f32x4 z;
  z[0] = z[1] = z[2] = z[3] = 0.0f;
  return z;
}

__device__ __forceinline__ f32x4 mf16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// D (NH tile halves x NB neuron blocks) -> X[tile][neuron]
template <int NH, int NB>
__device__ __forceinline__ void d_store(lds_f xs, const f32x4 (&D)[NH][NB], int j, int q) {
  MLP_WAVE_FENCE();
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int mb = 0; mb < NB; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) xs[(16 * h + j) * MLP_XS + 16 * mb + 4 * q + r] = D[h][mb][r];
  MLP_WAVE_FENCE();
}

// Linear without bias, K inputs from X, 16*NB outputs: 2*NB chains of K/4 steps
template <int K, int NH, int NB, typename PT>
__device__ __forceinline__ void layer16(PT A, lds_f xs, f32x4 (&D)[NH][NB], int lane) {
  constexpr int KS = K / 4;
  const int j = lane & 15, q = lane >> 4;
  float bb[NH][KS], aa[NB][KS];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int s = 0; s < KS; ++s) bb[h][s] = xs[(16 * h + j) * MLP_XS + 4 * s + q];
#pragma unroll
  for (int mb = 0; mb < NB; ++mb)
#pragma unroll
    for (int s = 0; s < KS; ++s) aa[mb][s] = A[(mb * KS + s) * 64 + lane];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int mb = 0; mb < NB; ++mb) D[h][mb] = zero4();
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int mb = 0; mb < NB; ++mb) D[h][mb] = mf16(aa[mb][s], bb[h][s], D[h][mb]);
}

// + bias per neuron
template <int NH, int NB, typename PT>
__device__ __forceinline__ void add_bias(f32x4 (&D)[NH][NB], PT b, int q) {
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int mb = 0; mb < NB; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) D[h][mb][r] = D[h][mb][r] + b[16 * mb + 4 * q + r];
}

// value of x in lane l ^ 16 / l ^ 32 (v_permlane16_swap / v_permlane32_swap:
// VALU lane swaps, no LDS round trip; tools/probe/permlane_probe.hip)
__device__ __forceinline__ float xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

// pairwise tree over the 16*NB neurons of one tile (oracle tree_sum order)
template <int NB>
__device__ __forceinline__ float tree16(const f32x4 (&d)[NB]) {
  float s[NB];
#pragma unroll
  for (int mb = 0; mb < NB; ++mb) {
    float v = (d[mb][0] + d[mb][1]) + (d[mb][2] + d[mb][3]);   // neurons 4q..4q+3
    v = v + xor16(v);                                            // 8: q, q^1
    v = v + xor32(v);                                            // 16: q pairs
    s[mb] = v;
  }
  if constexpr (NB == 2) return s[0] + s[1];
  else return (s[0] + s[1]) + (s[2] + s[3]);
}

// LayerNorm (oracle order: mean, d = x - mean, var of d*d, ((d*rstd)*g)+b)
template <int NB, typename PT>
__device__ __forceinline__ void layernorm16(f32x4 (&d)[NB], PT g, PT b, int q) {
  const float mean = tree16<NB>(d) / (float)(16 * NB);
  f32x4 sq[NB];
#pragma unroll
  for (int mb = 0; mb < NB; ++mb)
#pragma unroll
    for (int r = 0; r < 4; ++r) { d[mb][r] = d[mb][r] - mean; sq[mb][r] = d[mb][r] * d[mb][r]; }
  const float var = tree16<NB>(sq) / (float)(16 * NB);
  const float rstd = 1.0f / cr_sqrt(var + 1e-5f);
#pragma unroll
  for (int mb = 0; mb < NB; ++mb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = 16 * mb + 4 * q + r;
      d[mb][r] = ((d[mb][r] * rstd) * g[n]) + b[n];
    }
}

// BN eval with the folded per-neuron (alpha, beta), then ReLU
template <int NH, int NB, typename PT>
__device__ __forceinline__ void bn_relu16(f32x4 (&D)[NH][NB], PT alpha, PT beta, int q) {
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int mb = 0; mb < NB; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * mb + 4 * q + r;
        D[h][mb][r] = fmax_(D[h][mb][r] * alpha[n] + beta[n], 0.0f);
      }
}

// complexity MLP for the 16*NH tiles [t0, t0+16*NH) of one image; writes T_CMLP
template <int NH, typename PT, int TS = TILE_FLOATS>   // TS: floats per tile of `tiles`
__device__ void cmlp_block_mfma(PT P, float* tiles, int NT, int t0, int lane, lds_f xs, bool stamp = false) {
  const int j = lane & 15, q = lane >> 4;
  WSTAMP(stamp, 40);
  // layer 1: 8 -> 64 from phi (2 k-steps)
  f32x4 D1[NH][4];
  {
    float bb[NH][2], aa[4][2];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int t = t0 + 16 * h + j;
      const float* tp = tiles + (t < NT ? t : 0) * TS + T_PHI;
#pragma unroll
      for (int s = 0; s < 2; ++s) bb[h][s] = t < NT ? tp[4 * s + q] : 0.0f;
    }
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int s = 0; s < 2; ++s) aa[mb][s] = P[CMQ_W1 + (mb * 2 + s) * 64 + lane];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) D1[h][mb] = zero4();
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) D1[h][mb] = mf16(aa[mb][s], bb[h][s], D1[h][mb]);
  }
  add_bias<NH, 4>(D1, P + CM_B1, q);
  WSTAMP(stamp, 41);
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    layernorm16<4>(D1[h], P + CM_G1, P + CM_BE1, q);
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) D1[h][mb][r] = fmax_(D1[h][mb][r], 0.0f);
  }
  d_store<NH, 4>(xs, D1, j, q);
  WSTAMP(stamp, 42);
  // layer 2: 64 -> 32
  f32x4 D2[NH][2];
  layer16<64, NH, 2>(P + CMQ_W2, xs, D2, lane);
  add_bias<NH, 2>(D2, P + CM_B2, q);
  WSTAMP(stamp, 43);
#pragma unroll
  for (int h = 0; h < NH; ++h) layernorm16<2>(D2[h], P + CM_G2, P + CM_BE2, q);
  d_store<NH, 2>(xs, D2, j, q);
  WSTAMP(stamp, 44);
  // layer 3: 32 -> 1 (ReLU inside the sequential dot), sigmoid; lane = tile
  if (lane < 16 * NH) {
    const int t = t0 + lane;
    float acc = 0.0f;
#pragma unroll
    for (int n = 0; n < 32; ++n) acc = fmaf(fmax_(xs[lane * MLP_XS + n], 0.0f), P[CM_W3 + n], acc);
    const float z = acc + P[CM_B3];
    if (t < NT) tiles[t * TS + T_CMLP] = 1.0f / (1.0f + cr_exp(-z));
  }
  WSTAMP(stamp, 45);
}

// MLP bit mapper for the tiles [t0, t0+16*NH): pre-temperature bits into T_AUX
// ab: folded BN terms in LDS, alpha at [0,128) and beta at [128,256) for the
// 32 + 64 + 32 neurons of BN1/BN2/BN3 (mcaq_morph.h, bn fold)
template <int NH, typename PT, int TS = TILE_FLOATS>
__device__ void mapper_block_mfma(PT P, PT ab, float* tiles, int NT, int t0, int lane, int csrc, float min_bits,
                                  float max_bits, lds_f xs, bool stamp = false) {
  const int j = lane & 15, q = lane >> 4;
  WSTAMP(stamp, 48);
  // layer 1: 3 -> 32, features (c, c^2, log1p c, 0) on k = q
  f32x4 D1[NH][2];
  {
    // lane l < 16*NH evaluates log1p for tile l once; lanes (q = 2, j) of
    // half h take it from lane 16h + j
    const int tl = t0 + (lane & (16 * NH - 1));
    const float cl = clampf_(tl < NT ? tiles[tl * TS + csrc] : 0.0f, 0.0f, 1.0f);
    const float lg = lane < 16 * NH ? cr_log1p(cl) : 0.0f;
    float bb[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int t = t0 + 16 * h + j;
      float c = t < NT ? tiles[t * TS + csrc] : 0.0f;
      c = clampf_(c, 0.0f, 1.0f);
      const float lh = __shfl(lg, 16 * h + j, 64);
      bb[h] = q == 0 ? c : (q == 1 ? c * c : (q == 2 ? lh : 0.0f));
    }
    WSTAMP(stamp, 49);
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) D1[h][mb] = mf16(P[MMQ_W1 + mb * 64 + lane], bb[h], zero4());
  }
  add_bias<NH, 2>(D1, P + MM_B1, q);
  bn_relu16<NH, 2>(D1, ab, ab + 128, q);
  d_store<NH, 2>(xs, D1, j, q);
  WSTAMP(stamp, 50);
  // layer 2: 32 -> 64
  f32x4 D2[NH][4];
  layer16<32, NH, 4>(P + MMQ_W2, xs, D2, lane);
  add_bias<NH, 4>(D2, P + MM_B2, q);
  bn_relu16<NH, 4>(D2, ab + 32, ab + 160, q);
  d_store<NH, 4>(xs, D2, j, q);
  WSTAMP(stamp, 51);
  // layer 3: 64 -> 32
  f32x4 D3[NH][2];
  layer16<64, NH, 2>(P + MMQ_W3, xs, D3, lane);
  add_bias<NH, 2>(D3, P + MM_B3, q);
  bn_relu16<NH, 2>(D3, ab + 96, ab + 224, q);
  d_store<NH, 2>(xs, D3, j, q);
  WSTAMP(stamp, 52);
  // layer 4: 32 -> 1 sequential dot, sigmoid, affine to [min_bits, max_bits]; lane = tile
  if (lane < 16 * NH) {
    const int t = t0 + lane;
    float acc = 0.0f;
#pragma unroll
    for (int n = 0; n < 32; ++n) acc = fmaf(xs[lane * MLP_XS + n], P[MM_W4 + n], acc);
    const float z = acc + P[MM_B4];
    WSTAMP(stamp, 53);
    const float hs = 1.0f / (1.0f + cr_exp(-z));
    if (t < NT) tiles[t * TS + T_AUX] = min_bits + (max_bits - min_bits) * hs;
  }
  WSTAMP(stamp, 54);
}

}  // namespace mcaq
