// mcaq_mlp_mfma.h - the two tile MLPs on fp32 MFMA (gfx950 device code only).
//
// v_mfma_f32_32x32x2_f32 computes D = fma(a_k1, b_k1, fma(a_k0, b_k0, C)), a
// k-ordered fp32 FMA chain (cdna_hip_programming.md s3), so chaining K/2 of
// them from C = 0 reproduces the oracle's Linear exactly: sequential FMA over
// k = 0..K-1 from 0, then + bias.
//
// Layout (transposed product, M = neurons, N = tiles):
//   A (32 neurons x 2 k): lane l holds W[nb*32 + (l&31)][2s + (l>>5)]
//   B (2 k x 32 tiles)  : lane l holds X[tile (l&31)][2s + (l>>5)]
//   D (32 x 32)         : lane l, register r -> neuron (r&3) + 8(r>>2) + 4(l>>5),
//                         tile l&31.
// A layer's D feeds the next layer's B with one cross-half shuffle per k-step
// (neurons 2s and 2s+1 always live in the same lane half).  LayerNorm
// statistics use the pairwise tree of the oracle's tree_sum, which the
// in-register pairs + one xor-32 exchange reproduce exactly.
#pragma once
#include <hip/hip_runtime.h>
#include "mcaq_math.h"
// included by mcaq_morph.h after the layout enums / helpers it uses

namespace mcaq {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// host-permuted weight layouts appended after the plain blobs (params.py)
enum : int {
  // complexity MLP (plain block CM_SIZE floats first)
  CMQ_W1 = CM_SIZE,                 // 2 blocks x 4 steps x 64   = 512
  CMQ_W2 = CMQ_W1 + 512,            // 1 block x 32 steps x 64   = 2048
  CMQ_SIZE = CMQ_W2 + 2048,
  // mapper MLP (plain block MM_SIZE floats first)
  MMQ_W1 = MM_SIZE,                 // 1 block x 2 steps x 64 (K padded 3->4) = 128
  MMQ_W2 = MMQ_W1 + 128,            // 2 blocks x 16 steps x 64  = 2048
  MMQ_W3 = MMQ_W2 + 2048,           // 1 block x 32 steps x 64   = 2048
  MMQ_SIZE = MMQ_W3 + 2048,
};

// weight / folded-BN pointers of the tile MLPs: LDS-typed when the weights are
// staged in the workgroup's LDS (ds_read, issued ahead of the MFMA chain; a
// generic pointer compiles to flat loads that wait before every MFMA step)
typedef const __attribute__((address_space(3))) float* lds_cf;

// optional scheduling fence between groups of 8 k-steps (keeps the A-operand
// loads of a layer from being hoisted at once); pass B's 256-thread workgroups
// have the registers to hoist them, so it is off unless MCAQ_MLP_FENCE is set
#if defined(MCAQ_MLP_FENCE)
#define MLP_GROUP_FENCE __builtin_amdgcn_sched_barrier(0);
#else
#define MLP_GROUP_FENCE
#endif

// diagnostic build only (-DMCAQ_STAMPS): wave-level cycle stamps (no barrier)
#if defined(MCAQ_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
#define WSTAMP(on, k) do { if ((on) && (threadIdx.x & 63) == 0) g_mcaq_stamps[(k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define WSTAMP(on, k) do {} while (0)
#endif

__device__ __forceinline__ int d_neuron(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// value of x in lane l ^ 32 (v_permlane32_swap: a VALU lane swap, no LDS round trip)
__device__ __forceinline__ float xhalf(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

// B operand of k-step s built from a previous layer's D blocks
template <int S>
__device__ __forceinline__ float b_from_d(const f32x16* D, int half) {
  constexpr int n0 = (2 * S) & 31;
  constexpr int blk = (2 * S) >> 5;
  constexpr int H = (n0 >> 2) & 1;
  constexpr int r0 = (n0 & 3) + 4 * (n0 >> 3);
  const float x0 = D[blk][r0];
  const float x1 = D[blk][r0 + 1];
  if (H == 0) {
    const float t = xhalf(x1);
    return half == 0 ? x0 : t;
  } else {
    const float t = xhalf(x0);
    return half == 1 ? x1 : t;
  }
}

// sum over the 32 neurons of one D block (per tile), oracle tree order
__device__ __forceinline__ float tree32(const f32x16& d) {
  float q[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) q[g] = (d[4 * g] + d[4 * g + 1]) + (d[4 * g + 2] + d[4 * g + 3]);
  float u[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) u[g] = q[g] + xhalf(q[g]);
  return (u[0] + u[1]) + (u[2] + u[3]);
}

template <int NB, typename PT>
__device__ __forceinline__ void layernorm_d(f32x16* D, PT g, PT b, int half) {
  float s = tree32(D[0]);
  if constexpr (NB == 2) s = s + tree32(D[1]);
  const float mean = s / (float)(32 * NB);
  f32x16 sq[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) { D[k][r] = D[k][r] - mean; sq[k][r] = D[k][r] * D[k][r]; }
  float v = tree32(sq[0]);
  if constexpr (NB == 2) v = v + tree32(sq[1]);
  const float var = v / (float)(32 * NB);
  const float rstd = 1.0f / cr_sqrt(var + 1e-5f);
#pragma unroll
  for (int k = 0; k < NB; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = 32 * k + d_neuron(r, half);
      D[k][r] = ((D[k][r] * rstd) * g[n]) + b[n];
    }
}

// sequential dot over neurons 0..31 of one D block with w (N = 1 output layer)
template <typename PT>
__device__ __forceinline__ float dot32_seq(const f32x16& d, PT w, int half) {
  float other[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) other[r] = xhalf(d[r]);
  float acc = 0.0f;
#pragma unroll
  for (int n = 0; n < 32; ++n) {
    const int hh = (n >> 2) & 1;
    const int r = (n & 3) + 4 * (n >> 3);
    const float v = (hh == half) ? d[r] : other[r];
    acc = fmaf(v, w[n], acc);
  }
  return acc;
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.0f;
  return z;
}

// complexity MLP for the 32 tiles [t0, t0+32) of one image; writes T_CMLP
template <typename PT>
__device__ void cmlp_block_mfma(PT P, float* tiles, int NT, int t0, int lane, bool stamp = false) {
  WSTAMP(stamp, 40);
  const int half = lane >> 5, col = lane & 31;
  const int t = t0 + col;
  const bool valid = t < NT;
  const float* tp = tiles + (valid ? t : 0) * TILE_FLOATS + T_PHI;
  // layer 1: 8 -> 64
  f32x16 D1[2] = {zero16(), zero16()};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float bop = valid ? tp[2 * s + half] : 0.0f;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
      D1[nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(P[CMQ_W1 + (nb * 4 + s) * 64 + lane], bop, D1[nb], 0, 0, 0);
  }
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) D1[nb][r] = D1[nb][r] + P[CM_B1 + 32 * nb + d_neuron(r, half)];
  WSTAMP(stamp, 41);
  layernorm_d<2>(D1, P + CM_G1, P + CM_BE1, half);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) D1[nb][r] = fmax_(D1[nb][r], 0.0f);
  WSTAMP(stamp, 42);
  // layer 2: 64 -> 32
  f32x16 D2[1] = {zero16()};
#define CM_L2_STEP(S) D2[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(P[CMQ_W2 + (S) * 64 + lane], b_from_d<S>(D1, half), D2[0], 0, 0, 0);
  CM_L2_STEP(0) CM_L2_STEP(1) CM_L2_STEP(2) CM_L2_STEP(3) CM_L2_STEP(4) CM_L2_STEP(5) CM_L2_STEP(6) CM_L2_STEP(7) MLP_GROUP_FENCE
  CM_L2_STEP(8) CM_L2_STEP(9) CM_L2_STEP(10) CM_L2_STEP(11) CM_L2_STEP(12) CM_L2_STEP(13) CM_L2_STEP(14) CM_L2_STEP(15)
  CM_L2_STEP(16) CM_L2_STEP(17) CM_L2_STEP(18) CM_L2_STEP(19) CM_L2_STEP(20) CM_L2_STEP(21) CM_L2_STEP(22) CM_L2_STEP(23)
  CM_L2_STEP(24) CM_L2_STEP(25) CM_L2_STEP(26) CM_L2_STEP(27) CM_L2_STEP(28) CM_L2_STEP(29) CM_L2_STEP(30) CM_L2_STEP(31)
#undef CM_L2_STEP
#pragma unroll
  for (int r = 0; r < 16; ++r) D2[0][r] = D2[0][r] + P[CM_B2 + d_neuron(r, half)];
  WSTAMP(stamp, 43);
  layernorm_d<1>(D2, P + CM_G2, P + CM_BE2, half);
  WSTAMP(stamp, 44);
#pragma unroll
  for (int r = 0; r < 16; ++r) D2[0][r] = fmax_(D2[0][r], 0.0f);
  // layer 3: 32 -> 1, sigmoid
  const float z = dot32_seq(D2[0], P + CM_W3, half) + P[CM_B3];
  if (valid && half == 0) tiles[t * TILE_FLOATS + T_CMLP] = 1.0f / (1.0f + cr_exp(-z));
  WSTAMP(stamp, 45);
}

// BN eval on a D block with the folded per-neuron (alpha, beta), then ReLU
template <typename PT>
__device__ __forceinline__ void bn_relu_d(f32x16& d, PT alpha, PT beta, int nb, int half) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = 32 * nb + d_neuron(r, half);
    d[r] = fmax_(d[r] * alpha[j] + beta[j], 0.0f);
  }
}

// MLP bit mapper for the tiles [t0, t0+32): pre-temperature bits into T_AUX
// ab: folded BN terms in LDS, alpha at [0,128) and beta at [128,256) for the
// 32 + 64 + 32 neurons of BN1/BN2/BN3 (mcaq_morph.h, bn_fold)
template <typename PT>
__device__ void mapper_block_mfma(PT P, PT ab, float* tiles, int NT, int t0, int lane,
                                  int csrc, float min_bits, float max_bits, bool stamp = false) {
  WSTAMP(stamp, 48);
  const int half = lane >> 5, col = lane & 31;
  const int t = t0 + col;
  const bool valid = t < NT;
  float c = valid ? tiles[t * TILE_FLOATS + csrc] : 0.0f;
  c = clampf_(c, 0.0f, 1.0f);
  const float z0 = half == 0 ? c : c * c;              // k = 0, 1
  const float z1 = half == 0 ? cr_log1p(c) : 0.0f;     // k = 2, (3 = zero pad)
  WSTAMP(stamp, 49);
  // layer 1: 3 -> 32
  f32x16 D1[1] = {zero16()};
  D1[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(P[MMQ_W1 + 0 * 64 + lane], z0, D1[0], 0, 0, 0);
  D1[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(P[MMQ_W1 + 1 * 64 + lane], z1, D1[0], 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) D1[0][r] = D1[0][r] + P[MM_B1 + d_neuron(r, half)];
  bn_relu_d(D1[0], ab, ab + 128, 0, half);
  WSTAMP(stamp, 50);
  // layer 2: 32 -> 64
  f32x16 D2[2] = {zero16(), zero16()};
#define MM_L2_STEP(S)                                                                                  \
  {                                                                                                    \
    const float bop = b_from_d<S>(D1, half);                                                           \
    D2[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(P[MMQ_W2 + (0 * 16 + (S)) * 64 + lane], bop, D2[0], 0, 0, 0); \
    D2[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(P[MMQ_W2 + (1 * 16 + (S)) * 64 + lane], bop, D2[1], 0, 0, 0); \
  }
  MM_L2_STEP(0) MM_L2_STEP(1) MM_L2_STEP(2) MM_L2_STEP(3) MM_L2_STEP(4) MM_L2_STEP(5) MM_L2_STEP(6) MM_L2_STEP(7) MLP_GROUP_FENCE
  MM_L2_STEP(8) MM_L2_STEP(9) MM_L2_STEP(10) MM_L2_STEP(11) MM_L2_STEP(12) MM_L2_STEP(13) MM_L2_STEP(14) MM_L2_STEP(15)
#undef MM_L2_STEP
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) D2[nb][r] = D2[nb][r] + P[MM_B2 + 32 * nb + d_neuron(r, half)];
    bn_relu_d(D2[nb], ab + 32, ab + 160, nb, half);
  }
  WSTAMP(stamp, 51);
  // layer 3: 64 -> 32
  f32x16 D3[1] = {zero16()};
#define MM_L3_STEP(S) D3[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(P[MMQ_W3 + (S) * 64 + lane], b_from_d<S>(D2, half), D3[0], 0, 0, 0);
  MM_L3_STEP(0) MM_L3_STEP(1) MM_L3_STEP(2) MM_L3_STEP(3) MM_L3_STEP(4) MM_L3_STEP(5) MM_L3_STEP(6) MM_L3_STEP(7) MLP_GROUP_FENCE
  MM_L3_STEP(8) MM_L3_STEP(9) MM_L3_STEP(10) MM_L3_STEP(11) MM_L3_STEP(12) MM_L3_STEP(13) MM_L3_STEP(14) MM_L3_STEP(15)
  MM_L3_STEP(16) MM_L3_STEP(17) MM_L3_STEP(18) MM_L3_STEP(19) MM_L3_STEP(20) MM_L3_STEP(21) MM_L3_STEP(22) MM_L3_STEP(23)
  MM_L3_STEP(24) MM_L3_STEP(25) MM_L3_STEP(26) MM_L3_STEP(27) MM_L3_STEP(28) MM_L3_STEP(29) MM_L3_STEP(30) MM_L3_STEP(31)
#undef MM_L3_STEP
#pragma unroll
  for (int r = 0; r < 16; ++r) D3[0][r] = D3[0][r] + P[MM_B3 + d_neuron(r, half)];
  bn_relu_d(D3[0], ab + 96, ab + 224, 0, half);
  WSTAMP(stamp, 52);
  // layer 4: 32 -> 1, sigmoid, affine to [min_bits, max_bits]
  const float z = dot32_seq(D3[0], P + MM_W4, half) + P[MM_B4];
  WSTAMP(stamp, 53);
  const float h = 1.0f / (1.0f + cr_exp(-z));
  if (valid && half == 0) tiles[t * TILE_FLOATS + T_AUX] = min_bits + (max_bits - min_bits) * h;
  WSTAMP(stamp, 54);
}

}  // namespace mcaq
