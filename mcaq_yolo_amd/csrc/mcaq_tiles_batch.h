// mcaq_tiles_batch.h - pass B of the morphology as batch-wide tile kernels.
//
// The per-image pass B (morph_tiles) runs the tile chain of one image in a
// 256-thread workgroup holding ~130 KB of LDS (tile arrays + the staged
// weights) and 246 VGPRs per lane: one workgroup per CU for ~27 us, so its
// CU-time (~2,000 CU-us per config-2 batch) competes with the streaming
// passes.  For the hook's flag set (phi, complexity MLP,
// bilateral, MLP mapper, soft mask; no percentile normalisation, no linear
// mapper) the only per-image dependencies of the chain are neighbourhoods
// (the bilateral's 5x5 and the soft mask's 3x3 tile windows) and the soft
// mask's per-image activation maximum, so the chain splits into three
// launches over all tiles of all images, one wave per 64 tiles (lane = tile),
// weights read through the caches:
//
//   head   phi assembly from the pass-A partials + complexity MLP (fp32 MFMA,
//          two 32-tile blocks) -> raw complexity
//   map    bilateral (25 clamped taps of the raw complexity) + clamp -> C;
//          mean |x| per tile; MLP bit mapper (MFMA) + temperature / STE -> bits
//   mask   per-image max of the tile activations, 3x3 conv + 1x1 conv +
//          2-way softmax -> m(tile)
//
// Intermediates travel in the free slots of tile_tmp (TT_*).  The m(p) plane,
// when requested (debug, or pass 2 reading a plane), is a fourth per-pixel
// launch.  Every value is
// the one morph_tiles computes: the same per-tile operation sequences (the
// MFMA blocks are the kernels' own, checked against the scalar forms), the
// same ATen reduction orders (tail flags from the tile's flat position).
//
// Reference: morphology.py:81-97 (complexity MLP), :309-354 (bilateral),
// :576-739 + :860-864 (phi), bit_allocation.py:199-280 (mapper),
// quantization.py:213-239 (soft mask).
#pragma once

namespace mcaq {

#ifndef MCAQ_TB_TILES
#define MCAQ_TB_TILES 64
#endif
constexpr int TB_TILES = MCAQ_TB_TILES;   // tiles per workgroup (one wave, lane = tile; 32 or 64)
constexpr int TB_TS = 16;      // floats per tile of the wave's LDS tile array
enum : int { TT_ACT = 29, TT_BITS = 30, TT_CRAW = 31 };   // tile_tmp slots of the tile kernels

MCAQ_HD bool tiles_batch_eligible(const MorphScale& S) {
  const int need = F_PHI | F_CMLP | F_MAPPER;
  int S_ = 0;
  for (int s = 2; s <= S.tile; s *= 2) ++S_;
  return (S.flags & need) == need && !(S.flags & (F_NORM_C | F_MAP_LINEAR | F_TILES_IMAGE)) &&
         S.c_in == nullptr && S.bits_in == nullptr && 20 + S_ <= TT_ACT && S.cmlp != nullptr &&
         S.mapper != nullptr && S.tile_tmp != nullptr && (!(S.flags & F_SOFTMASK) || (S.smask && S.absmean && S.mt_out));
}

// bilateral of tile t = (th, tw) over the clamped 5x5 tile window of the raw
// complexity craw(.) (morphology.py:309-354): w = spatial * exp(-d^2 / 0.02),
// C = clamp(sum w p / (sum w + 1e-8)) with ATen's 25-row outer sums (vector
// column: rows 0..15 folded, then 16..24; tail column: 4 interleaved
// partials, row 24 into partial 0) - morph_tiles' bilateral stage
template <class CR>
MCAQ_HD float bilateral_tile(int t, int th, int tw, int ht, int wt, int NT, CR craw) {
  const float ct = craw(t);
  float pv[25], wv[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) {
    const int hh = imin_(imax_(th + k / 5 - 2, 0), ht - 1);
    const int ww = imin_(imax_(tw + k % 5 - 2, 0), wt - 1);
    pv[k] = craw(hh * wt + ww);
  }
#pragma unroll
  for (int k = 0; k < 25; ++k) {
    const float d = pv[k] - ct;
    wv[k] = bits_as_float(k_bilat_sp_bits[k]) * cr_exp((-(d * d)) / 0.02f);
  }
  const bool tail = t >= aten_tail_start(NT);
  float n0 = 0.0f, n1 = 0.0f, n2 = 0.0f, n3 = 0.0f, d0 = 0.0f, d1 = 0.0f, d2 = 0.0f, d3 = 0.0f;
#pragma unroll
  for (int k = 0; k < 25; ++k) {
    const float wp = wv[k] * pv[k];
    const int q = tail ? (k < 24 ? (k & 3) : 0) : (k < 16 ? 1 : 0);
    n0 = n0 + (q == 0 ? wp : 0.0f); d0 = d0 + (q == 0 ? wv[k] : 0.0f);
    n1 = n1 + (q == 1 ? wp : 0.0f); d1 = d1 + (q == 1 ? wv[k] : 0.0f);
    n2 = n2 + (q == 2 ? wp : 0.0f); d2 = d2 + (q == 2 ? wv[k] : 0.0f);
    n3 = n3 + (q == 3 ? wp : 0.0f); d3 = d3 + (q == 3 ? wv[k] : 0.0f);
  }
  float num, dsum;
  if (tail) { num = ((n0 + n1) + n2) + n3; dsum = ((d0 + d1) + d2) + d3; }
  else { num = n0 + n1; dsum = d0 + d1; }
  return clampf_(num / (dsum + 1e-8f), 0.0f, 1.0f);
}

// mean |x| over tile (i, j)'s adaptive_avg_pool2d window of the (H, W) plane am
MCAQ_HD float act_tile(const float* am, int H, int W, int ht, int wt, int i, int j) {
  const int KH = H / ht, KW = W / wt;
  const bool even = KH * ht == H && KW * wt == W && KH == KW;
  if (even && KH == 4) return (window_sum_t<4>(am, W, i * 4, j * 4) / 4.0f) / 4.0f;
  if (even && KH == 8) return (window_sum_t<8>(am, W, i * 8, j * 8) / 8.0f) / 8.0f;
  const int ha = (i * H) / ht, hb = ((i + 1) * H + ht - 1) / ht;
  const int wa = (j * W) / wt, wb = ((j + 1) * W + wt - 1) / wt;
  float s = 0.0f;
  for (int h = ha; h < hb; ++h)
    for (int w = wa; w < wb; ++w) s = s + am[h * W + w];
  return (s / (float)(hb - ha)) / (float)(wb - wa);
}

// soft-mask net of tile (i, j) (quantization.py:213-239): 3x3 conv (zero pad,
// (kh, kw) outer, input channel inner, FMA from 0) of the two tile features
// f0 (bits) / f1 (activation), bias, ReLU, 1x1 conv, 2-way softmax with the
// exp ATen's lane of this tile takes (vl: SLEEF, else glibc) -> m(tile)
template <class F0, class F1>
MCAQ_HD float smask_tile(const float* Pm, int i, int j, int ht, int wt, F0 f0a, F1 f1a, bool vl) {
  float f0[9], f1[9];
  bool ok[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int ii = i + q / 3 - 1, jj = j + q % 3 - 1;
    ok[q] = ii >= 0 && ii < ht && jj >= 0 && jj < wt;
    const int src = imin_(imax_(ii, 0), ht - 1) * wt + imin_(imax_(jj, 0), wt - 1);
    f0[q] = f0a(src); f1[q] = f1a(src);
  }
  float hid[8];
#pragma unroll
  for (int oc = 0; oc < 8; ++oc) {
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const float a0 = fmaf(Pm[SM_W1 + (oc * 2 + 0) * 9 + q], f0[q], acc);
      const float a1 = fmaf(Pm[SM_W1 + (oc * 2 + 1) * 9 + q], f1[q], a0);
      acc = ok[q] ? a1 : acc;
    }
    hid[oc] = acc;
  }
  float l0 = Pm[SM_B2 + 0], l1 = Pm[SM_B2 + 1];
#pragma unroll
  for (int ic = 0; ic < 8; ++ic) {
    const float hv = relu_nan(hid[ic] + Pm[SM_B1 + ic]);
    l0 = fmaf(Pm[SM_W2 + ic], hv, l0);
    l1 = fmaf(Pm[SM_W2 + 8 + ic], hv, l1);
  }
  const float mxl = fmax_(l0, l1);
  const bool first = l0 >= l1;
  const float ea = (first ? l1 : l0) - mxl;
  const float e = vl ? sleef_expf(ea) : cr_exp(ea);
  const float e0 = first ? 1.0f : e, e1 = first ? e : 1.0f;
  return e0 / (e0 + e1);
}

// folded eval BatchNorms of the mapper (alpha at [0,128), beta at [128,256)),
// entries j of the calling thread's share (same values as bn_eval)
MCAQ_HD void fold_mapper_bn(const float* Pmap, float* ab, int j) {
  const int L = j < 32 ? 0 : (j < 96 ? 1 : 2);
  const int n = L == 1 ? 64 : 32;
  const int jj = j - (L == 0 ? 0 : (L == 1 ? 32 : 96));
  const float* bn = Pmap + (L == 0 ? MM_BN1 : (L == 1 ? MM_BN2 : MM_BN3));
  const float inv = 1.0f / cr_sqrt(bn[3 * n + jj] + 1e-5f);
  ab[j] = inv * bn[jj];
  ab[128 + j] = bn[n + jj] - (bn[2 * n + jj] * inv) * bn[jj];
}

// m(p) of pixel (h, w) from the m(tile) values of one image (quantization.py:
// 235-238): nearest upsample, 5x5 Gaussian with replicate pad, taps row-major
// from 0 - the plane morph_tiles writes
MCAQ_HD float mplane_pixel(const float* mt, int H, int W, int ht, int wt, int h, int w) {
  int cs[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) cs[j] = nearest_src(imin_(imax_(w + j - 2, 0), W - 1), wt, W);
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int rb = nearest_src(imin_(imax_(h + i - 2, 0), H - 1), ht, H) * wt;
#pragma unroll
    for (int j = 0; j < 5; ++j) acc = fmaf(bits_as_float(k_smooth5_bits[i * 5 + j]), mt[rb + cs[j]], acc);
  }
  return acc;
}

}  // namespace mcaq
