// mcaq_band.h - pass A of the morphology as two small-footprint kernels.
//
// The round-3 pass A ran one 1024-thread workgroup per (image, role) with the
// whole image's fp32 planes in LDS (~104 KB at 80x80): every workgroup held an
// entire CU for its ~25 us chain, so the morphology's CU-time (workgroups x
// duration) could not hide under the streaming passes.  Here
// the same arithmetic is cut along the two per-image dependencies it has (the
// blur's Otsu histogram, and hysteresis over the whole edge map):
//
//   band kernel   one 256-thread workgroup per (image, band of 16 rows): G =
//                 normalise(gray) over the band + a 6-row halo, adaptive
//                 threshold (BIN), 5x5 blur (+ the band's Otsu histogram),
//                 Sobel of the blur, NMS -> the NMS value plane (global),
//                 Sobel of G, LBP labels, boundary / Euler quad planes ->
//                 every per-tile partial of the mask side (tile_tmp)
//   edge kernel   one workgroup per image: Otsu threshold from the bands'
//                 histograms, double threshold of the NMS plane, hysteresis
//                 (one wave, registers), box counts + edge counts (tile_tmp)
//
// Every value is computed by the same operation sequence as morph_edges (the
// host emulation checks tile_tmp bit for bit against it on every golden case,
// tests/test_emu_cpu.py), so pass B and everything after it are unchanged.
// LDS per band workgroup ~40 KB and per edge workgroup ~34 KB at 80x80, so a
// CU holds several of them beside the streaming waves of other batches.
//
// Eligible scales: default Canny ('cv2compat'), adaptive binarize, tile 4, 8
// or 16 and a map of at most 128 x 128 (every hook scale at 640x640); other
// launches keep the per-image pass A.
//
// Reference: morphology.py:379-383 (normalise), :458-509 (Canny cv2compat),
// :551-573 (adaptive threshold), :576-739 (phi1..phi5 partials), :826-873.
#pragma once

namespace mcaq {

MCAQ_HD int band_rows(int T) { return T >= 16 ? T : 16; }
MCAQ_HD int band_count(int Hc, int T) {
  const int r = band_rows(T);
  return (Hc + r - 1) / r;
}
MCAQ_HD bool band_eligible(const MorphScale& S) {
  return (S.flags & F_PHI) && !(S.flags & (F_CANNY_LEGACY | F_BIN_OTSU)) &&
         (S.tile == 4 || S.tile == 8 || S.tile == 16) && S.Hc <= 128 && S.Wc <= 128 && S.pwork != nullptr;
}
// pwork of one scale: the NMS value plane (B x Hc x Wc floats), then the
// per-band Otsu histograms of the blur (B x bands x 256 ints)
MCAQ_HD size_t band_work_bytes(int B, int Hc, int Wc, int T) {
  return (size_t)4 * B * Hc * Wc + (size_t)4 * B * band_count(Hc, T) * 256;
}
MCAQ_HD float* band_nms(const MorphScale& S) { return S.pwork; }
MCAQ_HD int* band_hist(const MorphScale& S) { return (int*)(S.pwork + (size_t)S.B * S.Hc * S.Wc); }

// LDS of one band workgroup: Shared | G, adaptive row pass (R + 12 rows each)
// | blur (R + 4) | Sobel magnitude (R + 2) | direction bytes (R + 2) | BIN
// bits (R + 2 rows) | BND, Q1, Q3, QD, LBP label 0..9 bits (R rows each)
MCAQ_HD int band_lds_bytes(int Wc, int T) {
  const int R = band_rows(T), WPR = words_per_row(Wc);
  return fixed_bytes() + 4 * Wc * (2 * (R + 12) + (R + 4) + (R + 2)) + (((R + 2) * Wc + 3) & ~3) +
         4 * WPR * ((R + 2) + 14 * R);
}
// LDS of one edge workgroup: Shared | NMS plane | E0, E1, WK bit planes
MCAQ_HD int edge_lds_bytes(int Hc, int Wc) {
  return fixed_bytes() + 4 * ((Hc * Wc + 3) & ~3) + 4 * 3 * Hc * words_per_row(Wc);
}

// rows per thread of the band kernel's column-strip stages (register budget)
constexpr int BSR = 4;

// exact 121-tap adaptive mean of 255*G at (h, w) from G rows [g0, ...) stored
// at Gp (row h of the image at Gp + (h - g0) * Wc); same order as exact_g11
MCAQ_HD float exact_g11_rows(const float* Gp, int g0, int Hc, int Wc, int h, int w) {
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    const float* row = Gp + (imin_(imax_(h + i - 5, 0), Hc - 1) - g0) * Wc;
    float v[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) v[j] = row[imin_(imax_(w + j - 5, 0), Wc - 1)] * 255.0f;
#pragma unroll
    for (int j = 0; j < 11; ++j) acc = fmaf(bits_as_float(k_gauss11_bits[i * 11 + j]), v[j], acc);
  }
  return acc;
}

// ---- band kernel body: band `band` of image b -------------------------------
MCAQ_HD void band_pass(const Ctx& ctx, const MorphScale& S, int b, int band, char* lds) {
  const int Hc = S.Hc, Wc = S.Wc, P = Hc * Wc, T = S.tile, wt = S.wt, NT = S.ht * wt;
  const int R = band_rows(T), nb = band_count(Hc, T);
  const int WPR = words_per_row(Wc), RS = WPR * 32;
  const int r0 = band * R, r1 = imin_(r0 + R, Hc);
  // row ranges held: G and the adaptive row pass [gA, gB), blur [aA, aB),
  // Sobel magnitude / direction and BIN [mA, mB), owned rows [r0, r1)
  const int gA = imax_(r0 - 6, 0), gB = imin_(r1 + 6, Hc);
  const int aA = imax_(r0 - 2, 0), aB = imin_(r1 + 2, Hc);
  const int mA = imax_(r0 - 1, 0), mB = imin_(r1 + 1, Hc);
  Shared sh;
  carve_shared(lds, sh);
  char* q = lds + fixed_bytes();
  float* Gp = (float*)q;
  q += 4 * (R + 12) * Wc;
  float* Hp = (float*)q;      // adaptive row pass; later gx of the owned rows
  q += 4 * (R + 12) * Wc;
  float* Ap = (float*)q;      // blur; later gy of the owned rows
  q += 4 * (R + 4) * Wc;
  float* Mp = (float*)q;
  q += 4 * (R + 2) * Wc;
  uint8_t* Dp = (uint8_t*)q;
  q += ((R + 2) * Wc + 3) & ~3;
  uint32_t* BINp = (uint32_t*)q;
  q += 4 * (R + 2) * WPR;
  uint32_t* BPp = (uint32_t*)q;   // 14 planes of R rows: BND, Q1, Q3, QD, L0..L9
  const int pw = R * WPR;
  uint32_t* BND = BPp;
  uint32_t* Q1 = BPp + pw;
  uint32_t* Q3 = BPp + 2 * pw;
  uint32_t* QD = BPp + 3 * pw;
  uint32_t* LB = BPp + 4 * pw;
  MSTAMP_INIT(b == 0 && band == 1 ? 56 : -1);   // diagnostic build: slots 56-62
  MSTAMP(0);

  // -- S0: per-image min / max of gray (every pixel), then G rows [gA, gB)
  const float* gin = S.gray + (size_t)b * P;
  MFOR(i, 256) sh.hist[i] = 0;   // the band's Otsu histogram, filled by the blur
  constexpr int K = 8;
  float lmn = 3.402823466e38f, lmx = -3.402823466e38f;
  for (int base = 0; base < P; base += K * ctx.nthr) {
    float v[K];
#pragma unroll
    for (int i = 0; i < K; ++i) v[i] = gin[imin_(base + ctx.tid + i * ctx.nthr, P - 1)];
#pragma unroll
    for (int i = 0; i < K; ++i) { lmn = fminp(lmn, v[i]); lmx = fmaxp(lmx, v[i]); }
  }
  float mn, mx;
  block_minmax(ctx, sh, lmn, lmx, mn, mx);
  MSTAMP(1);
  const float den = (mx - mn) + 1e-8f;
  {
    const int n = (gB - gA) * Wc;
    const float* src = gin + gA * Wc;
    for (int base = 0; base < n; base += K * ctx.nthr) {
      float v[K];
#pragma unroll
      for (int i = 0; i < K; ++i) v[i] = src[imin_(base + ctx.tid + i * ctx.nthr, n - 1)];
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int u = base + ctx.tid + i * ctx.nthr;
        if (u < n) Gp[u] = (v[i] - mn) / den;
      }
    }
  }
  MSYNC();
  MSTAMP(2);

  // -- S1a: adaptive threshold, horizontal 11-tap pass of 255*G, rows [gA, gB)
  {
    const int nst = (gB - gA + BSR - 1) / BSR;
    MFOR2(st, w, nst, Wc) {
      const int h0 = gA + st * BSR;
      float v[BSR][11];
#pragma unroll
      for (int r = 0; r < BSR; ++r) {
        const float* row = Gp + (imin_(h0 + r, gB - 1) - gA) * Wc;
#pragma unroll
        for (int j = 0; j < 11; ++j) v[r][j] = row[imin_(imax_(w + j - 5, 0), Wc - 1)] * 255.0f;
      }
#pragma unroll
      for (int r = 0; r < BSR; ++r) {
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < 11; ++j) acc = fmaf(bits_as_float(k_g11_sep_bits[j]), v[r][j], acc);
        if (h0 + r < gB) Hp[(h0 + r - gA) * Wc + w] = acc;
      }
    }
  }
  // -- S1b: 5x5 Gaussian blur (zero pad), rows [aA, aB); the owned rows feed
  //    the band's Otsu histogram
  {
    const int nst = (aB - aA + BSR - 1) / BSR;
    MFOR2(st, w, nst, Wc) {
      const int h0 = aA + st * BSR;
      float v[BSR + 4][5];
#pragma unroll
      for (int t = 0; t < BSR + 4; ++t) {
        const int hh = h0 + t - 2;
        const bool rv = hh >= 0 && hh < Hc;
        const float* row = Gp + (imin_(imax_(hh, gA), gB - 1) - gA) * Wc;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const int ww = w + j - 2;
          const float x = row[imin_(imax_(ww, 0), Wc - 1)];
          v[t][j] = (rv && ww >= 0 && ww < Wc) ? x : 0.0f;
        }
      }
#pragma unroll
      for (int r = 0; r < BSR; ++r) {
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
          for (int j = 0; j < 5; ++j) acc = fmaf(bits_as_float(k_gauss5_bits[i * 5 + j]), v[r + i][j], acc);
        const int h = h0 + r;
        if (h < aB) {
          Ap[(h - aA) * Wc + w] = acc;
          if (h >= r0 && h < r1) otsu_hist_add(sh, acc);
        }
      }
    }
  }
  MSYNC();
  MSTAMP(3);

  // -- S2a: adaptive threshold, vertical pass + exact fallback -> BIN rows [mA, mB)
  {
    const float marg = bits_as_float(k_g11_margin_bits[0]);
    const int nst = (mB - mA + BSR - 1) / BSR;
    MFOR2(st, sl, nst, RS) {
      const int k = sl >> 5, bit = sl & 31, w = sl;
      const int h0 = mA + st * BSR;
      bool on[BSR];
#pragma unroll
      for (int r = 0; r < BSR; ++r) on[r] = false;
      if (w < Wc) {
        float v[BSR + 10];
#pragma unroll
        for (int t = 0; t < BSR + 10; ++t) {
          const int hh = imin_(imax_(h0 + t - 5, 0), Hc - 1);
          v[t] = Hp[(imin_(imax_(hh, gA), gB - 1) - gA) * Wc + w];
        }
#pragma unroll
        for (int r = 0; r < BSR; ++r) {
          const int h = h0 + r;
          if (h >= mB) continue;
          float m = 0.0f;
#pragma unroll
          for (int i = 0; i < 11; ++i) m = fmaf(bits_as_float(k_g11_sep_bits[i]), v[r + i], m);
          const float g = Gp[(h - gA) * Wc + w] * 255.0f;
          const float t = m - 2.0f;
          if (fabsf(g - t) > marg) {
            on[r] = g > t;
          } else {
            on[r] = g > exact_g11_rows(Gp, gA, Hc, Wc, h, w) - 2.0f;
          }
        }
      }
#pragma unroll
      for (int r = 0; r < BSR; ++r)
        if (h0 + r < mB) put_bits(BINp, (h0 + r - mA) * WPR + k, bit, on[r]);
    }
  }
  // -- S2b: Sobel of 255*blur (zero pad) -> L1 magnitude + NMS direction, rows [mA, mB)
  {
    const int nst = (mB - mA + BSR - 1) / BSR;
    MFOR2(st, w, nst, Wc) {
      const int h0 = mA + st * BSR;
      float v[BSR + 2][3];
#pragma unroll
      for (int t = 0; t < BSR + 2; ++t) {
        const int hh = h0 + t - 1;
        const bool rv = hh >= 0 && hh < Hc;
        const float* row = Ap + (imin_(imax_(hh, aA), aB - 1) - aA) * Wc;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int ww = w + j - 1;
          const float x = row[imin_(imax_(ww, 0), Wc - 1)] * 255.0f;
          v[t][j] = (rv && ww >= 0 && ww < Wc) ? x : 0.0f;
        }
      }
#pragma unroll
      for (int r = 0; r < BSR; ++r) {
        float gx = 0.0f, gy = 0.0f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const float kx = (i == 1) ? 2.0f : 1.0f;
          const float ky = (float)(i - 1);
          gx = fmaf(-kx, v[r + i][0], gx);
          gx = fmaf(kx, v[r + i][2], gx);
          if (i != 1) {
            gy = fmaf(ky, v[r + i][0], gy);
            gy = fmaf(2.0f * ky, v[r + i][1], gy);
            gy = fmaf(ky, v[r + i][2], gy);
          }
        }
        if (h0 + r < mB) {
          const int p = (h0 + r - mA) * Wc + w;
          Mp[p] = fabsf(gx) + fabsf(gy);
          Dp[p] = (uint8_t)nms_dir(gx, gy);
        }
      }
    }
  }
  MSYNC();
  MSTAMP(4);

  // -- S3a: NMS (replicate-shifted neighbours) of the owned rows -> NMS plane
  float* nmsg = band_nms(S) + (size_t)b * P;
  MFOR2(hr, w, r1 - r0, Wc) {
    const int h = r0 + hr;
    const int d = Dp[(h - mA) * Wc + w];
    const float m = Mp[(h - mA) * Wc + w];
    const int dy1 = (d == 0) ? 0 : -1;
    const int dx1 = (d == 2) ? 0 : ((d == 3) ? -1 : 1);
    const int h1 = imin_(imax_(h + dy1, 0), Hc - 1), w1 = imin_(imax_(w + dx1, 0), Wc - 1);
    const int h2 = imin_(imax_(h - dy1, 0), Hc - 1), w2 = imin_(imax_(w - dx1, 0), Wc - 1);
    const float n1 = Mp[(h1 - mA) * Wc + w1], n2 = Mp[(h2 - mA) * Wc + w2];
    nmsg[h * Wc + w] = (m >= n1 && m >= n2) ? m : 0.0f;
  }
  // -- S3b: Sobel of G (zero pad, phi3) -> gx (row pass space), gy (blur
  //    space) and the uniform-LBP label planes, owned rows
  {
    const int nst = (r1 - r0 + BSR - 1) / BSR;
    MFOR2(st, sl, nst, RS) {
      const int k = sl >> 5, bit = sl & 31, w = sl;
      const int h0 = r0 + st * BSR;
      const int wc = imin_(w, Wc - 1);
      const int wm = imax_(wc - 1, 0), wp = imin_(wc + 1, Wc - 1);
      const bool cl = wc > 0, cr = wc + 1 < Wc;
      float c[BSR + 2][3];
#pragma unroll
      for (int t = 0; t < BSR + 2; ++t) {
        const int hh = imin_(imax_(h0 + t - 1, 0), Hc - 1);
        const float* row = Gp + (imin_(imax_(hh, gA), gB - 1) - gA) * Wc;
        c[t][0] = row[wm]; c[t][1] = row[wc]; c[t][2] = row[wp];
      }
#pragma unroll
      for (int r = 0; r < BSR; ++r) {
        const int h = h0 + r;
        int lab = -1;
        if (w < Wc && h < r1) {
          const bool ru = h > 0, rd = h + 1 < Hc;
          const float ctr = c[r + 1][1];
          const float z00 = (ru && cl) ? c[r][0] : 0.0f, z01 = ru ? c[r][1] : 0.0f;
          const float z02 = (ru && cr) ? c[r][2] : 0.0f;
          const float z10 = cl ? c[r + 1][0] : 0.0f, z12 = cr ? c[r + 1][2] : 0.0f;
          const float z20 = (rd && cl) ? c[r + 2][0] : 0.0f, z21 = rd ? c[r + 2][1] : 0.0f;
          const float z22 = (rd && cr) ? c[r + 2][2] : 0.0f;
          float gx = 0.0f, gy = 0.0f;
          gx = fmaf(-1.0f, z00, gx); gx = fmaf(1.0f, z02, gx);
          gx = fmaf(-2.0f, z10, gx); gx = fmaf(2.0f, z12, gx);
          gx = fmaf(-1.0f, z20, gx); gx = fmaf(1.0f, z22, gx);
          gy = fmaf(-1.0f, z00, gy); gy = fmaf(-2.0f, z01, gy); gy = fmaf(-1.0f, z02, gy);
          gy = fmaf(1.0f, z20, gy); gy = fmaf(2.0f, z21, gy); gy = fmaf(1.0f, z22, gy);
          Hp[(h - gA) * Wc + w] = gx;
          Ap[(h - aA) * Wc + w] = gy;
          int bt[8];
          bt[0] = c[r][0] >= ctr; bt[1] = c[r][1] >= ctr; bt[2] = c[r][2] >= ctr; bt[3] = c[r + 1][2] >= ctr;
          bt[4] = c[r + 2][2] >= ctr; bt[5] = c[r + 2][1] >= ctr; bt[6] = c[r + 2][0] >= ctr; bt[7] = c[r + 1][0] >= ctr;
          int n1 = 0, tr = 0;
#pragma unroll
          for (int qq = 0; qq < 8; ++qq) { n1 += bt[qq]; tr += bt[qq] != bt[(qq + 7) & 7]; }
          lab = tr <= 2 ? n1 : 9;
        }
        if (h < r1) {
#pragma unroll
          for (int qq = 0; qq < 10; ++qq) put_bits(LB + qq * pw, (h - r0) * WPR + k, bit, lab == qq);
        }
      }
    }
  }
  // -- S3c: boundary (m & ~erode3x3, in-bounds neighbours) and Euler quad
  //    classes of the owned rows from BIN
  MFOR2(hr, k, r1 - r0, WPR) {
    const int h = r0 + hr;
    const int nvalid = imin_(Wc - 32 * k, 32);
    const uint32_t vmask = nvalid >= 32 ? 0xFFFFFFFFu : ((1u << nvalid) - 1u);
    const uint32_t rim = (k + 1 == WPR) ? (1u << (nvalid - 1)) : 0u;
    uint32_t er = 0xFFFFFFFFu;
    for (int hh = imax_(h - 1, 0); hh <= imin_(h + 1, Hc - 1); ++hh) {
      const uint32_t* row = BINp + (hh - mA) * WPR;
      const uint32_t c = row[k];
      const uint32_t l = (c << 1) | (k > 0 ? row[k - 1] >> 31 : 1u);
      const uint32_t r = (c >> 1) | (k + 1 < WPR ? row[k + 1] << 31 : 0u) | rim;
      er &= c & l & r;
    }
    const uint32_t* rowm = BINp + (h - mA) * WPR;
    const uint32_t m = rowm[k];
    const int o = hr * WPR + k;
    BND[o] = m & ~er;
    const uint32_t Dq = m;
    const uint32_t Cc = (m << 1) | (k > 0 ? rowm[k - 1] >> 31 : 0u);
    const uint32_t* rowu = BINp + (h - 1 - mA) * WPR;   // read only when h > 0 (then h - 1 >= mA)
    const uint32_t Bq = h > 0 ? rowu[k] : 0u;
    const uint32_t Aq = h > 0 ? ((Bq << 1) | (k > 0 ? rowu[k - 1] >> 31 : 0u)) : 0u;
    const uint32_t odd = Aq ^ Bq ^ Cc ^ Dq;
    const uint32_t pairs = (Aq & Bq) | (Aq & Cc) | (Aq & Dq) | (Bq & Cc) | (Bq & Dq) | (Cc & Dq);
    Q1[o] = odd & ~pairs & vmask;
    Q3[o] = odd & pairs & vmask;
    QD[o] = (((Aq & Dq) & ~(Bq | Cc)) | ((Bq & Cc) & ~(Aq | Dq))) & vmask;
  }
  // -- S3d: the band's histogram out (complete since the S1 barrier); debug BIN
  MFOR(i, 256) band_hist(S)[((size_t)b * nb + band) * 256 + i] = sh.hist[i];
  if (S.bin_out)
    MFOR2(hr, w, r1 - r0, Wc)
      S.bin_out[(size_t)b * P + (r0 + hr) * Wc + w] = (BINp[(r0 + hr - mA) * WPR + (w >> 5)] >> (w & 31)) & 1u;
  MSYNC();
  MSTAMP(5);

  // -- S4: per-tile partials of the owned tile rows (tile_tmp items, as
  //    morph_edges role 1): gradient sums [0,4), LBP terms [4+S, 14+S),
  //    mask counts [15+S, 20+S)
  {
    int S_ = 0;
    for (int s = 2; s <= T; s *= 2) ++S_;
    const int tr0 = r0 / T, NTb = ((r1 - r0) / T) * wt;
    float* ttmp = S.tile_tmp + (size_t)b * NT * TT_STRIDE;
    const int nG = (4 * NTb + 63) & ~63;
    const int nR = 15 * NTb;
    const float inv_nb = 1.0f / (float)NTb, inv_wt = 1.0f / (float)wt;
    MFOR(u, nG + nR) {
      int it, tl;
      if (u < nG) {
        if (u >= 4 * NTb) continue;
        const int kq = div_small(u, NTb, inv_nb);
        it = kq; tl = u - kq * NTb;
      } else {
        const int v = u - nG, kk = div_small(v, NTb, inv_nb);
        tl = v - kk * NTb;
        it = kk < 10 ? 4 + S_ + kk : 15 + S_ + (kk - 10);
      }
      const int th = div_small(tl, wt, inv_wt), tw = tl - th * wt;
      const int h0 = (tr0 + th) * T, w0 = tw * T;
      float val;
      if (it < 4) {
        const float* plane = (it < 2) ? Hp + (h0 - gA) * Wc : Ap + (h0 - aA) * Wc;   // row h0
        const bool sqr = (it & 1) != 0;
        if (T == 4) val = sqr ? tile_sum_t<4, true>(plane, Wc, 0, w0) : tile_sum_t<4, false>(plane, Wc, 0, w0);
        else if (T == 8) val = sqr ? tile_sum_t<8, true>(plane, Wc, 0, w0) : tile_sum_t<8, false>(plane, Wc, 0, w0);
        else val = sqr ? tile_sum_t<16, true>(plane, Wc, 0, w0) : tile_sum_t<16, false>(plane, Wc, 0, w0);
      } else {
        const int kk = it - 4 - S_;   // 0..9 LBP labels, 11 BIN, 12 BND, 13 Q1, 14 Q3, 15 QD
        const uint32_t* plane = kk < 10 ? LB + kk * pw + (h0 - r0) * WPR
                              : (kk == 11 ? BINp + (h0 - mA) * WPR
                              : (kk == 12 ? BND : (kk == 13 ? Q1 : (kk == 14 ? Q3 : QD))) + (h0 - r0) * WPR);
        int cnt;
        if (T == 4) cnt = tile_pop_t<4>(plane, WPR, 0, w0);
        else if (T == 8) cnt = tile_pop_t<8>(plane, WPR, 0, w0);
        else cnt = tile_pop_t<16>(plane, WPR, 0, w0);
        if (kk < 10) val = bits_as_float(T == 4 ? k_lbp_t4_bits[cnt] : (T == 8 ? k_lbp_t8_bits[cnt] : k_lbp_t16_bits[cnt]));
        else val = (float)cnt;
      }
      ttmp[((tr0 + th) * wt + tw) * TT_STRIDE + it] = val;
    }
  }
  MSTAMP(6);
}

// ---- edge kernel body: image b -----------------------------------------------
MCAQ_HD void edge_image(const Ctx& ctx, const MorphScale& S, int b, char* lds) {
  const int Hc = S.Hc, Wc = S.Wc, P = Hc * Wc, T = S.tile, wt = S.wt, NT = S.ht * wt;
  const int nb = band_count(Hc, T), WPR = words_per_row(Wc), RS = WPR * 32;
  Shared sh;
  carve_shared(lds, sh);
  float* Np = (float*)(lds + fixed_bytes());
  uint32_t* E0 = (uint32_t*)(Np + ((P + 3) & ~3));
  uint32_t* E1 = E0 + Hc * WPR;
  uint32_t* WK = E1 + Hc * WPR;
  const float* nmsg = band_nms(S) + (size_t)b * P;
  const int* hp = band_hist(S) + (size_t)b * nb * 256;
  MSTAMP_INIT(b == 0 ? 16 : -1);   // diagnostic build: slots 16-21
  MSTAMP(0);
  // the image's Otsu histogram (integer sums of the bands', exact) and its
  // NMS plane, all loads in flight together
  MFOR(i, 256) {
    int s = 0;
    for (int k = 0; k < nb; ++k) s += hp[k * 256 + i];
    sh.hist[i] = s;
  }
  bcopy<32>(ctx, P, [&](int u) { return nmsg[u]; }, [&](int u, float v) { Np[u] = v; });
  MSYNC();
  MSTAMP(1);
  const float thr = otsu_from_hist(ctx, sh);
  MSTAMP(2);
  const float thr255 = thr * 255.0f;
  const float lo255 = 0.5f * thr255;
  // double threshold -> strong / weak bit planes
  MFOR2(h, sl, Hc, RS) {
    const int k = sl >> 5, bit = sl & 31;
    const float v = Np[h * Wc + imin_(sl, Wc - 1)];
    put_bits(E0, h * WPR + k, bit, sl < Wc && v > thr255);
    put_bits(WK, h * WPR + k, bit, sl < Wc && v > lo255);
  }
  MSYNC();
  MSTAMP(3);
  const uint32_t* edge = hysteresis_run(ctx, E0, E1, WK, Hc, WPR, S.hyst_iters < 1 ? 1 : S.hyst_iters);
  MSTAMP(4);
  // per-tile partials (as morph_edges role 0): box counts [4, 4+S), edge count 14+S
  int S_ = 0;
  for (int s = 2; s <= T; s *= 2) ++S_;
  float* ttmp = S.tile_tmp + (size_t)b * NT * TT_STRIDE;
  const int nG = (S_ * NT + 63) & ~63;
  const float inv_nt = 1.0f / (float)NT, inv_wt = 1.0f / (float)wt;
  MFOR(u, nG + NT) {
    int it, t;
    if (u < nG) {
      if (u >= S_ * NT) continue;
      const int kq = div_small(u, NT, inv_nt);
      it = 4 + kq; t = u - kq * NT;
    } else {
      t = u - nG; it = 14 + S_;
    }
    const int th = div_small(t, wt, inv_wt), tw = t - th * wt;
    const int h0 = th * T, w0 = tw * T;
    float val;
    if (it < 4 + S_) {
      const int s = 2 << (it - 4);
      int n;
      if (T == 4) n = box_count_t<4>(edge, WPR, h0, w0, s);
      else if (T == 8) n = box_count_t<8>(edge, WPR, h0, w0, s);
      else n = box_count_t<16>(edge, WPR, h0, w0, s);
      val = n <= 64 ? bits_as_float(k_lognp1_bits[n]) : cr_log((float)n + 1.0f);
    } else {
      int cnt;
      if (T == 4) cnt = tile_pop_t<4>(edge, WPR, h0, w0);
      else if (T == 8) cnt = tile_pop_t<8>(edge, WPR, h0, w0);
      else cnt = tile_pop_t<16>(edge, WPR, h0, w0);
      val = (float)cnt;
    }
    ttmp[t * TT_STRIDE + it] = val;
  }
  MSTAMP(5);
  if (S.edge_out)
    MFOR2(h, w, Hc, Wc) S.edge_out[(size_t)b * P + h * Wc + w] = (edge[h * WPR + (w >> 5)] >> (w & 31)) & 1u;
}

}  // namespace mcaq
