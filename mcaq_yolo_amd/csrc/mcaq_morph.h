// mcaq_morph.h - per-image morphology -> complexity -> bits -> soft mask.
//
// One workgroup owns one image of one hook scale (its planes live in LDS when
// they fit, else in a global workspace).  The body is written as thread loops
// (MFOR) separated by barriers (MSYNC) so that the identical source also runs
// on the host with one thread (tests/emu), where it is checked against the
// numpy oracle before it ever reaches the GPU.
//
// Reference (yooooonjae/mcaq-yolo):
//   morphology.py:826-873 (_phi_tiles_gpu) and helpers :379-739,
//   morphology.py:81-97 (complexity MLP), :309-354 (bilateral), :939-973,
//   bit_allocation.py:12-80 (LinearBitMapper), :199-280 (MLP mapper),
//   quantization.py:213-239 (LearnedSoftMask),
//   models/mcaq_yolo.py:426-442 (hook: analyzer -> normalize -> mapper).
#pragma once
#include "../../include/mcaq_hip.h"
#include "mcaq_math.h"
#include "mcaq_tables.h"

namespace mcaq {

// ---- packed parameter layouts (host packs the reference state_dict) --------
// complexity MLP: Linear(8,64) LN(64) ReLU Linear(64,32) LN(32) ReLU Linear(32,1)
enum : int {
  CM_W1 = 0, CM_B1 = 512, CM_G1 = 576, CM_BE1 = 640, CM_W2 = 704, CM_B2 = 2752,
  CM_G2 = 2784, CM_BE2 = 2816, CM_W3 = 2848, CM_B3 = 2880, CM_SIZE = 2881
};
// mapper MLP: Linear(3,32) BN ReLU Linear(32,64) BN ReLU Linear(64,32) BN ReLU
// Linear(32,1); each BN block is {gamma, beta, running_mean, running_var}.
enum : int {
  MM_W1 = 0, MM_B1 = 96, MM_BN1 = 128, MM_W2 = 256, MM_B2 = 2304, MM_BN2 = 2368,
  MM_W3 = 2624, MM_B3 = 4672, MM_BN3 = 4704, MM_W4 = 4832, MM_B4 = 4864, MM_SIZE = 4865
};
// soft mask: Conv2d(2,8,3,pad 1) ReLU Conv2d(8,2,1)
enum : int { SM_W1 = 0, SM_B1 = 144, SM_W2 = 152, SM_B2 = 168, SM_SIZE = 170 };

// stage flags
enum : int {
  F_PHI = 1,          // phi tiles from the gray plane
  F_CMLP = 2,         // complexity MLP + bilateral -> C
  F_MAPPER = 4,       // bits from C (computed or c_in)
  F_SOFTMASK = 8,     // m plane from bits (computed or bits_in)
  F_CONT = 16,        // return continuous bits (no STE round)
  F_HAS_T = 32,       // temperature given
  F_NORM_C = 64,      // per-image percentile normalisation of C before mapping
  F_MAP_LINEAR = 128, // LinearBitMapper instead of the MLP
  F_BIN_OTSU = 256,   // binarize_impl='otsu'
  F_NO_EULER = 512,   // contour_components=False
};

using MorphScale = mcaq_morph_scale;  // include/mcaq_hip.h

struct MorphArgs {
  MorphScale s[3];
  int nscales;
};

// bytes of per-image plane storage: 3 fp32 planes + 4 byte planes
MCAQ_HD int plane_bytes(int P) { return 16 * ((P + 3) & ~3); }
// bytes of per-image tile storage (fp32 [NT][TILE_FLOATS])
enum : int { TILE_FLOATS = 16 };
MCAQ_HD int tile_bytes(int NT) { return 4 * TILE_FLOATS * NT; }
// fixed shared scratch: 256 int hist + 2x256 double scan + reductions
enum : int { RED_N = 1024 };
MCAQ_HD int fixed_bytes() { return 256 * 4 + 2 * 256 * 8 * 2 + RED_N * 8 + 64; }

// tile array slots
enum : int {
  T_PHI = 0,   // 8 floats
  T_CMLP = 8, T_C = 9, T_CN = 10, T_BITS = 11, T_ACT = 12, T_MT = 13, T_SORT = 14, T_AUX = 15
};

// ---------------------------------------------------------------------------
// execution context: device = real threads; host emulation = one thread
// ---------------------------------------------------------------------------
struct Ctx { int tid, nthr; };

#if defined(__HIP_DEVICE_COMPILE__)
#define MSYNC() __syncthreads()
#define MATOMIC_ADD(p, v) atomicAdd((p), (v))
#define MATOMIC_OR(p, v) atomicOr((p), (v))
#else
#define MSYNC() do {} while (0)
#define MATOMIC_ADD(p, v) (*(p) += (v))
#define MATOMIC_OR(p, v) (*(p) |= (v))
#endif
#define MFOR(i, n) for (int i = ctx.tid; i < (n); i += ctx.nthr)

struct Shared {
  int* hist;       // 256
  double* scan0;   // 2 x 256 (ping-pong)
  double* scan1;   // 2 x 256
  float* redf;     // RED_N
  int* redi;       // RED_N
  int* flags;      // 16 ints
  float* tiles;    // NT * TILE_FLOATS
};

struct Planes {
  float *G, *A, *Bf;            // fp32 planes
  uint8_t *E0, *E1, *Wk, *Bin;  // byte planes
};

MCAQ_HD void carve_planes(char* base, int P, Planes& pl) {
  const int P4 = (P + 3) & ~3;
  pl.G = (float*)base;
  pl.A = pl.G + P4;
  pl.Bf = pl.A + P4;
  uint8_t* u = (uint8_t*)(pl.Bf + P4);
  pl.E0 = u; pl.E1 = u + P4; pl.Wk = u + 2 * P4; pl.Bin = u + 3 * P4;
}

MCAQ_HD void carve_shared(char* base, int NT, Shared& sh) {
  sh.hist = (int*)base;
  sh.scan0 = (double*)(base + 1024);
  sh.scan1 = sh.scan0 + 512;
  sh.redf = (float*)(sh.scan1 + 512);
  sh.redi = (int*)(sh.redf + RED_N);
  sh.flags = sh.redi + RED_N;
  sh.tiles = (float*)(sh.flags + 16);
  (void)NT;
}

// ---- block reductions through shared memory (tree; exact ops only) --------
MCAQ_HD void block_minmax(const Ctx& ctx, Shared& sh, float lmn, float lmx, float& mn, float& mx) {
  float* rmn = sh.redf;
  int* dummy = sh.redi; (void)dummy;
  float* rmx = (float*)sh.redi;
  rmn[ctx.tid] = lmn; rmx[ctx.tid] = lmx;
  MSYNC();
  for (int s = ctx.nthr / 2; s > 0; s >>= 1) {
    if (ctx.tid < s) {
      rmn[ctx.tid] = fmin_(rmn[ctx.tid], rmn[ctx.tid + s]);
      rmx[ctx.tid] = fmax_(rmx[ctx.tid], rmx[ctx.tid + s]);
    }
    MSYNC();
  }
  mn = rmn[0]; mx = rmx[0];
  MSYNC();
}

MCAQ_HD float block_max(const Ctx& ctx, Shared& sh, float v) {
  float* r = sh.redf;
  r[ctx.tid] = v;
  MSYNC();
  for (int s = ctx.nthr / 2; s > 0; s >>= 1) {
    if (ctx.tid < s) r[ctx.tid] = fmax_(r[ctx.tid], r[ctx.tid + s]);
    MSYNC();
  }
  float m = r[0];
  MSYNC();
  return m;
}

// ---- Otsu (morphology.py:398-418) on a [0,1] plane --------------------------
// Histogram counts are integers (exact in any order); the double prefix sums
// are exact because every partial sum fits in 53 bits, so a parallel scan
// reproduces ATen's sequential double cumsum.
MCAQ_HD float otsu_threshold(const Ctx& ctx, Shared& sh, const float* v, int P) {
  MFOR(i, 256) sh.hist[i] = 0;
  MSYNC();
  MFOR(p, P) {
    const float x = v[p];
    if (x >= 0.0f && x <= 1.0f) {
      int k = (int)(x * 256.0f);
      if (k > 255) k = 255;
      MATOMIC_ADD(&sh.hist[k], 1);
    }
  }
  MSYNC();
  // total count (exact)
  int* ri = sh.redi;
  {
    int loc = 0;
    MFOR(i, 256) loc += sh.hist[i];
    ri[ctx.tid] = loc;
    MSYNC();
    for (int s = ctx.nthr / 2; s > 0; s >>= 1) {
      if (ctx.tid < s) ri[ctx.tid] += ri[ctx.tid + s];
      MSYNC();
    }
  }
  const float total = fmax_((float)ri[0], 1.0f);
  MSYNC();
  double* w0 = sh.scan0;        // omega ping
  double* w1 = sh.scan0 + 256;  // omega pong
  double* m0 = sh.scan1;
  double* m1 = sh.scan1 + 256;
  MFOR(i, 256) {
    const float p = (float)sh.hist[i] / total;
    const float c = ((float)i + 0.5f) / 256.0f;
    w0[i] = (double)p;
    m0[i] = (double)(p * c);
  }
  MSYNC();
  for (int off = 1; off < 256; off <<= 1) {
    MFOR(i, 256) {
      w1[i] = w0[i] + (i >= off ? w0[i - off] : 0.0);
      m1[i] = m0[i] + (i >= off ? m0[i - off] : 0.0);
    }
    MSYNC();
    double* t = w0; w0 = w1; w1 = t;
    t = m0; m0 = m1; m1 = t;
  }
  const float mu_t = (float)m0[255];
  // sigma_b and first argmax
  float* rv = sh.redf;
  int* rix = sh.redi;
  float best = -1.0f; int bi = 0x7fffffff;
  MFOR(i, 256) {
    const float om = (float)w0[i];
    const float mu = (float)m0[i];
    float num = mu_t * om - mu;
    num = num * num;
    const float den = om * (1.0f - om) + 1e-12f;
    const float sb = num / den;
    if (sb > best || (sb == best && i < bi)) { best = sb; bi = i; }
  }
  rv[ctx.tid] = best; rix[ctx.tid] = bi;
  MSYNC();
  for (int s = ctx.nthr / 2; s > 0; s >>= 1) {
    if (ctx.tid < s) {
      const float a = rv[ctx.tid], b = rv[ctx.tid + s];
      const int ia = rix[ctx.tid], ib = rix[ctx.tid + s];
      if (b > a || (b == a && ib < ia)) { rv[ctx.tid] = b; rix[ctx.tid] = ib; }
    }
    MSYNC();
  }
  const int idx = rix[0];
  MSYNC();
  return ((float)idx + 0.5f) / 256.0f;
}

// ---- small fixed-size sums in ATen order ------------------------------------
// n <= 8 values: vector column = sequential; tail column = row_sum.
MCAQ_HD float small_sum(const float (&v)[8], int n, bool tail) {
  if (!tail) {
    float a = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) if (i < n) a = a + v[i];
    return a;
  }
  const int nilp = n / 4;
  float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if (r < nilp) p[k] = p[k] + v[4 * r + k];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i >= 4 * nilp && i < n) p[0] = p[0] + v[i];
  return ((p[0] + p[1]) + p[2]) + p[3];
}

template <int N>
MCAQ_HD float aten_sum_n(const float (&v)[N], bool tail) {
  if (!tail) {
    Cascade c; c.init();
#pragma unroll
    for (int r = 0; r < N; ++r) c.push(v[r]);
    return c.result();
  }
  constexpr int nilp = N / 4;
  Cascade c0, c1, c2, c3;
  c0.init(); c1.init(); c2.init(); c3.init();
#pragma unroll
  for (int r = 0; r < nilp; ++r) {
    c0.push(v[4 * r]); c1.push(v[4 * r + 1]); c2.push(v[4 * r + 2]); c3.push(v[4 * r + 3]);
  }
  float p0 = c0.result();
#pragma unroll
  for (int r = 4 * nilp; r < N; ++r) p0 = p0 + v[r];
  return ((p0 + c1.result()) + c2.result()) + c3.result();
}

// pairwise tree over N (power of two) values: the LayerNorm statistic order
template <int N>
MCAQ_HD float tree_sum(const float (&v)[N]) {
  float t[N];
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = v[i];
#pragma unroll
  for (int w = N; w > 1; w >>= 1) {
#pragma unroll
    for (int i = 0; i < w / 2; ++i) t[i] = t[2 * i] + t[2 * i + 1];
  }
  return t[0];
}

template <int N>
MCAQ_HD void layernorm(float (&h)[N], const float* g, const float* b) {
  const float mean = tree_sum<N>(h) / (float)N;
  float d2[N];
#pragma unroll
  for (int i = 0; i < N; ++i) { h[i] = h[i] - mean; d2[i] = h[i] * h[i]; }
  const float var = tree_sum<N>(d2) / (float)N;
  const float rstd = 1.0f / cr_sqrt(var + 1e-5f);
#pragma unroll
  for (int i = 0; i < N; ++i) h[i] = ((h[i] * rstd) * g[i]) + b[i];
}

MCAQ_HD float sigmoid_(float z) { return 1.0f / (1.0f + cr_exp(-z)); }

// complexity MLP on one tile's 8 features (morphology.py:81-97)
MCAQ_HD float complexity_mlp_tile(const float* P, const float (&phi)[8]) {
  float h1[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) a = fmaf(phi[k], P[CM_W1 + j * 8 + k], a);
    h1[j] = a + P[CM_B1 + j];
  }
  layernorm<64>(h1, P + CM_G1, P + CM_BE1);
#pragma unroll
  for (int j = 0; j < 64; ++j) h1[j] = fmax_(h1[j], 0.0f);
  float h2[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < 64; ++k) a = fmaf(h1[k], P[CM_W2 + j * 64 + k], a);
    h2[j] = a + P[CM_B2 + j];
  }
  layernorm<32>(h2, P + CM_G2, P + CM_BE2);
  float a = 0.0f;
#pragma unroll
  for (int k = 0; k < 32; ++k) a = fmaf(fmax_(h2[k], 0.0f), P[CM_W3 + k], a);
  return sigmoid_(a + P[CM_B3]);
}

// BatchNorm1d eval as ATen folds it: alpha = inv*g, beta = b - (rm*inv)*g
MCAQ_HD float bn_eval(float x, const float* bn, int n, int j) {
  const float inv = 1.0f / cr_sqrt(bn[3 * n + j] + 1e-5f);
  const float alpha = inv * bn[j];
  const float beta = bn[n + j] - (bn[2 * n + j] * inv) * bn[j];
  return x * alpha + beta;
}

// MLP mapper pre-temperature bits for one complexity value
// (bit_allocation.py:199-261)
MCAQ_HD float mapper_mlp_tile(const float* P, float c, float min_bits, float max_bits) {
  c = clampf_(c, 0.0f, 1.0f);
  const float z[3] = {c, c * c, cr_log1p(c)};
  float h1[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) a = fmaf(z[k], P[MM_W1 + j * 3 + k], a);
    h1[j] = fmax_(bn_eval(a + P[MM_B1 + j], P + MM_BN1, 32, j), 0.0f);
  }
  float h2[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; ++k) a = fmaf(h1[k], P[MM_W2 + j * 32 + k], a);
    h2[j] = fmax_(bn_eval(a + P[MM_B2 + j], P + MM_BN2, 64, j), 0.0f);
  }
  float a4 = 0.0f;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < 64; ++k) a = fmaf(h2[k], P[MM_W3 + j * 64 + k], a);
    const float h3 = fmax_(bn_eval(a + P[MM_B3 + j], P + MM_BN3, 32, j), 0.0f);
    a4 = fmaf(h3, P[MM_W4 + j], a4);
  }
  const float h = sigmoid_(a4 + P[MM_B4]);
  return min_bits + (max_bits - min_bits) * h;
}

// temperature, STE clamp, STE round forward values (bit_allocation.py:264-278)
MCAQ_HD float finish_bits(float bm, const MorphScale& S) {
  if (S.flags & F_HAS_T) bm = bm * S.temperature;  // temperature pre-clamped to >= 0.1 by host
  const float cl = clampf_(bm, S.min_bits, S.max_bits);
  float v = bm + (cl - bm);
  if (!(S.flags & F_CONT)) v = v + (rintf(v) - v);
  return v;
}

// torch.quantile(linear) of the n values sorted in `sorted`
MCAQ_HD float quantile_sorted(const float* sorted, int stride, int n, float q) {
  const float rank = q * (float)(n - 1);
  const int lo = (int)rank;
  const int hi = (int)ceilf(rank);
  const float w = rank - (float)lo;
  const float a = sorted[lo * stride], b = sorted[hi * stride];
  const float d = b - a;
  if (fabsf(w) < 0.5f) return fmaf(w, d, a);
  return fmaf(-d, 1.0f - w, b);
}

// sort slot src of the tile array into slot T_SORT (rank sort, exact)
MCAQ_HD void sort_tiles(const Ctx& ctx, float* tiles, int NT, int src) {
  MFOR(t, NT) {
    const float v = tiles[t * TILE_FLOATS + src];
    int r = 0;
    for (int u = 0; u < NT; ++u) {
      const float w = tiles[u * TILE_FLOATS + src];
      r += (w < v) || (w == v && u < t);
    }
    tiles[r * TILE_FLOATS + T_SORT] = v;
  }
  MSYNC();
}

// ---- the per-image pipeline -------------------------------------------------
MCAQ_HD void morph_image(const Ctx& ctx, const MorphScale& S, int b, Planes& pl, Shared& sh) {
  const int Hc = S.Hc, Wc = S.Wc, P = Hc * Wc, T = S.tile, ht = S.ht, wt = S.wt, NT = ht * wt;
  const int T2 = T * T;
  float* tiles = sh.tiles;
  const float K180 = (float)(180.0 / 3.14159265358979323846);
  const float FOURPI = (float)(4.0 * 3.14159265358979323846);
  const float LOG2_10 = (float)3.321928094887362;

  if (S.flags & F_PHI) {
    // -- gray (channel mean from the stats pass) + per-image normalise01
    const float* gin = S.gray + (size_t)b * P;
    float lmn = 3.402823466e38f, lmx = -3.402823466e38f;
    MFOR(p, P) { const float v = gin[p]; pl.G[p] = v; lmn = fmin_(lmn, v); lmx = fmax_(lmx, v); }
    float mn, mx;
    block_minmax(ctx, sh, lmn, lmx, mn, mx);
    const float den = (mx - mn) + 1e-8f;
    MFOR(p, P) pl.G[p] = (pl.G[p] - mn) / den;
    MSYNC();

    // -- Canny, cv2compat (morphology.py:458-509)
    // 5x5 Gaussian blur, zero pad, oneDNN tap order
    MFOR(p, P) {
      const int h = p / Wc, w = p - (p / Wc) * Wc;
      float acc = 0.0f;
      for (int i = 0; i < 5; ++i) {
        const int hh = h + i - 2;
        if (hh < 0 || hh >= Hc) continue;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const int ww = w + j - 2;
          if (ww < 0 || ww >= Wc) continue;
          acc = fmaf(bits_as_float(k_gauss5_bits[i * 5 + j]), pl.G[hh * Wc + ww], acc);
        }
      }
      pl.A[p] = acc;
    }
    MSYNC();
    const float thr = otsu_threshold(ctx, sh, pl.A, P);
    const float thr255 = thr * 255.0f;
    const float lo255 = 0.5f * thr255;
    // Sobel of 255*blur, L1 magnitude and direction bin
    uint8_t* dir = pl.E1;
    MFOR(p, P) {
      const int h = p / Wc, w = p - (p / Wc) * Wc;
      float gx = 0.0f, gy = 0.0f;
      for (int i = 0; i < 3; ++i) {
        const int hh = h + i - 1;
        if (hh < 0 || hh >= Hc) continue;
        for (int j = 0; j < 3; ++j) {
          const int ww = w + j - 1;
          if (ww < 0 || ww >= Wc) continue;
          const float v = pl.A[hh * Wc + ww] * 255.0f;
          const float kx = (float)((j - 1) * (i == 1 ? 2 : 1));
          const float ky = (float)((i - 1) * (j == 1 ? 2 : 1));
          if (kx != 0.0f) gx = fmaf(kx, v, gx);
          if (ky != 0.0f) gy = fmaf(ky, v, gy);
        }
      }
      pl.Bf[p] = fabsf(gx) + fabsf(gy);
      float ang = cr_atan2(gy, gx) * K180;
      if (ang < 0.0f) ang = ang + 180.0f;
      uint8_t d = 0;
      if (ang >= 22.5f && ang < 67.5f) d = 1;
      else if (ang >= 67.5f && ang < 112.5f) d = 2;
      else if (ang >= 112.5f && ang < 157.5f) d = 3;
      dir[p] = d;
    }
    MSYNC();
    // NMS (replicate-shifted neighbours) + double threshold
    MFOR(p, P) {
      const int h = p / Wc, w = p - (p / Wc) * Wc;
      const int d = dir[p];
      int dy1, dx1;
      if (d == 0) { dy1 = 0; dx1 = 1; }
      else if (d == 1) { dy1 = -1; dx1 = 1; }
      else if (d == 2) { dy1 = -1; dx1 = 0; }
      else { dy1 = -1; dx1 = -1; }
      const int h1 = imin_(imax_(h + dy1, 0), Hc - 1), w1 = imin_(imax_(w + dx1, 0), Wc - 1);
      const int h2 = imin_(imax_(h - dy1, 0), Hc - 1), w2 = imin_(imax_(w - dx1, 0), Wc - 1);
      const float m = pl.Bf[p];
      const bool keep = (m >= pl.Bf[h1 * Wc + w1]) && (m >= pl.Bf[h2 * Wc + w2]);
      const float nms = keep ? m : 0.0f;
      pl.E0[p] = nms > thr255 ? 1 : 0;
      pl.Wk[p] = nms > lo255 ? 1 : 0;
    }
    MSYNC();
    // hysteresis: Jacobi 3x3 dilation passes gated by weak, early exit when stable
    uint8_t* src = pl.E0;
    uint8_t* dst = pl.E1;
    if (ctx.tid == 0) { sh.flags[0] = 0; sh.flags[1] = 0; sh.flags[2] = 0; }
    MSYNC();
    const int iters = S.hyst_iters < 1 ? 1 : S.hyst_iters;
    for (int it = 0; it < iters; ++it) {
      int changed = 0;
      MFOR(p, P) {
        uint8_t v = src[p];
        if (!v && pl.Wk[p]) {
          const int h = p / Wc, w = p - (p / Wc) * Wc;
          for (int dy = -1; dy <= 1 && !v; ++dy) {
            const int hh = h + dy;
            if (hh < 0 || hh >= Hc) continue;
            for (int dx = -1; dx <= 1; ++dx) {
              const int ww = w + dx;
              if (ww < 0 || ww >= Wc) continue;
              if (src[hh * Wc + ww]) { v = 1; break; }
            }
          }
          changed |= v;
        }
        dst[p] = v;
      }
      if (ctx.tid == 0) sh.flags[(it + 1) % 3] = 0;
      if (changed) MATOMIC_OR(&sh.flags[it % 3], 1);
      MSYNC();
      const int any = sh.flags[it % 3];
      uint8_t* t = src; src = dst; dst = t;
      if (!any) break;
    }
    uint8_t* edge = src;     // final edge map
    uint8_t* lbl = dst;      // free byte plane (LBP labels below)
    MSYNC();

    // -- foreground mask for phi5
    if (S.flags & F_BIN_OTSU) {
      const float t2 = otsu_threshold(ctx, sh, pl.G, P);
      MFOR(p, P) pl.Bin[p] = pl.G[p] > t2 ? 1 : 0;
      MSYNC();
    } else {
      // adaptive threshold (morphology.py:551-573): g255 > G11(g255) - 2
      MFOR(p, P) pl.A[p] = pl.G[p] * 255.0f;
      MSYNC();
      MFOR(p, P) {
        const int h = p / Wc, w = p - (p / Wc) * Wc;
        float acc = 0.0f;
        for (int i = 0; i < 11; ++i) {
          const int hh = imin_(imax_(h + i - 5, 0), Hc - 1);
          const float* row = pl.A + hh * Wc;
#pragma unroll
          for (int j = 0; j < 11; ++j) {
            const int ww = imin_(imax_(w + j - 5, 0), Wc - 1);
            acc = fmaf(bits_as_float(k_gauss11_bits[i * 11 + j]), row[ww], acc);
          }
        }
        pl.Bin[p] = pl.A[p] > (acc - 2.0f) ? 1 : 0;
      }
      MSYNC();
    }

    // -- Sobel of the normalised gray (phi3) -> A = gx, Bf = gy; LBP labels
    MFOR(p, P) {
      const int h = p / Wc, w = p - (p / Wc) * Wc;
      float gx = 0.0f, gy = 0.0f;
      for (int i = 0; i < 3; ++i) {
        const int hh = h + i - 1;
        if (hh < 0 || hh >= Hc) continue;
        for (int j = 0; j < 3; ++j) {
          const int ww = w + j - 1;
          if (ww < 0 || ww >= Wc) continue;
          const float v = pl.G[hh * Wc + ww];
          const float kx = (float)((j - 1) * (i == 1 ? 2 : 1));
          const float ky = (float)((i - 1) * (j == 1 ? 2 : 1));
          if (kx != 0.0f) gx = fmaf(kx, v, gx);
          if (ky != 0.0f) gy = fmaf(ky, v, gy);
        }
      }
      pl.A[p] = gx;
      pl.Bf[p] = gy;
      // uniform LBP label (morphology.py:630-646), replicate pad, nb >= center
      const float c = pl.G[p];
      const int hm = imax_(h - 1, 0), hp = imin_(h + 1, Hc - 1);
      const int wm = imax_(w - 1, 0), wp = imin_(w + 1, Wc - 1);
      int bit[8];
      bit[0] = pl.G[hm * Wc + wm] >= c; bit[1] = pl.G[hm * Wc + w] >= c;
      bit[2] = pl.G[hm * Wc + wp] >= c; bit[3] = pl.G[h * Wc + wp] >= c;
      bit[4] = pl.G[hp * Wc + wp] >= c; bit[5] = pl.G[hp * Wc + w] >= c;
      bit[6] = pl.G[hp * Wc + wm] >= c; bit[7] = pl.G[h * Wc + wm] >= c;
      int n1 = 0, tr = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) { n1 += bit[k]; tr += bit[k] != bit[(k + 7) & 7]; }
      lbl[p] = (uint8_t)(tr <= 2 ? n1 : 9);
    }
    MSYNC();
    if (S.edge_out) MFOR(p, P) S.edge_out[(size_t)b * P + p] = edge[p];
    if (S.bin_out) MFOR(p, P) S.bin_out[(size_t)b * P + p] = pl.Bin[p];

    // -- per-tile descriptors phi1..phi5 + interactions
    int S_ = 0;
    for (int s = 2; s <= T; s *= 2) ++S_;
    const int Mcols = S.batch_total * NT;
    const int ycut = aten_tail_start(Mcols);
    // constants of the weighted regression (morphology.py:604-619)
    float xs[8], ws[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      xs[i] = i < S_ ? cr_log((float)(2 << i)) : 0.0f;
      ws[i] = i < S_ ? cr_exp(-0.1f * (float)i) : 0.0f;
    }
    const float w_sum = small_sum(ws, S_, true);
    float wx[8], wdx2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) wx[i] = ws[i] * xs[i];
    const float x_mean = small_sum(wx, S_, true) / w_sum;
#pragma unroll
    for (int i = 0; i < 8; ++i) { const float dx = xs[i] - x_mean; wdx2[i] = ws[i] * (dx * dx); }
    const float var = small_sum(wdx2, S_, true);

    MFOR(t, NT) {
      const int th = t / wt, tw = t - (t / wt) * wt;
      const int h0 = th * T, w0 = tw * T;
      // phi1: box counting (morphology.py:576-621)
      float p1 = 1.0f;
      if (S_ >= 2) {
        float ys[8];
        int si = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) ys[i] = 0.0f;
        for (int s = 2; s <= T; s *= 2, ++si) {
          int n = 0;
          for (int by = 0; by < T; by += s)
            for (int bx = 0; bx < T; bx += s) {
              int occ = 0;
              for (int yy = 0; yy < s && !occ; ++yy)
                for (int xx = 0; xx < s; ++xx)
                  if (edge[(h0 + by + yy) * Wc + w0 + bx + xx]) { occ = 1; break; }
              n += occ;
            }
          const float y = cr_log((float)n + 1.0f);
#pragma unroll
          for (int i = 0; i < 8; ++i) if (i == si) ys[i] = y;
        }
        const bool tail = ((S.batch_offset + b) * NT + t) >= ycut;
        float wy[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) wy[i] = ws[i] * ys[i];
        const float y_mean = small_sum(wy, S_, tail) / w_sum;
        float cv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) cv[i] = (ws[i] * (xs[i] - x_mean)) * (ys[i] - y_mean);
        const float cov = small_sum(cv, S_, tail);
        float df = -(cov / (var + 1e-12f));
        df = clampf_(df, 1.0f, 2.0f);
        p1 = df / 2.0f;
      } else {
        p1 = 1.0f / 2.0f;
      }
      // phi2: LBP histogram entropy; bins summed 8, 9, 0..7 (channels-last)
      int cnt[10];
#pragma unroll
      for (int k = 0; k < 10; ++k) cnt[k] = 0;
      // phi3 sums, phi4 count, phi5 area/perimeter/Euler
      float sgx = 0.0f, sgx2 = 0.0f, sgy = 0.0f, sgy2 = 0.0f;
      int ecount = 0, area = 0, perim = 0;
      float esum = 0.0f;
      for (int yy = 0; yy < T; ++yy) {
        const int h = h0 + yy;
        for (int xx = 0; xx < T; ++xx) {
          const int w = w0 + xx;
          const int q = h * Wc + w;
          const int lb = lbl[q];
#pragma unroll
          for (int k = 0; k < 10; ++k) cnt[k] += (lb == k);
          const float gx = pl.A[q], gy = pl.Bf[q];
          sgx = sgx + gx; sgx2 = sgx2 + gx * gx;
          sgy = sgy + gy; sgy2 = sgy2 + gy * gy;
          ecount += edge[q];
          const int m = pl.Bin[q];
          area += m;
          if (m) {
            int mn3 = 1;
            for (int dy = -1; dy <= 1; ++dy) {
              const int hh = h + dy;
              if (hh < 0 || hh >= Hc) continue;
              for (int dx = -1; dx <= 1; ++dx) {
                const int ww = w + dx;
                if (ww < 0 || ww >= Wc) continue;
                mn3 &= pl.Bin[hh * Wc + ww];
              }
            }
            perim += 1 - mn3;
          }
          // Euler quad of window (h, w): m[h-1][w-1]*1 + m[h-1][w]*2 + m[h][w-1]*4 + m[h][w]*8
          const int a = (h > 0 && w > 0) ? pl.Bin[q - Wc - 1] : 0;
          const int bq = (h > 0) ? pl.Bin[q - Wc] : 0;
          const int c = (w > 0) ? pl.Bin[q - 1] : 0;
          const int idx = a + 2 * bq + 4 * c + 8 * m;
          float e = 0.0f;
          if (idx == 1 || idx == 2 || idx == 4 || idx == 8) e = 0.25f;
          else if (idx == 7 || idx == 11 || idx == 13 || idx == 14) e = -0.25f;
          else if (idx == 6 || idx == 9) e = -0.5f;
          esum = esum + e;
        }
      }
      float terms[10];
      const float invT2 = (float)T2;
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        const float pk = (float)cnt[k] / invT2;
        terms[k] = pk * log2_ref(pk + 1e-10f);
      }
      float ent = 0.0f;
      ent = ent + terms[8]; ent = ent + terms[9];
#pragma unroll
      for (int k = 0; k < 8; ++k) ent = ent + terms[k];
      const float p2 = (-ent) / LOG2_10;
      // phi3
      const float mgx = sgx / invT2, mgx2 = sgx2 / invT2;
      const float mgy = sgy / invT2, mgy2 = sgy2 / invT2;
      const float vx = fmax_(mgx2 - mgx * mgx, 0.0f);
      const float vy = fmax_(mgy2 - mgy * mgy, 0.0f);
      const float v = vx + vy;
      const float p3 = v / (v + 1.0f);
      // phi4
      const float p4 = (float)ecount / invT2;
      // phi5
      const float fa = (float)area, fp = (float)perim;
      float ic = (fp * fp) / (FOURPI * fa + 1e-6f);
      if (!(S.flags & F_NO_EULER)) {
        const float Kr = (esum / invT2) * invT2;
        const float Kc = fmax_(rintf(Kr), 1.0f);
        ic = ic / Kc;
      }
      float p5 = 1.0f - 1.0f / fmax_(ic, 1.0f);
      if (!(area > 0)) p5 = 0.0f;
      const float p8 = cr_sqrt(p4 * p5 + 1e-12f);
      float* tp = tiles + t * TILE_FLOATS + T_PHI;
      tp[0] = p1; tp[1] = p2; tp[2] = p3; tp[3] = p4; tp[4] = p5;
      tp[5] = p1 * p2; tp[6] = p3 * p3; tp[7] = p8;
      if (S.phi_out) {
        float* o = S.phi_out + ((size_t)b * NT + t) * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = tp[k];
      }
    }
    MSYNC();
  }

  // -- complexity MLP + bilateral (morphology.py:959-968)
  if (S.flags & F_CMLP) {
    MFOR(t, NT) {
      float phi[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) phi[k] = tiles[t * TILE_FLOATS + T_PHI + k];
      const float c = complexity_mlp_tile(S.cmlp, phi);
      tiles[t * TILE_FLOATS + T_CMLP] = c;
      if (S.cmlp_out) S.cmlp_out[(size_t)b * NT + t] = c;
    }
    MSYNC();
    const int cut = aten_tail_start(NT);
    MFOR(t, NT) {
      const int th = t / wt, tw = t - (t / wt) * wt;
      const float ctr = tiles[t * TILE_FLOATS + T_CMLP];
      float wv[25], wp[25];
#pragma unroll
      for (int k = 0; k < 25; ++k) {
        const int i = k / 5, j = k % 5;
        const int hh = imin_(imax_(th + i - 2, 0), ht - 1);
        const int ww = imin_(imax_(tw + j - 2, 0), wt - 1);
        const float pv = tiles[(hh * wt + ww) * TILE_FLOATS + T_CMLP];
        const float d = pv - ctr;
        const float rw = cr_exp((-(d * d)) / 0.02f);
        wv[k] = bits_as_float(k_bilat_sp_bits[k]) * rw;
        wp[k] = wv[k] * pv;
      }
      const bool tail = t >= cut;
      const float num = aten_sum_n<25>(wp, tail);
      const float den = aten_sum_n<25>(wv, tail);
      const float c = clampf_(num / (den + 1e-8f), 0.0f, 1.0f);
      tiles[t * TILE_FLOATS + T_C] = c;
      if (S.c_out) S.c_out[(size_t)b * NT + t] = c;
    }
    MSYNC();
  } else if (S.c_in) {
    MFOR(t, NT) tiles[t * TILE_FLOATS + T_C] = S.c_in[(size_t)b * NT + t];
    MSYNC();
  }

  // -- optional percentile normalisation (models/mcaq_yolo.py:427-432) and mapper
  if (S.flags & F_MAPPER) {
    int csrc = T_C;
    if (S.flags & F_NORM_C) {
      sort_tiles(ctx, tiles, NT, T_C);
      const float lo = quantile_sorted(tiles + T_SORT, TILE_FLOATS, NT, 0.02f);
      const float hi = quantile_sorted(tiles + T_SORT, TILE_FLOATS, NT, 0.98f);
      MSYNC();
      const float den = (hi - lo) + 1e-8f;
      MFOR(t, NT) {
        const float c = tiles[t * TILE_FLOATS + T_C];
        tiles[t * TILE_FLOATS + T_CN] = clampf_((c - lo) / den, 0.0f, 1.0f);
      }
      MSYNC();
      csrc = T_CN;
    }
    if (S.flags & F_MAP_LINEAR) {
      // LinearBitMapper (bit_allocation.py:42-80)
      sort_tiles(ctx, tiles, NT, csrc);
      const float lo = quantile_sorted(tiles + T_SORT, TILE_FLOATS, NT, 0.02f);
      const float hi = quantile_sorted(tiles + T_SORT, TILE_FLOATS, NT, 0.98f);
      MSYNC();
      const float spread = hi - lo;
      MFOR(t, NT) {
        const float c = tiles[t * TILE_FLOATS + csrc];
        const float rel = clampf_((c - lo) / (spread + 1e-8f), 0.0f, 1.0f);
        const float cn = spread > 1e-3f ? rel : clampf_(c, 0.0f, 1.0f);
        const float bm = S.min_bits + (S.max_bits - S.min_bits) * cn;
        const float bv = finish_bits(bm, S);
        tiles[t * TILE_FLOATS + T_BITS] = bv;
        if (S.bits_out) S.bits_out[(size_t)b * NT + t] = bv;
      }
    } else {
      MFOR(t, NT) {
        const float bm = mapper_mlp_tile(S.mapper, tiles[t * TILE_FLOATS + csrc], S.min_bits, S.max_bits);
        const float bv = finish_bits(bm, S);
        tiles[t * TILE_FLOATS + T_BITS] = bv;
        if (S.bits_out) S.bits_out[(size_t)b * NT + t] = bv;
      }
    }
    MSYNC();
  } else if ((S.flags & F_SOFTMASK) && S.bits_in) {
    MFOR(t, NT) tiles[t * TILE_FLOATS + T_BITS] = S.bits_in[(size_t)b * NT + t];
    MSYNC();
  }

  // -- learned soft mask m(p) (quantization.py:213-239)
  if (S.flags & F_SOFTMASK) {
    const int H = S.H, W = S.W;
    const float* am = S.absmean + (size_t)b * H * W;
    float lmx = -3.402823466e38f;
    MFOR(t, NT) {
      const int i = t / wt, j = t - (t / wt) * wt;
      const int ha = (i * H) / ht, hb = ((i + 1) * H + ht - 1) / ht;
      const int wa = (j * W) / wt, wb = ((j + 1) * W + wt - 1) / wt;
      float s = 0.0f;
      for (int h = ha; h < hb; ++h)
        for (int w = wa; w < wb; ++w) s = s + am[h * W + w];
      const float a = (s / (float)(hb - ha)) / (float)(wb - wa);
      tiles[t * TILE_FLOATS + T_ACT] = a;
      lmx = fmax_(lmx, a);
    }
    const float amax = block_max(ctx, sh, lmx);
    MFOR(t, NT) {
      float* tp = tiles + t * TILE_FLOATS;
      tp[T_AUX] = clampf_((tp[T_BITS] - 2.0f) / 6.0f, 0.0f, 1.0f);
    }
    MSYNC();
    const float* Pm = S.smask;
    const float den = amax + 1e-8f;
    MFOR(t, NT) {
      const int i = t / wt, j = t - (t / wt) * wt;
      float hid[8];
#pragma unroll
      for (int oc = 0; oc < 8; ++oc) {
        float acc = 0.0f;
        for (int ki = 0; ki < 3; ++ki) {
          const int ii = i + ki - 1;
          if (ii < 0 || ii >= ht) continue;
          for (int kj = 0; kj < 3; ++kj) {
            const int jj = j + kj - 1;
            if (jj < 0 || jj >= wt) continue;
            const float* nb = tiles + (ii * wt + jj) * TILE_FLOATS;
            acc = fmaf(Pm[SM_W1 + ((oc * 2 + 0) * 3 + ki) * 3 + kj], nb[T_AUX], acc);
            acc = fmaf(Pm[SM_W1 + ((oc * 2 + 1) * 3 + ki) * 3 + kj], nb[T_ACT] / den, acc);
          }
        }
        hid[oc] = fmax_(acc + Pm[SM_B1 + oc], 0.0f);
      }
      float l0 = Pm[SM_B2 + 0], l1 = Pm[SM_B2 + 1];
#pragma unroll
      for (int ic = 0; ic < 8; ++ic) {
        l0 = fmaf(Pm[SM_W2 + ic], hid[ic], l0);
        l1 = fmaf(Pm[SM_W2 + 8 + ic], hid[ic], l1);
      }
      const float mxl = fmax_(l0, l1);
      const float e0 = cr_exp(l0 - mxl), e1 = cr_exp(l1 - mxl);
      tiles[t * TILE_FLOATS + T_MT] = e0 / (e0 + e1);
    }
    MSYNC();
    if (S.m_out) {
      float* mo = S.m_out + (size_t)b * H * W;
      MFOR(p, H * W) {
        const int h = p / W, w = p - (p / W) * W;
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const int hh = imin_(imax_(h + i - 2, 0), H - 1);
          const int si = nearest_src(hh, ht, H);
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            const int ww = imin_(imax_(w + j - 2, 0), W - 1);
            const int sj = nearest_src(ww, wt, W);
            acc = fmaf(bits_as_float(k_smooth5_bits[i * 5 + j]), tiles[(si * wt + sj) * TILE_FLOATS + T_MT], acc);
          }
        }
        mo[p] = acc;
      }
    }
    MSYNC();
  }
}

}  // namespace mcaq
