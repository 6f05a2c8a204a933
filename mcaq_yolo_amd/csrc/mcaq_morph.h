// mcaq_morph.h - per-image morphology -> complexity -> bits -> soft mask.
//
// One workgroup owns one image of one hook scale.  Its working set lives in
// LDS when it fits (else in a global workspace): three fp32 planes (gray,
// scratch, scratch), one byte plane (Canny direction) and 18 BIT planes
// (32 pixels per word, built with wave ballots): edges (2, ping-pong), weak
// edges, foreground mask, its boundary, the three Euler quad classes and the
// ten uniform-LBP labels.  Hysteresis, erosion and every per-tile count are
// word operations / popcounts on those bit planes.
//
// The body is written as thread loops (MFOR) separated by barriers (MSYNC) so
// that the identical source also runs on the host with one thread
// (tests/emu/), where it is checked bit-for-bit against the numpy oracle
// before it reaches the GPU.  Device-only fast paths (wave shuffles, ballots,
// fp32 MFMA) compute the same exact values as their host counterparts.
//
// Reference (yooooonjae/mcaq-yolo):
//   morphology.py:826-873 (_phi_tiles_gpu) and helpers :379-739,
//   morphology.py:81-97 (complexity MLP), :309-354 (bilateral), :939-973,
//   bit_allocation.py:12-80 (LinearBitMapper), :199-280 (MLP mapper),
//   quantization.py:213-239 (LearnedSoftMask),
//   models/mcaq_yolo.py:426-442 (hook: analyzer -> normalize -> mapper).
#pragma once
#include <utility>
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
// blob sizes including the MFMA A-operand copies appended by params.py
// (mcaq_mlp_mfma.h: CMQ_* / MMQ_*)
enum : int { CM_BLOB = 2881 + 512 + 2048, MM_BLOB = 4865 + 128 + 2048 + 2048 };
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
  F_CANNY_LEGACY = 1024,  // canny_impl='legacy'
  F_TILES_IMAGE = 2048,   // pass B per image (morph_tiles) even where the batch-wide tile kernels apply
  F_IMAGE_BATCH = 4096,   // every image as its own batch of one (batch_offset 0, batch_total 1): the
                          // values of the reference's batch-1 calls (compute_dataset_complexity)
};


using MorphScale = mcaq_morph_scale;  // include/mcaq_hip.h

// global position of image b in the batch whose ATen reductions the kernels
// reproduce, and that batch's size (F_IMAGE_BATCH: each image alone)
MCAQ_HD int img_global(const MorphScale& S, int b) { return (S.flags & F_IMAGE_BATCH) ? 0 : S.batch_offset + b; }
MCAQ_HD int img_batch_total(const MorphScale& S) { return (S.flags & F_IMAGE_BATCH) ? 1 : S.batch_total; }

constexpr int MORPH_MAXSEG = MCAQ_MAX_SEGMENTS;   // segments (hook scale x batch) per launch

struct MorphArgs {
  MorphScale s[MORPH_MAXSEG];
  int nscales;
  // pass A packing (set by the launcher): images per workgroup, LDS bytes per
  // image group (planes + shared, or shared only), plane bytes per image, and
  // the first workgroup of each segment (wg_begin[nscales] = pass A workgroups)
  int ipw[MORPH_MAXSEG], gstride[MORPH_MAXSEG], pstride[MORPH_MAXSEG], wg_begin[MORPH_MAXSEG + 1];
  // pass B packing: images per workgroup, LDS bytes per image, first workgroup
  int tipw[MORPH_MAXSEG], tgstride[MORPH_MAXSEG], twg_begin[MORPH_MAXSEG + 1];
  // band mode of pass A (mcaq_band.h): first band / edge workgroup of each segment
  int bwg_begin[MORPH_MAXSEG + 1], ewg_begin[MORPH_MAXSEG + 1];
  // batch-wide pass B (mcaq_tiles_batch.h): first 64-tile workgroup of each segment
  int tb_begin[MORPH_MAXSEG + 1];
};

// bit planes
enum : int { BP_E0 = 0, BP_E1, BP_WK, BP_BIN, BP_BND, BP_Q1, BP_Q3, BP_QD, BP_L0, BP_COUNT = BP_L0 + 10 };

MCAQ_HD int words_per_row(int Wc) { return (Wc + 31) >> 5; }
// bytes of per-image plane storage
MCAQ_HD int plane_bytes(int Hc, int Wc) {
  const int P4 = (Hc * Wc + 3) & ~3;
  return 13 * P4 + 4 * BP_COUNT * Hc * words_per_row(Wc);
}
// per-image tile storage: fp32 [NT][TS] with 48 slots used.  Pass B runs
// with rows padded to TILE_FLOATS_PAD = 52 floats when the image's tiles fit
// the LDS that way: per-tile accesses (lane = tile) then spread over 8 of the
// 32 banks a 4-byte LDS access uses (48: 2 banks, 16-way conflicts); a
// multiple of 4 keeps the 16-byte staging stores aligned.  Images with more
// tiles (e.g. 80x80 at grid 16: 400 tiles) keep TILE_FLOATS = 48.
enum : int { TILE_FLOATS = 48, TILE_FLOATS_PAD = 52 };
// per-tile partial quantities in the pass A -> pass B buffer (tile_tmp)
enum : int { TT_STRIDE = 32 };
MCAQ_HD int tile_bytes(int NT, int TS = TILE_FLOATS_PAD) { return 4 * TS * NT; }
// fixed shared scratch: 256-int histogram, 2 x 256 doubles, 2 x 64 reduction slots, flags
MCAQ_HD int fixed_bytes() { return 1024 + 4096 + 512 + 64; }
// after the tile array: folded mapper BatchNorms (256 floats), two compact
// per-tile arrays (2 NT floats), or one + the nearest-upsample source tables
// (NT floats + H + W ints)
MCAQ_HD int extra_bytes(int H, int W, int NT) { return 4 * imax_(256, (imax_(2 * NT, NT + H + W) + 3) & ~3); }

// tile array slots
enum : int {
  T_PHI = 0,   // 8 floats
  T_CMLP = 8, T_C = 9, T_CN = 10, T_BITS = 11, T_ACT = 12, T_MT = 13, T_SORT = 14, T_AUX = 15,
  T_TMP = 16   // up to 32 per-tile partials of the phi stage
};

// ---------------------------------------------------------------------------
// execution context: device = real threads; host emulation = one thread
// ---------------------------------------------------------------------------
struct Ctx { int tid, nthr; };

#if defined(__HIP_DEVICE_COMPILE__)
#define MSYNC() __syncthreads()
#define MATOMIC_ADD(p, v) atomicAdd((p), (v))
#define MATOMIC_FETCH_ADD(p, v) atomicAdd((p), (v))
#define MATOMIC_OR(p, v) atomicOr((p), (v))
#else
#define MSYNC() do {} while (0)
#define MATOMIC_ADD(p, v) (*(p) += (v))
#define MATOMIC_FETCH_ADD(p, v) ((*(p) += (v)) - (v))
#define MATOMIC_OR(p, v) (*(p) |= (v))
#endif
#define MFOR(i, n) for (int i = ctx.tid; i < (n); i += ctx.nthr)

// 2D thread loop over a rows x cols grid without per-element divisions
#define MFOR2(r_, c_, rows, cols)                                                              \
  for (int _i = ctx.tid, r_ = ctx.tid / (cols), c_ = ctx.tid - (ctx.tid / (cols)) * (cols),    \
           _dr = ctx.nthr / (cols), _dc = ctx.nthr - (ctx.nthr / (cols)) * (cols);             \
       _i < (rows) * (cols);                                                                   \
       _i += ctx.nthr, r_ += _dr, c_ += _dc, r_ += (c_ >= (cols)), c_ -= (c_ >= (cols)) ? (cols) : 0)

// diagnostic build only (-DMCAQ_STAMPS): per-stage cycle stamps of workgroup 0
#if defined(MCAQ_STAMPS) && defined(MCAQ_STAMPS_ACC) && defined(__HIP_DEVICE_COMPILE__)
// accumulating variant (-DMCAQ_STAMPS_ACC): slot k sums, over every launch,
// the cycles from the previous stamp to stamp k of scale 0's image 0
// (tools/probe/stamps_contended.py: stage times inside the pipelined step)
extern __device__ unsigned long long g_mcaq_stamps[64];
#define MSTAMP_INIT(base)                                                           \
  const int mstamp_base = (S.block_begin == 0) ? (base) : -1;                        \
  unsigned long long mstamp_last = __builtin_amdgcn_s_memtime()
#define MSTAMP(k)                                                                   \
  do {                                                                              \
    __syncthreads();                                                                \
    if (ctx.tid == 0 && mstamp_base >= 0) {                                         \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();                 \
      atomicAdd(&g_mcaq_stamps[mstamp_base + (k)], now_ - mstamp_last);             \
      mstamp_last = now_;                                                           \
    }                                                                               \
  } while (0)
#elif defined(MCAQ_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
extern __device__ unsigned long long g_mcaq_stamps[64];
#define MSTAMP_INIT(base) const int mstamp_base = (base)
#define MSTAMP(k)                                                                   \
  do {                                                                              \
    __syncthreads();                                                                \
    if (ctx.tid == 0 && mstamp_base >= 0) g_mcaq_stamps[mstamp_base + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define MSTAMP_INIT(base) do {} while (0)
#define MSTAMP(k) do {} while (0)
#endif

struct Shared {
  int* hist;       // 256
  double* om;      // 256 (Otsu omega prefix)
  double* mu;      // 256 (Otsu mu prefix)
  float* redf;     // 64
  int* redi;       // 64
  int* flags;      // 16: [8] Otsu argmax, [9] adaptive-threshold exact-list length
  float* tiles;    // NT * TILE_FLOATS
};

struct Planes {
  float *G, *A, *Bf;   // fp32 planes (P4 each)
  uint8_t* dir;        // byte plane
  uint32_t* bp;        // BP_COUNT bit planes of Hc * WPR words
  int WPR, plane_words;
  MCAQ_HD uint32_t* bits(int k) const { return bp + k * plane_words; }
};

MCAQ_HD void carve_planes(char* base, int Hc, int Wc, Planes& pl) {
  const int P4 = (Hc * Wc + 3) & ~3;
  pl.G = (float*)base;
  pl.A = pl.G + P4;
  pl.Bf = pl.A + P4;
  pl.bp = (uint32_t*)(pl.Bf + P4);
  pl.WPR = words_per_row(Wc);
  pl.plane_words = Hc * pl.WPR;
  pl.dir = (uint8_t*)(pl.bp + BP_COUNT * pl.plane_words);
}

MCAQ_HD void carve_shared(char* base, Shared& sh) {
  sh.hist = (int*)base;
  sh.om = (double*)(base + 1024);
  sh.mu = sh.om + 256;
  sh.redf = (float*)(sh.mu + 256);
  sh.redi = (int*)(sh.redf + 64);
  sh.flags = sh.redi + 64;
  sh.tiles = (float*)(sh.flags + 16);
}

// ---- reductions (exact operations only: min / max / integer / exact double) --
MCAQ_HD void block_minmax(const Ctx& ctx, Shared& sh, float lmn, float lmx, float& mn, float& mx) {
#if defined(__HIP_DEVICE_COMPILE__)
  // NaN-propagating, as torch.amin / amax
  for (int o = 32; o > 0; o >>= 1) { lmn = fminp(lmn, __shfl_xor(lmn, o, 64)); lmx = fmaxp(lmx, __shfl_xor(lmx, o, 64)); }
  const int nw = ctx.nthr >> 6;
  if ((ctx.tid & 63) == 0) { sh.redf[ctx.tid >> 6] = lmn; sh.redf[32 + (ctx.tid >> 6)] = lmx; }
  MSYNC();
  mn = sh.redf[0]; mx = sh.redf[32];
  for (int w = 1; w < nw; ++w) { mn = fminp(mn, sh.redf[w]); mx = fmaxp(mx, sh.redf[32 + w]); }
  MSYNC();
#else
  (void)ctx; (void)sh;
  mn = lmn; mx = lmx;
#endif
}

MCAQ_HD float block_max(const Ctx& ctx, Shared& sh, float v) {
  float mn = 0.0f, mx;
  block_minmax(ctx, sh, 0.0f, v, mn, mx);
  return mx;
}

MCAQ_HD int block_or(const Ctx& ctx, int v) {
#if defined(__HIP_DEVICE_COMPILE__)
  (void)ctx;
  return __syncthreads_or(v);
#else
  (void)ctx;
  return v;
#endif
}

// ---- Otsu (morphology.py:398-418) on a [0,1] plane --------------------------
// Histogram counts are integers (exact in any order); the double prefix sums
// are exact because every partial sum fits in 53 bits, so one wave's parallel
// scan reproduces ATen's sequential double cumsum.
MCAQ_HD void otsu_hist_add(Shared& sh, float x) {
  if (x >= 0.0f && x <= 1.0f) {   // histc ignores out-of-range values
    int k = (int)(x * 256.0f);
    if (k > 255) k = 255;
    MATOMIC_ADD(&sh.hist[k], 1);
  }
}
MCAQ_HD float otsu_from_hist(const Ctx& ctx, Shared& sh);
MCAQ_HD float otsu_threshold(const Ctx& ctx, Shared& sh, const float* v, int P) {
  MFOR(i, 256) sh.hist[i] = 0;
  MSYNC();
  MFOR(p, P) otsu_hist_add(sh, v[p]);
  MSYNC();
  return otsu_from_hist(ctx, sh);
}
// threshold from a complete histogram in sh.hist (all threads; ends synced)
MCAQ_HD float otsu_from_hist(const Ctx& ctx, Shared& sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (ctx.tid < 64) {
    const int l = ctx.tid;
    int hc[4], tot = 0;
    for (int k = 0; k < 4; ++k) { hc[k] = sh.hist[4 * l + k]; tot += hc[k]; }
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    const float total = fmax_((float)tot, 1.0f);
    float p[4];
    double w[4], m[4];
    for (int k = 0; k < 4; ++k) {
      p[k] = (float)hc[k] / total;
      const float c = ((float)(4 * l + k) + 0.5f) / 256.0f;
      w[k] = (double)p[k];
      m[k] = (double)(p[k] * c);
      if (k) { w[k] = w[k] + w[k - 1]; m[k] = m[k] + m[k - 1]; }
    }
    double sw = w[3], sm = m[3];     // inclusive scan of lane totals
    for (int o = 1; o < 64; o <<= 1) {
      const double uw = __shfl_up(sw, o, 64), um = __shfl_up(sm, o, 64);
      if (l >= o) { sw = sw + uw; sm = sm + um; }
    }
    const double ew = sw - w[3], em = sm - m[3];   // exclusive offsets (exact)
    const float mu_t = (float)__shfl(sm, 63, 64);
    float best = -1.0f;
    int bi = 0x7fffffff;
    for (int k = 0; k < 4; ++k) {
      const float om = (float)(ew + w[k]);
      const float mu = (float)(em + m[k]);
      float num = mu_t * om - mu;
      num = num * num;
      const float sb = num / (om * (1.0f - om) + 1e-12f);
      if (sb > best) { best = sb; bi = 4 * l + k; }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (l == 0) sh.flags[8] = bi;
  }
  MSYNC();
  const int idx = sh.flags[8];
  MSYNC();
#else
  int tot = 0;
  for (int i = 0; i < 256; ++i) tot += sh.hist[i];
  const float total = fmax_((float)tot, 1.0f);
  double cw = 0.0, cm = 0.0;
  for (int i = 0; i < 256; ++i) {
    const float p = (float)sh.hist[i] / total;
    cw = cw + (double)p;
    cm = cm + (double)(p * (((float)i + 0.5f) / 256.0f));
    sh.om[i] = cw; sh.mu[i] = cm;
  }
  const float mu_t = (float)sh.mu[255];
  float best = -1.0f;
  int idx = 0;
  for (int i = 0; i < 256; ++i) {
    const float om = (float)sh.om[i], mu = (float)sh.mu[i];
    float num = mu_t * om - mu;
    num = num * num;
    const float sb = num / (om * (1.0f - om) + 1e-12f);
    if (sb > best) { best = sb; idx = i; }
  }
#endif
  return ((float)idx + 0.5f) / 256.0f;
}

// ---- bit planes --------------------------------------------------------------
// Pack one predicate per (row h, word k, bit i) slot; every 32 consecutive
// threads of a wave form one word (device: ballot).
MCAQ_HD void put_bits(uint32_t* plane, int wi, int bit, bool pred) {
#if defined(__HIP_DEVICE_COMPILE__)
  const unsigned long long m = __ballot(pred);
  if (bit == 0) plane[wi] = (uint32_t)(m >> (threadIdx.x & 32));
#else
  if (bit == 0) plane[wi] = 0u;
  if (pred) plane[wi] |= 1u << bit;
#endif
}

MCAQ_HD int popc(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popc(x);
#else
  return __builtin_popcount(x);
#endif
}

// bits [x0, x0+n) of a row (n <= 32, may straddle a word boundary)
MCAQ_HD uint32_t row_field(const uint32_t* row, int x0, int n, int WPR) {
  const int k = x0 >> 5, s = x0 & 31;
  uint64_t v = row[k];
  if (s + n > 32 && k + 1 < WPR) v |= (uint64_t)row[k + 1] << 32;
  v >>= s;
  return (uint32_t)(n == 32 ? v : (v & ((1ull << n) - 1ull)));
}
// popcount of bits [x0, x0+n) of a row, any n
MCAQ_HD int row_pop(const uint32_t* row, int x0, int n, int WPR) {
  int c = 0;
  for (int o = 0; o < n; o += 32) c += popc(row_field(row, x0 + o, n - o < 32 ? n - o : 32, WPR));
  return c;
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
template <int TS>
MCAQ_HD void sort_tiles(const Ctx& ctx, float* tiles, int NT, int src) {
  MFOR(t, NT) {
    const float v = tiles[t * TS + src];
    int r = 0;
    for (int u = 0; u < NT; ++u) {
      const float w = tiles[u * TS + src];
      r += (w < v) || (w == v && u < t);
    }
    tiles[r * TS + T_SORT] = v;
  }
  MSYNC();
}

}  // namespace mcaq
// per-wave activation scratch of the MFMA tile MLPs (mcaq_mlp_mfma.h): 32 tiles
// x MLP_XS floats (MLP_XS = 68: the B-operand reads of 16 tiles x 4 k-rows hit
// 64 distinct banks)
#ifndef MCAQ_TILES_THREADS       // pass B workgroup size (256 or 512)
#define MCAQ_TILES_THREADS 256
#endif
constexpr int MLP_XS = 68;
// tiles per wave block of the MFMA MLPs: 16 (one 16x16 half) at 512 threads,
// 32 (two halves, more independent chains per wave) at 256
constexpr int MLP_NH = MCAQ_TILES_THREADS >= 512 ? 1 : 2;
constexpr int MLP_TPW = 16 * MLP_NH;
constexpr int MLP_SCRATCH_FLOATS = MLP_TPW * MLP_XS;

#if defined(__HIP_DEVICE_COMPILE__)
#include "mcaq_mlp_mfma.h"   // fp32 MFMA versions of the tile MLPs (device only)
#endif
namespace mcaq {

// NMS direction bin (morphology.py:430-444): the reference bins the fp32 angle
// a = atan2(gy, gx) * fp32(180/pi) (+180 when negative) at 22.5 / 67.5 /
// 112.5 / 157.5 degrees.  Fast path: the bin edges are the slopes tan(22.5)
// and tan(67.5), so |gy| against t*|gx| (plus the sign of gx*gy between them)
// decides every pixel whose slope is at least 3e-5*|gx| from an edge (>= 2.5e-4
// degrees, ten times the fp32 angle's error); the others, and gx = gy = 0, take
// the exact path: correctly rounded fp32 atan2 scaled by fp32(180/pi).
MCAQ_HD int nms_dir(float gx, float gy) {
  const float ax = fabsf(gx), ay = fabsf(gy);
  const float r1 = ay - 0.41421356237309503f * ax;
  const float r2 = ay - 2.4142135623730949f * ax;
  const float mg = 3e-5f * ax;
  if (fabsf(r1) > mg && fabsf(r2) > mg) {
    if (r1 < 0.0f) return 0;
    if (r2 > 0.0f) return 2;
    return ((gx > 0.0f) == (gy > 0.0f)) ? 1 : 3;
  }
  const float K180 = (float)(180.0 / 3.14159265358979323846);
  float a = cr_atan2(gy, gx) * K180;
  if (a < 0.0f) a = a + 180.0f;
  if (a >= 22.5f && a < 67.5f) return 1;
  if (a >= 67.5f && a < 112.5f) return 2;
  if (a >= 112.5f && a < 157.5f) return 3;
  return 0;
}

// 16-byte store of 4 consecutive floats (p 16-byte aligned)
MCAQ_HD void store4(float* p, const float (&v)[4]) {
#if defined(__HIP_DEVICE_COMPILE__)
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
#else
  p[0] = v[0]; p[1] = v[1]; p[2] = v[2]; p[3] = v[3];
#endif
}

#if defined(__HIPCC__)
// 3-wide horizontal dilation of word k of a 4-word register row
__device__ __forceinline__ uint32_t dil3(const uint32_t (&rw)[4], int k) {
  const uint32_t c = rw[k];
  const uint32_t l = (c << 1) | (k > 0 ? rw[k > 0 ? k - 1 : 0] >> 31 : 0u);
  const uint32_t r = (c >> 1) | (k < 3 ? rw[k < 3 ? k + 1 : 3] << 31 : 0u);
  return c | l | r;
}
#endif

// exact 121-tap adaptive mean of 255*G at (h, w), replicate pad, oneDNN
// order (kh-major, kw-minor, FMA from 0); each row's 11 loads issue together
MCAQ_HD float exact_g11(const float* G, int Hc, int Wc, int h, int w) {
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    const float* row = G + imin_(imax_(h + i - 5, 0), Hc - 1) * Wc;
    float v[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) v[j] = row[imin_(imax_(w + j - 5, 0), Wc - 1)] * 255.0f;
#pragma unroll
    for (int j = 0; j < 11; ++j) acc = fmaf(bits_as_float(k_gauss11_bits[i * 11 + j]), v[j], acc);
  }
  return acc;
}

#if defined(__HIP_DEVICE_COMPILE__)
// acc = fma(k[O + i], tap O + i, acc) for i = 0, 1, ..., tap O + i in lane i
// of v: exact_g11's FMA order with every weight an immediate (I are
// compile-time indices)
template <int... I, int O>
__device__ __forceinline__ void g11_chain(float& acc, float v, std::integer_sequence<int, I...>,
                                          std::integral_constant<int, O>) {
  ((acc = fmaf(bits_as_float(k_gauss11_bits[O + I]), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), I)), acc)), ...);
}
#endif

// row_field without a branch around the second word (loads issue together)
MCAQ_HD uint32_t row_field_bf(const uint32_t* row, int x0, int n, int WPR) {
  const int k = x0 >> 5, sft = x0 & 31;
  const uint64_t lo = row[k];
  const uint64_t hi = row[imin_(k + 1, WPR - 1)];
  uint64_t v = lo | ((sft + n > 32 && k + 1 < WPR) ? (hi << 32) : 0ull);
  v >>= sft;
  return n == 32 ? (uint32_t)v : (uint32_t)(v & ((1ull << n) - 1ull));
}

// popcount of a T x T window of a bit plane (T <= 32)
template <int T>
MCAQ_HD int tile_pop_t(const uint32_t* plane, int WPR, int h0, int w0) {
  uint32_t f[T];
#pragma unroll
  for (int yy = 0; yy < T; ++yy) f[yy] = row_field_bf(plane + (h0 + yy) * WPR, w0, T, WPR);
  int c = 0;
#pragma unroll
  for (int yy = 0; yy < T; ++yy) c += popc(f[yy]);
  return c;
}

// occupied S x S boxes of a T x T window (T <= 16): OR-fold S rows, then S columns
template <int T, int S>
MCAQ_HD int box_count_s(const uint32_t (&f)[T]) {
  uint32_t starts = 0u;
#pragma unroll
  for (int x = 0; x < T; x += S) starts |= 1u << x;
  int n = 0;
#pragma unroll
  for (int by = 0; by < T; by += S) {
    uint32_t o = 0u;
#pragma unroll
    for (int yy = 0; yy < S; ++yy) o |= f[by + yy];
#pragma unroll
    for (int sh2 = 1; sh2 < S; sh2 <<= 1) o |= o >> sh2;
    n += popc(o & starts);
  }
  return n;
}
template <int T>
MCAQ_HD int box_count_t(const uint32_t* plane, int WPR, int h0, int w0, int s) {
  uint32_t f[T];
#pragma unroll
  for (int yy = 0; yy < T; ++yy) f[yy] = row_field_bf(plane + (h0 + yy) * WPR, w0, T, WPR);
  if (s == 2) return box_count_s<T, 2>(f);
  if (s == 4) return box_count_s<T, (T >= 4 ? 4 : 2)>(f);
  if (s == 8) return box_count_s<T, (T >= 8 ? 8 : 2)>(f);
  return box_count_s<T, (T >= 16 ? 16 : 2)>(f);
}

// rows per thread of the column-strip convolution stages
constexpr int SR = 8;

// sequential row-major sum of a T x T window (avg_pool2d order), unrolled so
// all loads issue ahead of the dependent add chain
template <int T, bool SQ>
MCAQ_HD float tile_sum_t(const float* plane, int Wc, int h0, int w0) {
  float acc = 0.0f;
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (T % 4 == 0) {
    // 16-byte row loads (Wc and w0 are multiples of T, the planes 16-byte
    // aligned): lanes take consecutive tiles, T floats apart, so 4-byte loads
    // hit the same LDS bank every 32 / T lanes (8-way at T = 8)
    typedef float f4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int yy = 0; yy < T; ++yy) {
      const f4v* row = reinterpret_cast<const f4v*>(plane + (h0 + yy) * Wc + w0);
#pragma unroll
      for (int q = 0; q < T / 4; ++q) {
        const f4v v = row[q];
        acc = SQ ? acc + v.x * v.x : acc + v.x;
        acc = SQ ? acc + v.y * v.y : acc + v.y;
        acc = SQ ? acc + v.z * v.z : acc + v.z;
        acc = SQ ? acc + v.w * v.w : acc + v.w;
      }
    }
    return acc;
  }
#endif
#pragma unroll
  for (int yy = 0; yy < T; ++yy) {
    const float* row = plane + (h0 + yy) * Wc + w0;
#pragma unroll
    for (int xx = 0; xx < T; ++xx) acc = SQ ? acc + row[xx] * row[xx] : acc + row[xx];
  }
  return acc;
}

// Sobel of gsc*blur (zero pad) -> magnitude Bf, NMS direction dir; column
// strips as the blur.  Zero-weight taps are skipped and padded taps add
// fma(k, 0, g) == g (g never holds -0: it starts at +0).  Default: gsc = 255,
// L1 magnitude; canny_impl='legacy': gsc = 1, sqrt(gx^2 + gy^2 + 1e-12).
// Separate instantiations keep the default path's registers unchanged.
template <bool kLegacy>
MCAQ_HD void sobel_stage(const Ctx& ctx, Planes& pl, int Hc, int Wc) {
  {
    const int nsr = (Hc + SR - 1) / SR;
    MFOR2(st, w, nsr, Wc) {
      const int r0 = st * SR;
      float v[SR + 2][3];
#pragma unroll
      for (int t = 0; t < SR + 2; ++t) {
        const int hh = r0 + t - 1;
        const bool rv = hh >= 0 && hh < Hc;
        const float* row = pl.A + imin_(imax_(hh, 0), Hc - 1) * Wc;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int ww = w + j - 1;
          const float x = row[imin_(imax_(ww, 0), Wc - 1)] * (kLegacy ? 1.0f : 255.0f);
          v[t][j] = (rv && ww >= 0 && ww < Wc) ? x : 0.0f;
        }
      }
#pragma unroll
      for (int r = 0; r < SR; ++r) {
        float gx = 0.0f, gy = 0.0f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const float kx = (i == 1) ? 2.0f : 1.0f;    // gx taps (i,0) = -kx, (i,2) = +kx
          const float ky = (float)(i - 1);             // gy taps (i,j) = ky * {1,2,1}
          gx = fmaf(-kx, v[r + i][0], gx);
          gx = fmaf(kx, v[r + i][2], gx);
          if (i != 1) {
            gy = fmaf(ky, v[r + i][0], gy);
            gy = fmaf(2.0f * ky, v[r + i][1], gy);
            gy = fmaf(ky, v[r + i][2], gy);
          }
        }
        if (r0 + r < Hc) {
          const int p = (r0 + r) * Wc + w;
          pl.Bf[p] = kLegacy ? sqrtf((gx * gx + gy * gy) + 1e-12f) : fabsf(gx) + fabsf(gy);
          pl.dir[p] = (uint8_t)nms_dir(gx, gy);
        }
      }
    }
  }
}

// Canny hysteresis on bit planes (morphology.py:504-509): `iters` Jacobi
// sweeps e' = e | (weak & dilate3x3(e)), stopping early once a sweep changes
// nothing (every later sweep would be the identity).  E0 holds the strong
// pixels, E1 is scratch; returns the plane holding the result.  Ends synced.
MCAQ_HD const uint32_t* hysteresis_run(const Ctx& ctx, uint32_t* E0, uint32_t* E1, const uint32_t* WK, int Hc, int WPR,
                                       int iters) {
  uint32_t* src = E0;
  uint32_t* dst = E1;
#if defined(__HIP_DEVICE_COMPILE__)
  if (Hc <= 128 && WPR <= 4) {
    // one wave, planes in registers (lane l: rows 2l, 2l+1), neighbour rows by
    // lane shuffles: no barrier per iteration.  Same Jacobi sweeps and the
    // same stop rule as the workgroup loop below.
    if (ctx.tid < 64) {
      const int lane = ctx.tid;
      uint32_t e[2][4], wk[2][4];
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int row = 2 * lane + rr;
          const bool ok = row < Hc && k < WPR;
          e[rr][k] = ok ? src[row * WPR + k] : 0u;
          wk[rr][k] = ok ? WK[row * WPR + k] : 0u;
        }
      }
      for (int it = 0; it < iters; ++it) {
        uint32_t up[4], dn[4], d[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          // DPP wave_shr:1 / wave_shl:1 (lane l <- l-1 / l+1; 0 past the ends)
          up[k] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e[1][k], 0x138, 0xF, 0xF, false);
          dn[k] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e[0][k], 0x130, 0xF, 0xF, false);
        }
        // horizontal 3-dilation of the 4 rows up, e0, e1, dn
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[0][k] = dil3(up, k);
          d[1][k] = dil3(e[0], k);
          d[2][k] = dil3(e[1], k);
          d[3][k] = dil3(dn, k);
        }
        bool ch = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t n0 = e[0][k] | (wk[0][k] & (d[0][k] | d[1][k] | d[2][k]));
          const uint32_t n1 = e[1][k] | (wk[1][k] & (d[1][k] | d[2][k] | d[3][k]));
          ch = ch || (n0 != e[0][k]) || (n1 != e[1][k]);
          e[0][k] = n0; e[1][k] = n1;
        }
        if (!__any(ch)) break;
      }
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int row = 2 * lane + rr;
          if (row < Hc && k < WPR) src[row * WPR + k] = e[rr][k];
        }
      }
    }
    MSYNC();
  } else
#endif
  {
    for (int it = 0; it < iters; ++it) {
      int changed = 0;
      MFOR2(h, k, Hc, WPR) {
        const uint32_t cur = src[h * WPR + k];
        uint32_t g = 0u;
        for (int hh = imax_(h - 1, 0); hh <= imin_(h + 1, Hc - 1); ++hh) {
          const uint32_t* row = src + hh * WPR;
          const uint32_t c = row[k];
          const uint32_t l = (c << 1) | (k > 0 ? row[k - 1] >> 31 : 0u);
          const uint32_t r = (c >> 1) | (k + 1 < WPR ? row[k + 1] << 31 : 0u);
          g |= c | l | r;
        }
        const uint32_t nv = cur | (WK[h * WPR + k] & g);
        changed |= (nv != cur);
        dst[h * WPR + k] = nv;
      }
      const int any = block_or(ctx, changed);
      uint32_t* t = src; src = dst; dst = t;
      if (!any) break;
    }
  }
  return src;
}

// ---- pass A: per-image pixel work -> phi (one 1024-thread workgroup per image)
// kLegacy: the canny_impl='legacy' instantiation (a separate kernel on the
// device, so the default edge path keeps its register allocation)
template <bool kLegacy>
MCAQ_HD void morph_edges(const Ctx& ctx, const MorphScale& S, int b, int role, Planes& pl, Shared& sh) {
  const int Hc = S.Hc, Wc = S.Wc, P = Hc * Wc, T = S.tile, wt = S.wt, NT = S.ht * wt;
  const int WPR = pl.WPR, RS = WPR * 32;   // words / bit slots per row
  const float fT2 = (float)(T * T);

  MSTAMP_INIT(b == 0 ? 16 * role : -1);   // diagnostic build: image 0, slots 0-9 / 16-25
  MSTAMP(0);
  {
    // -- gray (channel mean from the stats pass) + per-image normalise01.
    //    Up to GPT pixels per thread are loaded at once and kept in registers.
    const float* gin = S.gray + (size_t)b * P;
    MFOR(i, 256) sh.hist[i] = 0;          // Otsu histogram, filled by the blur stage
    // mask role, tiles >= 8 px: per-tile uniform-LBP label counts, counted by
    // LDS atomics in the Sobel / LBP stage (in the direction byte plane, unused
    // by this role: 40 NT <= P bytes) instead of 10 label bit planes
    const bool lbp_cnt = role == 1 && T >= 8;
    int* lcnt = reinterpret_cast<int*>(pl.dir);
    const int tsh = __builtin_ctz((unsigned)T);   // tiles are powers of two
    if (lbp_cnt) MFOR(i, 10 * NT) lcnt[i] = 0;
    float lmn = 3.402823466e38f, lmx = -3.402823466e38f;
    constexpr int GPT = 8;
    const bool greg = P <= GPT * ctx.nthr;
    float gv[GPT];
    if (greg) {
#pragma unroll
      for (int i = 0; i < GPT; ++i) {
        const int p = ctx.tid + i * ctx.nthr;
        gv[i] = gin[p < P ? p : 0];
        if (p < P) { lmn = fminp(lmn, gv[i]); lmx = fmaxp(lmx, gv[i]); }
      }
    } else {
      MFOR(p, P) { const float v = gin[p]; pl.G[p] = v; lmn = fminp(lmn, v); lmx = fmaxp(lmx, v); }
    }
    float mn, mx;
    block_minmax(ctx, sh, lmn, lmx, mn, mx);
    const float den = (mx - mn) + 1e-8f;
    if (greg) {
#pragma unroll
      for (int i = 0; i < GPT; ++i) {
        const int p = ctx.tid + i * ctx.nthr;
        if (p < P) pl.G[p] = (gv[i] - mn) / den;
      }
    } else {
      MFOR(p, P) pl.G[p] = (pl.G[p] - mn) / den;
    }
    MSYNC();
    MSTAMP(1);

    const uint32_t* edge = nullptr;      // final edge bit plane (edge workgroup)
    uint32_t* BIN = pl.bits(BP_BIN);
    uint32_t* BND = pl.bits(BP_BND);
    uint32_t* Q1 = pl.bits(BP_Q1);
    uint32_t* Q3 = pl.bits(BP_Q3);
    uint32_t* QD = pl.bits(BP_QD);
    // Two workgroups per image run the two independent halves of the
    // descriptor pipeline side by side: role 0 = Canny edge plane (blur,
    // Otsu, Sobel, NMS, hysteresis), role 1 = foreground mask / LBP /
    // gradient planes.  Each reduces its planes to per-tile partial
    // quantities (tile_tmp); pass B assembles phi from both.
    if (role == 0) {
    // canny_impl='legacy' (morphology.py:512-540): Sobel of the blur itself,
    // L2 magnitude, Otsu of the min-max normalised NMS map, 2 hysteresis rounds
    constexpr bool legacy = kLegacy;
    // -- 5x5 Gaussian blur (zero pad; an out-of-image tap adds fma(w, 0, acc) == acc
    //    because acc >= +0), fused with the Otsu histogram of the result.
    //    Column strips of SR rows per thread: consecutive threads own consecutive
    //    columns (conflict-free LDS rows); all (SR+4) x 5 loads are branch-free
    //    (clamped address, zero select) so they issue together; every output
    //    still accumulates its 25 taps row-major from 0 (the oneDNN order).
    {
      const int nsr = (Hc + SR - 1) / SR;
      MFOR2(st, w, nsr, Wc) {
        const int r0 = st * SR;
        float v[SR + 4][5];
#pragma unroll
        for (int t = 0; t < SR + 4; ++t) {
          const int hh = r0 + t - 2;
          const bool rv = hh >= 0 && hh < Hc;
          const float* row = pl.G + imin_(imax_(hh, 0), Hc - 1) * Wc;
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            const int ww = w + j - 2;
            const float x = row[imin_(imax_(ww, 0), Wc - 1)];
            v[t][j] = (rv && ww >= 0 && ww < Wc) ? x : 0.0f;
          }
        }
#pragma unroll
        for (int r = 0; r < SR; ++r) {
          float acc = 0.0f;
#pragma unroll
          for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) acc = fmaf(bits_as_float(k_gauss5_bits[i * 5 + j]), v[r + i][j], acc);
          if (r0 + r < Hc) {
            pl.A[(r0 + r) * Wc + w] = acc;
#ifndef MCAQ_PROBE_NO_HIST   // timing probe only (wrong Otsu threshold)
            if (!legacy) otsu_hist_add(sh, acc);
#endif
          }
        }
      }
    }
    MSYNC();
    MSTAMP(2);
    const float thr = legacy ? 0.0f : otsu_from_hist(ctx, sh);
    const float thr255 = thr * 255.0f;
    const float lo255 = 0.5f * thr255;
    MSTAMP(3);

    // -- Sobel (-> Bf magnitude, dir direction), see sobel_stage
    sobel_stage<kLegacy>(ctx, pl, Hc, Wc);
    MSYNC();
    MSTAMP(4);
    // -- NMS (replicate-shifted neighbours) + double threshold -> bit planes.
    //    Column strips: directions + magnitudes of SR rows (one round trip),
    //    then both neighbours of every row (one more), then the ballots.
    uint32_t* E0 = pl.bits(BP_E0);
    uint32_t* E1 = pl.bits(BP_E1);
    uint32_t* WK = pl.bits(BP_WK);
    if constexpr (!legacy) {
      const int nsr = (Hc + SR - 1) / SR;
      MFOR2(st, sl, nsr, RS) {
        const int k = sl >> 5, bit = sl & 31, w = sl;
        const int r0 = st * SR;
        const int wc = imin_(w, Wc - 1);
        int d[SR];
        float m[SR], n1[SR], n2[SR];
#pragma unroll
        for (int r = 0; r < SR; ++r) {
          const int p = imin_(r0 + r, Hc - 1) * Wc + wc;
          d[r] = pl.dir[p];
          m[r] = pl.Bf[p];
        }
#pragma unroll
        for (int r = 0; r < SR; ++r) {
          const int h = imin_(r0 + r, Hc - 1);
          const int dy1 = (d[r] == 0) ? 0 : -1;
          const int dx1 = (d[r] == 2) ? 0 : ((d[r] == 3) ? -1 : 1);
          const int h1 = imin_(imax_(h + dy1, 0), Hc - 1), w1 = imin_(imax_(wc + dx1, 0), Wc - 1);
          const int h2 = imin_(imax_(h - dy1, 0), Hc - 1), w2 = imin_(imax_(wc - dx1, 0), Wc - 1);
          n1[r] = pl.Bf[h1 * Wc + w1];
          n2[r] = pl.Bf[h2 * Wc + w2];
        }
#pragma unroll
        for (int r = 0; r < SR; ++r) {
          if (r0 + r >= Hc) continue;
          const bool keep = (m[r] >= n1[r]) && (m[r] >= n2[r]);
          const float nms = keep ? m[r] : 0.0f;
          put_bits(E0, (r0 + r) * WPR + k, bit, w < Wc && nms > thr255);
          put_bits(WK, (r0 + r) * WPR + k, bit, w < Wc && nms > lo255);
        }
      }
      MSYNC();
    } else {
      // legacy: the NMS map itself (into the blur plane, free after Sobel),
      // normalise01, its Otsu threshold t, strong > t, weak > t/2
      float lmn = 3.402823466e38f, lmx = -3.402823466e38f;
      MFOR(p, P) {
        const int h = p / Wc, w = p - (p / Wc) * Wc;
        const int d = pl.dir[p];
        const float m = pl.Bf[p];
        const int dy1 = (d == 0) ? 0 : -1;
        const int dx1 = (d == 2) ? 0 : ((d == 3) ? -1 : 1);
        const int h1 = imin_(imax_(h + dy1, 0), Hc - 1), w1 = imin_(imax_(w + dx1, 0), Wc - 1);
        const int h2 = imin_(imax_(h - dy1, 0), Hc - 1), w2 = imin_(imax_(w - dx1, 0), Wc - 1);
        const float nms = (m >= pl.Bf[h1 * Wc + w1] && m >= pl.Bf[h2 * Wc + w2]) ? m : 0.0f;
        pl.A[p] = nms;
        lmn = fminp(lmn, nms); lmx = fmaxp(lmx, nms);
      }
      float mn, mx;
      block_minmax(ctx, sh, lmn, lmx, mn, mx);
      const float den = (mx - mn) + 1e-8f;
      MFOR(p, P) {
        const float v = (pl.A[p] - mn) / den;
        pl.A[p] = v;
        otsu_hist_add(sh, v);
      }
      MSYNC();
      const float t = otsu_from_hist(ctx, sh);
      const float tl = 0.5f * t;
      MFOR2(h, sl, Hc, RS) {
        const int k = sl >> 5, bit = sl & 31;
        const float v = pl.A[h * Wc + imin_(sl, Wc - 1)];
        put_bits(E0, h * WPR + k, bit, sl < Wc && v > t);
        put_bits(WK, h * WPR + k, bit, sl < Wc && v > tl);
      }
      MSYNC();
    }
    MSTAMP(5);
    // -- hysteresis on words: e' = e | (weak & dilate3x3(e)), Jacobi, early exit
    edge = hysteresis_run(ctx, E0, E1, WK, Hc, WPR, legacy ? 2 : (S.hyst_iters < 1 ? 1 : S.hyst_iters));
    MSTAMP(6);

    } else {
    // -- foreground mask for phi5 -> BIN bit plane
    if (S.flags & F_BIN_OTSU) {
      const float t2 = otsu_threshold(ctx, sh, pl.G, P);
      MFOR2(h, sl, Hc, RS) {
        const int k = sl >> 5, bit = sl & 31;
        put_bits(BIN, h * WPR + k, bit, sl < Wc && pl.G[h * Wc + sl] > t2);
      }
    } else {
      // adaptive threshold (morphology.py:551-573): g255 > G11(g255, replicate) - 2.
      // A separable fp32 estimate decides every pixel whose distance to the
      // threshold exceeds the proven error bound k_g11_margin (tools/
      // gen_tables.py); the others get the exact 121-tap sum in oneDNN order
      // (taps kh-major / kw-minor, FMA from 0), i.e. the reference's value.
      // g255 = G * 255 is recomputed where read (same rounding as a stored plane).
      float* rowp = pl.Bf;    // horizontal 11-tap pass, column strips, loads issued together
      const int nsr = (Hc + SR - 1) / SR;
      // pixels within the margin are listed (in the blur plane A, free in
      // this role until the Sobel stage) and get their exact sums after the
      // vertical pass, one pixel per thread, instead of a divergent 121-tap
      // chain inside each wave that meets one
      int* xlist = reinterpret_cast<int*>(pl.A);
      int* nx = sh.flags + 9;
      if (ctx.tid == 0) *nx = 0;
      MFOR2(st, w, nsr, Wc) {
        const int r0 = st * SR;
        float v[SR][11];
#pragma unroll
        for (int r = 0; r < SR; ++r) {
          const float* row = pl.G + imin_(r0 + r, Hc - 1) * Wc;
#pragma unroll
          for (int j = 0; j < 11; ++j) v[r][j] = row[imin_(imax_(w + j - 5, 0), Wc - 1)] * 255.0f;
        }
#pragma unroll
        for (int r = 0; r < SR; ++r) {
          float acc = 0.0f;
#pragma unroll
          for (int j = 0; j < 11; ++j) acc = fmaf(bits_as_float(k_g11_sep_bits[j]), v[r][j], acc);
          if (r0 + r < Hc) rowp[(r0 + r) * Wc + w] = acc;
        }
      }
      MSYNC();
      MSTAMP(2);
      const float marg = bits_as_float(k_g11_margin_bits[0]);
      MFOR2(st, sl, nsr, RS) {   // vertical pass: column strips of SR rows, word-aligned lanes
        const int k = sl >> 5, bit = sl & 31, w = sl;
        const int r0 = st * SR;
        bool on[SR];
#pragma unroll
        for (int r = 0; r < SR; ++r) on[r] = false;
        if (w < Wc) {
          float v[SR + 10];
#pragma unroll
          for (int t = 0; t < SR + 10; ++t) v[t] = rowp[imin_(imax_(r0 + t - 5, 0), Hc - 1) * Wc + w];
#pragma unroll
          for (int r = 0; r < SR; ++r) {
            if (r0 + r >= Hc) continue;
            const int h = r0 + r;
            float m = 0.0f;
#pragma unroll
            for (int i = 0; i < 11; ++i) m = fmaf(bits_as_float(k_g11_sep_bits[i]), v[r + i], m);
            const float g = pl.G[h * Wc + w] * 255.0f;
            const float t = m - 2.0f;
#ifdef MCAQ_PROBE_NO_EXACT_G11   // timing probe only (separable estimate everywhere)
            if (true) {
#else
            if (fabsf(g - t) > marg) {
#endif
              on[r] = g > t;
            } else {
              xlist[MATOMIC_FETCH_ADD(nx, 1)] = h * Wc + w;   // decided below
            }
          }
        }
#pragma unroll
        for (int r = 0; r < SR; ++r) if (r0 + r < Hc) put_bits(BIN, (r0 + r) * WPR + k, bit, on[r]);
      }
      MSYNC();
      MSTAMP(3);
      const int nxs = *nx;
#if defined(__HIP_DEVICE_COMPILE__)
      // one wave per listed pixel: its lanes load the 121 taps at once (lane
      // l: taps l and l + 64), then the FMA chain of exact_g11 runs in that
      // order on the taps read back lane by lane (a single-lane chain waits
      // on 11 LDS round trips: ~5.5 k cycles per pixel, stage stamps)
      {
        const int lane = ctx.tid & 63;
        for (int i = ctx.tid >> 6; i < nxs; i += ctx.nthr >> 6) {
          const int p = xlist[i], h = p / Wc, w = p - (p / Wc) * Wc;
          const int ta = lane, tb = imin_(lane + 64, 120);
          const int ia = ta / 11, ib = tb / 11;
          const float va = pl.G[imin_(imax_(h + ia - 5, 0), Hc - 1) * Wc + imin_(imax_(w + (ta - 11 * ia) - 5, 0), Wc - 1)] * 255.0f;
          const float vb = pl.G[imin_(imax_(h + ib - 5, 0), Hc - 1) * Wc + imin_(imax_(w + (tb - 11 * ib) - 5, 0), Wc - 1)] * 255.0f;
          float acc = 0.0f;
          g11_chain(acc, va, std::make_integer_sequence<int, 64>{}, std::integral_constant<int, 0>{});
          g11_chain(acc, vb, std::make_integer_sequence<int, 57>{}, std::integral_constant<int, 64>{});
          if (lane == 0 && pl.G[p] * 255.0f > acc - 2.0f) MATOMIC_OR(&BIN[h * WPR + (w >> 5)], 1u << (w & 31));
        }
      }
#else
      MFOR(i, nxs) {
        const int p = xlist[i], h = p / Wc, w = p - (p / Wc) * Wc;
        if (pl.G[p] * 255.0f > exact_g11(pl.G, Hc, Wc, h, w) - 2.0f) MATOMIC_OR(&BIN[h * WPR + (w >> 5)], 1u << (w & 31));
      }
#endif
    }
    MSYNC();
    MSTAMP(7);

    // -- Sobel of the normalised gray (phi3) -> A = gx, Bf = gy; uniform LBP label planes.
    //    Column strips: the (SR+2) x 3 replicate-clamped window values load
    //    together; the zero-padded Sobel taps select 0 outside the image.
    {
      const int nsr = (Hc + SR - 1) / SR;
      MFOR2(st, sl, nsr, RS) {
        const int k = sl >> 5, bit = sl & 31, w = sl;
        const int r0 = st * SR;
        const int wc = imin_(w, Wc - 1);
        const int wm = imax_(wc - 1, 0), wp = imin_(wc + 1, Wc - 1);
        const bool cl = wc > 0, cr = wc + 1 < Wc;
        float c[SR + 2][3];
#pragma unroll
        for (int t = 0; t < SR + 2; ++t) {
          const float* row = pl.G + imin_(imax_(r0 + t - 1, 0), Hc - 1) * Wc;
          c[t][0] = row[wm]; c[t][1] = row[wc]; c[t][2] = row[wp];
        }
#pragma unroll
        for (int r = 0; r < SR; ++r) {
          const int h = r0 + r;
          int lab = -1;
          if (w < Wc && h < Hc) {
            const bool ru = h > 0, rd = h + 1 < Hc;
            const float ctr = c[r + 1][1];
            // zero-padded Sobel taps, row-major
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
#ifndef MCAQ_PROBE_NO_GRAD_PLANES   // timing probe only
            pl.A[h * Wc + w] = gx;
            pl.Bf[h * Wc + w] = gy;
#endif
            // LBP (morphology.py:630-646): replicate pad, nb >= center, circular order
            int bt[8];
            bt[0] = c[r][0] >= ctr; bt[1] = c[r][1] >= ctr; bt[2] = c[r][2] >= ctr; bt[3] = c[r + 1][2] >= ctr;
            bt[4] = c[r + 2][2] >= ctr; bt[5] = c[r + 2][1] >= ctr; bt[6] = c[r + 2][0] >= ctr; bt[7] = c[r + 1][0] >= ctr;
            int n1 = 0, tr = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) { n1 += bt[q]; tr += bt[q] != bt[(q + 7) & 7]; }
            lab = tr <= 2 ? n1 : 9;
          }
          if (lbp_cnt) {
            if (lab >= 0) MATOMIC_ADD(&lcnt[((h >> tsh) * wt + (w >> tsh)) * 10 + lab], 1);
          } else if (h < Hc) {
#pragma unroll
            for (int q = 0; q < 10; ++q) put_bits(pl.bits(BP_L0 + q), h * WPR + k, bit, lab == q);
          }
        }
      }
    }
    MSTAMP(4);
    // boundary (m & ~erode3x3 with in-bounds neighbours) and Euler quad classes
    // of the windows anchored at (h, w) over m[h-1..h][w-1..w] (zero padded)
    MFOR2(h, k, Hc, WPR) {
      const int nvalid = imin_(Wc - 32 * k, 32);
      const uint32_t vmask = nvalid >= 32 ? 0xFFFFFFFFu : ((1u << nvalid) - 1u);
      // pixel w+1 outside the image counts as 1 for the erosion (min over in-bounds)
      const uint32_t rim = (k + 1 == WPR) ? (1u << (nvalid - 1)) : 0u;
      uint32_t er = 0xFFFFFFFFu;
      for (int hh = imax_(h - 1, 0); hh <= imin_(h + 1, Hc - 1); ++hh) {
        const uint32_t* row = BIN + hh * WPR;
        const uint32_t c = row[k];
        const uint32_t l = (c << 1) | (k > 0 ? row[k - 1] >> 31 : 1u);
        const uint32_t r = (c >> 1) | (k + 1 < WPR ? row[k + 1] << 31 : 0u) | rim;
        er &= c & l & r;
      }
      const uint32_t m = BIN[h * WPR + k];
      BND[h * WPR + k] = m & ~er;
      const uint32_t D = m;
      const uint32_t Cc = (m << 1) | (k > 0 ? BIN[h * WPR + k - 1] >> 31 : 0u);
      const uint32_t Bq = h > 0 ? BIN[(h - 1) * WPR + k] : 0u;
      const uint32_t Aq = h > 0 ? ((Bq << 1) | (k > 0 ? BIN[(h - 1) * WPR + k - 1] >> 31 : 0u)) : 0u;
      const uint32_t odd = Aq ^ Bq ^ Cc ^ D;
      const uint32_t pairs = (Aq & Bq) | (Aq & Cc) | (Aq & D) | (Bq & Cc) | (Bq & D) | (Cc & D);
      Q1[h * WPR + k] = odd & ~pairs & vmask;
      Q3[h * WPR + k] = odd & pairs & vmask;
      QD[h * WPR + k] = (((Aq & D) & ~(Bq | Cc)) | ((Bq & Cc) & ~(Aq | D))) & vmask;
    }
    MSYNC();
    }
    if (role == 0 && S.edge_out) MFOR2(h, w, Hc, Wc) S.edge_out[(size_t)b * P + h * Wc + w] = (edge[h * WPR + (w >> 5)] >> (w & 31)) & 1u;
    if (role == 1 && S.bin_out) MFOR2(h, w, Hc, Wc) S.bin_out[(size_t)b * P + h * Wc + w] = (BIN[h * WPR + (w >> 5)] >> (w & 31)) & 1u;
    MSTAMP(8);

    // -- per-tile partial quantities, one thread per (tile, item):
    //    items [0,4)            gradient window sums gx, gx^2, gy, gy^2 (row-major order)
    //    items [4,4+S)          log(n_s + 1), n_s = occupied s x s boxes of the edge map
    //    items [4+S,14+S)       p_k * log2(p_k + 1e-10) of the uniform-LBP label k
    //    items [14+S,20+S)      counts: edges, mask area, boundary, Euler quads q1, q3, qd
    int S_ = 0;
    for (int s = 2; s <= T; s *= 2) ++S_;
    // items of this workgroup: edge role = box counts [4, 4+S) and the edge
    // count 14+S; mask role = gradient sums [0,4), LBP terms [4+S, 14+S) and
    // the mask counts [15+S, 20+S).  Item-major order (consecutive lanes =
    // consecutive tiles of one item), each item group padded to whole waves.
    float* ttmp = S.tile_tmp + (size_t)b * NT * TT_STRIDE;
    const int nG = role ? (4 * NT + 63) & ~63 : (S_ * NT + 63) & ~63;
    const int nR = role ? 15 * NT : NT;
    const float inv_nt = 1.0f / (float)NT, inv_wt = 1.0f / (float)wt;
    MFOR(u, nG + nR) {
      int it, t;
      if (u < nG) {
        const int nit = role ? 4 : S_;
        if (u >= nit * NT) continue;
        const int kq = div_small(u, NT, inv_nt);
        it = (role ? 0 : 4) + kq; t = u - kq * NT;
      } else {
        const int v = u - nG, kk = div_small(v, NT, inv_nt);
        t = v - kk * NT;
        it = role ? (kk < 10 ? 4 + S_ + kk : 15 + S_ + (kk - 10)) : 14 + S_;
      }
      const int th = div_small(t, wt, inv_wt), tw = t - th * wt;
      const int h0 = th * T, w0 = tw * T;
      float val;
      if (it < 4) {
        const float* plane = (it < 2) ? pl.A : pl.Bf;
        const bool sq = (it & 1) != 0;
        if (T == 4) val = sq ? tile_sum_t<4, true>(plane, Wc, h0, w0) : tile_sum_t<4, false>(plane, Wc, h0, w0);
        else if (T == 8) val = sq ? tile_sum_t<8, true>(plane, Wc, h0, w0) : tile_sum_t<8, false>(plane, Wc, h0, w0);
        else if (T == 16) val = sq ? tile_sum_t<16, true>(plane, Wc, h0, w0) : tile_sum_t<16, false>(plane, Wc, h0, w0);
        else {
          float acc = 0.0f;
          for (int yy = 0; yy < T; ++yy) {
            const float* row = plane + (h0 + yy) * Wc + w0;
            if (sq) { for (int xx = 0; xx < T; ++xx) acc = acc + row[xx] * row[xx]; }
            else { for (int xx = 0; xx < T; ++xx) acc = acc + row[xx]; }
          }
          val = acc;
        }
      } else if (it < 4 + S_) {
        // box counting (morphology.py:576-621): OR-fold s rows, then s columns
        const int s = 2 << (it - 4);
        int n = 0;
        if (T == 4) n = box_count_t<4>(edge, WPR, h0, w0, s);
        else if (T == 8) n = box_count_t<8>(edge, WPR, h0, w0, s);
        else if (T == 16) n = box_count_t<16>(edge, WPR, h0, w0, s);
        else for (int by = 0; by < T; by += s) {
          if (s <= 32) {
            const int fw = T < 32 ? T : 32;
            uint32_t starts = 0u;
            for (int x = 0; x < fw; x += s) starts |= 1u << x;
            for (int fx = 0; fx < T; fx += fw) {
              uint32_t o = 0u;
              for (int yy = 0; yy < s; ++yy) o |= row_field(edge + (h0 + by + yy) * WPR, w0 + fx, fw, WPR);
              for (int sh2 = 1; sh2 < s; sh2 <<= 1) o |= o >> sh2;     // group OR onto its first bit
              n += popc(o & starts);
            }
          } else {   // s >= 64: whole-word boxes
            for (int bx = 0; bx < T; bx += s) {
              int any = 0;
              for (int yy = 0; yy < s && !any; ++yy) any = row_pop(edge + (h0 + by + yy) * WPR, w0 + bx, s, WPR) > 0;
              n += any;
            }
          }
        }
        val = n <= 64 ? bits_as_float(k_lognp1_bits[n]) : cr_log((float)n + 1.0f);
      } else {
        const int k = it - 4 - S_;
        const uint32_t* plane = k < 10 ? pl.bits(BP_L0 + k)
                              : (k == 10 ? edge : (k == 11 ? BIN : (k == 12 ? BND : (k == 13 ? Q1 : (k == 14 ? Q3 : QD)))));
        int cnt = 0;
        if (k < 10 && lbp_cnt) cnt = lcnt[t * 10 + k];
        else if (T == 4) cnt = tile_pop_t<4>(plane, WPR, h0, w0);
        else if (T == 8) cnt = tile_pop_t<8>(plane, WPR, h0, w0);
        else if (T == 16) cnt = tile_pop_t<16>(plane, WPR, h0, w0);
        else for (int yy = 0; yy < T; ++yy) cnt += row_pop(plane + (h0 + yy) * WPR, w0, T, WPR);
        if (k < 10) {
          // exact table of p * log2(p + 1e-10), p = cnt / T^2 (tools/gen_tables.py)
          if (T == 4) val = bits_as_float(k_lbp_t4_bits[cnt]);
          else if (T == 8) val = bits_as_float(k_lbp_t8_bits[cnt]);
          else if (T == 16) val = bits_as_float(k_lbp_t16_bits[cnt]);
          else {
            const float pk = (float)cnt / fT2;
            val = pk * log2_ref(pk + 1e-10f);
          }
        } else {
          val = (float)cnt;
        }
      }
      ttmp[t * TT_STRIDE + it] = val;
    }
    MSYNC();

  }
  MSTAMP(9);
}

// phi1..phi5 + interactions of tile t of image b from its per-tile partial
// quantities tv[0..20+S) (morphology.py:576-739, :860-864) into tp[0..8)
MCAQ_HD void phi_of_tile(const MorphScale& S, int b, int t, const float* tv, float* tp) {
  const int T = S.tile, NT = S.ht * S.wt;
  const float fT2 = (float)(T * T);
  int S_ = 0;
  for (int s = 2; s <= T; s *= 2) ++S_;
  // phi1: weighted log-log regression slope (morphology.py:596-621)
  float p1;
  if (S_ >= 2) {
    const int ycut = aten_tail_start(img_batch_total(S) * NT);
    float xs[8], ws[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      xs[i] = i < S_ ? bits_as_float(k_frac_x_bits[i]) : 0.0f;
      ws[i] = i < S_ ? bits_as_float(k_frac_w_bits[i]) : 0.0f;
    }
    const float w_sum = bits_as_float(k_frac_st_bits[4 * S_ + 0]);
    const float x_mean = bits_as_float(k_frac_st_bits[4 * S_ + 1]);
    const float var = bits_as_float(k_frac_st_bits[4 * S_ + 2]);
    const bool tail = (img_global(S, b) * NT + t) >= ycut;
    float ys[8], wy[8], cv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ys[i] = i < S_ ? tv[4 + i] : 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) wy[i] = ws[i] * ys[i];
    const float y_mean = small_sum(wy, S_, tail) / w_sum;
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = (ws[i] * (xs[i] - x_mean)) * (ys[i] - y_mean);
    const float cov = small_sum(cv, S_, tail);
    p1 = clampf_(-(cov / (var + 1e-12f)), 1.0f, 2.0f) / 2.0f;
  } else {
    p1 = 1.0f / 2.0f;
  }
  // phi2: LBP entropy, bins summed 8, 9, 0..7 (channels-last inner sum)
  const float* terms = tv + 4 + S_;
  float ent = 0.0f;
  ent = ent + terms[8];
  ent = ent + terms[9];
#pragma unroll
  for (int k = 0; k < 8; ++k) ent = ent + terms[k];
  const float p2 = (-ent) / (float)3.321928094887362;
  // phi3: gradient variance
  const float mgx = tv[0] / fT2, mgx2 = tv[1] / fT2, mgy = tv[2] / fT2, mgy2 = tv[3] / fT2;
  const float v = fmax_(mgx2 - mgx * mgx, 0.0f) + fmax_(mgy2 - mgy * mgy, 0.0f);
  const float p3 = v / (v + 1.0f);
  // phi4 edge density, phi5 contour complexity
  const float* cn = tv + 14 + S_;
  const float p4 = cn[0] / fT2;
  const float fa = cn[1], fp = cn[2];
  float ic = (fp * fp) / ((float)(4.0 * 3.14159265358979323846) * fa + 1e-6f);
  if (!(S.flags & F_NO_EULER)) {
    // Euler sum = (q1 - q3 - 2 qd) / 4: a multiple of 0.25, exact in fp32
    const float esum = (cn[3] - cn[4] - 2.0f * cn[5]) * 0.25f;
    ic = ic / fmax_(rintf((esum / fT2) * fT2), 1.0f);
  }
  const float p5 = fa > 0.0f ? 1.0f - 1.0f / fmax_(ic, 1.0f) : 0.0f;
  const float p8 = cr_sqrt(p4 * p5 + 1e-12f);
  tp[0] = p1; tp[1] = p2; tp[2] = p3; tp[3] = p4; tp[4] = p5;
  tp[5] = p1 * p2; tp[6] = p3 * p3; tp[7] = p8;
}

// phi of every tile of image b from the partials staged in tiles[t][T_TMP..] (pass B)
template <int TS>
MCAQ_HD void assemble_phi(const Ctx& ctx, const MorphScale& S, int b, float* tiles) {
  const int NT = S.ht * S.wt;
  MFOR(t, NT) {
    float* tp = tiles + t * TS + T_PHI;
    phi_of_tile(S, b, t, tiles + t * TS + T_TMP, tp);
    if (S.phi_out) {
      float* o = S.phi_out + ((size_t)b * NT + t) * 8;
      for (int k = 0; k < 8; ++k) o[k] = tp[k];
    }
  }
  MSYNC();
}

// batched copy of n values: every thread issues up to K loads before its
// first store (a runtime-trip-count loop would pay one memory latency per
// iteration); fs(u) loads item u, fd(u, v) stores it
template <int K, class FS, class FD>
MCAQ_HD void bcopy(const Ctx& ctx, int n, FS fs, FD fd) {
  if (n <= K * ctx.nthr) {
    float v[K];
#pragma unroll
    for (int i = 0; i < K; ++i) { const int u = ctx.tid + i * ctx.nthr; v[i] = u < n ? fs(u) : 0.0f; }
#pragma unroll
    for (int i = 0; i < K; ++i) { const int u = ctx.tid + i * ctx.nthr; if (u < n) fd(u, v[i]); }
  } else {
    MFOR(u, n) fd(u, fs(u));
  }
}

// weight blobs staged in the tile kernel's LDS (float offsets, 16-B aligned)
enum : int {
  WL_CM = 0,
  WL_MM = (CM_BLOB + 3) & ~3,
  WL_SM = WL_MM + ((MM_BLOB + 3) & ~3),
  WL_FLOATS = WL_SM + ((SM_SIZE + 3) & ~3),
};
MCAQ_HD int weights_lds_bytes() { return 4 * WL_FLOATS; }
// sequential row-major sum of a K x K window of a global plane (adaptive_avg_pool
// order), all loads issued together
template <int K>
MCAQ_HD float window_sum_t(const float* a, int W, int h0, int w0) {
  float v[K * K];
#pragma unroll
  for (int y = 0; y < K; ++y)
#pragma unroll
    for (int x = 0; x < K; ++x) v[y * K + x] = a[(h0 + y) * W + w0 + x];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < K * K; ++i) s = s + v[i];
  return s;
}

// Copy of the weight ranges the device MLPs read into the staged blob `wl`
// (every thread of the workgroup; wtid / wnthr: its index and count), and of
// this image's tile partials into tiles[t][T_TMP..T_TMP+32), all loads issued
// before the first store; addresses by selects only (no divergent branches
// between the loads).
#if defined(__HIP_DEVICE_COMPILE__)
template <int TS>
MCAQ_HD void stage_tiles(const Ctx& ctx, const MorphScale& S, int b, float* tiles, float* wl, int wtid, int wnthr) {
  const int NT = S.ht * S.wt;
  // tile partials: NT rows of 8 float4 (tile_tmp rows are contiguous)
  const int q_t = (S.flags & F_PHI) ? NT * 8 : 0;
  const float4* tsrc = reinterpret_cast<const float4*>(S.tile_tmp + (size_t)b * NT * TT_STRIDE);
  // weights: [CM_B1, CM_W2) + [CM_B2, end) of the complexity MLP, [MM_B1, MM_W2) +
  // [MM_B2, MM_W3) + [MM_B3, end) of the mapper, the whole soft-mask net
  const int c1 = (CM_W2 - CM_B1) >> 2, c2 = ((CM_BLOB + 3) >> 2) - (CM_B2 >> 2);
  const int m1 = (MM_W2 - MM_B1) >> 2, m2 = (MM_W3 - MM_B2) >> 2, m3 = ((MM_BLOB + 3) >> 2) - (MM_B3 >> 2);
  const int q_c = (wl && (S.flags & F_CMLP)) ? c1 + c2 : 0;
  const int q_m = (wl && (S.flags & F_MAPPER) && !(S.flags & F_MAP_LINEAR)) ? m1 + m2 + m3 : 0;
  const int q_s = (wl && (S.flags & F_SOFTMASK)) ? (SM_SIZE + 3) >> 2 : 0;
  const int nw = q_c + q_m + q_s;
  const uintptr_t pc = (uintptr_t)S.cmlp, pm = (uintptr_t)S.mapper, ps = (uintptr_t)S.smask;
  // float4 index u of the weight copy -> source address, float4 offset in wl
  struct WSrc { const float4* p; int dq; };
  auto wsrc = [&](int u) -> WSrc {
    const int v = u - q_c, z = v - q_m;
    const int qc = u < c1 ? (CM_B1 >> 2) + u : (CM_B2 >> 2) + (u - c1);
    const int qm = v < m1 ? (MM_B1 >> 2) + v : (v < m1 + m2 ? (MM_B2 >> 2) + (v - m1) : (MM_B3 >> 2) + (v - m1 - m2));
    const bool inc = u < q_c, inm = !inc && v < q_m;
    const int q = inc ? qc : (inm ? qm : z);
    // bit-mask select (a ternary chain becomes a private-memory lookup table)
    const uintptr_t mc = (uintptr_t)0 - (uintptr_t)inc, mm = (uintptr_t)0 - (uintptr_t)inm;
    const uintptr_t base = (pc & mc) | (pm & mm) | (ps & ~(mc | mm));
    return WSrc{reinterpret_cast<const float4*>(base) + q, (inc ? (WL_CM >> 2) : (inm ? (WL_MM >> 2) : (WL_SM >> 2))) + q};
  };
  constexpr int KT = 4, KW = 8;
  float4* wl4 = reinterpret_cast<float4*>(wl);
  if (q_t <= KT * ctx.nthr && nw <= KW * wnthr) {
    float4 vt[KT], vw[KW];
    int dw[KW];
#pragma unroll
    for (int i = 0; i < KW; ++i) {
      const int u = wtid + i * wnthr;
      const WSrc ws = wsrc(u < nw ? u : 0);
      dw[i] = ws.dq;
      vw[i] = nw > 0 ? *ws.p : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < KT; ++i) {
      const int u = ctx.tid + i * ctx.nthr;
      vt[i] = q_t > 0 ? tsrc[u < q_t ? u : 0] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < KW; ++i) if (wtid + i * wnthr < nw) wl4[dw[i]] = vw[i];
#pragma unroll
    for (int i = 0; i < KT; ++i) {
      const int u = ctx.tid + i * ctx.nthr;
      if (u < q_t) reinterpret_cast<float4*>(tiles + (u >> 3) * TS + T_TMP)[u & 7] = vt[i];
    }
  } else {
    for (int u = wtid; u < nw; u += wnthr) { const WSrc ws = wsrc(u); wl4[ws.dq] = *ws.p; }
    MFOR(u, q_t) reinterpret_cast<float4*>(tiles + (u >> 3) * TS + T_TMP)[u & 7] = tsrc[u];
  }
}
#endif

// ---- pass B: per-image tile work, one group of threads per image (small
// images share a workgroup): phi assembly, complexity MLP, bilateral,
// normalisation, bit mapper, soft mask (tile values; the m plane itself only
// on request).  LDS per image: Shared (fixed + tiles) | extra | bilateral
// weights (25 NT floats); the staged weight blobs `wl` (or null) belong to the
// workgroup.
MCAQ_HD int tiles_lds_bytes(int H, int W, int NT, int TS = TILE_FLOATS_PAD) {
  return fixed_bytes() + tile_bytes(NT, TS) + extra_bytes(H, W, NT) + 100 * NT;
}

// per-tile mean |x| activation of the soft mask (adaptive_avg_pool2d windows)
MCAQ_HD float smask_act_tile(const float* am, int H, int W, int ht, int wt, float inv_wt, int t) {
  const int KH = H / ht, KW = W / wt;
  const bool even = KH * ht == H && KW * wt == W && KH == KW;
  const int i = div_small(t, wt, inv_wt), j = t - i * wt;
  if (even && KH == 4) return (window_sum_t<4>(am, W, i * 4, j * 4) / 4.0f) / 4.0f;
  if (even && KH == 8) return (window_sum_t<8>(am, W, i * 8, j * 8) / 8.0f) / 8.0f;
  const int ha = (i * H) / ht, hb = ((i + 1) * H + ht - 1) / ht;
  const int wa = (j * W) / wt, wb = ((j + 1) * W + wt - 1) / wt;
  float s = 0.0f;
  for (int h = ha; h < hb; ++h)
    for (int w = wa; w < wb; ++w) s = s + am[h * W + w];
  return (s / (float)(hb - ha)) / (float)(wb - wa);
}

// xs: the workgroup's MLP activation scratch (MLP_SCRATCH_FLOATS per wave), device only
// kSmo: a soft-mask-only launch (every scale F_SOFTMASK with bits_in and at
// most one tile per thread of its image group; host-checked)
template <int TS = TILE_FLOATS_PAD, bool kSmo = false>
MCAQ_HD void morph_tiles(const Ctx& ctx, const MorphScale& S, int b, Shared& sh, float* wl, int wtid, int wnthr,
                         float* xs) {
  const int ht = S.ht, wt = S.wt, NT = ht * wt;
  const float inv_wt = 1.0f / (float)wt;
  float* tiles = sh.tiles;
  float* extra = tiles + NT * TS;            // compact per-tile arrays / tables
  float* wbuf = (float*)((char*)extra + extra_bytes(S.H, S.W, NT));
  const float* Pc = S.cmlp;
  const float* Pmap = S.mapper;
  const float* Pm = S.smask;
  MSTAMP_INIT(b == 0 ? 0 : -1);
  MSTAMP(10);
  // soft-mask-only launch (the train step's m planes, bits given): each
  // thread's tile bits and pooled activation are loaded before the weight
  // staging - one memory latency instead of three, the same values
  float pre_b = 0.0f, pre_a = 0.0f;
  if constexpr (kSmo) {
    if (ctx.tid < NT) {
      pre_b = S.bits_in[(size_t)b * NT + ctx.tid];
      pre_a = smask_act_tile(S.absmean + (size_t)b * S.H * S.W, S.H, S.W, ht, wt, inv_wt, ctx.tid);
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  stage_tiles<TS>(ctx, S, b, tiles, wl, wtid, wnthr);
  if (wl && (S.flags & F_CMLP)) Pc = wl + WL_CM;
  if (wl && (S.flags & F_MAPPER) && !(S.flags & F_MAP_LINEAR)) Pmap = wl + WL_MM;
  if (wl && (S.flags & F_SOFTMASK)) Pm = wl + WL_SM;
#else
  (void)wl; (void)wtid; (void)wnthr; (void)xs;
  int S_ = 0;
  for (int s = 2; s <= S.tile; s *= 2) ++S_;
  const int NI = 20 + S_;
  const float* ttmp = S.tile_tmp + (size_t)b * NT * TT_STRIDE;
  if (S.flags & F_PHI)
    MFOR(u, NT * NI) {
      const int t = u / NI, it = u - (u / NI) * NI;
      tiles[t * TS + T_TMP + it] = ttmp[t * TT_STRIDE + it];
    }
#endif
  if (S.flags & F_PHI) {
    // partial quantities of the edge and mask workgroups -> phi
    MSYNC();
    MSTAMP(26);
    assemble_phi<TS>(ctx, S, b, tiles);
    MSTAMP(27);
  } else if (S.flags & F_CMLP) {
    bcopy<16>(ctx, NT * 8, [&](int u) { return S.phi_out[(size_t)b * NT * 8 + u]; },
              [&](int u, float v) { tiles[(u >> 3) * TS + T_PHI + (u & 7)] = v; });
    MSYNC();
  } else {
    MSYNC();   // staged weights visible
  }

  // -- complexity MLP + bilateral (morphology.py:959-968)
  if (S.flags & F_CMLP) {
#if defined(__HIP_DEVICE_COMPILE__)
    for (int blk = ctx.tid >> 6; blk * MLP_TPW < NT; blk += ctx.nthr >> 6) {
      const bool st = b == 0 && blk == 0 && ctx.nthr == MCAQ_TILES_THREADS;
      const lds_f xw = (lds_f)(xs + (threadIdx.x >> 6) * MLP_SCRATCH_FLOATS);
      if (wl) cmlp_block_mfma<MLP_NH, lds_cf, TS>((lds_cf)Pc, tiles, NT, blk * MLP_TPW, ctx.tid & 63, xw, st);
      else cmlp_block_mfma<MLP_NH, const float*, TS>(Pc, tiles, NT, blk * MLP_TPW, ctx.tid & 63, xw, st);
    }
    MSTAMP(28);
#else
    MFOR(t, NT) {
      float phi[8];
      for (int k = 0; k < 8; ++k) phi[k] = tiles[t * TS + T_PHI + k];
      tiles[t * TS + T_CMLP] = complexity_mlp_tile(Pc, phi);
    }
#endif
    MSYNC();
    MFOR(t, NT) {
      const float v = tiles[t * TS + T_CMLP];
      extra[t] = v;
      if (S.cmlp_out) S.cmlp_out[(size_t)b * NT + t] = v;
    }
    MSYNC();
    MSTAMP(11);
    // range weights w = spatial * exp(-(d^2)/0.02), one thread per (tile, tap),
    // up to BK items per thread with their exps in flight together
    {
      constexpr int BK = 12;
      auto wgt = [&](int u) {
        const int t = u / 25, k = u - (u / 25) * 25;
        const int th = div_small(t, wt, inv_wt), tw = t - th * wt;
        const int hh = imin_(imax_(th + k / 5 - 2, 0), ht - 1);
        const int ww = imin_(imax_(tw + k % 5 - 2, 0), wt - 1);
        const float d = extra[hh * wt + ww] - extra[t];
        return bits_as_float(k_bilat_sp_bits[k]) * cr_exp((-(d * d)) / 0.02f);
      };
      bcopy<BK>(ctx, NT * 25, wgt, [&](int u, float v) { wbuf[u] = v; });
      MSYNC();
    }
    MSTAMP(29);
    const int cut = aten_tail_start(NT);
    MFOR(t, NT) {
      const int th = div_small(t, wt, inv_wt), tw = t - th * wt;
      // 25-row ATen outer sums of w*p and w: vector column = rows 0..15 folded,
      // then 16..24 in a0; tail column = 4 interleaved partials (rows 4i+q),
      // row 24 into partial 0.  Adding an exact +0 is an identity (sums never
      // hold -0), so both orders are accumulated with selects in one loop.
      const bool tail = t >= cut;
      float pv[25], wv[25];
#pragma unroll
      for (int k = 0; k < 25; ++k) {
        const int hh = imin_(imax_(th + k / 5 - 2, 0), ht - 1);
        const int ww = imin_(imax_(tw + k % 5 - 2, 0), wt - 1);
        pv[k] = extra[hh * wt + ww];
        wv[k] = wbuf[t * 25 + k];
      }
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
      const float c = clampf_(num / (dsum + 1e-8f), 0.0f, 1.0f);
      tiles[t * TS + T_C] = c;
      if (S.c_out) S.c_out[(size_t)b * NT + t] = c;
    }
    MSYNC();
  } else if (S.c_in) {
    bcopy<16>(ctx, NT, [&](int u) { return S.c_in[(size_t)b * NT + u]; },
              [&](int u, float v) { tiles[u * TS + T_C] = v; });
    MSYNC();
  }
  MSTAMP(12);

  // -- optional percentile normalisation (models/mcaq_yolo.py:427-432) and mapper
  if (S.flags & F_MAPPER) {
    int csrc = T_C;
    if (S.flags & F_NORM_C) {
      sort_tiles<TS>(ctx, tiles, NT, T_C);
      const float lo = quantile_sorted(tiles + T_SORT, TS, NT, 0.02f);
      const float hi = quantile_sorted(tiles + T_SORT, TS, NT, 0.98f);
      MSYNC();
      const float den = (hi - lo) + 1e-8f;
      MFOR(t, NT) {
        const float c = tiles[t * TS + T_C];
        tiles[t * TS + T_CN] = clampf_((c - lo) / den, 0.0f, 1.0f);
      }
      MSYNC();
      csrc = T_CN;
    }
    if (S.flags & F_MAP_LINEAR) {
      // LinearBitMapper (bit_allocation.py:42-80)
      sort_tiles<TS>(ctx, tiles, NT, csrc);
      const float lo = quantile_sorted(tiles + T_SORT, TS, NT, 0.02f);
      const float hi = quantile_sorted(tiles + T_SORT, TS, NT, 0.98f);
      MSYNC();
      const float spread = hi - lo;
      MFOR(t, NT) {
        const float c = tiles[t * TS + csrc];
        const float rel = clampf_((c - lo) / (spread + 1e-8f), 0.0f, 1.0f);
        const float cn = spread > 1e-3f ? rel : clampf_(c, 0.0f, 1.0f);
        tiles[t * TS + T_AUX] = S.min_bits + (S.max_bits - S.min_bits) * cn;
      }
    } else {
#if defined(__HIP_DEVICE_COMPILE__)
      // fold the three eval BatchNorms once per workgroup: alpha = inv*g,
      // beta = b - (rm*inv)*g, inv = 1/sqrt(rv + eps)  (same values as bn_eval)
      float* ab = extra;
      MFOR(j, 128) {
        const int L = j < 32 ? 0 : (j < 96 ? 1 : 2);
        const int n = L == 1 ? 64 : 32;
        const int jj = j - (L == 0 ? 0 : (L == 1 ? 32 : 96));
        const float* bn = Pmap + (L == 0 ? MM_BN1 : (L == 1 ? MM_BN2 : MM_BN3));
        const float inv = 1.0f / cr_sqrt(bn[3 * n + jj] + 1e-5f);
        ab[j] = inv * bn[jj];
        ab[128 + j] = bn[n + jj] - (bn[2 * n + jj] * inv) * bn[jj];
      }
      MSYNC();
      MSTAMP(30);
      for (int blk = ctx.tid >> 6; blk * MLP_TPW < NT; blk += ctx.nthr >> 6) {
        const bool st = b == 0 && blk == 0 && ctx.nthr == MCAQ_TILES_THREADS;
        const lds_f xw = (lds_f)(xs + (threadIdx.x >> 6) * MLP_SCRATCH_FLOATS);
        if (wl) mapper_block_mfma<MLP_NH, lds_cf, TS>((lds_cf)Pmap, (lds_cf)ab, tiles, NT, blk * MLP_TPW, ctx.tid & 63, csrc, S.min_bits,
                                  S.max_bits, xw, st);
        else mapper_block_mfma<MLP_NH, const float*, TS>((const float*)Pmap, (const float*)ab, tiles, NT, blk * MLP_TPW, ctx.tid & 63, csrc,
                               S.min_bits, S.max_bits, xw, st);
      }
#else
      MFOR(t, NT) tiles[t * TS + T_AUX] =
          mapper_mlp_tile(Pmap, tiles[t * TS + csrc], S.min_bits, S.max_bits);
#endif
    }
    MSYNC();
    MFOR(t, NT) {
      const float bv = finish_bits(tiles[t * TS + T_AUX], S);
      tiles[t * TS + T_BITS] = bv;
      if (S.bits_out) S.bits_out[(size_t)b * NT + t] = bv;
    }
    MSYNC();
  } else if (kSmo) {
    if (ctx.tid < NT) tiles[ctx.tid * TS + T_BITS] = pre_b;
    MSYNC();
  } else if ((S.flags & F_SOFTMASK) && S.bits_in) {
    bcopy<16>(ctx, NT, [&](int u) { return S.bits_in[(size_t)b * NT + u]; },
              [&](int u, float v) { tiles[u * TS + T_BITS] = v; });
    MSYNC();
  }
  MSTAMP(13);

  // -- learned soft mask m(p) (quantization.py:213-239)
  if (S.flags & F_SOFTMASK) {
    const int H = S.H, W = S.W;
    const float* am = S.absmean + (size_t)b * H * W;
    float lmx = -3.402823466e38f;
    MFOR(t, NT) {
      const float a = kSmo ? pre_a : smask_act_tile(am, H, W, ht, wt, inv_wt, t);
      tiles[t * TS + T_ACT] = a;
      lmx = fmaxp(lmx, a);          // torch.amax: a NaN activation makes the image's max NaN
    }
    const float amax = block_max(ctx, sh, lmx);
    MSTAMP(31);
    const float den = amax + 1e-8f;
    // the two conv input features, compact: f0 = bits feature, f1 = activation
    float* f0a = extra;
    float* f1a = extra + NT;
    MFOR(t, NT) {
      f0a[t] = clampf_((tiles[t * TS + T_BITS] - 2.0f) / 6.0f, 0.0f, 1.0f);
      f1a[t] = tiles[t * TS + T_ACT] / den;
    }
    MSYNC();
    MFOR(t, NT) {
      const int i = div_small(t, wt, inv_wt), j = t - i * wt;
      // 3x3 window (zero pad): (kh, kw) outer, ic inner, FMA from 0, + bias;
      // out-of-grid taps are skipped exactly as the reference's zero taps
      float f0[9], f1[9];
      bool ok[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        const int ii = i + q / 3 - 1, jj = j + q % 3 - 1;
        ok[q] = ii >= 0 && ii < ht && jj >= 0 && jj < wt;
        const int src = imin_(imax_(ii, 0), ht - 1) * wt + imin_(imax_(jj, 0), wt - 1);
        f0[q] = f0a[src]; f1[q] = f1a[src];
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
      // softmax over 2: the larger logit's term is exp(+0) = 1 exactly (both
      // exps); the other is SLEEF's or glibc's by ATen's lane of this tile
      const float mxl = fmax_(l0, l1);
      const bool first = l0 >= l1;
      const float ea = (first ? l1 : l0) - mxl;
      const bool vl = aten_softmax_vec_lane((long long)img_global(S, b) * NT + t,
                                            (long long)img_batch_total(S) * NT, NT, S.softmax_threads);
      const float e = vl ? sleef_expf(ea) : cr_exp(ea);
      const float e0 = first ? 1.0f : e, e1 = first ? e : 1.0f;
      const float mtv = e0 / (e0 + e1);
      tiles[t * TS + T_MT] = mtv;
      if (S.mt_out) S.mt_out[(size_t)b * NT + t] = mtv;
    }
    MSYNC();
    MSTAMP(14);
    if (S.m_out) {
      // compact m(tile) and the nearest-upsample source of every row / column
      float* mt = extra;
      int* rsrc = (int*)(extra + NT);
      int* csrc = rsrc + H;
      MFOR(t, NT) mt[t] = tiles[t * TS + T_MT];
      MFOR(h, H) rsrc[h] = nearest_src(h, ht, H) * wt;
      MFOR(w, W) csrc[w] = nearest_src(w, wt, W);
      MSYNC();
      float* mo = S.m_out + (size_t)b * H * W;
      const int qpr = (W + 3) >> 2;
      MFOR(q, H * qpr) {
        const int h = q / qpr, w0 = (q - h * qpr) * 4;
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        int cs[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) cs[u] = csrc[imin_(imax_(w0 - 2 + u, 0), W - 1)];
        for (int i = 0; i < 5; ++i) {
          const int rb = rsrc[imin_(imax_(h + i - 2, 0), H - 1)];
          float seg[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) seg[u] = mt[rb + cs[u]];
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            const float k = bits_as_float(k_smooth5_bits[i * 5 + j]);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = fmaf(k, seg[r + j], acc[r]);
          }
        }
        if (w0 + 3 < W && (W & 3) == 0) {
          store4(mo + h * W + w0, acc);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) if (w0 + r < W) mo[h * W + w0 + r] = acc[r];
        }
      }
    }
    MSYNC();
  }
  MSTAMP(15);
}

}  // namespace mcaq

#include "mcaq_band.h"   // pass A as band + edge workgroups
#include "mcaq_tiles_batch.h"   // pass B as batch-wide tile kernels
