// mcaq_kernels.hip - gfx950 (CDNA4) kernels of the MCAQ hook path and the
// extern "C" launchers declared in include/mcaq_hip.h.
//
//   pass 1  mcaq_stats_kernel     one read of x: per-pixel channel sums in
//                                 ATen order (gray, |x|) + per-channel min/max
//                                 partials                      (HBM bound)
//           mcaq_finalize_kernel  channel min/max -> scale/zero-point table
//   morph   mcaq_morph_kernel     one workgroup per (scale, image): Canny,
//                                 adaptive mask, phi1..5, MLP, bilateral,
//                                 mapper, soft mask (LDS resident planes)
//   pass 2  mcaq_quant_kernel     one read of x + one write of y: tile-wise
//                                 2..8-bit quant/dequant fused with m(p)
//
// Built with -ffp-contract=off (see mcaq_math.h).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/mcaq_hip.h"
#include "mcaq_math.h"
#include "mcaq_morph.h"

using namespace mcaq;

#if defined(MCAQ_STAMPS)
namespace mcaq { __device__ unsigned long long g_mcaq_stamps[64]; }
extern "C" int mcaq_read_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(mcaq::g_mcaq_stamps), sizeof(mcaq::g_mcaq_stamps));
}
#endif

// ---------------------------------------------------------------------------
// pass 1
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

struct StatsArgs {
  mcaq_stats_scale s[3];
  int nscales;
  int units_total;
};

constexpr int ST_PIX = 256;   // pixels per workgroup (one per lane)
constexpr int ST_CG = 16;     // channels per load group (= one ATen cascade block)

// unit = one 256-thread workgroup = 256 consecutive pixels of one image.
// Lane = pixel: the channel loop runs the ATen cascade in registers; each
// 16-channel group is one cascade block (a0 summed from 0, then folded).
// Channel min/max: the group's values go through an LDS transpose
// [16 ch][256 px] and are reduced by 16 threads per channel.
__global__ __launch_bounds__(256) void mcaq_stats_kernel(StatsArgs a) {
  __shared__ float tmn[ST_CG][ST_PIX + 4];
  __shared__ float tmx[ST_CG][ST_PIX + 4];
  const int unit = blockIdx.x;
  int si = 0;
  while (si + 1 < a.nscales && unit >= a.s[si + 1].unit_begin) ++si;
  const mcaq_stats_scale& S = a.s[si];
  const int tid = threadIdx.x;
  const int lu = unit - S.unit_begin;
  const int HW = S.H * S.W;
  const int upi = (HW + ST_PIX - 1) / ST_PIX;
  const int b = lu / upi, chunk = lu - b * upi;
  const int C = S.C;
  const float* xb = S.x + (size_t)b * C * HW;
  const bool cropped = (S.Hc != S.H) || (S.Wc != S.W);
  const int p = chunk * ST_PIX + tid;
  const bool valid = p < HW;
  const bool want_g = S.gray != nullptr, want_a = S.absmean != nullptr, want_m = S.pmin != nullptr;
  const float* px = xb + (valid ? p : 0);

  float g1 = 0.0f, g2 = 0.0f, g3 = 0.0f;   // cascade levels 1..3 (gray)
  float a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;   // cascade levels 1..3 (|x|)
  float ga0 = 0.0f, aa0 = 0.0f;            // open (partial) block
  float sq = 0.0f;                          // sequential sum (cropped view)
  int nblk = 0;
  for (int c0 = 0; c0 < C; c0 += ST_CG) {
    const int nc = C - c0 < ST_CG ? C - c0 : ST_CG;
    float v[ST_CG];
#pragma unroll
    for (int i = 0; i < ST_CG; ++i) v[i] = (valid && i < nc) ? px[(size_t)(c0 + i) * HW] : 0.0f;
    float gb = 0.0f, ab = 0.0f;
#pragma unroll
    for (int i = 0; i < ST_CG; ++i) {
      if (i < nc) { gb = gb + v[i]; ab = ab + fabsf(v[i]); sq = sq + v[i]; }
    }
    if (nc == ST_CG) {       // a full cascade block: fold (Cascade::push at i % 16 == 0)
      ++nblk;
      g1 = g1 + gb; a1 = a1 + ab;
      if ((nblk & 15) == 0) {
        g2 = g2 + g1; g1 = 0.0f; a2 = a2 + a1; a1 = 0.0f;
        if ((nblk & 255) == 0) { g3 = g3 + g2; g2 = 0.0f; a3 = a3 + a2; a2 = 0.0f; }
      }
    } else {
      ga0 = gb; aa0 = ab;   // trailing partial block stays in a0
    }
    if (want_m) {
#pragma unroll
      for (int i = 0; i < ST_CG; ++i) {
        tmn[i][tid] = valid ? v[i] : 3.402823466e38f;
        tmx[i][tid] = valid ? v[i] : -3.402823466e38f;
      }
      __syncthreads();
      const int ci = tid >> 4, part = tid & 15;
      float mn = tmn[ci][part * 16], mx = tmx[ci][part * 16];
#pragma unroll
      for (int k = 1; k < 16; ++k) { mn = fminf(mn, tmn[ci][part * 16 + k]); mx = fmaxf(mx, tmx[ci][part * 16 + k]); }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) { mn = fminf(mn, __shfl_xor(mn, o, 64)); mx = fmaxf(mx, __shfl_xor(mx, o, 64)); }
      if (part == 0 && ci < nc) {
        S.pmin[(size_t)lu * C + c0 + ci] = mn;
        S.pmax[(size_t)lu * C + c0 + ci] = mx;
      }
      __syncthreads();
    }
  }
  if (!valid) return;
  const float fC = (float)C;
  const bool tail = p >= aten_tail_start(HW);
  if (want_a) {
    float s = ((aa0 + a1) + a2) + a3;
    if (tail) s = aten_sum(C, true, [&](int r) { return fabsf(xb[(size_t)r * HW + p]); });
    S.absmean[(size_t)b * HW + p] = s / fC;
  }
  if (want_g) {
    const int h = p / S.W, w = p - (p / S.W) * S.W;
    if (cropped) {
      if (h < S.Hc && w < S.Wc) S.gray[((size_t)b * S.Hc + h) * S.Wc + w] = sq / fC;
    } else {
      float s = ((ga0 + g1) + g2) + g3;
      if (tail) s = aten_sum(C, true, [&](int r) { return xb[(size_t)r * HW + p]; });
      S.gray[(size_t)b * HW + p] = s / fC;
    }
  }
}

// ---------------------------------------------------------------------------
// finalize: channel min/max over the partials of pass 1
// ---------------------------------------------------------------------------
struct FinalizeArgs {
  mcaq_finalize_scale s[3];
  int nscales;
};

// one workgroup = 64 channels x 4 unit-parts
__global__ __launch_bounds__(256) void mcaq_finalize_kernel(FinalizeArgs a) {
  __shared__ float rmn[4][64], rmx[4][64];
  int si = 0;
  while (si + 1 < a.nscales && (int)blockIdx.x >= a.s[si + 1].block_begin) ++si;
  const mcaq_finalize_scale& S = a.s[si];
  const int cl = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int c = ((int)blockIdx.x - S.block_begin) * 64 + cl;
  const bool cv = c < S.C;
  float mn = 3.402823466e38f, mx = -3.402823466e38f;
  if (cv) {
    if (S.pmin) {
      int u = part;
      for (; u + 12 < S.nunits; u += 16) {
        const float m0 = S.pmin[(size_t)u * S.C + c], m1 = S.pmin[(size_t)(u + 4) * S.C + c];
        const float m2 = S.pmin[(size_t)(u + 8) * S.C + c], m3 = S.pmin[(size_t)(u + 12) * S.C + c];
        const float x0 = S.pmax[(size_t)u * S.C + c], x1 = S.pmax[(size_t)(u + 4) * S.C + c];
        const float x2 = S.pmax[(size_t)(u + 8) * S.C + c], x3 = S.pmax[(size_t)(u + 12) * S.C + c];
        mn = fminf(mn, fminf(fminf(m0, m1), fminf(m2, m3)));
        mx = fmaxf(mx, fmaxf(fmaxf(x0, x1), fmaxf(x2, x3)));
      }
      for (; u < S.nunits; u += 4) {
        mn = fminf(mn, S.pmin[(size_t)u * S.C + c]);
        mx = fmaxf(mx, S.pmax[(size_t)u * S.C + c]);
      }
    } else if (part == 0) {
      mn = S.min_in[(size_t)S.min_stride * c];
      mx = S.max_in[(size_t)S.min_stride * c];
    }
  }
  rmn[part][cl] = mn; rmx[part][cl] = mx;
  __syncthreads();
  if (part == 0 && cv) {
    S.min_out[c] = fminf(fminf(rmn[0][cl], rmn[1][cl]), fminf(rmn[2][cl], rmn[3][cl]));
    S.max_out[c] = fmaxf(fmaxf(rmx[0][cl], rmx[1][cl]), fmaxf(rmx[2][cl], rmx[3][cl]));
  }
}

// ---------------------------------------------------------------------------
// morph pass A: one 1024-thread workgroup per (scale, image), planes in LDS
// morph pass B: one 256-thread workgroup per (scale, image), tile grid in LDS
// ---------------------------------------------------------------------------
constexpr int MORPH_THREADS = 1024;
constexpr int TILES_THREADS = 256;

__device__ __forceinline__ int morph_scale_of(const MorphArgs& a) {
  int si = 0;
  while (si + 1 < a.nscales && (int)blockIdx.x >= a.s[si + 1].block_begin) ++si;
  return si;
}

template <bool kLDS>
__global__ __launch_bounds__(MORPH_THREADS) void mcaq_morph_kernel(MorphArgs a, int plane_stride) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const MorphScale& S = a.s[morph_scale_of(a)];
  const int b = (int)blockIdx.x - S.block_begin;
  if (b >= S.B || !(S.flags & F_PHI)) return;
  Ctx ctx{(int)threadIdx.x, (int)blockDim.x};
  Shared sh;
  Planes pl;
  if (kLDS) {
    carve_planes(smem, S.Hc, S.Wc, pl);
    carve_shared(smem + plane_stride, sh);
  } else {
    carve_planes((char*)S.gscratch + (size_t)b * plane_stride, S.Hc, S.Wc, pl);
    carve_shared(smem, sh);
  }
  morph_edges(ctx, S, b, pl, sh);
}

__global__ __launch_bounds__(TILES_THREADS) void mcaq_tiles_kernel(MorphArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const MorphScale& S = a.s[morph_scale_of(a)];
  const int b = (int)blockIdx.x - S.block_begin;
  if (b >= S.B) return;
  Ctx ctx{(int)threadIdx.x, (int)blockDim.x};
  Shared sh;
  carve_shared(smem, sh);
  morph_tiles(ctx, S, b, sh);
}

// ---------------------------------------------------------------------------
// pass 2: y = dequant(quant_b(x)) * m, one wave = 256 pixels x a channel slice
// ---------------------------------------------------------------------------
struct QuantArgs {
  mcaq_quant_scale s[3];
  int nscales;
  int units_total;
};

constexpr int QSLICE = 16;     // channels per unit
constexpr int QMAXBITS = 15;   // max entries per channel in the LDS table

__global__ __launch_bounds__(64) void mcaq_quant_kernel(QuantArgs a) {
  __shared__ float qt[QSLICE * QMAXBITS * 2];
  const int unit = blockIdx.x;
  int si = 0;
  while (si + 1 < a.nscales && unit >= a.s[si + 1].unit_begin) ++si;
  const mcaq_quant_scale& S = a.s[si];
  const int lane = threadIdx.x;
  const int HW = S.H * S.W;
  const int upi = (HW + 255) / 256;
  const int nsl = (S.C + QSLICE - 1) / QSLICE;
  int lu = unit - S.unit_begin;
  const int slice = lu % nsl; lu /= nsl;
  const int chunk = lu % upi;
  const int b = lu / upi;
  const int c0 = slice * QSLICE;
  const int nc = imin_(QSLICE, S.C - c0);
  const int NB = S.nbits;
  for (int i = lane; i < nc * NB; i += 64) {
    const int c = i / NB, k = i - (i / NB) * NB;
    const QParam q = qparam(S.xmin[c0 + c], S.xmax[c0 + c], S.bits_lo + k);
    qt[2 * i + 0] = q.scale;
    qt[2 * i + 1] = q.zp;
  }
  __syncthreads();

  const int p0 = chunk * 256 + lane * 4;
  bool valid[4];
  int kb[4];
  float mv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = p0 + k;
    valid[k] = p < HW;
    kb[k] = 0; mv[k] = 1.0f;
    if (!valid[k]) continue;
    const int h = p / S.W, w = p - (p / S.W) * S.W;
    int th, tw;
    if (S.compat_tile_h > 0) {   // spatial_quantize contract: h / tile_h, clamped
      th = imin_(h / S.compat_tile_h, S.ht - 1);
      tw = imin_(w / S.compat_tile_w, S.wt - 1);
    } else {                     // PyTorch path: nearest upsample of the bit map
      th = nearest_src(h, S.ht, S.H);
      tw = nearest_src(w, S.wt, S.W);
    }
    const float bv = S.bits[((size_t)b * S.ht + th) * S.wt + tw];
    int bi = (int)rintf(bv);
    bi = imin_(imax_(bi, S.bits_lo), S.bits_lo + NB - 1);
    kb[k] = bi - S.bits_lo;
    if (S.m) mv[k] = S.m[(size_t)b * HW + p];
  }
  const bool vec4 = ((HW & 3) == 0) && valid[3];
  const float* xb = S.x + ((size_t)b * S.C + c0) * HW;
  float* yb = S.y + ((size_t)b * S.C + c0) * HW;
  const bool has_m = S.m != nullptr;
  for (int c = 0; c < nc; ++c) {
    const float* row = xb + (size_t)c * HW;
    float* orow = yb + (size_t)c * HW;
    float v[4];
    if (vec4) {
      const float4 q = *reinterpret_cast<const float4*>(row + p0);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = valid[k] ? row[p0 + k] : 0.0f;
    }
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      QParam q;
      q.scale = qt[(c * NB + kb[k]) * 2 + 0];
      q.zp = qt[(c * NB + kb[k]) * 2 + 1];
      const int bb = S.bits_lo + kb[k];
      q.qmin = (float)(-(1 << (bb - 1)));
      q.qmax = (float)((1 << (bb - 1)) - 1);
      float d = quant_dequant(v[k], q);
      if (has_m) d = d * mv[k];
      o[k] = d;
    }
    if (vec4) {
      *reinterpret_cast<float4*>(orow + p0) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) if (valid[k]) orow[p0 + k] = o[k];
    }
  }
}

// ---------------------------------------------------------------------------
// extern "C" launchers
// ---------------------------------------------------------------------------
extern "C" {

int mcaq_abi_version(void) { return MCAQ_ABI_VERSION; }

int mcaq_launch_spatial_quantization(const float* input, const float* bit_map, const float* min_vals,
                                     const float* max_vals, const float* mask, float* output, int N, int C,
                                     int H, int W, int tile_h, int tile_w, int n_tiles_h, int n_tiles_w,
                                     hipStream_t stream) {
  if (N < 1 || C < 1 || H < 1 || W < 1 || tile_h < 1 || tile_w < 1 || n_tiles_h < 1 || n_tiles_w < 1)
    return (int)hipErrorInvalidValue;
  mcaq_quant_scale q{};
  q.x = input; q.y = output; q.bits = bit_map; q.m = mask; q.xmin = min_vals; q.xmax = max_vals;
  q.B = N; q.C = C; q.H = H; q.W = W; q.ht = n_tiles_h; q.wt = n_tiles_w;
  q.bits_lo = 2; q.nbits = 7;
  q.compat_tile_h = tile_h; q.compat_tile_w = tile_w;
  return mcaq_quant(&q, 1, stream);
}

int mcaq_stats(const mcaq_stats_scale* scales, int nscales, hipStream_t stream) {
  if (nscales < 1 || nscales > 3) return (int)hipErrorInvalidValue;
  StatsArgs a;
  int units = 0;
  for (int i = 0; i < nscales; ++i) {
    a.s[i] = scales[i];
    a.s[i].unit_begin = units;
    const int HW = scales[i].H * scales[i].W;
    if (scales[i].B < 1 || scales[i].C < 1 || HW < 1) return (int)hipErrorInvalidValue;
    units += scales[i].B * ((HW + ST_PIX - 1) / ST_PIX);
  }
  a.nscales = nscales;
  a.units_total = units;
  hipLaunchKernelGGL(mcaq_stats_kernel, dim3(units), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

int mcaq_stats_units(int B, int H, int W) { return B * ((H * W + 255) / 256); }

int mcaq_finalize(const mcaq_finalize_scale* scales, int nscales, hipStream_t stream) {
  if (nscales < 1 || nscales > 3) return (int)hipErrorInvalidValue;
  FinalizeArgs a;
  int blocks = 0;
  for (int i = 0; i < nscales; ++i) {
    a.s[i] = scales[i];
    a.s[i].block_begin = blocks;
    if (scales[i].C < 1 || !scales[i].min_out || !scales[i].max_out) return (int)hipErrorInvalidValue;
    blocks += (scales[i].C + 63) / 64;
  }
  a.nscales = nscales;
  hipLaunchKernelGGL(mcaq_finalize_kernel, dim3(blocks), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

// dynamic LDS available to the morph kernel: 160 KiB minus its static LDS
// (the runtime rejects a launch whose static + dynamic LDS exceeds the CU's)
static int morph_lds_budget() {
  static int budget = -1;
  if (budget < 0) {
    hipFuncAttributes fa, fb;
    if (hipFuncGetAttributes(&fa, (const void*)mcaq_morph_kernel<true>) != hipSuccess ||
        hipFuncGetAttributes(&fb, (const void*)mcaq_morph_kernel<false>) != hipSuccess)
      return MCAQ_MORPH_LDS_LIMIT - 4096;   // no device yet: conservative, not cached
    const int st = imax_((int)fa.sharedSizeBytes, (int)fb.sharedSizeBytes);
    budget = MCAQ_MORPH_LDS_LIMIT - ((st + 255) & ~255);
  }
  return budget;
}

static int morph_plan(const MorphScale* s, int n, int* lds_mode, int* plane_stride, size_t* dyn) {
  int pb = 0, rest = 0;
  for (int i = 0; i < n; ++i) {
    pb = imax_(pb, (plane_bytes(s[i].Hc, s[i].Wc) + 15) & ~15);
    rest = imax_(rest, fixed_bytes() + tile_bytes(s[i].ht * s[i].wt));
  }
  const int limit = morph_lds_budget();
  if (pb + rest <= limit) {
    *lds_mode = 1; *plane_stride = pb; *dyn = (size_t)(pb + rest);
  } else if (rest <= limit) {
    *lds_mode = 0; *plane_stride = pb; *dyn = (size_t)rest;
  } else {
    return (int)hipErrorInvalidValue;
  }
  return 0;
}

size_t mcaq_morph_scratch_bytes(int B, int Hc, int Wc, int ht, int wt) {
  MorphScale s{};
  s.Hc = Hc; s.Wc = Wc; s.ht = ht; s.wt = wt; s.H = 2 * Hc; s.W = 2 * Wc;  // conservative: H < Hc + tile
  int mode, stride; size_t dyn;
  if (morph_plan(&s, 1, &mode, &stride, &dyn)) return 0;
  return mode ? 0 : (size_t)B * stride;
}

int mcaq_morph(const mcaq_morph_scale* scales, int nscales, hipStream_t stream) {
  if (nscales < 1 || nscales > 3) return (int)hipErrorInvalidValue;
  MorphArgs a;
  int blocks = 0, any_phi = 0, any_tiles = 0, tlds = 0;
  for (int i = 0; i < nscales; ++i) {
    memcpy(&a.s[i], &scales[i], sizeof(MorphScale));
    MorphScale& S = a.s[i];
    if (S.B < 1 || S.ht < 1 || S.wt < 1) return (int)hipErrorInvalidValue;
    if (S.tile < 4 || (S.tile & (S.tile - 1)) || S.tile > 64) return (int)hipErrorInvalidValue;
    if (S.Hc != S.ht * S.tile || S.Wc != S.wt * S.tile || S.Hc > S.H || S.Wc > S.W) return (int)hipErrorInvalidValue;
    // phi_out carries phi from pass A to pass B
    if ((S.flags & F_PHI) && !S.phi_out) return (int)hipErrorInvalidValue;
    if ((S.flags & F_CMLP) && (!S.phi_out || !S.cmlp)) return (int)hipErrorInvalidValue;
    if ((S.flags & F_SOFTMASK) && (!S.smask || !S.absmean)) return (int)hipErrorInvalidValue;
    S.block_begin = blocks;
    blocks += S.B;
    any_phi |= (S.flags & F_PHI) != 0;
    const int tf = S.flags & (F_CMLP | F_MAPPER | F_SOFTMASK);
    any_tiles |= tf != 0;
    if (tf) tlds = imax_(tlds, tiles_lds_bytes(S.H, S.W, S.ht * S.wt));
  }
  a.nscales = nscales;
  if (any_phi) {
    int mode, stride; size_t dyn;
    int e = morph_plan(a.s, nscales, &mode, &stride, &dyn);
    if (e) return e;
    if (!mode)
      for (int i = 0; i < nscales; ++i)
        if (!a.s[i].gscratch && (a.s[i].flags & F_PHI)) return (int)hipErrorInvalidValue;
    if (mode) {
      static int set_true = 0;  // raise the dynamic LDS limit once (not during graph capture)
      if ((int)dyn > set_true) {
        hipError_t ae = hipFuncSetAttribute((const void*)mcaq_morph_kernel<true>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, morph_lds_budget());
        if (ae != hipSuccess) return (int)ae;
        set_true = morph_lds_budget();
      }
      hipLaunchKernelGGL(mcaq_morph_kernel<true>, dim3(blocks), dim3(MORPH_THREADS), dyn, stream, a, stride);
    } else {
      static int set_false = 0;
      if ((int)dyn > set_false) {
        hipError_t ae = hipFuncSetAttribute((const void*)mcaq_morph_kernel<false>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, morph_lds_budget());
        if (ae != hipSuccess) return (int)ae;
        set_false = morph_lds_budget();
      }
      hipLaunchKernelGGL(mcaq_morph_kernel<false>, dim3(blocks), dim3(MORPH_THREADS), dyn, stream, a, stride);
    }
    hipError_t le = hipGetLastError();
    if (le != hipSuccess) return (int)le;
  }
  if (any_tiles) {
    if (tlds > MCAQ_MORPH_LDS_LIMIT - 1024) return (int)hipErrorInvalidValue;
    static int set_tiles = 0;
    if (tlds > set_tiles) {
      hipError_t ae = hipFuncSetAttribute((const void*)mcaq_tiles_kernel,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, MCAQ_MORPH_LDS_LIMIT - 1024);
      if (ae != hipSuccess) return (int)ae;
      set_tiles = MCAQ_MORPH_LDS_LIMIT - 1024;
    }
    hipLaunchKernelGGL(mcaq_tiles_kernel, dim3(blocks), dim3(TILES_THREADS), (size_t)tlds, stream, a);
  }
  return (int)hipGetLastError();
}

int mcaq_quant(const mcaq_quant_scale* scales, int nscales, hipStream_t stream) {
  if (nscales < 1 || nscales > 3) return (int)hipErrorInvalidValue;
  QuantArgs a;
  int units = 0;
  for (int i = 0; i < nscales; ++i) {
    a.s[i] = scales[i];
    a.s[i].unit_begin = units;
    const int HW = scales[i].H * scales[i].W;
    if (scales[i].nbits < 1 || scales[i].nbits > QMAXBITS || scales[i].bits_lo < 1 ||
        scales[i].bits_lo + scales[i].nbits - 1 > 16 || HW < 1 || scales[i].C < 1 ||
        scales[i].ht < 1 || scales[i].wt < 1 || !scales[i].x || !scales[i].y || !scales[i].bits ||
        !scales[i].xmin || !scales[i].xmax)
      return (int)hipErrorInvalidValue;
    units += scales[i].B * ((HW + 255) / 256) * ((scales[i].C + QSLICE - 1) / QSLICE);
  }
  a.nscales = nscales;
  a.units_total = units;
  hipLaunchKernelGGL(mcaq_quant_kernel, dim3(units), dim3(64), 0, stream, a);
  return (int)hipGetLastError();
}

}  // extern "C"
