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
//   QAT     mcaq_qat_kernel       fractional-bit forward / STE backward
//                                 (mcaq_qat.h)
//
// Built with -ffp-contract=off (see mcaq_math.h).
#include <hip/hip_ext.h>
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
extern "C" int mcaq_reset_stamps(void) {
  static const unsigned long long z[64] = {};
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(mcaq::g_mcaq_stamps), z, sizeof(z));
}
#endif

// ---------------------------------------------------------------------------
// pass 1
// ---------------------------------------------------------------------------
constexpr int MAXSEG = MCAQ_MAX_SEGMENTS;   // segments (hook scale x batch) per launch

struct StatsArgs {
  mcaq_stats_scale s[MAXSEG];
  int ppl[MAXSEG];     // pixels per lane of each segment (1, 2 or 4)
  int nscales;
  int units_total;
};

constexpr int ST_CG = 16;     // channels per block (= one ATen cascade block)
constexpr int ST_WAVES = 4;   // waves per workgroup; wave w owns blocks w, w+4, ...
constexpr int ST_LDS = 4096;  // floats of LDS (block sums; tail block sums)

// Pixels per lane: enough pixels per unit for 16-byte rows when one round of
// blocks covers the channels, fewer (more units in flight) when the channel
// loop needs several rounds.  Requires H*W % ppl == 0.
#ifndef MCAQ_STATS_MAXPPL
#define MCAQ_STATS_MAXPPL 4
#endif
#ifndef MCAQ_STATS_MINW
#define MCAQ_STATS_MINW 4
#endif
#ifndef MCAQ_STATS_PPL_R2   // pixels per lane when the channels take 2 rounds of blocks
#define MCAQ_STATS_PPL_R2 4
#endif
#ifndef MCAQ_STATS_PPL_R4   // ... 3 or more rounds
#define MCAQ_STATS_PPL_R4 1
#endif
#ifndef MCAQ_STATS_LANE_FLOATS   // x values a lane loads before reducing
#define MCAQ_STATS_LANE_FLOATS 64
#endif
static inline int stats_ppl(int C, int HW) {
  const int nblk = (C + ST_CG - 1) / ST_CG;
  const int rounds = (nblk + ST_WAVES - 1) / ST_WAVES;
  int ppl = rounds <= 1 ? 4 : (rounds == 2 ? MCAQ_STATS_PPL_R2 : MCAQ_STATS_PPL_R4);
  if (ppl > MCAQ_STATS_MAXPPL) ppl = MCAQ_STATS_MAXPPL;
  while (ppl > 1 && HW % ppl) ppl >>= 1;
  return ppl;
}

// Per-lane values of 16 channels -> per-channel reduction over the wave.
// Reduce-scatter inside each 16-lane row with DPP lane swaps (partners l^8,
// l^7, l^2, l^1: each flips the bit that picks the kept half and keeps the
// bits picked before, so lane l ends with one channel reduced over all 16
// lanes of its row), then two cross-row exchanges.  Min and max are exact in
// any order.
// NaN-propagating min / max (v_minimum3_f32 / v_maximum3_f32 on gfx950, as
// ATen's amin/amax propagate NaN): unlike fminf/fmaxf in IEEE mode they need
// no v_max_f32 canonicalisation of loaded or DPP-moved operands, which was a
// third of pass 1's min/max VALU work.  Exact in any order.
#ifndef MCAQ_STATS_PERMLANE
#define MCAQ_STATS_PERMLANE 0
#endif
#ifndef MCAQ_STATS_TAIL_PXMAJOR   // tail items pixel-major over the lanes (A/B)
#define MCAQ_STATS_TAIL_PXMAJOR 0
#endif

__device__ __forceinline__ float vmin_(float a, float b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ float vmax_(float a, float b) { return __builtin_elementwise_maximum(a, b); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int H, int CTRL>
__device__ __forceinline__ void rs_step(float (&mn)[16], float (&mx)[16], bool up) {
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const float smn = up ? mn[i] : mn[i + H], kmn = up ? mn[i + H] : mn[i];
    const float smx = up ? mx[i] : mx[i + H], kmx = up ? mx[i + H] : mx[i];
    mn[i] = vmin_(kmn, dpp_f<CTRL>(smn));
    mx[i] = vmax_(kmx, dpp_f<CTRL>(smx));
  }
}
// returns channel c(l) = 8*b3 + 4*b2 + 2*b1 + b0 of lane l (b = bits of l & 15)
__device__ __forceinline__ void wave_minmax16(float (&mn)[ST_CG], float (&mx)[ST_CG], int lane, float& omn, float& omx) {
  rs_step<8, 0x128>(mn, mx, (lane & 8) != 0);   // row_ror:8      (l ^ 8)
  rs_step<4, 0x141>(mn, mx, (lane & 4) != 0);   // row_half_mirror (l ^ 7)
  rs_step<2, 0x4E>(mn, mx, (lane & 2) != 0);    // quad_perm 2301 (l ^ 2)
  rs_step<1, 0xB1>(mn, mx, (lane & 1) != 0);    // quad_perm 1032 (l ^ 1)
  float a = mn[0], b = mx[0];
#if MCAQ_STATS_PERMLANE
  // cross-row exchanges on the VALU (gfx950 v_permlane16_swap / 32_swap with
  // the value as both operands: each lane sees its own value and lane l ^ 16
  // (l ^ 32) among the two results) instead of two LDS bpermutes per step
  {
    const auto pa = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
    const auto pb = __builtin_amdgcn_permlane16_swap(__float_as_uint(b), __float_as_uint(b), false, false);
    a = vmin_(vmin_(a, __uint_as_float(pa[0])), __uint_as_float(pa[1]));
    b = vmax_(vmax_(b, __uint_as_float(pb[0])), __uint_as_float(pb[1]));
  }
  {
    const auto pa = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
    const auto pb = __builtin_amdgcn_permlane32_swap(__float_as_uint(b), __float_as_uint(b), false, false);
    a = vmin_(vmin_(a, __uint_as_float(pa[0])), __uint_as_float(pa[1]));
    b = vmax_(vmax_(b, __uint_as_float(pb[0])), __uint_as_float(pb[1]));
  }
#else
  a = vmin_(a, __shfl_xor(a, 16, 64)); b = vmax_(b, __shfl_xor(b, 16, 64));
  a = vmin_(a, __shfl_xor(a, 32, 64)); b = vmax_(b, __shfl_xor(b, 32, 64));
#endif
  omn = a; omx = b;
}

// ---- feature element types (MCAQ_DTYPE_*): fp32, or the fp16 / bf16 maps an
// autocast region hands the hooks.  Loads widen exactly to fp32 (all
// arithmetic stays fp32: the analyzer's gray / |x| sums are those of
// x.float(), morphology.py:834-837); stores round to nearest even.
typedef float mcaq_f4v __attribute__((ext_vector_type(4)));
typedef _Float16 mcaq_h4v __attribute__((ext_vector_type(4)));
typedef unsigned short mcaq_u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float bf16_f(unsigned short u) { return __uint_as_float((unsigned)u << 16); }
__device__ __forceinline__ unsigned short f_bf16(float f) {
  const unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40u);   // quiet NaN
  return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
// The nontemporal choice is a template argument: a runtime `nt ? ntload(p)
// : *p` lets LLVM merge the two loads of one address and drop the
// nontemporal bit (round 6: pass 1's x loads lost `nt` that way, -10 % on
// the config-2 step until caught by an ISA diff).
template <bool NT, typename V>
__device__ __forceinline__ V ld_v(const V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename V>
__device__ __forceinline__ void st_v(V* p, V v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <typename T> struct ElemIO;
template <> struct ElemIO<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  template <bool NT> static __device__ __forceinline__ mcaq_f4v ld4(const float* p) {
    return ld_v<NT>(reinterpret_cast<const mcaq_f4v*>(p));
  }
  static __device__ __forceinline__ float2 ld2(const float* p) { return *reinterpret_cast<const float2*>(p); }
  template <bool NT> static __device__ __forceinline__ void st4(float* p, mcaq_f4v v) {
    st_v<NT>(reinterpret_cast<mcaq_f4v*>(p), v);
  }
};
template <> struct ElemIO<_Float16> {
  static __device__ __forceinline__ float ld(const _Float16* p) { return (float)*p; }
  template <bool NT> static __device__ __forceinline__ mcaq_f4v ld4(const _Float16* p) {
    return __builtin_convertvector(ld_v<NT>(reinterpret_cast<const mcaq_h4v*>(p)), mcaq_f4v);
  }
  static __device__ __forceinline__ float2 ld2(const _Float16* p) { return make_float2((float)p[0], (float)p[1]); }
  template <bool NT> static __device__ __forceinline__ void st4(_Float16* p, mcaq_f4v v) {
    st_v<NT>(reinterpret_cast<mcaq_h4v*>(p), __builtin_convertvector(v, mcaq_h4v));
  }
};
struct Bf16 { unsigned short u; };
template <> struct ElemIO<Bf16> {
  static __device__ __forceinline__ float ld(const Bf16* p) { return bf16_f(p->u); }
  template <bool NT> static __device__ __forceinline__ mcaq_f4v ld4(const Bf16* p) {
    const mcaq_u4v u = ld_v<NT>(reinterpret_cast<const mcaq_u4v*>(p));
    return mcaq_f4v{bf16_f(u.x), bf16_f(u.y), bf16_f(u.z), bf16_f(u.w)};
  }
  static __device__ __forceinline__ float2 ld2(const Bf16* p) { return make_float2(bf16_f(p[0].u), bf16_f(p[1].u)); }
  template <bool NT> static __device__ __forceinline__ void st4(Bf16* p, mcaq_f4v v) {
    st_v<NT>(reinterpret_cast<mcaq_u4v*>(p), mcaq_u4v{f_bf16(v.x), f_bf16(v.y), f_bf16(v.z), f_bf16(v.w)});
  }
};

// Fold one 16-row block sum into cascade levels a1..a3 (Cascade::push at i % 16 == 0).
struct Fold {
  float a0, a1, a2, a3;
  int n;
  __device__ __forceinline__ void init() { a0 = a1 = a2 = a3 = 0.0f; n = 0; }
  __device__ __forceinline__ void full(float s) {
    ++n;
    a1 = a1 + s;
    if ((n & 15) == 0) {
      a2 = a2 + a1; a1 = 0.0f;
      if ((n & 255) == 0) { a3 = a3 + a2; a2 = 0.0f; }
    }
  }
  __device__ __forceinline__ float result() const { return ((a0 + a1) + a2) + a3; }
};

// Tail-column order (ATen row_sum: 4 interleaved cascades over channels
// c = 4r + k, leftovers into partial 0) of pixel p, for x and |x| at once;
// the per-pixel slow path (C > 1024).
template <typename T>
__device__ __noinline__ void tail_sums(const T* xb, int HW, int p, int C, float& og, float& oa) {
  Cascade cg[4], ca[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) { cg[k].init(); ca[k].init(); }
  const int n4 = (C / 4) * 4;
  for (int c0 = 0; c0 < n4; c0 += 16) {
    const int n = imin_(16, n4 - c0);
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = ElemIO<T>::ld(xb + (size_t)(c0 + (i < n ? i : 0)) * HW + p);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i < n) { cg[i & 3].push(v[i]); ca[i & 3].push(fabsf(v[i])); }
    }
  }
  float g0 = cg[0].result(), a0 = ca[0].result();
  for (int r = n4; r < C; ++r) {
    const float v = ElemIO<T>::ld(xb + (size_t)r * HW + p);
    g0 = g0 + v; a0 = a0 + fabsf(v);
  }
  og = ((g0 + cg[1].result()) + cg[2].result()) + cg[3].result();
  oa = ((a0 + ca[1].result()) + ca[2].result()) + ca[3].result();
}

// sequential channel sum of pixel p (the order of a cropped view's mean)
template <typename T>
__device__ __noinline__ float seq_sum(const T* xb, int HW, int p, int C) {
  float sq = 0.0f;
  for (int c0 = 0; c0 < C; c0 += 16) {
    const int n = imin_(16, C - c0);
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = ElemIO<T>::ld(xb + (size_t)(c0 + (i < n ? i : 0)) * HW + p);
#pragma unroll
    for (int i = 0; i < 16; ++i) if (i < n) sq = sq + v[i];
  }
  return sq;
}

// unit = one 256-thread workgroup = 64*PPL consecutive pixels of one image,
// all channels.  Lane l of every wave owns pixels PPL*l .. PPL*l+PPL-1 (one
// 4*PPL-byte load per channel row); the channels are cut into 16-row ATen
// cascade blocks, wave w takes blocks w, w+4, ... and produces each block's
// per-pixel sums (rows added sequentially from 0, the cascade's a0).  Per
// round the four waves' block sums meet in LDS and thread t folds them, in
// block order, into pixel t's cascade levels a1..a3: the exact CPU-ATen order
// of x.mean(dim=1).  Channel min/max partials of the unit go straight from
// registers.  The last (< 32) pixels of an image reduce in ATen's row_sum
// order instead: their 4 x ceil(C/64) independent 16-row block sums are spread
// over the workgroup (one load round trip), then folded per pixel.
template <int PPL, bool kVec, typename T>
__device__ __forceinline__ void stats_unit(const mcaq_stats_scale& S, int lu, float* lds, const int only_round = -1) {
  float (*bsg)[256] = reinterpret_cast<float (*)[256]>(lds);
  float (*bsa)[256] = reinterpret_cast<float (*)[256]>(lds + ST_WAVES * 256);
  constexpr int UPIX = 64 * PPL;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int HW = S.H * S.W;
  const int upi = (HW + UPIX - 1) / UPIX;
  const int b = lu / upi, chunk = lu - b * upi;
  const int C = S.C;
  const T* xb = reinterpret_cast<const T*>(S.x) + (size_t)b * C * HW;
  const bool cropped = (S.Hc != S.H) || (S.Wc != S.W);
#ifdef MCAQ_PROBE_STATS_NO_MINMAX   // timing probe only (no min/max partials)
  const bool want_g = S.gray != nullptr, want_a = S.absmean != nullptr, want_m = false;
#else
  const bool want_g = S.gray != nullptr, want_a = S.absmean != nullptr, want_m = S.pmin != nullptr;
#endif
  const int base = chunk * UPIX;
  const int q0 = base + lane * PPL;                    // first pixel of this lane
  bool pv[PPL];
#pragma unroll
  for (int k = 0; k < PPL; ++k) pv[k] = q0 + k < HW;
  const int nblk = (C + ST_CG - 1) / ST_CG;
  const int rounds = (nblk + ST_WAVES - 1) / ST_WAVES;

  // ---- tail columns (row_sum order), all in the image's last unit
  const int tstart = imax_(aten_tail_start(HW), base);
  const int tend = imin_(HW, base + UPIX);
  const int ntail = tend - tstart;
  const int nilp = C >> 2;                        // rows per interleaved cascade
  const int nbt = (nilp + 15) >> 4;               // 16-row blocks per cascade
#ifdef MCAQ_PROBE_STATS_NO_TAIL   // timing probe only (wrong tail sums): tools/probe/stats_probe.sh
  const bool need_tail = false;
#else
  const bool need_tail = ntail > 0 && (want_a || (want_g && !cropped));
#endif
  const bool coop = nbt <= 16;                    // 31 px x 4 x 16 x 2 floats fit the LDS
  const int titems = need_tail && coop ? ntail * 4 * nbt : 0;
#ifdef MCAQ_STATS_TAIL_EARLY
  // the tail's strided loads are issued before the channel rounds, so their
  // latency overlaps the rounds' instead of following them (C <= 512)
  constexpr int TE = 1;
  const bool early = PPL == 1 && titems > 0 && titems <= TE * 256;   // the many-channel scales
  float tv[TE][16];
  if (early) {
#pragma unroll
    for (int e2 = 0; e2 < TE; ++e2) {
      const int it = imin_(tid + e2 * 256, titems - 1);
      const int i = it / (4 * nbt), rem = it - i * (4 * nbt);
      const int k = rem / nbt, j = rem - k * nbt;
      const int p = tstart + i;
      const int r0 = 16 * j, n = imin_(16, nilp - r0);
#pragma unroll
      for (int e = 0; e < 16; ++e) tv[e2][e] = ElemIO<T>::ld(xb + (size_t)(4 * (r0 + (e < n ? e : 0)) + k) * HW + p);
    }
  }
#else
  constexpr bool early = false;
#endif

  Fold fg, fa;   // pixel `tid` (tid < UPIX)
  fg.init(); fa.init();
  // MR rounds of 16-row blocks are loaded before the first is reduced (MR * 16
  // * PPL = 64 floats per lane), so a unit with several channel rounds still
  // pays about one memory latency per MR rounds
  constexpr int MR = MCAQ_STATS_LANE_FLOATS / (ST_CG * PPL) > 0 ? MCAQ_STATS_LANE_FLOATS / (ST_CG * PPL) : 1;
#ifdef MCAQ_PROBE_STATS_SPLIT
  // timing probe only (wrong outputs): this workgroup loads one channel round
  // of the unit and stores its block sums, no fold, no tail
  if (only_round >= 0) {
    const int r = only_round;
    const int blk = imin_(r * ST_WAVES + wv, nblk - 1);
    const int c0 = blk * ST_CG, nc = imin_(ST_CG, C - c0);
    const int qa = pv[0] ? q0 : 0;
    float v[ST_CG][PPL];
#pragma unroll
    for (int i = 0; i < ST_CG; ++i) {
      const T* row = xb + (size_t)(c0 + (i < nc ? i : 0)) * HW;
      if (kVec && PPL == 4) {
        const mcaq_f4v t = ElemIO<T>::template ld4<true>(row + qa);
        v[i][0] = t.x; v[i][1 % PPL] = t.y; v[i][2 % PPL] = t.z; v[i][3 % PPL] = t.w;
      } else {
#pragma unroll
        for (int k = 0; k < PPL; ++k) v[i][k] = ElemIO<T>::ld(row + imin_(q0 + k, HW - 1));
      }
    }
    float gb[PPL], ab[PPL];
#pragma unroll
    for (int k = 0; k < PPL; ++k) { gb[k] = 0.0f; ab[k] = 0.0f; }
#pragma unroll
    for (int i = 0; i < ST_CG; ++i)
      if (i < nc) {
#pragma unroll
        for (int k = 0; k < PPL; ++k) { gb[k] = gb[k] + v[i][k]; ab[k] = ab[k] + fabsf(v[i][k]); }
      }
    if (want_m) {
      float mn[ST_CG], mx[ST_CG];
#pragma unroll
      for (int i = 0; i < ST_CG; ++i) {
        float lo = v[i][0], hi = v[i][0];
#pragma unroll
        for (int k = 1; k < PPL; ++k) { lo = vmin_(lo, v[i][k]); hi = vmax_(hi, v[i][k]); }
        mn[i] = lo; mx[i] = hi;
      }
      float omn, omx;
      wave_minmax16(mn, mx, lane, omn, omx);
      if (lane < 16 && lane < nc) { S.pmin[(size_t)lu * C + c0 + lane] = omn; S.pmax[(size_t)lu * C + c0 + lane] = omx; }
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k)
      if (pv[k] && want_g) S.gray[(size_t)b * HW + q0 + k] = gb[k] + ab[k];
    return;
  }
#endif
  for (int r0 = 0; r0 < rounds; r0 += MR) {
    float v[MR][ST_CG][PPL];
    const int qa = pv[0] ? q0 : 0;
#pragma unroll
    for (int rr = 0; rr < MR; ++rr) {
      if (r0 + rr >= rounds) break;                                 // uniform
      const int blk = imin_((r0 + rr) * ST_WAVES + wv, nblk - 1);   // clamped: branch-free loads
      const int c0 = blk * ST_CG;
      const int nc = imin_(ST_CG, C - c0);
#pragma unroll
      for (int i = 0; i < ST_CG; ++i) {
        const T* row = xb + (size_t)(c0 + (i < nc ? i : 0)) * HW;
        if (kVec && PPL == 4) {
          // streaming load: x is far larger than L2, and leaving L2 to the
          // morphology of the other in-flight batches gains ~3 % per step
          // (profiles/r01_stats_ntl_ab/)
#if defined(MCAQ_STATS_PLAIN_LOADS)
          const mcaq_f4v t = ElemIO<T>::template ld4<false>(row + qa);
#else
          const mcaq_f4v t = ElemIO<T>::template ld4<true>(row + qa);
#endif
          v[rr][i][0] = t.x; v[rr][i][1 % PPL] = t.y; v[rr][i][2 % PPL] = t.z; v[rr][i][3 % PPL] = t.w;
        } else if (kVec && PPL == 2) {
          const float2 t = ElemIO<T>::ld2(row + qa);
          v[rr][i][0] = t.x; v[rr][i][1 % PPL] = t.y;
        } else {
#pragma unroll
          for (int k = 0; k < PPL; ++k) v[rr][i][k] = ElemIO<T>::ld(row + imin_(q0 + k, HW - 1));
        }
      }
    }
#pragma unroll
    for (int rr = 0; rr < MR; ++rr) {
      const int r = r0 + rr;
      if (r >= rounds) break;
      const int blk = r * ST_WAVES + wv;
      if (blk < nblk) {
        const int c0 = blk * ST_CG;
        const int nc = imin_(ST_CG, C - c0);
        float gb[PPL], ab[PPL];
#pragma unroll
        for (int k = 0; k < PPL; ++k) { gb[k] = 0.0f; ab[k] = 0.0f; }
#pragma unroll
        for (int i = 0; i < ST_CG; ++i) {
          if (i < nc) {
#pragma unroll
            for (int k = 0; k < PPL; ++k) { gb[k] = gb[k] + v[rr][i][k]; ab[k] = ab[k] + fabsf(v[rr][i][k]); }
          }
        }
#pragma unroll
        for (int k = 0; k < PPL; ++k) { bsg[wv][lane * PPL + k] = gb[k]; bsa[wv][lane * PPL + k] = ab[k]; }
        if (want_m) {
          // no valid-pixel masking: PPL divides HW, so a lane's pixels are all
          // in the image or the lane loaded pixels 0.. of the same channel row
          // (qa = 0 / clamped index) - genuine values, which cannot move a min
          // or max over the batch (r02 probe: the masks were ~1/3 of pass 1's
          // min/max VALU work, tools/probe/stats_probe.sh)
          float mn[ST_CG], mx[ST_CG];
#pragma unroll
          for (int i = 0; i < ST_CG; ++i) {
            float lo = v[rr][i][0], hi = v[rr][i][0];
#pragma unroll
            for (int k = 1; k < PPL; ++k) {
              lo = vmin_(lo, v[rr][i][k]);
              hi = vmax_(hi, v[rr][i][k]);
            }
            mn[i] = lo; mx[i] = hi;
          }
          float omn, omx;
          wave_minmax16(mn, mx, lane, omn, omx);
          if (lane < 16 && lane < nc) {
            S.pmin[(size_t)lu * C + c0 + lane] = omn;
            S.pmax[(size_t)lu * C + c0 + lane] = omx;
          }
        }
      }
      __syncthreads();
      if (tid < UPIX) {
        const int nslot = imin_(ST_WAVES, nblk - r * ST_WAVES);
        for (int s = 0; s < nslot; ++s) {
          const int blk2 = r * ST_WAVES + s;
          if (C - blk2 * ST_CG >= ST_CG) { fg.full(bsg[s][tid]); fa.full(bsa[s][tid]); }
          else { fg.a0 = bsg[s][tid]; fa.a0 = bsa[s][tid]; }   // trailing partial block stays in a0
        }
      }
      __syncthreads();
    }
  }

  float tg = 0.0f, ta = 0.0f;
  if (need_tail && coop) {
    float* tsg = lds;                             // [px][k][j]
    float* tsa = lds + ST_LDS / 2;
    const int items = titems;
#ifdef MCAQ_STATS_TAIL_EARLY
    if (early) {
#pragma unroll
      for (int e2 = 0; e2 < TE; ++e2) {
        const int it = tid + e2 * 256;
        if (it < items) {
          const int r0 = 16 * ((it % (4 * nbt)) % nbt), n = imin_(16, nilp - r0);
          float sg = 0.0f, sa = 0.0f;
#pragma unroll
          for (int e = 0; e < 16; ++e) if (e < n) { sg = sg + tv[e2][e]; sa = sa + fabsf(tv[e2][e]); }
          tsg[it] = sg; tsa[it] = sa;
        }
      }
    }
#endif
    for (int it = early ? items : tid; it < items; it += 256) {
#if MCAQ_STATS_TAIL_PXMAJOR
      // consecutive lanes on consecutive tail pixels of one (cascade, block):
      // each load instruction touches a few rows, not one row per lane
      const int i = it % ntail, rem = it / ntail;
      const int k = rem / nbt, j = rem - k * nbt;
      const int slot = (i * 4 + k) * nbt + j;
#else
      const int i = it / (4 * nbt), rem = it - i * (4 * nbt);
      const int k = rem / nbt, j = rem - k * nbt;
      const int slot = it;
#endif
      const int p = tstart + i;
      const int r0 = 16 * j, n = imin_(16, nilp - r0);
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = ElemIO<T>::ld(xb + (size_t)(4 * (r0 + (e < n ? e : 0)) + k) * HW + p);
      float sg = 0.0f, sa = 0.0f;
#pragma unroll
      for (int e = 0; e < 16; ++e) if (e < n) { sg = sg + v[e]; sa = sa + fabsf(v[e]); }
      tsg[slot] = sg; tsa[slot] = sa;
    }
    __syncthreads();
    const int i = tid - (tstart - base);
    if (i >= 0 && i < ntail) {
      const int p = tstart + i;
      float rg[4], ra[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        Fold cg, ca;
        cg.init(); ca.init();
        for (int j = 0; j < nbt; ++j) {
          const float sg = tsg[(i * 4 + k) * nbt + j], sa = tsa[(i * 4 + k) * nbt + j];
          if (nilp - 16 * j >= 16) { cg.full(sg); ca.full(sa); } else { cg.a0 = sg; ca.a0 = sa; }
        }
        rg[k] = cg.result(); ra[k] = ca.result();
      }
      for (int rr = 4 * nilp; rr < C; ++rr) {      // leftover rows into partial 0
        const float v = ElemIO<T>::ld(xb + (size_t)rr * HW + p);
        rg[0] = rg[0] + v; ra[0] = ra[0] + fabsf(v);
      }
      tg = ((rg[0] + rg[1]) + rg[2]) + rg[3];
      ta = ((ra[0] + ra[1]) + ra[2]) + ra[3];
    }
  }

  if (tid >= UPIX) return;
  const int p = base + tid;
  if (p >= HW) return;
  const float fC = (float)C;
  float sg = fg.result(), sa = fa.result();
  if (need_tail && p >= tstart) {
    if (coop) { sg = tg; sa = ta; }
    else tail_sums(xb, HW, p, C, sg, sa);
  }
  if (want_a) S.absmean[(size_t)b * HW + p] = sa / fC;
  if (want_g) {
    const int h = p / S.W, w = p - h * S.W;
    if (cropped) {
      // a cropped (non-contiguous) view reduces sequentially (L2-hot re-read)
      if (h < S.Hc && w < S.Wc) {
        const float sq = seq_sum(xb, HW, p, C);
        S.gray[((size_t)b * S.Hc + h) * S.Wc + w] = sq / fC;
      }
    } else {
      S.gray[(size_t)b * HW + p] = sg / fC;
    }
  }
}

// XCD-aware unit order: workgroups are placed on the 8 XCDs round-robin by
// blockIdx, so consecutive units of one image land on different XCDs, and a
// 128-byte line that two of them share (a channel row not 128-byte aligned,
// as C5's 1,600-byte rows on every other channel) is fetched once per XCD.
// Permuted so that every unit of image b runs on XCD b % 8, the shared line
// is fetched once and the neighbour reads it from that XCD's L2 (needs the
// scale's block range to start at a multiple of 8 and B % 8 == 0; else the
// plain order).  0: plain order (A/B).
#ifndef MCAQ_STATS_XCD
#define MCAQ_STATS_XCD 1
#endif
// > 0: pass 1 and pass 2 (tile kernel) launch at most MCAQ_STREAM_CAP
// workgroups per CU (x 256 CUs, a multiple of 8: the XCD order holds) that
// loop over their units, so the streaming passes never hold more than that
// share of a CU and the latency-bound morphology of other batches in flight
// finds room beside them.  0: one workgroup per unit (A/B).
#ifndef MCAQ_STREAM_CAP
#define MCAQ_STREAM_CAP 0
#endif

template <bool kVec, typename T = float>   // kVec: 8/16-byte row accesses for ppl 2/4 (host checks alignment)
__device__ __forceinline__ void stats_dispatch(const StatsArgs& a, float* lds, const int bid) {
  // heaviest (most channels per pixel) scales are the last ones: start them first
  const int unit = a.units_total - 1 - bid;
  int si = 0;
  while (si + 1 < a.nscales && unit >= a.s[si + 1].unit_begin) ++si;
  int lu = unit - a.s[si].unit_begin;
  const mcaq_stats_scale S = a.s[si];   // wave-uniform index: scalar loads from the kernarg segment
  const int ppl = a.ppl[si];
#if MCAQ_STATS_XCD && !defined(MCAQ_PROBE_STATS_SPLIT)
  {
    const int n = (si + 1 < a.nscales ? a.s[si + 1].unit_begin : a.units_total) - a.s[si].unit_begin;
    const int x0 = a.units_total - a.s[si].unit_begin - n;     // first blockIdx of this scale
    const int upi = (S.H * S.W + 64 * ppl - 1) / (64 * ppl);   // units per image
    if ((x0 & 7) == 0 && (S.B & 7) == 0) {
      const int j = bid - x0, slot = j >> 3, q = slot / upi;
      lu = ((j & 7) + 8 * q) * upi + (slot - q * upi);
    }
  }
#endif
#ifdef MCAQ_PROBE_STATS_SPLIT
  int rnd = -1;
  {
    const int nb = (S.C + ST_CG - 1) / ST_CG, R = (nb + ST_WAVES - 1) / ST_WAVES;
    if (R >= 2) { rnd = lu % R; lu /= R; }
  }
#else
  const int rnd = -1;
#endif
  if constexpr (MCAQ_STATS_MAXPPL >= 4) {
    if (ppl == 4) { stats_unit<4, kVec, T>(S, lu, lds, rnd); return; }
  }
  if constexpr (MCAQ_STATS_MAXPPL >= 2) {
    if (ppl == 2) { stats_unit<2, kVec, T>(S, lu, lds, rnd); return; }
  }
  stats_unit<1, kVec, T>(S, lu, lds, rnd);
}

template <bool kVec, typename T = float>
__global__ __launch_bounds__(256, MCAQ_STATS_MINW) void mcaq_stats_kernel(StatsArgs a) {
  __shared__ float lds[ST_LDS];
#if MCAQ_STREAM_CAP > 0
  for (int u = (int)blockIdx.x; u < a.units_total; u += (int)gridDim.x) {
    stats_dispatch<kVec, T>(a, lds, u);
    __syncthreads();    // the LDS of this unit is free for the next
  }
#else
  stats_dispatch<kVec, T>(a, lds, (int)blockIdx.x);
#endif
}

// ---------------------------------------------------------------------------
// finalize: channel min/max over the partials of pass 1
// ---------------------------------------------------------------------------
struct FinalizeArgs {
  mcaq_finalize_scale s[MAXSEG];
  int nscales;
  int nblocks;
};

// one workgroup = 64 channels x (blockDim / 64) unit-parts; `red` holds
// 2 * blockDim floats of LDS.  Runs as its own kernel or as extra workgroups
// of the morph launch (which leaves most CUs idle: the reduction is free there).
__device__ __forceinline__ void finalize_body(const FinalizeArgs& a, int blk, float* red) {
  int si = 0;
  while (si + 1 < a.nscales && blk >= a.s[si + 1].block_begin) ++si;
  const mcaq_finalize_scale& S = a.s[si];
  const int nthr = (int)blockDim.x, parts = nthr >> 6;
  if (S.per_tensor) {   // one workgroup: every (unit, channel) partial, then broadcast
    float mn = __builtin_huge_valf(), mx = -__builtin_huge_valf();
    const int tid = (int)threadIdx.x;
    if (S.pmin) {
      const size_t n = (size_t)S.nunits * S.C;
      for (size_t i = tid; i < n; i += nthr) { mn = vmin_(mn, S.pmin[i]); mx = vmax_(mx, S.pmax[i]); }
    } else {
      for (int c = tid; c < (S.min_stride ? S.C : 1); c += nthr) {
        mn = vmin_(mn, S.min_in[(size_t)S.min_stride * c]);
        mx = vmax_(mx, S.max_in[(size_t)S.min_stride * c]);
      }
    }
    red[tid] = mn;
    red[nthr + tid] = mx;
    __syncthreads();
    for (int h = nthr >> 1; h > 0; h >>= 1) {
      if (tid < h) { red[tid] = vmin_(red[tid], red[tid + h]); red[nthr + tid] = vmax_(red[nthr + tid], red[nthr + tid + h]); }
      __syncthreads();
    }
    mn = red[0];
    mx = red[nthr];
    if (S.neg_min) mn = -mn;
    for (int c = tid; c < S.C; c += nthr) { S.min_out[c] = mn; S.max_out[c] = mx; }
    return;
  }
  const int cl = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int c = (blk - S.block_begin) * 64 + cl;
  const bool cv = c < S.C;
  float mn = __builtin_huge_valf(), mx = -__builtin_huge_valf();
  if (cv) {
    if (S.pmin) {
      const float* pn = S.pmin + c;
      const float* px = S.pmax + c;
      const size_t st = (size_t)S.C * parts;
      int u = part;
      for (; u + 3 * parts < S.nunits; u += 4 * parts) {
        const size_t o = (size_t)u * S.C;
        const float m0 = pn[o], m1 = pn[o + st], m2 = pn[o + 2 * st], m3 = pn[o + 3 * st];
        const float x0 = px[o], x1 = px[o + st], x2 = px[o + 2 * st], x3 = px[o + 3 * st];
        mn = vmin_(mn, vmin_(vmin_(m0, m1), vmin_(m2, m3)));
        mx = vmax_(mx, vmax_(vmax_(x0, x1), vmax_(x2, x3)));
      }
      for (; u < S.nunits; u += parts) {
        mn = vmin_(mn, pn[(size_t)u * S.C]);
        mx = vmax_(mx, px[(size_t)u * S.C]);
      }
    } else if (part == 0) {
      mn = S.min_in[(size_t)S.min_stride * c];
      mx = S.max_in[(size_t)S.min_stride * c];
    }
  }
  red[part * 64 + cl] = mn;
  red[nthr + part * 64 + cl] = mx;
  __syncthreads();
  if (part == 0 && cv) {
    for (int k = 1; k < parts; ++k) { mn = vmin_(mn, red[k * 64 + cl]); mx = vmax_(mx, red[nthr + k * 64 + cl]); }
    S.min_out[c] = S.neg_min ? -mn : mn;
    S.max_out[c] = mx;
  }
}

// kernel arguments live in the dispatch's kernarg segment (4 KiB)
static_assert(sizeof(MorphArgs) + sizeof(FinalizeArgs) <= 4096, "morph kernel arguments exceed 4 KiB");

__global__ __launch_bounds__(256) void mcaq_finalize_kernel(FinalizeArgs a) {
  __shared__ float red[2 * 256];
  finalize_body(a, (int)blockIdx.x, red);
}

// ---------------------------------------------------------------------------
// morph pass A: one 1024-thread workgroup per (scale, image), planes in LDS
// morph pass B: one 256-thread workgroup per (scale, image), tile grid in LDS
// ---------------------------------------------------------------------------
constexpr int TILES_THREADS = MCAQ_TILES_THREADS;
constexpr int TILES_SCRATCH_BYTES = 4 * (TILES_THREADS / 64) * MLP_SCRATCH_FLOATS;   // 34816 at 256 or 512
#ifndef MCAQ_MORPH_THREADS
#define MCAQ_MORPH_THREADS 1024
#endif
#ifndef MCAQ_MORPH_MINW     // min waves per SIMD of pass A: 4 -> <= 128 VGPRs
#define MCAQ_MORPH_MINW 4
#endif
#ifndef MCAQ_MORPH_PRIO     // wave priority of passes A and B (0..3) against the streaming passes
#define MCAQ_MORPH_PRIO 2
#endif
#ifndef MCAQ_TILES_MINW     // min waves per SIMD of pass B (register budget 512 / MINW)
#define MCAQ_TILES_MINW 1
#endif
constexpr int MORPH_THREADS = MCAQ_MORPH_THREADS;

__device__ __forceinline__ int morph_scale_of(const MorphArgs& a, int img) {
  int si = 0;
  while (si + 1 < a.nscales && img >= a.s[si + 1].block_begin) ++si;
  return si;
}

// Pass A packs several small images into one 1024-thread workgroup: image
// group g owns threads [g*G, (g+1)*G), G = 1024 / ipw, and its own LDS planes.
// The per-image chain is latency bound, so a 20x20 image needs no more than
// 128 threads to finish as fast as alone -- packing 8 of them frees 7 CUs.
// Every group runs the same barrier sequence (stage loops depend on the
// scale's geometry only); a group past the batch end recomputes the last
// image (identical values written twice) instead of idling at the barriers.
template <bool kLDS, bool kLegacy = false>
__global__ __launch_bounds__(MORPH_THREADS, MCAQ_MORPH_MINW) void mcaq_morph_kernel(MorphArgs a, FinalizeArgs f) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nwg = a.wg_begin[a.nscales];
  if ((int)blockIdx.x >= nwg) {   // channel min/max workgroups ride along
    finalize_body(f, (int)blockIdx.x - nwg, reinterpret_cast<float*>(smem));
    return;
  }
  // latency-bound per-image chain: win VALU / LDS issue arbitration against
  // co-resident streaming waves of other batches in flight
  __builtin_amdgcn_s_setprio(MCAQ_MORPH_PRIO);
  int si = 0;
  while (si + 1 < a.nscales && (int)blockIdx.x >= a.wg_begin[si + 1]) ++si;
  const MorphScale& S = a.s[si];
  // two workgroups per image group: role 0 = edge plane, role 1 = mask planes
  const int wg = (int)blockIdx.x - a.wg_begin[si];
  const int grp = wg >> 1, role = wg & 1;
  const int ipw = a.ipw[si], G = MORPH_THREADS / ipw;
  const int g = (int)threadIdx.x / G;
  const int b = imin_(grp * ipw + g, S.B - 1);
  Ctx ctx{(int)threadIdx.x - g * G, G};
  Shared sh;
  Planes pl;
  char* base = smem + (size_t)g * a.gstride[si];
  if (kLDS) {
    carve_planes(base, S.Hc, S.Wc, pl);
    carve_shared(base + a.pstride[si], sh);
  } else {
    carve_planes((char*)S.gscratch + (size_t)(2 * b + role) * a.pstride[si], S.Hc, S.Wc, pl);
    carve_shared(base, sh);
  }
  morph_edges<kLegacy>(ctx, S, b, role, pl, sh);
}

// pass A in band mode (mcaq_band.h): one 256-thread workgroup per (scale,
// image, 16-row band) with its halo rows in ~40 KB of LDS, then one per
// (scale, image) for the Otsu threshold, hysteresis and box counts.  The
// channel min/max workgroups ride along with the band launch.
#ifndef MCAQ_BAND_MINW      // min waves per SIMD of the band kernel (register budget 512 / MINW)
#define MCAQ_BAND_MINW 4
#endif
#ifndef MCAQ_EDGE_MINW
#define MCAQ_EDGE_MINW 4
#endif
#ifndef MCAQ_BAND_PRIO      // wave priority of the band / edge kernels
#define MCAQ_BAND_PRIO MCAQ_MORPH_PRIO
#endif
__global__ __launch_bounds__(256, MCAQ_BAND_MINW) void mcaq_band_kernel(MorphArgs a, FinalizeArgs f) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nwg = a.bwg_begin[a.nscales];
  if ((int)blockIdx.x >= nwg) {
    finalize_body(f, (int)blockIdx.x - nwg, reinterpret_cast<float*>(smem));
    return;
  }
  __builtin_amdgcn_s_setprio(MCAQ_BAND_PRIO);
  int si = 0;
  while (si + 1 < a.nscales && (int)blockIdx.x >= a.bwg_begin[si + 1]) ++si;
  const MorphScale& S = a.s[si];
  const int wg = (int)blockIdx.x - a.bwg_begin[si];
  const int nb = band_count(S.Hc, S.tile);
  const int b = wg / nb;
  Ctx ctx{(int)threadIdx.x, 256};
#ifdef MCAQ_TWICE   // diagnostic: a second, identical run finds the code in the instruction cache
  band_pass(ctx, S, b, wg - b * nb, smem);
  __syncthreads();
#endif
  band_pass(ctx, S, b, wg - b * nb, smem);
}

__global__ __launch_bounds__(256, MCAQ_EDGE_MINW) void mcaq_edge_kernel(MorphArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __builtin_amdgcn_s_setprio(MCAQ_BAND_PRIO);
  int si = 0;
  while (si + 1 < a.nscales && (int)blockIdx.x >= a.ewg_begin[si + 1]) ++si;
  const MorphScale& S = a.s[si];
  Ctx ctx{(int)threadIdx.x, 256};
#ifdef MCAQ_TWICE
  edge_image(ctx, S, (int)blockIdx.x - a.ewg_begin[si], smem);
  __syncthreads();
#endif
  edge_image(ctx, S, (int)blockIdx.x - a.ewg_begin[si], smem);
}

// pass B, batch-wide (mcaq_tiles_batch.h): one 64-thread workgroup (one wave,
// lane = tile) per 64 consecutive tiles of a scale's batch, ~14 KB of LDS
__device__ __forceinline__ int tb_scale_of(const MorphArgs& a) {
  int si = 0;
  while (si + 1 < a.nscales && (int)blockIdx.x >= a.tb_begin[si + 1]) ++si;
  return si;
}

__global__ __launch_bounds__(64) void mcaq_tb_head_kernel(MorphArgs a) {
  __shared__ float tiles[TB_TILES * TB_TS];
  __shared__ float xs[MLP_SCRATCH_FLOATS];
  __builtin_amdgcn_s_setprio(MCAQ_MORPH_PRIO);
  const int si = tb_scale_of(a);
  const MorphScale& S = a.s[si];
  const int NT = S.ht * S.wt;
  const int u0 = ((int)blockIdx.x - a.tb_begin[si]) * TB_TILES;
  const int n = imin_(TB_TILES, S.B * NT - u0);
  const int lane = (int)threadIdx.x, u = u0 + imin_(lane, n - 1);
  const int b = div_small(u, NT, 1.0f / (float)NT), t = u - b * NT;
  float* tt = S.tile_tmp + (size_t)u * TT_STRIDE;
  {
    float tv[28];   // the pass-A partials [0, 20 + S) of this tile (S <= 7)
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const float4 q = reinterpret_cast<const float4*>(tt)[i];
      tv[4 * i] = q.x; tv[4 * i + 1] = q.y; tv[4 * i + 2] = q.z; tv[4 * i + 3] = q.w;
    }
    float p[8];
    phi_of_tile(S, b, t, tv, p);
    if (lane < n) {
#pragma unroll
      for (int k = 0; k < 8; ++k) tiles[lane * TB_TS + T_PHI + k] = p[k];
      if (S.phi_out) {
        float4* o = reinterpret_cast<float4*>(S.phi_out + (size_t)u * 8);
        o[0] = make_float4(p[0], p[1], p[2], p[3]);
        o[1] = make_float4(p[4], p[5], p[6], p[7]);
      }
    }
  }
  __syncthreads();
#if defined(__HIP_DEVICE_COMPILE__)
  cmlp_block_mfma<2, const float*, TB_TS>(S.cmlp, tiles, n, 0, lane, (lds_f)xs);
  if (n > 32) cmlp_block_mfma<2, const float*, TB_TS>(S.cmlp, tiles, n, 32, lane, (lds_f)xs);
#else
  (void)xs;
#endif
  __syncthreads();
  if (lane < n) {
    const float c = tiles[lane * TB_TS + T_CMLP];
    tt[TT_CRAW] = c;
    if (S.cmlp_out) S.cmlp_out[u] = c;
  }
}

__global__ __launch_bounds__(64) void mcaq_tb_map_kernel(MorphArgs a) {
  __shared__ float tiles[TB_TILES * TB_TS];
  __shared__ float xs[MLP_SCRATCH_FLOATS];
  __shared__ float ab[256];
  __builtin_amdgcn_s_setprio(MCAQ_MORPH_PRIO);
  const int si = tb_scale_of(a);
  const MorphScale& S = a.s[si];
  const int NT = S.ht * S.wt;
  const int u0 = ((int)blockIdx.x - a.tb_begin[si]) * TB_TILES;
  const int n = imin_(TB_TILES, S.B * NT - u0);
  const int lane = (int)threadIdx.x, u = u0 + imin_(lane, n - 1);
  const int b = div_small(u, NT, 1.0f / (float)NT), t = u - b * NT;
  const int th = div_small(t, S.wt, 1.0f / (float)S.wt), tw = t - th * S.wt;
  float* tt = S.tile_tmp + (size_t)u * TT_STRIDE;
  for (int j = lane; j < 128; j += 64) fold_mapper_bn(S.mapper, ab, j);
  const float* crow = S.tile_tmp + (size_t)b * NT * TT_STRIDE + TT_CRAW;
  const float c = bilateral_tile(t, th, tw, S.ht, S.wt, NT, [&](int k) { return crow[(size_t)k * TT_STRIDE]; });
  float act = 0.0f;
  if (S.flags & F_SOFTMASK) act = act_tile(S.absmean + (size_t)b * S.H * S.W, S.H, S.W, S.ht, S.wt, th, tw);
  if (lane < n) {
    tiles[lane * TB_TS + T_C] = c;
    if (S.c_out) S.c_out[u] = c;
    if (S.flags & F_SOFTMASK) tt[TT_ACT] = act;
  }
  __syncthreads();
#if defined(__HIP_DEVICE_COMPILE__)
  mapper_block_mfma<2, const float*, TB_TS>(S.mapper, (const float*)ab, tiles, n, 0, lane, T_C, S.min_bits, S.max_bits,
                                           (lds_f)xs);
  if (n > 32)
    mapper_block_mfma<2, const float*, TB_TS>(S.mapper, (const float*)ab, tiles, n, 32, lane, T_C, S.min_bits,
                                             S.max_bits, (lds_f)xs);
#else
  (void)xs;
#endif
  __syncthreads();
  if (lane < n) {
    const float bv = finish_bits(tiles[lane * TB_TS + T_AUX], S);
    tt[TT_BITS] = bv;
    if (S.bits_out) S.bits_out[u] = bv;
  }
}

__global__ __launch_bounds__(64) void mcaq_tb_mask_kernel(MorphArgs a) {
  __builtin_amdgcn_s_setprio(MCAQ_MORPH_PRIO);
  const int si = tb_scale_of(a);
  const MorphScale& S = a.s[si];
  if (!(S.flags & F_SOFTMASK)) return;
  const int NT = S.ht * S.wt;
  const float rnt = 1.0f / (float)NT;
  const int u0 = ((int)blockIdx.x - a.tb_begin[si]) * TB_TILES;
  const int n = imin_(TB_TILES, S.B * NT - u0);
  const int lane = (int)threadIdx.x, u = u0 + imin_(lane, n - 1);
  const int b = div_small(u, NT, rnt), t = u - b * NT;
  const int th = div_small(t, S.wt, 1.0f / (float)S.wt), tw = t - th * S.wt;
  // max of the tile activations of every image this block touches (NaN-propagating, as torch.amax)
  float amax = 0.0f;
  const int bf = div_small(u0, NT, rnt), bl = div_small(u0 + n - 1, NT, rnt);
  for (int bb = bf; bb <= bl; ++bb) {
    float lm = -3.402823466e38f;
    for (int j = lane; j < NT; j += 64) lm = fmaxp(lm, S.tile_tmp[((size_t)bb * NT + j) * TT_STRIDE + TT_ACT]);
    for (int o = 32; o > 0; o >>= 1) lm = fmaxp(lm, __shfl_xor(lm, o, 64));
    if (bb == b) amax = lm;
  }
  const float den = amax + 1e-8f;
  const float* row = S.tile_tmp + (size_t)b * NT * TT_STRIDE;
  const bool vl = aten_softmax_vec_lane((long long)img_global(S, b) * NT + t, (long long)img_batch_total(S) * NT, NT,
                                        S.softmax_threads);
  const float mtv = smask_tile(
      S.smask, th, tw, S.ht, S.wt,
      [&](int s) { return clampf_((row[(size_t)s * TT_STRIDE + TT_BITS] - 2.0f) / 6.0f, 0.0f, 1.0f); },
      [&](int s) { return row[(size_t)s * TT_STRIDE + TT_ACT] / den; }, vl);
  if (lane < n && S.mt_out) S.mt_out[u] = mtv;
}

// the m(p) plane of the batch-wide pass B (debug / m_plane): one thread per pixel
__global__ __launch_bounds__(256) void mcaq_tb_mplane_kernel(MorphArgs a, int total) {
  const int g = (int)(blockIdx.x * 256 + threadIdx.x);
  if (g >= total) return;
  int si = 0, o = g;
  while (si + 1 < a.nscales && o >= a.s[si].B * a.s[si].H * a.s[si].W) { o -= a.s[si].B * a.s[si].H * a.s[si].W; ++si; }
  const MorphScale& S = a.s[si];
  if (!S.m_out || !(S.flags & F_SOFTMASK)) return;
  const int HW = S.H * S.W, b = o / HW, p = o - b * HW, h = p / S.W, w = p - h * S.W;
  S.m_out[o] = mplane_pixel(S.mt_out + (size_t)b * S.ht * S.wt, S.H, S.W, S.ht, S.wt, h, w);
}

// pass B: image group g of a workgroup owns threads [g*G, (g+1)*G) and its own
// LDS tile arrays; the staged weights are shared by the workgroup.  A group
// past the batch end recomputes the last image (identical values written twice).
// TS: floats per tile row of the LDS tile arrays (TILE_FLOATS_PAD when the
// launch's images fit that way, else TILE_FLOATS; mcaq_morph.h)
template <int TS, bool kSmo = false>
__device__ __forceinline__ void tiles_body(const MorphArgs& a, int wlds) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __builtin_amdgcn_s_setprio(MCAQ_MORPH_PRIO);
  int si = 0;
  while (si + 1 < a.nscales && (int)blockIdx.x >= a.twg_begin[si + 1]) ++si;
  const MorphScale& S = a.s[si];
  const int ipw = a.tipw[si], G = TILES_THREADS / ipw;
  const int g = (int)threadIdx.x / G;
  const int b = imin_(((int)blockIdx.x - a.twg_begin[si]) * ipw + g, S.B - 1);
  float* wl = wlds ? reinterpret_cast<float*>(smem) : nullptr;
  float* xs = reinterpret_cast<float*>(smem + (wlds ? weights_lds_bytes() : 0));   // MLP scratch, per wave
  char* base = smem + (wlds ? weights_lds_bytes() : 0) + TILES_SCRATCH_BYTES + (size_t)g * a.tgstride[si];
  Ctx ctx{(int)threadIdx.x - g * G, G};
  Shared sh;
  carve_shared(base, sh);
  morph_tiles<TS, kSmo>(ctx, S, b, sh, wl, (int)threadIdx.x, TILES_THREADS, xs);
}
template <int TS>
__global__ __launch_bounds__(TILES_THREADS, MCAQ_TILES_MINW) void mcaq_tiles_kernel(MorphArgs a, int wlds) {
  tiles_body<TS>(a, wlds);
}

// ---------------------------------------------------------------------------
// pass 2: y = dequant(quant_b(x)) * m
// ---------------------------------------------------------------------------
struct QuantArgs {
  mcaq_quant_scale s[MAXSEG];
  int nscales;
  int units_total;
  // tile-aligned path (mcaq_quant_tile_kernel): H = ht << sh, W = wt << sw;
  // reciprocals of the slice count, units per image and W for div_small
  int sh[MAXSEG], sw[MAXSEG];
  float rnsl[MAXSEG], rupi[MAXSEG], rw[MAXSEG];
};

#ifndef MCAQ_QSLICE
#define MCAQ_QSLICE 32
#endif
constexpr int QSLICE = MCAQ_QSLICE;   // channels per unit (8 per wave)
// mcaq_quant_tile_kernel stores one [bits][channel] table entry per thread
// (bit width tid / 32, channel tid % 32) for 8 widths x QSLICE channels
static_assert(QSLICE == 32, "the tile-aligned pass 2 assumes 32-channel slices");
constexpr int QCW = QSLICE / 4;       // channels per wave
constexpr int QMAXBITS = 15;   // max entries per channel in the LDS table
constexpr int QMAXNT = 1024;   // max tiles per image whose m values are staged in LDS (more: read from L2)

// unit = 256 pixels x 32 channels of one image; lane l of every wave owns
// pixels 4l..4l+3 (16-byte accesses), wave w channels 8w..8w+7 of the slice,
// all eight rows loaded before any is computed.  Per-pixel tile bits and the
// soft-mask value are fetched once; per-(channel, bits) scale / zero-point
// come from an LDS table built by the workgroup (IEEE divisions, as
// QuantizationParameters computes them).
// 6 resident workgroups per CU (79 VGPRs, no spills): the prologue's early
// loads raised the unbounded kernel to 91 VGPRs / 5 workgroups; r02 A/B
// 29.7 vs 30.4-30.6 us back to back (profiles/r02_probes/ab_round2_late.txt);
// 7 spills 16 VGPRs
#ifndef MCAQ_QUANT_MINW
#define MCAQ_QUANT_MINW 6
#endif
#define MCAQ_QUANT_LB __launch_bounds__(256, MCAQ_QUANT_MINW)
// m(p) source of a pass-2 instantiation (compile time, so that no load sits
// behind a runtime branch: the compiler's wait counts then stay exact and the
// x rows stay in flight through the prologue -- with the loads behind
// branches it waited for every x row before the first barrier, r03)
enum : int { QM_NONE = 0, QM_MT_LDS = 1, QM_MT_L2 = 2, QM_PLANE = 3 };

// pixel -> tile row / column: the reference's nearest source index
// floor(o * fp32(in / out)), clamped (exact for the o >> k and o >> 1 special
// cases of ATen's nearest_idx too: in / out is then a power of two), or the
// spatial_quantize contract o / tile, clamped; branch-free
__device__ __forceinline__ int q_tile_of(int o, int in, float sc, int compat_tile) {
  const int ns = imin_((int)floorf((float)o * sc), in - 1);
  const int ct = imin_(o / imax_(compat_tile, 1), in - 1);
  return compat_tile > 0 ? ct : ns;
}

template <bool kVec, bool kNTL, bool kNTS, int kM, bool kBig>
__global__ MCAQ_QUANT_LB void mcaq_quant_kernel(QuantArgs a) {
  __shared__ float4 qt[QSLICE * QMAXBITS];   // scale, zp, 1/scale
  __shared__ float mts[kM == QM_MT_LDS ? QMAXNT : 1];
  __shared__ float mq[256];
  __shared__ int qany[QSLICE];               // channel needs quant_dequant_any
  const int unit = blockIdx.x;
  int si = 0;
  while (si + 1 < a.nscales && unit >= a.s[si + 1].unit_begin) ++si;
  const mcaq_quant_scale& S = a.s[si];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
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
  const int NTq = S.ht * S.wt;
  const int ntab = nc * NB;
  // ---- 1. small operands, unconditional (clamped indices): this thread's
  // table entry's min / max, its m(tile) value, the lane's 4 tile bits (and
  // m(p) values when the plane is given)
  const int tc = imin_(tid / NB, nc - 1);
  const float tmn0 = S.xmin[c0 + tc], tmx = S.xmax[c0 + tc];
  const float tmn = S.neg_min ? -tmn0 : tmn0;
  float mtv = 0.0f;
  if (kM == QM_MT_LDS) mtv = S.mt[(size_t)b * NTq + imin_(tid, NTq - 1)];
  const int q0 = chunk * 256 + lane * 4;
  const float sch = (float)S.ht / (float)S.H, scw = (float)S.wt / (float)S.W;
  bool pv[4];
  float bv[4], mv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = imin_(q0 + k, HW - 1);
    pv[k] = q0 + k < HW;
    const int h = p / S.W, w = p - h * S.W;
    const int th = q_tile_of(h, S.ht, sch, S.compat_tile_h);
    const int tw = q_tile_of(w, S.wt, scw, S.compat_tile_w);
    bv[k] = S.bits[((size_t)b * S.ht + th) * S.wt + tw];
    mv[k] = kM == QM_PLANE ? S.m[(size_t)b * HW + p] : 1.0f;
  }
  // ---- 2. the x rows (8 x 16 B per lane), in flight through the prologue
  const int cw = wv * QCW;                 // first channel of this wave in the slice
  const int ncw = imin_(QCW, nc - cw);     // may be <= 0 for a short last slice
  const size_t rowbase = ((size_t)b * S.C + c0 + imax_(imin_(cw, nc - 1), 0)) * HW;
  const float* xb = S.x + rowbase;
  float* yb = S.y + rowbase;
  float v[QCW][4];
  const int qa = pv[0] ? q0 : 0;
#pragma unroll
  for (int c = 0; c < QCW; ++c) {
    const float* row = xb + (size_t)imin_(c, imax_(ncw - 1, 0)) * HW;
    if (kVec) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      const f4v t = kNTL ? __builtin_nontemporal_load(reinterpret_cast<const f4v*>(row + qa))
                        : *reinterpret_cast<const f4v*>(row + qa);
      v[c][0] = t.x; v[c][1] = t.y; v[c][2] = t.z; v[c][3] = t.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[c][k] = row[imin_(q0 + k, HW - 1)];
    }
  }
  // ---- 3. scale / zero-point table and staged m values (no global loads
  // behind a branch on the common path; > 256 entries only in kBig builds)
  {
    // every thread computes an entry (tid >= ntab: an unused slot of the
    // 480-entry table), so the min / max loads have an unconditional use and
    // are not sunk into a branch behind the x rows
    const int kq = imin_(tid - tc * NB, QMAXBITS - 1);
    const QParam q = qparam(tmn, tmx, S.bits_lo + kq);
    qt[tid] = make_float4(q.scale, q.zp, q.rs, 0.0f);
    if (kq == 0) qany[tc] = (!S.stats_cover_x || stats_need_any(tmn, tmx)) ? 1 : 0;
  }
  if (kBig) {
    for (int i = tid + 256; i < ntab; i += 256) {   // > 256 entries: continuous bit ranges
      const int c = i / NB, k = i - (i / NB) * NB;
      const float mn = S.neg_min ? -S.xmin[c0 + c] : S.xmin[c0 + c];
      const QParam q = qparam(mn, S.xmax[c0 + c], S.bits_lo + k);
      qt[i] = make_float4(q.scale, q.zp, q.rs, 0.0f);
      if (k == 0) qany[c] = (!S.stats_cover_x || stats_need_any(mn, S.xmax[c0 + c])) ? 1 : 0;
    }
  }
  if (kM == QM_MT_LDS) {
    if (tid < NTq) mts[tid] = mtv;
    if (kBig)
      for (int i = tid + 256; i < NTq; i += 256) mts[i] = S.mt[(size_t)b * NTq + i];
  }
  int kb[4];
  float qlo[4], qhi[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    kb[k] = imin_(imax_((int)rintf(bv[k]), S.bits_lo), S.bits_lo + NB - 1) - S.bits_lo;
    const int bb = S.bits_lo + kb[k];
    qlo[k] = (float)(-(1 << (bb - 1)));
    qhi[k] = (float)((1 << (bb - 1)) - 1);
  }
  __syncthreads();   // qt, mts ready
#ifndef MCAQ_PROBE_Q_NOM
  if (kM == QM_MT_LDS || kM == QM_MT_L2) {
#else
  if (false) {
#endif
    // m(p) = 5x5 Gaussian (replicate pad) of the nearest-upsampled tile values,
    // taps row-major from 0 - the m plane LearnedSoftMask produces
    // (quantization.py:235-238), generated here instead of read from HBM.
    // Wave w computes pixel w of every lane's quad; the quads meet in LDS.
    const float* mtab = kM == QM_MT_LDS ? mts : S.mt + (size_t)b * NTq;
    {
      const int p = imin_(q0 + wv, HW - 1);
      const int h = p / S.W, w = p - h * S.W;
      int cs[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) cs[j] = q_tile_of(imin_(imax_(w + j - 2, 0), S.W - 1), S.wt, scw, 0);
      float acc = 0.0f;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int rb = q_tile_of(imin_(imax_(h + i - 2, 0), S.H - 1), S.ht, sch, 0) * S.wt;
#pragma unroll
        for (int j = 0; j < 5; ++j) acc = fmaf(bits_as_float(k_smooth5_bits[i * 5 + j]), mtab[rb + cs[j]], acc);
      }
      mq[lane * 4 + wv] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) mv[k] = mq[lane * 4 + k];
  }
  if (ncw <= 0) return;
  // one wave-uniform choice for the wave's channels: the short arithmetic
  // unless a channel's statistics do not cover x or are not finite
  int anyc = 0;
#pragma unroll
  for (int c = 0; c < QCW; ++c) anyc |= c < ncw ? qany[cw + c] : 0;
  const bool any_x = __builtin_amdgcn_readfirstlane(anyc) != 0;
#pragma unroll
  for (int c = 0; c < QCW; ++c) {
    if (c >= ncw) break;
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 sz = qt[(cw + c) * NB + kb[k]];
      QParam q;
      q.scale = sz.x; q.zp = sz.y; q.rs = sz.z; q.qmin = qlo[k]; q.qmax = qhi[k];
#ifdef MCAQ_PROBE_Q_NOQ
      float d = v[c][k] * q.scale;
#else
      float d = any_x ? quant_dequant_any(v[c][k], q) : quant_dequant(v[c][k], q);
#endif
      if (kM != QM_NONE) d = d * mv[k];
      o[k] = d;
    }
    float* orow = yb + (size_t)c * HW;
    if (kVec) {
      if (pv[0]) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v ov = {o[0], o[1], o[2], o[3]};
        // y is written once and not re-read by this step: streaming store
        if (kNTS) __builtin_nontemporal_store(ov, reinterpret_cast<f4v*>(orow + q0));
        else *reinterpret_cast<f4v*>(orow + q0) = ov;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) if (pv[k]) orow[q0 + k] = o[k];
    }
  }
}

// Pass 2, tile-aligned path.  When every scale's map is a power-of-two
// multiple of its tile grid (H = ht << sh, W = wt << sw, sw >= 2 - every hook
// scale), a lane's 4 consecutive pixels lie in ONE tile: one bit width, so one
// (scale, zp, 1/scale) table entry per channel serves all 4, read from a
// [bits][channel] LDS table at an immediate offset, and the quantizer runs on
// pixel pairs with packed fp32 instructions (v_pk_mul / v_pk_fma / v_pk_add,
// each an IEEE fp32 operation per component: the values are those of
// quant_dequant).  Pixel -> tile and m(p)'s source rows / columns are shifts;
// no integer division anywhere (the general kernel spent ~2/3 of its ~1,070
// VALU instructions per wave on index arithmetic and its integer divisions:
// rocprofv3 SQ_INSTS_VALU, profiles/r04_sq/).  Soft mask: none or m(tile)
// values (QM_NONE / QM_MT_LDS); at most 8 bit widths.
typedef float qt_f4v __attribute__((ext_vector_type(4)));

// the x rows of one unit (8 x 16 B per lane) into v: step 2 of quant_tile_unit,
// issued ahead of time by the pipelined kernel
template <bool kNTL, typename T>
__device__ __forceinline__ void quant_tile_load(const QuantArgs& a, const int unit, qt_f4v (&v)[QCW]) {
  int si = 0;
  while (si + 1 < a.nscales && unit >= a.s[si + 1].unit_begin) ++si;
  const mcaq_quant_scale& S = a.s[si];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int HW = S.H * S.W;
  const int nsl = (S.C + QSLICE - 1) / QSLICE, upi = (HW + 255) >> 8;
  const int lu = unit - S.unit_begin;
  const int q1 = div_small(lu, nsl, a.rnsl[si]);
  const int slice = lu - q1 * nsl;
  const int b = div_small(q1, upi, a.rupi[si]);
  const int chunk = q1 - b * upi;
  const int c0 = slice * QSLICE;
  const int nc = imin_(QSLICE, S.C - c0);
  const int q0 = chunk * 256 + lane * 4;
  const int qa = q0 < HW ? q0 : 0;
  const int cw = wv * QCW;
  const int ncw = imin_(QCW, nc - cw);
  const size_t rowbase = ((size_t)b * S.C + c0 + imax_(imin_(cw, nc - 1), 0)) * HW;
  const T* xb = reinterpret_cast<const T*>(S.x) + rowbase;
#pragma unroll
  for (int c = 0; c < QCW; ++c) v[c] = ElemIO<T>::template ld4<kNTL>(xb + (size_t)imin_(c, imax_(ncw - 1, 0)) * HW + qa);
}

template <bool kNTL, bool kNTS, int kM, typename T, typename TO, bool kPre = false>
__device__ __forceinline__ void quant_tile_unit(const QuantArgs& a, const int unit, float4* qt, float* mts, float4* mq4,
                                                int* qany, qt_f4v (*pre)[QCW] = nullptr) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  int si = 0;
  while (si + 1 < a.nscales && unit >= a.s[si + 1].unit_begin) ++si;
  const mcaq_quant_scale& S = a.s[si];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int H = S.H, W = S.W, HW = H * W;
  const int sh = a.sh[si], sw = a.sw[si];
  const float rnsl = a.rnsl[si], rupi = a.rupi[si], rw = a.rw[si];
  const int nsl = (S.C + QSLICE - 1) / QSLICE, upi = (HW + 255) >> 8;
  const int lu = unit - S.unit_begin;
  const int q1 = div_small(lu, nsl, rnsl);
  const int slice = lu - q1 * nsl;
  const int b = div_small(q1, upi, rupi);
  const int chunk = q1 - b * upi;
  const int c0 = slice * QSLICE;
  const int nc = imin_(QSLICE, S.C - c0);
  const int NB = S.nbits;
  const int NTq = S.ht * S.wt;
  // ---- 1. small operands: this thread's table entry (bit width tid / 32,
  // channel tid % 32), its m(tile) value, the lane's tile bits (one load: its
  // 4 pixels share the tile)
  const int tc = imin_(tid & (QSLICE - 1), nc - 1);
  const float tmn0 = S.xmin[c0 + tc], tmx = S.xmax[c0 + tc];
  const float tmn = S.neg_min ? -tmn0 : tmn0;
  float mtv = 0.0f;
  if (kM == QM_MT_LDS) mtv = S.mt[(size_t)b * NTq + imin_(tid, NTq - 1)];
  const int q0 = chunk * 256 + lane * 4;
  const bool pv = q0 < HW;                     // HW % 4 == 0: all 4 pixels in or out
  const int qa = pv ? q0 : 0;
  const int h0 = div_small(qa, W, rw), w0 = qa - h0 * W;
  const float bv = S.bits[((size_t)b * S.ht + (h0 >> sh)) * S.wt + (w0 >> sw)];
  // ---- 2. the x rows (8 x 16 B per lane), in flight through the prologue
  const int cw = wv * QCW;
  const int ncw = imin_(QCW, nc - cw);
  const size_t rowbase = ((size_t)b * S.C + c0 + imax_(imin_(cw, nc - 1), 0)) * HW;
  const T* xb = reinterpret_cast<const T*>(S.x) + rowbase;
  TO* yb = reinterpret_cast<TO*>(S.y) + rowbase;
  typedef float f4v __attribute__((ext_vector_type(4)));
  f4v v[QCW];
  if constexpr (kPre) {
#pragma unroll
    for (int c = 0; c < QCW; ++c) v[c] = (*pre)[c];
  } else {
#pragma unroll
    for (int c = 0; c < QCW; ++c) v[c] = ElemIO<T>::template ld4<kNTL>(xb + (size_t)imin_(c, imax_(ncw - 1, 0)) * HW + qa);
  }
  // ---- 3. the table (IEEE divisions of QuantizationParameters), staged m(tile)
  {
    const int kq = imin_(tid >> 5, NB - 1);     // every thread stores an entry (unused rows harmless)
    const QParam q = qparam(tmn, tmx, S.bits_lo + kq);
    qt[tid] = make_float4(q.scale, q.zp, q.rs, 0.0f);
    if (tid < QSLICE) qany[tid] = (!S.stats_cover_x || stats_need_any(tmn, tmx)) ? 1 : 0;
  }
  if (kM == QM_MT_LDS) {
    if (tid < NTq) mts[tid] = mtv;
    for (int i = tid + 256; i < NTq; i += 256) mts[i] = S.mt[(size_t)b * NTq + i];
  }
  const int kb = imin_(imax_((int)rintf(bv), S.bits_lo), S.bits_lo + NB - 1) - S.bits_lo;
  const int hb = 1 << (S.bits_lo + kb - 1);
  const float qlo = (float)(-hb), qhi = (float)(hb - 1);
  __syncthreads();   // qt, mts ready
  // ---- 4. m(p) = 5x5 Gaussian (replicate pad) of the nearest-upsampled tile
  // values, taps row-major from 0 (quantization.py:235-238); wave w computes
  // pixel w of every lane's quad
  f2 m01 = {1.0f, 1.0f}, m23 = {1.0f, 1.0f};
  if (kM == QM_MT_LDS) {
    const int w = w0 + wv;
    int cs[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) cs[j] = imin_(imax_(w + j - 2, 0), W - 1) >> sw;
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int rb = (imin_(imax_(h0 + i - 2, 0), H - 1) >> sh) * S.wt;
#pragma unroll
      for (int j = 0; j < 5; ++j) acc = fmaf(bits_as_float(k_smooth5_bits[i * 5 + j]), mts[rb + cs[j]], acc);
    }
    reinterpret_cast<float*>(mq4)[lane * 4 + wv] = acc;
    __syncthreads();
    const float4 mm = mq4[lane];
    m01 = f2{mm.x, mm.y};
    m23 = f2{mm.z, mm.w};
  }
  if (ncw <= 0) return;
  int anyc = 0;
#pragma unroll
  for (int c = 0; c < QCW; ++c) anyc |= c < ncw ? qany[cw + c] : 0;
  const bool any_x = __builtin_amdgcn_readfirstlane(anyc) != 0;
  const float4* qrow = qt + kb * QSLICE + cw;   // the lane's entries: immediate offsets c * 16
#pragma unroll
  for (int c = 0; c < QCW; ++c) {
    if (c >= ncw) break;
    const float4 e = qrow[c];
    f4v o;
    if (!any_x) {
      // quant_dequant (mcaq_math.h) on pixel pairs: x / s by the reciprocal
      // and one FMA correction, + zp, round half to even, clamp, - zp, * s, * m
      const f2 x01 = f2{v[c].x, v[c].y}, x23 = f2{v[c].z, v[c].w};
      const f2 s2 = f2{e.x, e.x}, r2 = f2{e.z, e.z};
      const f2 p01 = x01 * e.z, p23 = x23 * e.z;
      const f2 d01 = __builtin_elementwise_fma(__builtin_elementwise_fma(-p01, s2, x01), r2, p01);
      const f2 d23 = __builtin_elementwise_fma(__builtin_elementwise_fma(-p23, s2, x23), r2, p23);
      f2 t01 = d01 + e.y, t23 = d23 + e.y;
      t01.x = __builtin_amdgcn_fmed3f(rintf(t01.x), qlo, qhi);
      t01.y = __builtin_amdgcn_fmed3f(rintf(t01.y), qlo, qhi);
      t23.x = __builtin_amdgcn_fmed3f(rintf(t23.x), qlo, qhi);
      t23.y = __builtin_amdgcn_fmed3f(rintf(t23.y), qlo, qhi);
      f2 y01 = (t01 - e.y) * e.x, y23 = (t23 - e.y) * e.x;
      if (kM != QM_NONE) { y01 = y01 * m01; y23 = y23 * m23; }
      o = f4v{y01.x, y01.y, y23.x, y23.y};
    } else {
      QParam q;
      q.scale = e.x; q.zp = e.y; q.rs = e.z; q.qmin = qlo; q.qmax = qhi;
      o = f4v{quant_dequant_any(v[c].x, q), quant_dequant_any(v[c].y, q), quant_dequant_any(v[c].z, q),
              quant_dequant_any(v[c].w, q)};
      if (kM != QM_NONE) o = o * f4v{m01.x, m01.y, m23.x, m23.y};
    }
    if (pv) ElemIO<TO>::template st4<kNTS>(yb + (size_t)c * HW + q0, o);
  }
}

template <bool kNTL, bool kNTS, int kM, typename T = float, typename TO = T>
__global__ MCAQ_QUANT_LB void mcaq_quant_tile_kernel(QuantArgs a) {
  __shared__ float4 qt[8 * QSLICE];           // [kb][c]: scale, zp, 1/scale
  __shared__ float mts[kM == QM_MT_LDS ? QMAXNT : 1];
  __shared__ float4 mq4[64];                  // m(p) of each lane's 4 pixels
  __shared__ int qany[QSLICE];
#if MCAQ_STREAM_CAP > 0
  for (int u = (int)blockIdx.x; u < a.units_total; u += (int)gridDim.x) {
    quant_tile_unit<kNTL, kNTS, kM, T, TO>(a, u, qt, mts, mq4, qany);
    __syncthreads();    // LDS of this unit free for the next
  }
#else
  quant_tile_unit<kNTL, kNTS, kM, T, TO>(a, (int)blockIdx.x, qt, mts, mq4, qany);
#endif
}

// Pipelined persistent form (MCAQ_QUANT_PIPE workgroups per CU, A/B): each
// workgroup walks units u, u + grid, ...; the x rows of its NEXT unit are in
// flight while the current one runs its prologue and stores (a 2-deep
// register pipeline, as tools/probe/narrow_probe.hip's D2 copy).  Same
// per-element arithmetic as mcaq_quant_tile_kernel.
#ifndef MCAQ_QUANT_PIPE
#define MCAQ_QUANT_PIPE 0
#endif
template <bool kNTL, bool kNTS, int kM, typename T = float, typename TO = T>
__global__ __launch_bounds__(256, 2) void mcaq_quant_tile_pipe_kernel(QuantArgs a) {
  __shared__ float4 qt[8 * QSLICE];
  __shared__ float mts[kM == QM_MT_LDS ? QMAXNT : 1];
  __shared__ float4 mq4[64];
  __shared__ int qany[QSLICE];
  qt_f4v va[QCW], vb[QCW];
  const int grid = (int)gridDim.x, total = a.units_total;
  int u = (int)blockIdx.x;
  if (u < total) quant_tile_load<kNTL, T>(a, u, va);
  for (; u < total; u += 2 * grid) {
    const int un = u + grid;
    if (un < total) quant_tile_load<kNTL, T>(a, un, vb);
    quant_tile_unit<kNTL, kNTS, kM, T, TO, true>(a, u, qt, mts, mq4, qany, &va);
    __syncthreads();
    if (un >= total) break;
    const int unn = un + grid;
    if (unn < total) quant_tile_load<kNTL, T>(a, unn, va);
    quant_tile_unit<kNTL, kNTS, kM, T, TO, true>(a, un, qt, mts, mq4, qany, &vb);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// extern "C" launchers
// ---------------------------------------------------------------------------
// Kernel timing (mcaq_time_next_launch): the next pass-1 / pass-2 launch of
// the calling thread goes through hipExtLaunchKernel with start/stop events,
// which the runtime stamps at the dispatch's own start and end (the interval
// a kernel trace reports), instead of event packets around it on the stream.
static thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
static thread_local int t_ev_skip = 0;
template <typename F, typename... Args>
static void launch_k(F kernel, dim3 grid, dim3 block, size_t shmem, hipStream_t stream, Args... args) {
  if ((t_ev_start || t_ev_stop) && t_ev_skip-- == 0) {
    hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)shmem, stream, t_ev_start, t_ev_stop, 0u, args...);
    t_ev_start = t_ev_stop = nullptr;
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shmem, stream, args...);
  }
}

extern "C" {

int mcaq_time_next_launch(hipEvent_t start, hipEvent_t stop) {
  return mcaq_time_launch(0, start, stop);
}

int mcaq_time_launch(int skip, hipEvent_t start, hipEvent_t stop) {
  if (skip < 0) return (int)hipErrorInvalidValue;
  t_ev_start = start;
  t_ev_stop = stop;
  t_ev_skip = skip;
  return 0;
}

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

// the arguments of a pass-1 launch; returns 0 or a hipError_t (vec: 16-byte rows)
static int stats_args(const mcaq_stats_scale* scales, int nscales, StatsArgs& a, bool& vec) {
  if (nscales < 1 || nscales > MAXSEG) return (int)hipErrorInvalidValue;
  int units = 0;
  for (int i = 0; i < nscales; ++i) {
    a.s[i] = scales[i];
    a.s[i].unit_begin = units;
    const int HW = scales[i].H * scales[i].W;
    if (scales[i].B < 1 || scales[i].C < 1 || HW < 1 || !scales[i].x) return (int)hipErrorInvalidValue;
    if ((scales[i].pmin == nullptr) != (scales[i].pmax == nullptr)) return (int)hipErrorInvalidValue;
    if (scales[i].dtype != scales[0].dtype || scales[i].dtype < MCAQ_DTYPE_F32 || scales[i].dtype > MCAQ_DTYPE_BF16)
      return (int)hipErrorInvalidValue;    // one element type per launch
    a.ppl[i] = stats_ppl(scales[i].C, HW);
    units += mcaq_stats_units(scales[i].B, scales[i].C, scales[i].H, scales[i].W);
#ifdef MCAQ_PROBE_STATS_SPLIT
    {
      const int nb = (scales[i].C + ST_CG - 1) / ST_CG, R = (nb + ST_WAVES - 1) / ST_WAVES;
      if (R >= 2) units += (R - 1) * mcaq_stats_units(scales[i].B, scales[i].C, scales[i].H, scales[i].W);
    }
#endif
  }
  a.nscales = nscales;
  a.units_total = units;
  // 16-byte (ppl 4) / 8-byte (ppl 2) rows need 16/8-byte aligned bases
  vec = true;
  for (int i = 0; i < nscales; ++i) vec = vec && ((uintptr_t)scales[i].x & 15) == 0;
  return 0;
}

int mcaq_stats(const mcaq_stats_scale* scales, int nscales, hipStream_t stream) {
  StatsArgs a;
  bool vec;
  const int e = stats_args(scales, nscales, a, vec);
  if (e) return e;
  const dim3 g(MCAQ_STREAM_CAP > 0 ? imin_(a.units_total, MCAQ_STREAM_CAP * 256) : a.units_total);
  switch (scales[0].dtype * 2 + (vec ? 1 : 0)) {
    case 0: launch_k(mcaq_stats_kernel<false>, g, dim3(256), 0, stream, a); break;
    case 1: launch_k(mcaq_stats_kernel<true>, g, dim3(256), 0, stream, a); break;
    case 2: launch_k(mcaq_stats_kernel<false, _Float16>, g, dim3(256), 0, stream, a); break;
    case 3: launch_k(mcaq_stats_kernel<true, _Float16>, g, dim3(256), 0, stream, a); break;
    case 4: launch_k(mcaq_stats_kernel<false, Bf16>, g, dim3(256), 0, stream, a); break;
    default: launch_k(mcaq_stats_kernel<true, Bf16>, g, dim3(256), 0, stream, a); break;
  }
  return (int)hipGetLastError();
}

int mcaq_stats_units(int B, int C, int H, int W) {
  const int HW = H * W;
  return B * ((HW + 64 * stats_ppl(C, HW) - 1) / (64 * stats_ppl(C, HW)));
}

static int finalize_args(const mcaq_finalize_scale* scales, int nscales, FinalizeArgs& a) {
  if (nscales < 1 || nscales > MAXSEG) return (int)hipErrorInvalidValue;
  int blocks = 0;
  for (int i = 0; i < nscales; ++i) {
    a.s[i] = scales[i];
    a.s[i].block_begin = blocks;
    if (scales[i].C < 1 || !scales[i].min_out || !scales[i].max_out) return (int)hipErrorInvalidValue;
    if (scales[i].pmin ? (!scales[i].pmax || scales[i].nunits < 1) : (!scales[i].min_in || !scales[i].max_in))
      return (int)hipErrorInvalidValue;
    blocks += scales[i].per_tensor ? 1 : (scales[i].C + 63) / 64;
  }
  a.nscales = nscales;
  a.nblocks = blocks;
  return 0;
}

int mcaq_finalize(const mcaq_finalize_scale* scales, int nscales, hipStream_t stream) {
  FinalizeArgs a;
  const int e = finalize_args(scales, nscales, a);
  if (e) return e;
  hipLaunchKernelGGL(mcaq_finalize_kernel, dim3(a.nblocks), dim3(256), 0, stream, a);
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

// LDS mode for a set of scales: planes in LDS when every scale's image fits
static int morph_plan(const MorphScale* s, int n, int* lds_mode, int* plane_stride, size_t* dyn) {
  int pb = 0;
  for (int i = 0; i < n; ++i) pb = imax_(pb, (plane_bytes(s[i].Hc, s[i].Wc) + 15) & ~15);
  const int rest = fixed_bytes();   // pass A keeps no tile array in LDS
  const int limit = morph_lds_budget();
#ifdef MCAQ_MORPH_GLOBAL_PLANES
  const bool lds_fit = false;   // A/B: planes in global scratch (small LDS footprint beside streaming waves)
#else
  const bool lds_fit = pb + rest <= limit;
#endif
  if (lds_fit) {
    *lds_mode = 1; *plane_stride = pb; *dyn = (size_t)(pb + rest);
  } else if (rest <= limit) {
    *lds_mode = 0; *plane_stride = pb; *dyn = (size_t)rest;
  } else {
    return (int)hipErrorInvalidValue;
  }
  return 0;
}

// images per pass A workgroup: the most (power of two, <= 16) whose planes fit
// the LDS budget while each image keeps >= 64 threads and <= 4 pixels per thread
#ifndef MCAQ_PPT
#define MCAQ_PPT 4   // max pixels per thread of a packed image (build-time experiment define)
#endif
static int morph_ipw(const MorphScale& S, int mode, int limit) {
  if (!mode) return 1;   // planes in global scratch: one image per workgroup
  const int per = ((plane_bytes(S.Hc, S.Wc) + 15) & ~15) + fixed_bytes();
  const int P = S.Hc * S.Wc;
  int ipw = 16;
  // every image group a whole number of waves (ballots / shuffles are per image)
  while (ipw > 1 && (ipw * per > limit || MORPH_THREADS / ipw < 64 || (MORPH_THREADS / ipw) % 64 != 0 ||
                     P > MCAQ_PPT * (MORPH_THREADS / ipw)))
    ipw >>= 1;
  return ipw;
}

size_t mcaq_morph_scratch_bytes_global(int B, int Hc, int Wc) {
  return (size_t)2 * B * ((plane_bytes(Hc, Wc) + 15) & ~15);   // edge + mask workgroup per image
}

size_t mcaq_morph_work_bytes(int B, int Hc, int Wc, int tile) {
  if (B < 1 || Hc < 1 || Wc < 1 || Hc > 128 || Wc > 128 || !(tile == 4 || tile == 8 || tile == 16)) return 0;
  return band_work_bytes(B, Hc, Wc, tile);
}

size_t mcaq_morph_scratch_bytes(int B, int Hc, int Wc, int ht, int wt) {
  MorphScale s{};
  s.Hc = Hc; s.Wc = Wc; s.ht = ht; s.wt = wt; s.H = 2 * Hc; s.W = 2 * Wc;  // conservative: H < Hc + tile
  int mode, stride; size_t dyn;
  if (morph_plan(&s, 1, &mode, &stride, &dyn)) return 0;
  return mode ? 0 : (size_t)2 * B * stride;   // edge + mask workgroup per image
}

int mcaq_morph(const mcaq_morph_scale* scales, int nscales, hipStream_t stream) {
  return mcaq_morph_finalize(scales, nscales, nullptr, 0, stream);
}

}  // extern "C"

// Launch configuration of the morph passes for a set of scales (validated):
// pass A (+ the channel min/max workgroups riding along) and pass B.
struct MorphLaunch {
  MorphArgs a;
  FinalizeArgs fa;
  int any_phi, any_tiles;
  int grid_a, var_a;       // pass A grid (0: no pass A) and kernel variant (2 * legacy + lds mode)
  size_t dyn_a;
  int grid_b, wlds;        // pass B grid (0: no pass B), weights staged in LDS
  int ts;                  // pass B tile row floats (TILE_FLOATS_PAD or TILE_FLOATS)
  size_t dyn_b;
  int band, grid_e;        // pass A in band mode: band grid = grid_a, edge grid
  size_t dyn_e;
  int tb, any_mask;        // pass B as batch-wide tile kernels (grid_b = 64-tile workgroups)
};

static int morph_launch_config(const mcaq_morph_scale* scales, int nscales, const mcaq_finalize_scale* fscales,
                               int nfscales, MorphLaunch& L) {
  if (nscales < 1 || nscales > MAXSEG) return (int)hipErrorInvalidValue;
  FinalizeArgs& fa = L.fa;
  fa = FinalizeArgs{};
  if (nfscales > 0) {
    const int fe = finalize_args(fscales, nfscales, fa);
    if (fe) return fe;
  }
  MorphArgs& a = L.a;
  int blocks = 0, any_phi = 0, any_tiles = 0;
  for (int i = 0; i < nscales; ++i) {
    memcpy(&a.s[i], &scales[i], sizeof(MorphScale));
    MorphScale& S = a.s[i];
    if (S.B < 1 || S.ht < 1 || S.wt < 1) return (int)hipErrorInvalidValue;
    if (S.tile < 4 || (S.tile & (S.tile - 1)) || S.tile > 128) return (int)hipErrorInvalidValue;
    if (S.Hc != S.ht * S.tile || S.Wc != S.wt * S.tile || S.Hc > S.H || S.Wc > S.W) return (int)hipErrorInvalidValue;
    // tile_tmp carries the per-tile partials from pass A to pass B; without
    // F_PHI the complexity MLP reads phi from phi_out
    if ((S.flags & F_PHI) && !S.tile_tmp) return (int)hipErrorInvalidValue;
    if ((S.flags & F_CMLP) && (!S.cmlp || (!(S.flags & F_PHI) && !S.phi_out))) return (int)hipErrorInvalidValue;
    if ((S.flags & F_SOFTMASK) && (!S.smask || !S.absmean)) return (int)hipErrorInvalidValue;
    S.block_begin = blocks;
    blocks += S.B;
    any_phi |= (S.flags & F_PHI) != 0;
    const int tf = S.flags & (F_PHI | F_CMLP | F_MAPPER | F_SOFTMASK);
    any_tiles |= tf != 0;
  }
  a.nscales = nscales;
  L.any_phi = any_phi;
  L.any_tiles = any_tiles;
  L.grid_a = 0; L.grid_b = 0; L.dyn_a = 0; L.dyn_b = 0; L.var_a = 0; L.wlds = 0;
  L.band = 0; L.grid_e = 0; L.dyn_e = 0;
  bool band = any_phi != 0;
  for (int i = 0; i < nscales; ++i)
    if ((a.s[i].flags & F_PHI) && !band_eligible(a.s[i])) band = false;
#ifdef MCAQ_NO_BAND
  band = false;   // A/B: the per-image pass A
#endif
  if (band) {
    int wg = 0, ewg = 0, dynb = 0, dyne = 0;
    for (int i = 0; i < nscales; ++i) {
      const MorphScale& S = a.s[i];
      a.bwg_begin[i] = wg;
      a.ewg_begin[i] = ewg;
      if (!(S.flags & F_PHI)) continue;
      wg += S.B * band_count(S.Hc, S.tile);
      ewg += S.B;
      dynb = imax_(dynb, (band_lds_bytes(S.Wc, S.tile) + 15) & ~15);
      dyne = imax_(dyne, (edge_lds_bytes(S.Hc, S.Wc) + 15) & ~15);
    }
    a.bwg_begin[nscales] = wg;
    a.ewg_begin[nscales] = ewg;
    if (fa.nblocks > 0) dynb = imax_(dynb, 8 * 256);   // finalize_body's LDS
    L.band = 1;
    L.grid_a = wg + fa.nblocks;
    L.dyn_a = (size_t)dynb;
    L.grid_e = ewg;
    L.dyn_e = (size_t)dyne;
  } else if (any_phi) {
    int mode, stride; size_t dyn;
    int e = morph_plan(a.s, nscales, &mode, &stride, &dyn);
    if (e) return e;
    const int limit = morph_lds_budget();
    int wg = 0;
    dyn = 0;
    for (int i = 0; i < nscales; ++i) {
      const MorphScale& S = a.s[i];
      a.wg_begin[i] = wg;
      a.ipw[i] = 1; a.pstride[i] = 0; a.gstride[i] = 0;
      if (!(S.flags & F_PHI)) continue;
      if (!mode && !S.gscratch) return (int)hipErrorInvalidValue;
      const int pb = (plane_bytes(S.Hc, S.Wc) + 15) & ~15;
      a.ipw[i] = morph_ipw(S, mode, limit);
      a.pstride[i] = pb;   // this scale's own plane bytes (global scratch: 2 B of them, mcaq_morph_scratch_bytes_global)
      a.gstride[i] = (mode ? pb : 0) + fixed_bytes();
      dyn = imax_((int)dyn, a.ipw[i] * a.gstride[i]);
      wg += 2 * ((S.B + a.ipw[i] - 1) / a.ipw[i]);
    }
    a.wg_begin[nscales] = wg;
    if (fa.nblocks > 0 && dyn < (size_t)(8 * MORPH_THREADS)) dyn = 8 * MORPH_THREADS;  // finalize_body's LDS
#ifdef MCAQ_MORPH_EXCL
    dyn = (size_t)limit;   // A/B: one pass-A workgroup per CU (no streaming waves beside it)
#endif
    // canny_impl='legacy' is an analyzer option: one value for every scale of a launch
    const int leg = (a.s[0].flags & F_CANNY_LEGACY) ? 1 : 0;
    for (int i = 1; i < nscales; ++i)
      if (((a.s[i].flags & F_CANNY_LEGACY) ? 1 : 0) != leg) return (int)hipErrorInvalidValue;
    L.grid_a = wg + fa.nblocks;
    L.var_a = 2 * leg + mode;
    L.dyn_a = dyn;
  }
  L.tb = 0; L.any_mask = 0; L.ts = TILE_FLOATS_PAD;
  bool tb = any_tiles != 0;
  for (int i = 0; i < nscales; ++i) {
    const int tf = a.s[i].flags & (F_PHI | F_CMLP | F_MAPPER | F_SOFTMASK);
    if (tf && !tiles_batch_eligible(a.s[i])) tb = false;
  }
#ifdef MCAQ_NO_TILES_BATCH
  tb = false;   // A/B: the per-image pass B
#endif
  if (tb) {
    int blk = 0;
    for (int i = 0; i < nscales; ++i) {
      const MorphScale& S = a.s[i];
      a.tb_begin[i] = blk;
      if (!(S.flags & (F_PHI | F_CMLP | F_MAPPER | F_SOFTMASK))) continue;
      blk += (S.B * S.ht * S.wt + TB_TILES - 1) / TB_TILES;
      L.any_mask |= (S.flags & F_SOFTMASK) != 0;
    }
    a.tb_begin[nscales] = blk;
    L.tb = 1;
    L.grid_b = blk;
  } else if (any_tiles) {
    // pass B packing: the waves an image needs for one MLP block of MLP_TPW
    // tiles each (at most the whole workgroup); small images share a workgroup
    const int lim = MCAQ_MORPH_LDS_LIMIT - 1024;
    int twg = 0, per = 0;
    for (int ts : {(int)TILE_FLOATS_PAD, (int)TILE_FLOATS}) {   // padded rows when they fit
      twg = 0; per = 0;
      for (int i = 0; i < nscales; ++i) {
        const MorphScale& S = a.s[i];
        a.twg_begin[i] = twg;
        a.tipw[i] = 1; a.tgstride[i] = 0;
        if (!(S.flags & (F_PHI | F_CMLP | F_MAPPER | F_SOFTMASK))) continue;
        const int NT = S.ht * S.wt;
        const int G = imin_(TILES_THREADS, 64 * ((NT + MLP_TPW - 1) / MLP_TPW));
        a.tipw[i] = TILES_THREADS / G;
        a.tgstride[i] = (tiles_lds_bytes(S.H, S.W, NT, ts) + 15) & ~15;
        per = imax_(per, a.tipw[i] * a.tgstride[i]);
        twg += (S.B + a.tipw[i] - 1) / a.tipw[i];
      }
      L.ts = ts;
      if (per + TILES_SCRATCH_BYTES <= lim) break;
    }
    a.twg_begin[nscales] = twg;
    if (per + TILES_SCRATCH_BYTES > lim) return (int)hipErrorInvalidValue;
    // stage the weight blobs in LDS when they fit beside the tile arrays and the MLP scratch
    L.wlds = per + TILES_SCRATCH_BYTES + weights_lds_bytes() <= lim;
#ifdef MCAQ_TILES_NO_WLDS
    L.wlds = 0;   // A/B: weights read through the caches (smaller LDS footprint per workgroup)
#endif
#ifdef MCAQ_TILES_EXCL
    L.dyn_b = (size_t)lim;   // A/B: one pass-B workgroup per CU (no streaming waves beside it)
#else
    L.dyn_b = (size_t)per + TILES_SCRATCH_BYTES + (L.wlds ? weights_lds_bytes() : 0);
#endif
    L.grid_b = twg;
  }
  return 0;
}

// passes: bit 0 = pass A (+ channel min/max workgroups), bit 1 = pass B
static int morph_launch(const MorphLaunch& L, int passes, hipStream_t stream) {
  const MorphArgs& a = L.a;
  const FinalizeArgs& fa = L.fa;
  if ((passes & 1) && !L.any_phi && fa.nblocks > 0) {   // nothing to ride along with
    hipLaunchKernelGGL(mcaq_finalize_kernel, dim3(fa.nblocks), dim3(256), 0, stream, fa);
    const hipError_t fe = hipGetLastError();
    if (fe != hipSuccess) return (int)fe;
  }
  if ((passes & 1) && L.band) {
    static int set_band = 0;   // raise the dynamic LDS limit once (not during graph capture)
    if (!set_band) {
      hipError_t ae = hipFuncSetAttribute((const void*)mcaq_band_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          MCAQ_MORPH_LDS_LIMIT - 1024);
      if (ae == hipSuccess)
        ae = hipFuncSetAttribute((const void*)mcaq_edge_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 MCAQ_MORPH_LDS_LIMIT - 1024);
      if (ae != hipSuccess) return (int)ae;
      set_band = 1;
    }
    hipLaunchKernelGGL(mcaq_band_kernel, dim3(L.grid_a), dim3(256), L.dyn_a, stream, a, fa);
    hipError_t le = hipGetLastError();
    if (le != hipSuccess) return (int)le;
    hipLaunchKernelGGL(mcaq_edge_kernel, dim3(L.grid_e), dim3(256), L.dyn_e, stream, a);
    le = hipGetLastError();
    if (le != hipSuccess) return (int)le;
  } else if ((passes & 1) && L.grid_a > 0) {
    const int limit = morph_lds_budget();
    static int set[4] = {0, 0, 0, 0};  // raise the dynamic LDS limit once (not during graph capture)
    const int var = L.var_a;
    const void* fns[4] = {(const void*)mcaq_morph_kernel<false>, (const void*)mcaq_morph_kernel<true>,
                          (const void*)mcaq_morph_kernel<false, true>, (const void*)mcaq_morph_kernel<true, true>};
    if ((int)L.dyn_a > set[var]) {
      hipError_t ae = hipFuncSetAttribute(fns[var], hipFuncAttributeMaxDynamicSharedMemorySize, limit);
      if (ae != hipSuccess) return (int)ae;
      set[var] = limit;
    }
    const dim3 g(L.grid_a), t(MORPH_THREADS);
    switch (var) {
      case 0: hipLaunchKernelGGL((mcaq_morph_kernel<false>), g, t, L.dyn_a, stream, a, fa); break;
      case 1: hipLaunchKernelGGL((mcaq_morph_kernel<true>), g, t, L.dyn_a, stream, a, fa); break;
      case 2: hipLaunchKernelGGL((mcaq_morph_kernel<false, true>), g, t, L.dyn_a, stream, a, fa); break;
      default: hipLaunchKernelGGL((mcaq_morph_kernel<true, true>), g, t, L.dyn_a, stream, a, fa); break;
    }
    hipError_t le = hipGetLastError();
    if (le != hipSuccess) return (int)le;
  }
  if ((passes & 2) && L.tb && L.grid_b > 0) {
    hipLaunchKernelGGL(mcaq_tb_head_kernel, dim3(L.grid_b), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(mcaq_tb_map_kernel, dim3(L.grid_b), dim3(64), 0, stream, a);
    if (L.any_mask) hipLaunchKernelGGL(mcaq_tb_mask_kernel, dim3(L.grid_b), dim3(64), 0, stream, a);
    int px = 0;
    bool mp = false;
    for (int i = 0; i < a.nscales; ++i) {
      px += a.s[i].B * a.s[i].H * a.s[i].W;
      mp = mp || (a.s[i].m_out && (a.s[i].flags & F_SOFTMASK));
    }
    if (mp) hipLaunchKernelGGL(mcaq_tb_mplane_kernel, dim3((px + 255) / 256), dim3(256), 0, stream, a, px);
  } else if ((passes & 2) && L.grid_b > 0) {
    const int lim = MCAQ_MORPH_LDS_LIMIT - 1024;
    static int set_tiles = 0;
    if ((int)L.dyn_b > set_tiles) {
      hipError_t ae = hipFuncSetAttribute((const void*)mcaq_tiles_kernel<TILE_FLOATS_PAD>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, lim);
      if (ae == hipSuccess)
        ae = hipFuncSetAttribute((const void*)mcaq_tiles_kernel<TILE_FLOATS>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
      if (ae != hipSuccess) return (int)ae;
      set_tiles = lim;
    }
    if (L.ts == TILE_FLOATS_PAD)
      hipLaunchKernelGGL(mcaq_tiles_kernel<TILE_FLOATS_PAD>, dim3(L.grid_b), dim3(TILES_THREADS), L.dyn_b, stream, a, L.wlds);
    else
      hipLaunchKernelGGL(mcaq_tiles_kernel<TILE_FLOATS>, dim3(L.grid_b), dim3(TILES_THREADS), L.dyn_b, stream, a, L.wlds);
  }
  return (int)hipGetLastError();
}

extern "C" {

int mcaq_morph_finalize(const mcaq_morph_scale* scales, int nscales, const mcaq_finalize_scale* fscales,
                        int nfscales, hipStream_t stream) {
  return mcaq_morph_pass(scales, nscales, fscales, nfscales, 3, stream);
}

int mcaq_morph_pass(const mcaq_morph_scale* scales, int nscales, const mcaq_finalize_scale* fscales,
                    int nfscales, int passes, hipStream_t stream) {
  if (passes < 1 || passes > 3) return (int)hipErrorInvalidValue;
  MorphLaunch L;
  const int e = morph_launch_config(scales, nscales, fscales, nfscales, L);
  if (e) return e;
  return morph_launch(L, passes, stream);
}

int mcaq_quant(const mcaq_quant_scale* scales, int nscales, hipStream_t stream) {
  if (nscales < 1 || nscales > MAXSEG) return (int)hipErrorInvalidValue;
  QuantArgs a;
  int units = 0;
  for (int i = 0; i < nscales; ++i) {
    a.s[i] = scales[i];
    a.s[i].unit_begin = units;
    const int HW = scales[i].H * scales[i].W;
    if (scales[i].nbits < 1 || scales[i].nbits > QMAXBITS || scales[i].bits_lo < 1 ||
        scales[i].bits_lo + scales[i].nbits - 1 > 16 || HW < 1 || scales[i].C < 1 ||
        scales[i].ht < 1 || scales[i].wt < 1 || !scales[i].x || !scales[i].y || !scales[i].bits ||
        !scales[i].xmin || !scales[i].xmax || scales[i].dtype != scales[0].dtype ||
        scales[i].dtype < MCAQ_DTYPE_F32 || scales[i].dtype > MCAQ_DTYPE_BF16 ||
        scales[i].ydtype != scales[0].ydtype ||
        (scales[i].ydtype != scales[i].dtype && scales[i].ydtype != MCAQ_DTYPE_F32))
      return (int)hipErrorInvalidValue;
    units += scales[i].B * ((HW + 255) / 256) * ((scales[i].C + QSLICE - 1) / QSLICE);
  }
  a.nscales = nscales;
  a.units_total = units;
  // 16-byte rows: HW % 4 == 0 and 16-byte aligned x / y bases (a contiguous
  // view may start at any float offset), else the scalar kernel
  bool vec = true;
  for (int i = 0; i < nscales; ++i)
    vec = vec && ((scales[i].H * scales[i].W) & 3) == 0 && (((uintptr_t)scales[i].x | (uintptr_t)scales[i].y) & 15) == 0;
  // nontemporal policy (measured): bit 0 = streaming stores of
  // y, bit 1 = nontemporal loads of x.  NT stores always; NT loads only when
  // the launch reads > 256 MB of x (config 3), where nothing of x survives in
  // L2/MALL anyway.  MCAQ_QUANT_NT (build-time define) pins it for A/B builds.
#ifdef MCAQ_QUANT_NT
  const int nt = MCAQ_QUANT_NT;
#else
  size_t xbytes = 0;
  for (int i = 0; i < nscales; ++i)
    xbytes += (size_t)scales[i].B * scales[i].C * scales[i].H * scales[i].W * (scales[0].dtype ? 2 : sizeof(float));
  const int nt = xbytes > ((size_t)256 << 20) ? 3 : 1;
#endif
  // m(p) source: one kind for every scale of the launch (the hook always
  // passes m(tile) values or nothing; the reference op a plane or nothing)
  int kind = -1;
  bool big = false;
  for (int i = 0; i < nscales; ++i) {
    const mcaq_quant_scale& q = scales[i];
    const int NT = q.ht * q.wt;
    const int k = q.mt ? (NT <= QMAXNT ? QM_MT_LDS : QM_MT_L2) : (q.m ? QM_PLANE : QM_NONE);
    if (kind >= 0 && k != kind) {
      // mixed kinds: one launch per scale
      for (int j = 0; j < nscales; ++j) {
        const int e = mcaq_quant(&scales[j], 1, stream);
        if (e) return e;
      }
      return 0;
    }
    kind = k;
    big = big || imin_(QSLICE, q.C) * q.nbits > 256 || (k == QM_MT_LDS && NT > 256);
  }
  const dim3 g(units), t(256);
#ifndef MCAQ_TRUE_DIV
  // tile-aligned path: every scale's map a power-of-two multiple of its tile
  // grid (tiles >= 4 pixels wide), <= 8 bit widths, no plane / compat indexing
  bool tile_ok = vec && (kind == QM_NONE || kind == QM_MT_LDS);
  for (int i = 0; i < nscales && tile_ok; ++i) {
    const mcaq_quant_scale& q = scales[i];
    int sh = 0, sw = 0;
    while ((q.ht << sh) < q.H) ++sh;
    while ((q.wt << sw) < q.W) ++sw;
    tile_ok = (q.ht << sh) == q.H && (q.wt << sw) == q.W && sw >= 2 && q.nbits <= 8 && q.compat_tile_h <= 0 &&
              q.compat_tile_w <= 0 && q.ht * q.wt <= QMAXNT;
    a.sh[i] = sh; a.sw[i] = sw;
    a.rnsl[i] = 1.0f / (float)((q.C + QSLICE - 1) / QSLICE);
    a.rupi[i] = 1.0f / (float)((q.H * q.W + 255) / 256);
    a.rw[i] = 1.0f / (float)q.W;
  }
#ifdef MCAQ_NO_QUANT_TILE
  tile_ok = false;   // A/B: the general kernel
#endif
  const int dt = scales[0].dtype;
  if (dt != MCAQ_DTYPE_F32) {
    // fp16 / bf16 maps: the tile-aligned kernel only (any nontemporal policy:
    // NT loads and stores)
    if (!tile_ok) return (int)hipErrorNotSupported;
    const dim3 g(MCAQ_STREAM_CAP > 0 ? imin_(units, MCAQ_STREAM_CAP * 256) : units);
    const bool yf = scales[0].ydtype == MCAQ_DTYPE_F32;
    switch ((kind == QM_NONE ? 0 : 1) + (dt == MCAQ_DTYPE_BF16 ? 2 : 0) + (yf ? 4 : 0)) {
      case 0: launch_k(mcaq_quant_tile_kernel<true, true, QM_NONE, _Float16>, g, t, 0, stream, a); break;
      case 1: launch_k(mcaq_quant_tile_kernel<true, true, QM_MT_LDS, _Float16>, g, t, 0, stream, a); break;
      case 2: launch_k(mcaq_quant_tile_kernel<true, true, QM_NONE, Bf16>, g, t, 0, stream, a); break;
      case 3: launch_k(mcaq_quant_tile_kernel<true, true, QM_MT_LDS, Bf16>, g, t, 0, stream, a); break;
      case 4: launch_k(mcaq_quant_tile_kernel<true, true, QM_NONE, _Float16, float>, g, t, 0, stream, a); break;
      case 5: launch_k(mcaq_quant_tile_kernel<true, true, QM_MT_LDS, _Float16, float>, g, t, 0, stream, a); break;
      case 6: launch_k(mcaq_quant_tile_kernel<true, true, QM_NONE, Bf16, float>, g, t, 0, stream, a); break;
      default: launch_k(mcaq_quant_tile_kernel<true, true, QM_MT_LDS, Bf16, float>, g, t, 0, stream, a); break;
    }
    return (int)hipGetLastError();
  }
#if MCAQ_QUANT_PIPE > 0
  if (tile_ok) {
    const dim3 gp(imin_(units, MCAQ_QUANT_PIPE * 256));
    switch ((kind == QM_NONE ? 0 : 4) + (nt & 3)) {
      case 0: launch_k(mcaq_quant_tile_pipe_kernel<false, false, QM_NONE>, gp, t, 0, stream, a); break;
      case 1: launch_k(mcaq_quant_tile_pipe_kernel<false, true, QM_NONE>, gp, t, 0, stream, a); break;
      case 2: launch_k(mcaq_quant_tile_pipe_kernel<true, false, QM_NONE>, gp, t, 0, stream, a); break;
      case 3: launch_k(mcaq_quant_tile_pipe_kernel<true, true, QM_NONE>, gp, t, 0, stream, a); break;
      case 4: launch_k(mcaq_quant_tile_pipe_kernel<false, false, QM_MT_LDS>, gp, t, 0, stream, a); break;
      case 5: launch_k(mcaq_quant_tile_pipe_kernel<false, true, QM_MT_LDS>, gp, t, 0, stream, a); break;
      case 6: launch_k(mcaq_quant_tile_pipe_kernel<true, false, QM_MT_LDS>, gp, t, 0, stream, a); break;
      default: launch_k(mcaq_quant_tile_pipe_kernel<true, true, QM_MT_LDS>, gp, t, 0, stream, a); break;
    }
    return (int)hipGetLastError();
  }
#endif
  if (tile_ok) {
    const dim3 g(MCAQ_STREAM_CAP > 0 ? imin_(units, MCAQ_STREAM_CAP * 256) : units);
    switch ((kind == QM_NONE ? 0 : 4) + (nt & 3)) {
      case 0: launch_k(mcaq_quant_tile_kernel<false, false, QM_NONE>, g, t, 0, stream, a); break;
      case 1: launch_k(mcaq_quant_tile_kernel<false, true, QM_NONE>, g, t, 0, stream, a); break;
      case 2: launch_k(mcaq_quant_tile_kernel<true, false, QM_NONE>, g, t, 0, stream, a); break;
      case 3: launch_k(mcaq_quant_tile_kernel<true, true, QM_NONE>, g, t, 0, stream, a); break;
      case 4: launch_k(mcaq_quant_tile_kernel<false, false, QM_MT_LDS>, g, t, 0, stream, a); break;
      case 5: launch_k(mcaq_quant_tile_kernel<false, true, QM_MT_LDS>, g, t, 0, stream, a); break;
      case 6: launch_k(mcaq_quant_tile_kernel<true, false, QM_MT_LDS>, g, t, 0, stream, a); break;
      default: launch_k(mcaq_quant_tile_kernel<true, true, QM_MT_LDS>, g, t, 0, stream, a); break;
    }
    return (int)hipGetLastError();
  }
#endif
  if (scales[0].dtype != MCAQ_DTYPE_F32) return (int)hipErrorNotSupported;   // fp16 / bf16: tile kernel only
#define MCAQ_Q_LAUNCH(V, L, S_)                                                                              \
  do {                                                                                                       \
    switch (kind * 2 + (big ? 1 : 0)) {                                                                      \
      case 0: launch_k((mcaq_quant_kernel<V, L, S_, QM_NONE, false>), g, t, 0, stream, a); break;           \
      case 1: launch_k((mcaq_quant_kernel<V, L, S_, QM_NONE, true>), g, t, 0, stream, a); break;            \
      case 2: launch_k((mcaq_quant_kernel<V, L, S_, QM_MT_LDS, false>), g, t, 0, stream, a); break;         \
      case 3: launch_k((mcaq_quant_kernel<V, L, S_, QM_MT_LDS, true>), g, t, 0, stream, a); break;          \
      case 4: case 5: launch_k((mcaq_quant_kernel<V, L, S_, QM_MT_L2, true>), g, t, 0, stream, a); break;  \
      case 6: launch_k((mcaq_quant_kernel<V, L, S_, QM_PLANE, false>), g, t, 0, stream, a); break;          \
      default: launch_k((mcaq_quant_kernel<V, L, S_, QM_PLANE, true>), g, t, 0, stream, a); break;          \
    }                                                                                                        \
  } while (0)
  if (!vec) MCAQ_Q_LAUNCH(false, false, false);
  else if (nt == 3) MCAQ_Q_LAUNCH(true, true, true);
  else if (nt == 1) MCAQ_Q_LAUNCH(true, false, true);
  else if (nt == 2) MCAQ_Q_LAUNCH(true, true, false);
  else MCAQ_Q_LAUNCH(true, false, false);
#undef MCAQ_Q_LAUNCH
  return (int)hipGetLastError();
}

}  // extern "C"

#include "mcaq_qat.h"
#include "mcaq_nms.h"
#include "mcaq_train.h"
#include "mcaq_optim.h"
#include "mcaq_dp.h"

// C++-linkage drop-in for the reference's declaration (include/mcaq_hip.h):
// same name, argument list and void return as MCAQPlugin.cpp:15-23.  An
// argument error launches nothing and is reported on stderr (the reference
// would launch with the bad sizes).
void launch_spatial_quantization(const float* input, const float* bit_map, const float* min_vals,
                                 const float* max_vals, const float* mask, float* output, int N, int C, int H,
                                 int W, int tile_h, int tile_w, int n_tiles_h, int n_tiles_w, hipStream_t stream) {
  const int e = mcaq_launch_spatial_quantization(input, bit_map, min_vals, max_vals, mask, output, N, C, H, W, tile_h,
                                                 tile_w, n_tiles_h, n_tiles_w, stream);
  if (e) fprintf(stderr, "launch_spatial_quantization: error %d (%s)\n", e, hipGetErrorString((hipError_t)e));
}
