// mcaq_math.h - exact fp32 arithmetic shared by the gfx950 kernels and the
// host emulation build (tests/emu).  Every function here is a fixed sequence
// of IEEE operations; the numpy oracle (oracle/mcaq_oracle.py) states the same
// sequence, and tests compare the two bit for bit.
//
// Build rule: compile with -ffp-contract=off.  The reference (CPU ATen) never
// fuses a multiply into an add except where it calls an FMA explicitly, so
// every fused operation below is an explicit fmaf().
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP_DEVICE_COMPILE__)
#include <hip/hip_runtime.h>
#define MCAQ_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define MCAQ_HD inline
#endif

#include <math.h>

namespace mcaq {

// Correctly rounded fp32 transcendentals: evaluate in double, round once.
// (ocml double and glibc double are both < 1 double-ulp, so the fp32 rounding
// agrees except at points within ~1e-16 of an fp32 midpoint.)
// (out of line on the device: one copy of each ocml double routine keeps the
// kernels' instruction footprint small)
#if defined(__HIPCC__) || defined(__HIP_DEVICE_COMPILE__)
#define MCAQ_CR __host__ __device__ __forceinline__
#else
#define MCAQ_CR inline
#endif
MCAQ_CR float cr_exp(float x) { return (float)exp((double)x); }
MCAQ_CR float cr_log(float x) { return (float)log((double)x); }
MCAQ_CR float cr_log2(float x) { return (float)log2((double)x); }
MCAQ_CR float cr_log1p(float x) { return (float)log1p((double)x); }
MCAQ_HD float cr_sqrt(float x) { return (float)sqrt((double)x); }
MCAQ_CR float cr_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }

MCAQ_HD float bits_as_float(uint32_t u) {
  union { uint32_t u; float f; } c; c.u = u; return c.f;
}

// exp as CPU ATen's vectorized float kernels evaluate it: SLEEF's
// expf_u10 (AVX-512 build in libtorch_cpu: Cody-Waite reduction by ln2 with
// two FMAs, degree-6 polynomial by FMA, 1 + s^2 u + s, scale by 2^(q>>1) and
// 2^(q - q>>1)).  Not correctly rounded: it differs from exp() in the last bit
// for ~9 % of arguments, which reaches the soft mask's softmax output
// (quantization.py:231) in about one tile in 10^4.  Constants read from the
// libtorch_cpu.so the fixtures were generated with.
MCAQ_HD float sleef_expf(float d) {
  const float qf = rintf(d * 1.44269502162933349609375f);
  const int q = (int)qf;
  float s = fmaf(qf, -0.693145751953125f, d);
  s = fmaf(qf, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = fmaf(u, s, 0.00139304355252534151077271f);
  u = fmaf(u, s, 0.00833336077630519866943359f);
  u = fmaf(u, s, 0.0416664853692054748535156f);
  u = fmaf(u, s, 0.166666671633720397949219f);
  u = fmaf(u, s, 0.5f);
  u = 1.0f + fmaf(s * s, u, s);
  const int a = q >> 1, b = q - a;
  u = u * bits_as_float((uint32_t)(a + 127) << 23);
  u = u * bits_as_float((uint32_t)(b + 127) << 23);
  if (d < -104.0f) u = 0.0f;
  if (d > 100.0f) u = __builtin_inff();
  return u;
}

// Which exp ATen's channel softmax (dim=1 of (B, 2, ht, wt), SoftMaxKernel
// _vec_softmax) applies to flattened position `flat` of N = B*NT: at::parallel_for
// cuts [0, N) into ceil(N / T) chunks for T threads; within a chunk each
// image's run is vectorized 16 lanes at a time (SLEEF) and its last < 16
// positions go through scalar std::exp (glibc, correctly rounded).  T is the
// reference process's torch.get_num_threads(); verified against torch.softmax
// for T = 1..16 on batch / grid shapes of all three hook scales.
MCAQ_HD bool aten_softmax_vec_lane(long long flat, long long N, int NT, int T) {
  const long long nthr = T < 1 ? 1 : (T < N ? T : N);
  const long long chunk = (N + nthr - 1) / nthr;
  const long long cs = (flat / chunk) * chunk, ce = cs + chunk < N ? cs + chunk : N;
  const long long img = flat / NT;
  const long long ss = cs > img * NT ? cs : img * NT;
  const long long se = ce < (img + 1) * NT ? ce : (img + 1) * NT;
  return flat < ss + ((se - ss) / 16) * 16;
}
MCAQ_HD uint32_t float_as_bits(float f) {
  union { uint32_t u; float f; } c; c.f = f; return c.u;
}

// CPU torch.log2 of the LBP arguments k/T^2 + 1e-10 is correctly rounded
// except at these arguments (oracle LOG2_OVERRIDES, pinned by tests).
MCAQ_HD float log2_ref(float a) {
  const uint32_t b = float_as_bits(a);
  switch (b) {
    case 0x3F4ABC00u: return bits_as_float(0xBEAC50B0u);
    case 0x3F553400u: return bits_as_float(0xBE871FE6u);
    case 0x3F5F7400u: return bits_as_float(0xBE48E134u);
    case 0x3F6C9400u: return bits_as_float(0xBDE91E32u);
    case 0x3F78CC00u: return bits_as_float(0xBD28A796u);
    case 0x3F7A7C00u: return bits_as_float(0xBD00B59Cu);
    case 0x3F7B8000u: return bits_as_float(0xBCD1987Eu);
    case 0x3F7BE800u: return bits_as_float(0xBCBE853Eu);
    case 0x3F7CA400u: return bits_as_float(0xBC9C1DC6u);
    case 0x3F7FFC00u: return bits_as_float(0xB8B8ABACu);
    default: return cr_log2(a);
  }
}

MCAQ_HD float fmax_(float a, float b) { return a > b ? a : b; }
// NaN-propagating max / ReLU (torch.amax, torch.relu keep NaN)
MCAQ_HD float fmaxp(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_elementwise_maximum(a, b);
#else
  return a != a ? a : (b != b ? b : (a > b ? a : b));
#endif
}
MCAQ_HD float fminp(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_elementwise_minimum(a, b);
#else
  return a != a ? a : (b != b ? b : (a < b ? a : b));
#endif
}
MCAQ_HD float relu_nan(float x) { return (x > 0.0f || x != x) ? x : 0.0f; }
MCAQ_HD float fmin_(float a, float b) { return a < b ? a : b; }
MCAQ_HD float clampf_(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
MCAQ_HD int imin_(int a, int b) { return a < b ? a : b; }
MCAQ_HD int imax_(int a, int b) { return a > b ? a : b; }

// ATen CPU multi_row_sum cascade (level_power 4, valid for n < 2^20):
// rows are added into a0; after every full block of 16 the block folds into
// a1, every 16 blocks a1 folds into a2, every 256 blocks a2 into a3.
struct Cascade {
  float a0, a1, a2, a3;
  int i;
  MCAQ_HD void init() { a0 = a1 = a2 = a3 = 0.0f; i = 0; }
  MCAQ_HD void push(float v) {
    a0 = a0 + v;
    ++i;
    if ((i & 15) == 0) {
      a1 = a1 + a0; a0 = 0.0f;
      if (i & 0xF0) return;
      a2 = a2 + a1; a1 = 0.0f;
      if (i & 0xF00) return;
      a3 = a3 + a2; a2 = 0.0f;
    }
  }
  MCAQ_HD float result() const { return ((a0 + a1) + a2) + a3; }
};

// Sum of n strided values in ATen's contiguous outer-reduction order.
// tail == false: vectorized column (plain cascade); tail == true: row_sum
// (4 interleaved cascades over rows k, k+4, ...; leftovers into partial 0).
template <typename Load>
MCAQ_HD float aten_sum(int n, bool tail, Load load) {
  if (!tail) {
    Cascade c; c.init();
    for (int r = 0; r < n; ++r) c.push(load(r));
    return c.result();
  }
  const int nilp = n / 4;
  Cascade c0, c1, c2, c3;
  c0.init(); c1.init(); c2.init(); c3.init();
  for (int r = 0; r < nilp; ++r) {
    c0.push(load(4 * r + 0));
    c1.push(load(4 * r + 1));
    c2.push(load(4 * r + 2));
    c3.push(load(4 * r + 3));
  }
  float p0 = c0.result();
  for (int r = 4 * nilp; r < n; ++r) p0 = p0 + load(r);
  return ((p0 + c1.result()) + c2.result()) + c3.result();
}

// Column index where ATen's tail (row_sum) order starts for M columns.
MCAQ_HD int aten_tail_start(int M) { return (M / 32) * 32; }

// a / b for 0 <= a < 2^24, b >= 1 without an integer division: the fp32
// estimate is within one of the quotient, then corrected (exact)
MCAQ_HD int div_small(int a, int b, float inv_b) {
  int q = (int)((float)a * inv_b);
  q -= (q * b > a) ? 1 : 0;
  q += ((q + 1) * b <= a) ? 1 : 0;
  return q;
}

// PyTorch upsample 'nearest' source index (UpSampleKernel nearest_idx).
MCAQ_HD int nearest_src(int o, int in_size, int out_size) {
  if (out_size == in_size) return o;
  if (out_size == 2 * in_size) return o >> 1;
  const float scale = (float)in_size / (float)out_size;
  const int s = (int)floorf((float)o * scale);
  return s < in_size - 1 ? s : in_size - 1;
}

// nearest_src with the ratio resolved once (per workgroup): when out = in *
// 2^k (a whole number of power-of-two tiles, the usual hook case) the source
// index is o >> k exactly (in/out = 2^-k is exact in fp32), else nearest_src.
struct NearestMap { int in, out, shift; };
MCAQ_HD NearestMap nearest_map(int in_size, int out_size) {
  NearestMap m{in_size, out_size, -1};
  if (in_size > 0 && out_size % in_size == 0) {
    const int r = out_size / in_size;
    if ((r & (r - 1)) == 0) { int k = 0; while ((1 << k) < r) ++k; m.shift = k; }
  }
  return m;
}
MCAQ_HD int nearest_apply(const NearestMap& m, int o) {
  return m.shift >= 0 ? (o >> m.shift) : nearest_src(o, m.in, m.out);
}

// Quantization parameters (quantization.py:26-66) for integer bits b.
struct QParam { float scale, zp, qmin, qmax, rs; };   // rs = RN(1 / scale)
MCAQ_HD QParam qparam(float xmin, float xmax, int b) {
  QParam q;
  const int qmin = -(1 << (b - 1)), qmax = (1 << (b - 1)) - 1;
  float rng = xmax - xmin;
  rng = rng < 1e-8f ? 1e-8f : rng;              // clamp(min=1e-8)
  q.scale = rng / (float)(qmax - qmin);
  float zp = (float)qmin - xmin / q.scale;
  q.qmin = (float)qmin; q.qmax = (float)qmax;
  q.zp = clampf_(zp, q.qmin, q.qmax);
  q.rs = 1.0f / q.scale;
  return q;
}

// x / s, correctly rounded, from rs = RN(1/s): q0 = RN(x rs), r = x - q0 s
// (exact by FMA), RN(q0 + r rs) (Markstein's correction; 0 mismatches vs IEEE
// division over 1.3e8 (x, s) pairs incl. all-ones-mantissa divisors,
// tests/test_oracle_cpu.py::test_reciprocal_division_is_correctly_rounded).
// 3 VALU ops instead of the ~10 of the v_div_scale/fmas/fixup sequence.  Where
// it can differ - subnormal x, the sign of a zero quotient - the quotient
// is < 1e-20 and the + zp that follows (0 or |zp| >= 6e-8) absorbs it, so
// quant_dequant is unchanged.  MCAQ_TRUE_DIV builds keep the IEEE division.
// x / s, correctly rounded, for |x rs| < FLT_MAX (finite statistics cover x:
// the fast path of pass 2)
MCAQ_HD float div_by(float x, float s, float rs) {
#ifdef MCAQ_TRUE_DIV
  (void)rs;
  return x / s;
#else
  const float q0 = x * rs;
  const float r = fmaf(-q0, s, x);
  return fmaf(r, rs, q0);
#endif
}

// The same for any x: when q0 = x rs is +-inf (x = +-inf, or an overflowing
// product) the remainder fma(-q0, s, x) is NaN; it is mapped to -FLT_MAX
// (v_med3_f32 returns its smallest operand when one is NaN), so the result is
// q0 = +-inf = x / s, as the reference's IEEE division gives.  NaN x stays NaN
// (q0 is NaN).  Finite remainders pass unchanged.
MCAQ_HD float rem_finite(float r) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_fmed3f(r, -3.40282347e38f, 3.40282347e38f);
#else
  return r != r ? -3.40282347e38f : clampf_(r, -3.40282347e38f, 3.40282347e38f);
#endif
}
MCAQ_HD float div_by_any(float x, float s, float rs) {
#ifdef MCAQ_TRUE_DIV
  (void)rs;
  return x / s;
#else
  const float q0 = x * rs;
  const float r = rem_finite(fmaf(-q0, s, x));
  return fmaf(r, rs, q0);
#endif
}

// clamp of a finite value into [lo, hi] (lo <= hi): one v_med3_f32 on the
// device instead of two compare + select pairs
MCAQ_HD float clamp_med3(float x, float lo, float hi) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_fmed3f(x, lo, hi);
#else
  return clampf_(x, lo, hi);
#endif
}

// torch.clamp(v, lo, hi) (lo <= hi): +-inf clamp to a bound, NaN stays NaN.
// On the device v_maximum_f32 / v_minimum_f32 (gfx950, NaN-propagating); a
// single v_med3_f32 would turn NaN into lo (it returns min3 when an operand
// is NaN).
MCAQ_HD float clamp_nan(float x, float lo, float hi) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_elementwise_minimum(__builtin_elementwise_maximum(x, lo), hi);
#else
  return clampf_(x, lo, hi);
#endif
}

// y = (clamp(rint(x/s + zp)) - zp) * s     (quantization.py:597-600), for
// finite x with |x / s| well inside the fp32 range: the fast path, taken by
// the kernels where the channel's own batch min/max are finite and < 1e20
// in magnitude (then every x of the channel is, and |x rs| < 3e30)
MCAQ_HD float quant_dequant(float x, const QParam& q) {
  float t = div_by(x, q.scale, q.rs) + q.zp;
  float r = clamp_med3(rintf(t), q.qmin, q.qmax);
  return (r - q.zp) * q.scale;
}

// the same for any x, with the reference's non-finite behaviour: x = +-inf
// -> the qmax / qmin level, x = NaN -> NaN (2 more VALU operations)
MCAQ_HD float quant_dequant_any(float x, const QParam& q) {
  float t = div_by_any(x, q.scale, q.rs) + q.zp;
  float r = clamp_nan(rintf(t), q.qmin, q.qmax);
  return (r - q.zp) * q.scale;
}

// true when a channel with batch statistics [xmin, xmax] needs
// quant_dequant_any (a NaN or +-inf in the channel, or huge magnitudes)
MCAQ_HD bool stats_need_any(float xmin, float xmax) {
  return !(fabsf(xmin) < 1e20f && fabsf(xmax) < 1e20f);
}

}  // namespace mcaq
