// mcaq_qat.h - gfx950 kernels of the QAT (training) quantizer: the
// fractional-bit forward and the straight-through backward of
// SpatialAdaptiveQuantization._forward_pytorch, training branch
// (mcaq_yolo/core/quantization.py:699-727, 733-737), the EMA running
// statistics (update_running_stats, quantization.py:319-353), and their
// extern "C" launchers (include/mcaq_hip.h).  Included by mcaq_kernels.hip.
//
// Per pixel p with tile bits b (nearest upsample of the continuous bit map),
// lo = floor(b), f = b - lo, hi = lo + 1 (lo past 8):
//   forward   xq = (1 - f) * Q_lo(x) + f * Q_hi(x),  y = xq * m
//   backward  gm = g * m                      (g * 1 without a mask)
//             grad_x    = gm * (1 - f) + gm * f          (STE, elementwise)
//             grad_m(p) = sum_c g * xq                  (channel sum)
//             grad_b(t) = sum_{p in t} sum_c (gm * Q_hi - gm * Q_lo)
// Q_b is the inference quant/dequant with per-channel running min/max.
// The HBM traffic: forward reads x (+ m plane) and writes y; backward reads
// g and x (+ m) and writes grad_x, plus per-slice channel partials of the two
// sums ((C/32) x 2 planes of B*H*W floats) that a small per-image kernel folds.
#pragma once

namespace mcaq {

// the train step's bit budget riding on the QAT forward launch (nseg = 0: none)
struct QatBudget { const float* bits[3]; int n[3]; int nseg; float target; float* avg; float* loss; };

struct QatArgs {
  mcaq_qat_scale s[3];
  int nscales;
  int units_total;
  QatBudget bb;
};

#ifndef MCAQ_QAT_MINW
#define MCAQ_QAT_MINW 4
#endif
constexpr int QAT_LO = 1;   // table widths QAT_LO .. 8 (the reference's bc_int <= 8)
constexpr int QAT_NB = 8;

// one workgroup per (scale, image, tile row): the band of pixel rows whose
// nearest tile row is th (binary search: nearest_src is monotone).  The
// per-slice channel partials of the backward kernel are summed per pixel,
// slices in order, the slice loads of a pixel issued together -> grad_m and
// an LDS chunk of the band; each pixel column is summed over the band's rows,
// then each tile over its columns (short dependent chains: rows + columns,
// not rows x columns).  fp32 sums in a different order than the reference's
// upsample backward: grad_bits is checked to a tolerance.
constexpr int QAT_FOLD_LDS = 8192;    // floats of pixel chunk
constexpr int QAT_FOLD_SL = 8;        // slices loaded together

// first index i in [0, n) with nearest_src(i, in, n) >= v (n if none)
__device__ __forceinline__ int band_start(int v, int in, int n) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (nearest_src(mid, in, n) >= v) hi = mid; else lo = mid + 1;
  }
  return lo;
}

constexpr int QAT_FOLD_PX = 4;        // pixels per thread per round

// per thread: pixels i0 + 256 j (j < QAT_FOLD_PX, i < np) of the chunk at p0;
// all slice loads of a round issued before the first add, slices summed in order
__device__ __forceinline__ void slice_sums(const float* pm, const float* pf, size_t plane, int nsl, int p0,
                                           int i0, int np, float (&am)[QAT_FOLD_PX], float (&af)[QAT_FOLD_PX]) {
  for (int s0 = 0; s0 < nsl; s0 += QAT_FOLD_SL) {
    float vm[QAT_FOLD_PX][QAT_FOLD_SL], vf[QAT_FOLD_PX][QAT_FOLD_SL];
#pragma unroll
    for (int j = 0; j < QAT_FOLD_PX; ++j) {
      const int p = p0 + imin_(i0 + 256 * j, np - 1);
#pragma unroll
      for (int k = 0; k < QAT_FOLD_SL; ++k) {
        const size_t o = (size_t)imin_(s0 + k, nsl - 1) * plane + p;
        vm[j][k] = pm[o];
        vf[j][k] = pf[o];
      }
    }
#pragma unroll
    for (int j = 0; j < QAT_FOLD_PX; ++j)
#pragma unroll
      for (int k = 0; k < QAT_FOLD_SL; ++k)
        if (s0 + k < nsl) {
          am[j] = (s0 + k == 0) ? vm[j][k] : am[j] + vm[j][k];
          af[j] = (s0 + k == 0) ? vf[j][k] : af[j] + vf[j][k];
        }
  }
}

// Fold of one (image b, tile row th) band by one 256-thread workgroup: the
// band's pixel rows in chunks of `cap` pixels (pl); per pixel the slice
// partials in slice order -> grad_m and pl; per pixel column the band's rows
// in order (col, W floats); per tile its columns in order -> grad_bits.  The
// separate fold kernel runs it per block; the backward kernel's last unit of
// a band runs it inside its own launch.
__device__ void qat_fold_band(const mcaq_qat_scale& S, int b, int th, float* pl, float* col, int cap) {
  const int H = S.H, W = S.W, HW = H * W, wt = S.wt;
  const int nsl = (S.C + 31) / 32;
  const size_t plane = (size_t)S.B * HW;
  const float* pm = S.work + (size_t)b * HW;
  const float* pf = S.work + (size_t)nsl * plane + (size_t)b * HW;
  const int rs = band_start(th, S.ht, H), re = band_start(th + 1, S.ht, H);
  const int rows_per_chunk = imax_(1, cap / W);
  for (int w = threadIdx.x; w < W; w += 256) col[w] = 0.0f;
  for (int r0 = rs; r0 < re; r0 += rows_per_chunk) {
    const int r1 = imin_(re, r0 + rows_per_chunk);
    const int p0 = r0 * W, np = (r1 - r0) * W;
    for (int i0 = threadIdx.x; i0 < np; i0 += 256 * QAT_FOLD_PX) {
      float am[QAT_FOLD_PX], af[QAT_FOLD_PX];
      slice_sums(pm, pf, plane, nsl, p0, i0, np, am, af);
#pragma unroll
      for (int j = 0; j < QAT_FOLD_PX; ++j) {
        const int i = i0 + 256 * j;
        if (i < np) {
          if (S.gm) S.gm[(size_t)b * HW + p0 + i] = am[j];
          pl[i] = af[j];
        }
      }
    }
    __syncthreads();
    // per pixel column: the band's rows of this chunk, in order
    if (S.gb)
      for (int w = threadIdx.x; w < W; w += 256) {
        float t = col[w];
        for (int r = 0; r < r1 - r0; ++r) t += pl[r * W + w];
        col[w] = t;
      }
    __syncthreads();
  }
  if (!S.gb) return;
  // tile tw: its columns, in order
  for (int tw = threadIdx.x; tw < wt; tw += 256) {
    const int cs = band_start(tw, wt, W), ce = band_start(tw + 1, wt, W);
    float t = 0.0f;
    for (int w = cs; w < ce; ++w) t += col[w];
    S.gb[((size_t)b * S.ht + th) * wt + tw] = t;
  }
}

// in-launch fold: the backward kernel's LDS lent to the band fold
constexpr int QAT_FUSED_BUF = 2048;   // floats: col (QAT_FUSED_MAXW) + pixel chunk
constexpr int QAT_FUSED_MAXW = 512;

// unit = 256 pixels x 32 channels of one image (the pass-2 layout): lane l of
// wave w owns pixels 4l..4l+3 and channels 8w..8w+7 of the slice (channel
// loop fully unrolled: the compiler schedules the loads).  Measured slower at
// config 5: all loads issued ahead of the table and barrier;
// two channels at a time under an 8-workgroup/CU register cap; one-wave
// workgroups walking all 32 channels of a slice (every unit resident at once).
// the bit budget of the train step (models/mcaq_yolo.py:572-577 avg_bits =
// mean_k mean(bits_k); MCAQLoss.compute_bit_budget_loss :110-118) as ONE extra
// workgroup of the QAT forward launch, which reads the same bit maps: per
// segment 8 loads a thread in flight (clamped index, no load behind a
// branch), a fixed shuffle tree per wave, the 4 waves summed in order
__device__ __forceinline__ void qat_budget_block(const QatBudget& B, float* red) {
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float total = 0.0f;
  for (int k = 0; k < B.nseg; ++k) {
    const float* p = k == 0 ? B.bits[0] : (k == 1 ? B.bits[1] : B.bits[2]);
    const int n = k == 0 ? B.n[0] : (k == 1 ? B.n[1] : B.n[2]);
    float s = 0.0f;
    for (int i0 = tid; i0 < n; i0 += 256 * 8) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = p[imin_(i0 + 256 * r, n - 1)];
#pragma unroll
      for (int r = 0; r < 8; ++r) s += i0 + 256 * r < n ? v[r] : 0.0f;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) red[wv] = s;
    __syncthreads();
    total = total + ((red[0] + red[1]) + (red[2] + red[3])) * (1.0f / (float)n);
    __syncthreads();
  }
  if (tid == 0) {
    const float avg = total * (1.0f / (float)B.nseg);
    B.avg[0] = avg;
    if (B.loss) B.loss[0] = (avg - B.target) * (avg - B.target);
  }
}

// kTile: every scale's map is a power-of-two multiple of its tile grid with
// tiles >= 4 pixels wide (host-checked): a lane's 4 pixels share one tile, so
// one bit-map load and one (lo, hi) table pair per channel serve all four
template <bool kBwd, bool kVec, bool kTile = false>
__global__ __launch_bounds__(256, MCAQ_QAT_MINW) void mcaq_qat_kernel(QatArgs a) {
  __shared__ float4 qt[32 * QAT_NB];   // scale, zp, 1/scale
  __shared__ float red[2][4][256];
  __shared__ int s_last;   // bands completed by this unit (bit per band)
  if (!kBwd && (int)blockIdx.x >= a.units_total) {   // the bit-budget workgroup (forward only)
    qat_budget_block(a.bb, &red[0][0][0]);
    return;
  }
  const int unit = blockIdx.x;
  int si = 0;
  while (si + 1 < a.nscales && unit >= a.s[si + 1].unit_begin) ++si;
  const mcaq_qat_scale S = si == 0 ? a.s[0] : si == 1 ? a.s[1] : a.s[2];   // by value: no indexed kernarg copy
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int HW = S.H * S.W;
  const int upi = (HW + 255) / 256;
  const int nsl = (S.C + 31) / 32;
  int lu = unit - S.unit_begin;
  const int slice = lu % nsl; lu /= nsl;
  const int chunk = lu % upi;
  const int b = lu / upi;
  const int c0 = slice * 32;
  const int nc = imin_(32, S.C - c0);
  const int q0 = chunk * 256 + lane * 4;
  const int cw = wv * 8;
  const int ncw = imin_(8, nc - cw);
  const size_t rowbase = ((size_t)b * S.C + c0 + imax_(0, imin_(cw, nc - 1))) * HW;
  const float* xb = S.x + rowbase;
  const int qa = q0 < HW ? q0 : 0;
  // ---- the wave's 8 x rows first, unconditionally (clamped channel and
  // pixel indices): in flight through the table build and the per-pixel
  // prologue, as pass 2 issues them (the backward's g rows follow in the
  // channel loop: both sets at once spill 84 B a lane at 128 VGPRs)
  float xv[8][4];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const size_t ro = (size_t)imin_(c, imax_(ncw - 1, 0)) * HW;
    if (kVec) {
      const float4 t = *reinterpret_cast<const float4*>(xb + ro + qa);
      xv[c][0] = t.x; xv[c][1] = t.y; xv[c][2] = t.z; xv[c][3] = t.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) xv[c][k] = xb[ro + imin_(q0 + k, HW - 1)];
    }
  }
  for (int i = tid; i < nc * QAT_NB; i += 256) {
    const int c = i / QAT_NB, k = i - c * QAT_NB;
    const QParam q = qparam(S.xmin[c0 + c], S.xmax[c0 + c], QAT_LO + k);
    qt[i] = make_float4(q.scale, q.zp, q.rs, 0.0f);
  }
  const NearestMap nmh = nearest_map(S.ht, S.H), nmw = nearest_map(S.wt, S.W);
  bool pv[4];
  int kl[4], kh[4];
  float fu[4], omf[4], mv[4];
  const bool has_m = S.m != nullptr;
  if constexpr (kTile) {
    // one tile for the lane's 4 pixels: the same values in every k slot
    // (the channel loop's table reads and parameters fold into one per channel)
    const int h0 = qa / S.W, w0 = qa - h0 * S.W;
    const float bv = S.bits[((size_t)b * S.ht + (h0 >> nmh.shift)) * S.wt + (w0 >> nmw.shift)];
    const float fl = floorf(bv);
    const float f0 = bv - fl;
    const int lo = imin_(imax_((int)fl, QAT_LO), QAT_LO + QAT_NB - 1);
    float4 m4 = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
    if (has_m) m4 = *reinterpret_cast<const float4*>(S.m + (size_t)b * HW + qa);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pv[k] = q0 + k < HW;
      fu[k] = f0;
      omf[k] = 1.0f - f0;
      kl[k] = lo - QAT_LO;
      kh[k] = (lo < 8 ? lo + 1 : lo) - QAT_LO;
    }
    mv[0] = m4.x; mv[1] = m4.y; mv[2] = m4.z; mv[3] = m4.w;
  } else {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = imin_(q0 + k, HW - 1);
    pv[k] = q0 + k < HW;
    const int h = p / S.W, w = p - (p / S.W) * S.W;
    const float bv = S.bits[((size_t)b * S.ht + nearest_apply(nmh, h)) * S.wt + nearest_apply(nmw, w)];
    const float fl = floorf(bv);
    fu[k] = bv - fl;                 // exact (Sterbenz) for b >= 1
    omf[k] = 1.0f - fu[k];
    const int lo = imin_(imax_((int)fl, QAT_LO), QAT_LO + QAT_NB - 1);
    kl[k] = lo - QAT_LO;
    kh[k] = (lo < 8 ? lo + 1 : lo) - QAT_LO;    // Q_hi := Q_lo past 8 bits (frac is 0 there)
    mv[k] = S.m ? S.m[(size_t)b * HW + p] : 1.0f;
  }
  }
  __syncthreads();   // qt ready
  float sgm[4] = {0.f, 0.f, 0.f, 0.f}, sgf[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    if (c >= ncw) break;
    const float* v = xv[c];
    float gv[4];
    if (kBwd) {
      const size_t ro = (size_t)c * HW;
      if (kVec) {
        const float4 u = *reinterpret_cast<const float4*>(S.g + rowbase + ro + qa);
        gv[0] = u.x; gv[1] = u.y; gv[2] = u.z; gv[3] = u.w;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) gv[k] = S.g[rowbase + ro + imin_(q0 + k, HW - 1)];
      }
    }
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 zl = qt[(cw + c) * QAT_NB + kl[k]];
      const float4 zh = qt[(cw + c) * QAT_NB + kh[k]];
      const int lo = kl[k] + QAT_LO, hi = kh[k] + QAT_LO;
      QParam L, Hq;
      L.scale = zl.x; L.zp = zl.y; L.rs = zl.z;
      L.qmin = (float)(-(1 << (lo - 1))); L.qmax = (float)((1 << (lo - 1)) - 1);
      Hq.scale = zh.x; Hq.zp = zh.y; Hq.rs = zh.z;
      Hq.qmin = (float)(-(1 << (hi - 1))); Hq.qmax = (float)((1 << (hi - 1)) - 1);
      const float ql = quant_dequant_any(v[k], L);
      const float qh = quant_dequant_any(v[k], Hq);
      const float xq = omf[k] * ql + fu[k] * qh;      // two rounded products, one rounded add
      if (!kBwd) {
        o[k] = has_m ? xq * mv[k] : xq;
      } else {
        const float g = gv[k];
        const float gm = has_m ? g * mv[k] : g;
        o[k] = gm * omf[k] + gm * fu[k];
        sgm[k] += g * xq;
        sgf[k] += gm * qh - gm * ql;
      }
    }
    float* orow = (kBwd ? S.gx : S.y) + rowbase + (size_t)c * HW;
    if (kVec) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      const f4v ov = {o[0], o[1], o[2], o[3]};
      if (pv[0]) __builtin_nontemporal_store(ov, reinterpret_cast<f4v*>(orow + q0));   // written once, streamed
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) if (pv[k]) orow[q0 + k] = o[k];
    }
  }
  if (!kBwd) return;
  // channel partials of this slice: waves in order, then one write per pixel
#pragma unroll
  for (int k = 0; k < 4; ++k) { red[0][wv][lane * 4 + k] = sgm[k]; red[1][wv][lane * 4 + k] = sgf[k]; }
  __syncthreads();
  const int p = chunk * 256 + tid;
  if (p < HW) {
    const float tm = ((red[0][0][tid] + red[0][1][tid]) + red[0][2][tid]) + red[0][3][tid];
    const float tf = ((red[1][0][tid] + red[1][1][tid]) + red[1][2][tid]) + red[1][3][tid];
    const size_t plane = (size_t)S.B * HW;
    const size_t o = ((size_t)slice * S.B + b) * HW + p;
    if (S.arrive) {
      // handed to the image's last unit inside this launch: write-through
      // (sc1) stores, no release fence (cdna_hip_programming.md Guideline 16)
      __hip_atomic_store(S.work + o, tm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(S.work + (size_t)nsl * plane + o, tf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      S.work[o] = tm;
      S.work[(size_t)nsl * plane + o] = tf;
    }
  }
  if (!S.arrive || (!S.gm && !S.gb)) return;
  // last-arriver fold per (image, tile row): every storing wave drains its
  // sc1 stores; one lane per tile-row band this unit's pixels touch counts
  // the unit in (a band is complete after nsl x the chunks overlapping it);
  // a unit that completes a band takes ONE agent-scope acquire and folds it
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int plo = chunk * 256, phi = imin_(HW, plo + 256) - 1;
  const int thA = nearest_src(plo / S.W, S.ht, S.H), thB = nearest_src(phi / S.W, S.ht, S.H);
  if (tid == 0) s_last = 0;
  __syncthreads();
  if (tid <= thB - thA) {
    const int th = thA + tid;
    const int rs = band_start(th, S.ht, S.H), re = band_start(th + 1, S.ht, S.H);
    const int need = nsl * ((re * S.W + 255) / 256 - (rs * S.W) / 256);
    const int old = __hip_atomic_fetch_add(S.arrive + (size_t)b * S.ht + th, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    if (old == need - 1) atomicOr(&s_last, 1 << tid);
  }
  __syncthreads();
  const int done = s_last;
  if (!done) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  float* buf = &red[0][0][0];
  for (int k = 0; k <= thB - thA; ++k)
    if (done & (1 << k)) {
      qat_fold_band(S, b, thA + k, buf + QAT_FUSED_MAXW, buf, QAT_FUSED_BUF - QAT_FUSED_MAXW);
      __syncthreads();
      if (tid == 0)   // zeroed for the next launch
        __hip_atomic_store(S.arrive + (size_t)b * S.ht + thA + k, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ __launch_bounds__(256) void mcaq_qat_fold_kernel(QatArgs a) {
  __shared__ float pl[QAT_FOLD_LDS];
  __shared__ float col[QAT_FOLD_LDS];
  const int blk = blockIdx.x;
  int si = 0;
  while (si + 1 < a.nscales && blk >= a.s[si + 1].block_begin) ++si;
  const mcaq_qat_scale S = si == 0 ? a.s[0] : si == 1 ? a.s[1] : a.s[2];
  if (S.arrive) return;   // folded inside the backward launch
  const int lb = blk - S.block_begin;
  const int b = lb / S.ht, th = lb - (lb / S.ht) * S.ht;
  qat_fold_band(S, b, th, pl, col, QAT_FOLD_LDS);
}

// running <- a * running + c * batch (first batch: running <- batch),
// a = fp32(momentum), c = fp32(1 - momentum) as Python evaluates them.
__global__ __launch_bounds__(256) void mcaq_ema_kernel(const float* bmin, const float* bmax, float* rmin,
                                                       float* rmax, int C, float am, float cm, int first,
                                                       float* cmin, float* cmax, long long* nbt) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c == 0 && nbt) nbt[0] += 1;     // num_batches_tracked (one thread of the launch)
  if (c >= C) return;
  float lo, hi;
  if (first) {
    lo = bmin[c];
    hi = bmax[c];
  } else {
    lo = am * rmin[c] + cm * bmin[c];
    hi = am * rmax[c] + cm * bmax[c];
  }
  rmin[c] = lo;
  rmax[c] = hi;
  if (cmin) cmin[c] = lo;             // copies for the quantizer of this step
  if (cmax) cmax[c] = hi;
}

// several EMA updates in one launch: segment of workgroup blockIdx.x by the
// running workgroup offsets (one per segment, 256 channels per workgroup)
struct EmaSeg { const float *bmin, *bmax; float *rmin, *rmax, *cmin, *cmax; long long* nbt; int C, first, wg0; float am, cm; };
struct EmaMulti { EmaSeg s[3]; int nseg; };
__device__ __forceinline__ void ema_multi_body(const EmaMulti& M, int x) {
  const EmaSeg& g = (M.nseg > 2 && x >= M.s[2].wg0) ? M.s[2] : ((M.nseg > 1 && x >= M.s[1].wg0) ? M.s[1] : M.s[0]);
  const int c = (x - g.wg0) * 256 + threadIdx.x;
  if (c == 0 && g.nbt) g.nbt[0] += 1;
  if (c >= g.C) return;
  float lo, hi;
  if (g.first) {
    lo = g.bmin[c];
    hi = g.bmax[c];
  } else {
    lo = g.am * g.rmin[c] + g.cm * g.bmin[c];
    hi = g.am * g.rmax[c] + g.cm * g.bmax[c];
  }
  g.rmin[c] = lo;
  g.rmax[c] = hi;
  if (g.cmin) g.cmin[c] = lo;
  if (g.cmax) g.cmax[c] = hi;
}
__global__ __launch_bounds__(256) void mcaq_ema_multi_kernel(EmaMulti M) { ema_multi_body(M, (int)blockIdx.x); }

}  // namespace mcaq

namespace mcaq {
// 16-byte vector rows need 16-byte aligned bases of every per-element array
// the EMA segments of a launch; returns its workgroup count, or -1
static inline int ema_multi_args(const mcaq_ema_seg* segs, int nseg, EmaMulti& M) {
  int wg = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_ema_seg& e = segs[k];
    if (e.C < 1 || !e.batch_min || !e.batch_max || !e.running_min || !e.running_max) return -1;
    M.s[k] = EmaSeg{e.batch_min, e.batch_max, e.running_min, e.running_max, e.copy_min, e.copy_max,
                    reinterpret_cast<long long*>(e.num_batches), e.C, e.first ? 1 : 0, wg, (float)e.momentum,
                    (float)(1.0 - e.momentum)};
    wg += (e.C + 255) / 256;
  }
  M.nseg = nseg;
  return wg;
}
// kTile launches: power-of-two tile multiples, tiles >= 4 pixels wide,
// 16-byte rows (and m plane)
static inline bool qat_tile_ok(const mcaq_qat_scale* sc, int n) {
  for (int i = 0; i < n; ++i) {
    const NearestMap mh = nearest_map(sc[i].ht, sc[i].H), mw = nearest_map(sc[i].wt, sc[i].W);
    if (mh.shift < 0 || mw.shift < 2 || (sc[i].W & 3) != 0 || (((uintptr_t)sc[i].m) & 15) != 0) return false;
  }
  return true;
}
static inline bool qat_aligned16(const mcaq_qat_scale& s, bool bwd) {
  uintptr_t u = (uintptr_t)s.x;
  u |= bwd ? ((uintptr_t)s.g | (uintptr_t)s.gx) : (uintptr_t)s.y;
  return (u & 15) == 0;
}
}  // namespace mcaq

extern "C" {

size_t mcaq_qat_work_floats(int B, int C, int H, int W) {
  return 2 * (size_t)((C + 31) / 32) * (size_t)B * (size_t)H * (size_t)W;
}

static int qat_args(const mcaq_qat_scale* scales, int nscales, bool bwd, mcaq::QatArgs& a, int& blocks) {
  if (nscales < 1 || nscales > 3 || !scales) return (int)hipErrorInvalidValue;
  int units = 0;
  blocks = 0;
  for (int i = 0; i < nscales; ++i) {
    const mcaq_qat_scale& s = scales[i];
    if (s.B < 1 || s.C < 1 || s.H < 1 || s.W < 1 || s.ht < 1 || s.wt < 1 || s.ht > s.H || s.wt > s.W ||
        s.W > QAT_FOLD_LDS ||
        !s.x || !s.bits || !s.xmin || !s.xmax)
      return (int)hipErrorInvalidValue;
    if (bwd ? (!s.g || !s.gx || !s.work) : !s.y) return (int)hipErrorInvalidValue;
    // in-launch fold: col fits the lent LDS, and a 256-pixel unit touches < 32 bands
    if (bwd && s.arrive && (s.W > QAT_FUSED_MAXW || s.W < 16)) return (int)hipErrorInvalidValue;
    a.s[i] = s;
    a.s[i].unit_begin = units;
    a.s[i].block_begin = blocks;
    units += s.B * ((s.H * s.W + 255) / 256) * ((s.C + 31) / 32);
    blocks += s.B * s.ht;          // fold: one workgroup per (image, tile row)
  }
  a.nscales = nscales;
  a.units_total = units;
  a.bb = mcaq::QatBudget{};
  return 0;
}

int mcaq_qat_forward(const mcaq_qat_scale* scales, int nscales, hipStream_t stream) {
  mcaq::QatArgs a;
  int blocks;
  const int e = qat_args(scales, nscales, false, a, blocks);
  if (e) return e;
  bool vec = true;
  for (int i = 0; i < nscales; ++i)
    vec = vec && ((scales[i].H * scales[i].W) & 3) == 0 && mcaq::qat_aligned16(scales[i], false);
  if (vec && mcaq::qat_tile_ok(scales, nscales))
    launch_k((mcaq::mcaq_qat_kernel<false, true, true>), dim3(a.units_total), dim3(256), 0, stream, a);
  else if (vec)
    launch_k((mcaq::mcaq_qat_kernel<false, true>), dim3(a.units_total), dim3(256), 0, stream, a);
  else
    launch_k((mcaq::mcaq_qat_kernel<false, false>), dim3(a.units_total), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

int mcaq_qat_forward_budget(const mcaq_qat_scale* scales, int nscales, const float* const* bits, const int* n,
                            int nseg, float target, float* avg, float* loss, hipStream_t stream) {
  mcaq::QatArgs a;
  int blocks;
  const int e = qat_args(scales, nscales, false, a, blocks);
  if (e) return e;
  if (!bits || !n || nseg < 1 || nseg > 3 || !avg) return (int)hipErrorInvalidValue;
  for (int k = 0; k < nseg; ++k) {
    if (!bits[k] || n[k] < 1) return (int)hipErrorInvalidValue;
    a.bb.bits[k] = bits[k];
    a.bb.n[k] = n[k];
  }
  a.bb.nseg = nseg; a.bb.target = target; a.bb.avg = avg; a.bb.loss = loss;
  bool vec = true;
  for (int i = 0; i < nscales; ++i)
    vec = vec && ((scales[i].H * scales[i].W) & 3) == 0 && mcaq::qat_aligned16(scales[i], false);
  if (vec && mcaq::qat_tile_ok(scales, nscales))
    launch_k((mcaq::mcaq_qat_kernel<false, true, true>), dim3(a.units_total + 1), dim3(256), 0, stream, a);
  else if (vec)
    launch_k((mcaq::mcaq_qat_kernel<false, true>), dim3(a.units_total + 1), dim3(256), 0, stream, a);
  else
    launch_k((mcaq::mcaq_qat_kernel<false, false>), dim3(a.units_total + 1), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

int mcaq_qat_backward(const mcaq_qat_scale* scales, int nscales, hipStream_t stream) {
  mcaq::QatArgs a;
  int blocks;
  const int e = qat_args(scales, nscales, true, a, blocks);
  if (e) return e;
  bool vec = true;
  for (int i = 0; i < nscales; ++i)
    vec = vec && ((scales[i].H * scales[i].W) & 3) == 0 && mcaq::qat_aligned16(scales[i], true);
  if (vec && mcaq::qat_tile_ok(scales, nscales))
    launch_k((mcaq::mcaq_qat_kernel<true, true, true>), dim3(a.units_total), dim3(256), 0, stream, a);
  else if (vec)
    launch_k((mcaq::mcaq_qat_kernel<true, true>), dim3(a.units_total), dim3(256), 0, stream, a);
  else
    launch_k((mcaq::mcaq_qat_kernel<true, false>), dim3(a.units_total), dim3(256), 0, stream, a);
  hipError_t le = hipGetLastError();
  if (le != hipSuccess) return (int)le;
  // the separate fold only for scales without arrival counters
  bool fold = false;
  for (int i = 0; i < nscales; ++i) fold = fold || ((scales[i].gm || scales[i].gb) && !a.s[i].arrive);
  if (fold) launch_k(mcaq::mcaq_qat_fold_kernel, dim3(blocks), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

int mcaq_ema_stats(const float* batch_min, const float* batch_max, float* running_min, float* running_max,
                   int C, double momentum, int first, hipStream_t stream) {
  if (C < 1 || !batch_min || !batch_max || !running_min || !running_max) return (int)hipErrorInvalidValue;
  const float am = (float)momentum, cm = (float)(1.0 - momentum);
  hipLaunchKernelGGL(mcaq::mcaq_ema_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, batch_min, batch_max,
                     running_min, running_max, C, am, cm, first ? 1 : 0, (float*)nullptr, (float*)nullptr,
                     (long long*)nullptr);
  return (int)hipGetLastError();
}

int mcaq_ema_stats_multi(const mcaq_ema_seg* segs, int nseg, hipStream_t stream) {
  if (!segs || nseg < 1 || nseg > 3) return (int)hipErrorInvalidValue;
  mcaq::EmaMulti M{};
  const int wg = ema_multi_args(segs, nseg, M);
  if (wg < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mcaq::mcaq_ema_multi_kernel, dim3(wg), dim3(256), 0, stream, M);
  return (int)hipGetLastError();
}

int mcaq_ema_stats_ex(const float* batch_min, const float* batch_max, float* running_min, float* running_max,
                      int C, double momentum, int first, float* copy_min, float* copy_max, long long* num_batches,
                      hipStream_t stream) {
  if (C < 1 || !batch_min || !batch_max || !running_min || !running_max) return (int)hipErrorInvalidValue;
  const float am = (float)momentum, cm = (float)(1.0 - momentum);
  hipLaunchKernelGGL(mcaq::mcaq_ema_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, batch_min, batch_max,
                     running_min, running_max, C, am, cm, first ? 1 : 0, copy_min, copy_max, num_batches);
  return (int)hipGetLastError();
}

}  // extern "C"
