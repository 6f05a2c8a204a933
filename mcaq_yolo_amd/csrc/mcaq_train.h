// mcaq_train.h - train-mode (QAT, BASELINE config 5) tile networks of the
// hook as fused kernels, replacing ~700 small ATen kernels of autograd glue
// per step (r02 DESIGN s.8) (included by mcaq_kernels.hip; C ABI in
// include/mcaq_hip.h):
//
//   bit mapper, train mode (bit_allocation.py:218-280, 120-130):
//     z = [C, C^2, log1p C] -> 3 x (Linear, BatchNorm1d over the batch's
//     tiles, ReLU) -> Linear -> sigmoid -> b_min + (b_max - b_min) h, x T,
//     straight-through clamp (and round);  forward = 4 launches (one per
//     batch-statistics barrier), backward = 4 + 1 (parameter reduction); or
//     (round 6) ONE launch per direction, the batch statistics exchanged
//     inside it as write-through granules (mapx_*, *_fused)
//   analyzer head backward (morphology.py:81-97, 309-354, 959-968):
//     bilateral adjoint per image, then the complexity MLP (Linear-LN-ReLU x2,
//     Linear, sigmoid) recomputed and differentiated per tile
//   soft mask backward (quantization.py:213-239): 5x5 smoothing and nearest
//     upsample adjoints, softmax, 1x1 conv, ReLU, 3x3 conv (zero pad)
//
// Forward values of the analyzer and the soft mask stay those of the morph
// kernel (bit-exact with the reference); these kernels are fp32 with their
// own summation orders (train-mode gradients are tolerance-checked, DESIGN
// s.4).  Parameter gradients: every workgroup writes partial sums of its
// tiles; one reduction launch sums them in workgroup order (deterministic).
#pragma once

namespace mcaq {

// v_mfma_f32_16x16x4_f32 (D = a k-ordered fp32 FMA chain over its 4 k; lane
// l: A[l & 15][l >> 4], B[l >> 4][l & 15], D rows 4 (l >> 4) + r, column l & 15)
typedef float tr_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ tr_f4 tr_mfma4(float a, float b, tr_f4 c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
#else
  return c;
#endif
}

// diagnostic build only (-DMCAQ_STAMPS): stage cycle stamps of the train
// kernels' workgroup 0 (tools/probe/train_stamps.py), slots 32..63
#if defined(MCAQ_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
#define TSTAMP(k)                                                                            \
  do {                                                                                       \
    __syncthreads();                                                                         \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_mcaq_stamps[(k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define TSTAMP(k) do {} while (0)
#endif


// ---- shared helpers --------------------------------------------------------
constexpr int TR_TPB = 64;          // tiles per workgroup (one per lane of a wave)

__device__ __forceinline__ float tr_sigmoid(float a) { return 1.0f / (1.0f + expf(-a)); }

// sum over the 64 lanes of a wave (every lane gets the total): DPP within
// rows of 16 (quad xor 1, xor 2, half-row and row mirrors), then the gfx950
// lane swaps across rows - no LDS round trips
template <int CTRL>
__device__ __forceinline__ float tr_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  v += tr_dpp<0xB1>(v);     // quad_perm [1,0,3,2]
  v += tr_dpp<0x4E>(v);     // quad_perm [2,3,0,1]
  v += tr_dpp<0x141>(v);    // row_half_mirror
  v += tr_dpp<0x140>(v);    // row_mirror
  {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v += __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
  }
  {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v += __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
  }
#endif
  return v;
}

// Chan / Welford combination of per-workgroup (count, mean, M2) partials in
// workgroup order -> batch mean and biased variance
__device__ __forceinline__ void chan_combine(const float* part, int nwg, int stride, int j, int nfeat,
                                             const float* cnt, float& mean, float& var) {
  float n = 0.0f, m = 0.0f, M2 = 0.0f;
  for (int w = 0; w < nwg; ++w) {
    const float nb = cnt[w];
    if (nb <= 0.0f) continue;
    const float mb = part[(size_t)w * stride + j], M2b = part[(size_t)w * stride + nfeat + j];
    const float nn = n + nb;
    const float d = mb - m;
    m = m + d * (nb / nn);
    M2 = M2 + M2b + d * d * (n * nb / nn);
    n = nn;
  }
  mean = m;
  var = n > 0.0f ? M2 / n : 0.0f;
}

// ---- parameter-gradient reduction ------------------------------------------
// sum_w part[w * stride + e] in workgroup order; the loads of 16 partials
// are issued before their adds (the sum is a chain of dependent adds, the
// loads are not: one memory latency per 16 partials instead of per partial)
// - the last, partial group too (clamped index, the surplus not added)
__device__ __forceinline__ float tr_ordered_sum(const float* __restrict__ part, int nwg, int stride, int e) {
  float s = 0.0f;
  for (int w = 0; w < nwg; w += 16) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = part[(size_t)imin_(w + k, nwg - 1) * stride + e];
#pragma unroll
    for (int k = 0; k < 16; ++k) s = w + k < nwg ? s + v[k] : s;
  }
  return s;
}

// out[e] (+)= sum_w part[w * stride + e], e < count, w in order
__global__ __launch_bounds__(256) void mcaq_tr_reduce_kernel(const float* __restrict__ part, int nwg, int stride,
                                                             int count, float* __restrict__ out, int accumulate) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= count) return;
  const float s = tr_ordered_sum(part, nwg, stride, e);
  out[e] = accumulate ? out[e] + s : s;
}

// ============================================================================
// bit mapper, train mode
// ============================================================================
// gradient layout (flat, floats): the torch parameter order of mapping_network
enum : int {
  MG_W1 = 0, MG_B1 = 96, MG_G1 = 128, MG_BE1 = 160, MG_W2 = 192, MG_B2 = 2240, MG_G2 = 2304, MG_BE2 = 2368,
  MG_W3 = 2432, MG_B3 = 4480, MG_G3 = 4512, MG_BE3 = 4544, MG_W4 = 4576, MG_B4 = 4608, MG_SIZE = 4609
};

struct MapperTrainArgs {
  mcaq_mapper_params P;
  const float* c;       // (n) complexity
  const float* gbits;   // (n) upstream gradient of the bit map (backward)
  float* bits;          // (n) forward output
  float* gc;            // (n) gradient of c (backward)
  float* work;          // mcaq_mapper_work_floats(n)
  float* gpart;         // backward parameter partials [nwg][MG_SIZE]
  int n, nwg;
  float min_bits, max_bits, temperature, momentum;   // temperature <= 0: none
  int round_bits, update_stats;
  // batch sharded over `gworld` ranks (process-group BatchNorm, one stage per
  // launch): gstat = every rank's (mean[64], M2[64], n) of the previous layer
  // (all-gathered, RANK_ENT floats each), read instead of this launch's
  // workgroup partials; gbsum = the BN sums (S1[64], S2[64]) of this stage's
  // layer all-reduced over the ranks; gstat1 = the gathered layer-1 entries
  // (their counts give the global tile count).  gworld = 0: one process.
  const float* gstat;
  const float* gbsum;
  const float* gstat1;
  int gworld;
  int wg0;              // first workgroup of this segment in a multi-segment launch (else 0)
  // fused launches (mcaq_mapper_train_forward_fused / _backward_fused): this
  // segment's granule region (3 exchanges x nwg x MAPX_STRIDE), its epoch
  // word and the buffer's status word (mapx_* below)
  unsigned long long* gx;
  unsigned* gep;
  unsigned* gst;
};
constexpr int RANK_ENT = 129;   // (mean[64], M2[64], n) of one rank

// work layout (floats)
struct MapperWork {
  // pre-BN activations (32 / 64 / 32 x n), sigmoid out, gradient scratch
  // (64 x n): feature-major, so a wave's 64 tiles (lanes) of one feature are
  // 256 contiguous bytes - coalesced loads and stores (tile-major rows made
  // every access 64 separate lines: the forward layer's stores and the
  // backward's g_y stores took ~6 us of a stage)
  float *a1, *a2, *a3, *o, *gy;
  float *part, *cnt;              // per-workgroup (mean[64], M2[64]) and counts
  float *stat;                    // 3 layers x (mean[64], rstd[64])
  float *bpart;                   // backward BN partials [2][nwg][2 x 64]
  float *rstat;                   // update_stats == 2: 3 layers x (mean[64], unbiased var[64]), deferred update
  int nwg;
  __host__ __device__ float* fpart(int layer) const { return part + (size_t)(layer & 1) * nwg * 128; }
  __host__ __device__ float* bpart_of(int stage) const { return bpart + (size_t)(stage & 1) * nwg * 128; }
};
// part / bpart are double-buffered by layer parity: a launch reads the
// partials the previous launch wrote while writing its own
__host__ __device__ inline size_t mapper_work_floats(int n) {
  const int nwg = (n + TR_TPB - 1) / TR_TPB;
  return (size_t)n * (32 + 64 + 32 + 1 + 64) + (size_t)2 * nwg * 128 + nwg + 3 * 128 + (size_t)2 * nwg * 128 + 64 +
         3 * 128;
}
__host__ __device__ inline MapperWork mapper_work(float* w, int n) {
  const int nwg = (n + TR_TPB - 1) / TR_TPB;
  MapperWork m;
  m.a1 = w; m.a2 = m.a1 + (size_t)n * 32; m.a3 = m.a2 + (size_t)n * 64; m.o = m.a3 + (size_t)n * 32;
  m.gy = m.o + n; m.part = m.gy + (size_t)n * 64; m.cnt = m.part + (size_t)2 * nwg * 128; m.stat = m.cnt + nwg;
  m.bpart = m.stat + 3 * 128;
  m.rstat = m.bpart + (size_t)2 * nwg * 128 + 64;
  m.nwg = nwg;
  return m;
}

// layer input dims / output dims: L1 3->32, L2 32->64, L3 64->32, L4 32->1
template <int L> struct MapL;
template <> struct MapL<1> { enum { K = 3, N = 32 }; };
template <> struct MapL<2> { enum { K = 32, N = 64 }; };
template <> struct MapL<3> { enum { K = 64, N = 32 }; };
template <> struct MapL<4> { enum { K = 32, N = 1 }; };
template <> struct MapL<0> { enum { K = 1, N = 1 }; };

// BN layer parameters of layer L (1..3)
__device__ __forceinline__ void map_bn(const mcaq_mapper_params& P, int L, const float*& g, const float*& be, float*& rm,
                                       float*& rv, long long*& nbt) {
  g = L == 1 ? P.g1 : (L == 2 ? P.g2 : P.g3);
  be = L == 1 ? P.be1 : (L == 2 ? P.be2 : P.be3);
  rm = L == 1 ? P.rm1 : (L == 2 ? P.rm2 : P.rm3);
  rv = L == 1 ? P.rv1 : (L == 2 ? P.rv2 : P.rv3);
  nbt = L == 1 ? P.nbt1 : (L == 2 ? P.nbt2 : P.nbt3);
}

constexpr int MW = 8;               // waves per mapper workgroup (lane = tile, waves split the features)
constexpr int MAPPER_COOP_MAX_WG = 256;   // one-launch mapper (grid barrier / granule exchanges) up to this many workgroups
constexpr int MTH = 64 * MW;

// ---- fused mapper launches: the batch-statistic partials exchanged inside
// the launch.  Each of the three exchanges per direction (forward: layer
// moments of stages 1..3; backward: BN sums of stages 4..2) is a region of
// nwg x MAPX_STRIDE 8-byte granules {tag, value}: the data is the flag
// (cdna_hip_programming.md s.6 Guideline 16, R2) - every producer store and
// every consumer load of a granule is an agent-scope (write-through, sc1)
// access and the consumer re-reads until every tag matches, so neither side
// takes a fence or a counter.  tag = epoch * 8 + exchange: the segment's
// epoch word is read by every wave at launch and advanced by the segment's
// first workgroup after its last exchange (every workgroup of the segment has
// read it by then), so granules of earlier launches never match.  A buffer
// serves one segment layout and starts zeroed (train_step._sync_buffer).
// Bounded spins: a timeout sets the status word and goes on (tests check it).
#ifndef MCAQ_MAPX_SLEEP   // s_sleep between two sweeps of unpublished granules (A/B build option)
#define MCAQ_MAPX_SLEEP 2
#endif
typedef unsigned long long mapx_t;
#if defined(MCAQ_STAMPS_WG)
__device__ unsigned long long g_mapx_wg[64];   // diagnostic build only (tools/probe/mapx_skew.py)
#endif
constexpr int MAPX_STRIDE = 129;   // granules per workgroup per exchange: [0, 128) partials, 128 count
constexpr int MAPX_HDR = 64;       // header words (epochs of the segments, status at MAPX_STATUS)
constexpr int MAPX_STATUS = 32;

__device__ __forceinline__ void mapx_put(mapx_t* g, unsigned tag, float v) {
  __hip_atomic_store(g, ((mapx_t)tag << 32) | (mapx_t)__float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
#ifndef MCAQ_MAPX_PIPE   // > 0: polls issued every s_sleep(MCAQ_MAPX_PIPE) with the previous one in flight (A/B)
#define MCAQ_MAPX_PIPE 0
#endif
template <int R>
__device__ __forceinline__ void mapx_get(mapx_t* const (&g)[R], unsigned tag, float (&v)[R], unsigned* status) {
  if constexpr (MCAQ_MAPX_PIPE > 0) {
    // two polls in flight: the next batch of loads is issued before the
    // previous one is checked, so a publish is seen about one round trip
    // after it lands instead of up to two
    mapx_t a[R];
#pragma unroll
    for (int r = 0; r < R; ++r) a[r] = __hip_atomic_load(g[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned spins = 0;; ++spins) {
      __builtin_amdgcn_s_sleep(MCAQ_MAPX_PIPE);
      mapx_t b[R];
#pragma unroll
      for (int r = 0; r < R; ++r) b[r] = __hip_atomic_load(g[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bool ok = true;
#pragma unroll
      for (int r = 0; r < R; ++r) ok = ok && (unsigned)(a[r] >> 32) == tag;
      if (ok) {
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = __uint_as_float((unsigned)a[r]);
        return;
      }
      if (spins >= (1u << 20)) {
        __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = __uint_as_float((unsigned)b[r]);
        return;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) a[r] = b[r];
    }
  }
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const mapx_t x = __hip_atomic_load(g[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v[r] = __uint_as_float((unsigned)x);
      ok = ok && (unsigned)(x >> 32) == tag;
    }
    if (ok) return;
    if (spins >= (1u << 20)) {
      __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if constexpr (MCAQ_MAPX_SLEEP > 0) __builtin_amdgcn_s_sleep(MCAQ_MAPX_SLEEP);
  }
}
// this launch's epoch of the segment, in a register of every wave
__device__ __forceinline__ unsigned mapx_epoch(const MapperTrainArgs& A) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(A.gep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ mapx_t* mapx_region(const MapperTrainArgs& A, int x) {
  return A.gx + (size_t)(x - 1) * A.nwg * MAPX_STRIDE;
}

// per-workgroup (mean, M2) of feature j over this workgroup's valid tiles;
// MW waves x 64 tiles, each wave 1/MW of the features.
// v[f]: this lane's tile's value of feature f0 + f (f < NQ); kX: published
// as granules of `gx` with `tag` instead of stored to `part`
template <int NQ, bool kX = false>
__device__ __forceinline__ void wg_moments(const float (&v)[NQ], bool valid, float nvalid, int f0, float* part, int nfeat,
                                           mapx_t* gx = nullptr, unsigned tag = 0) {
#pragma unroll
  for (int f = 0; f < NQ; ++f) {
    const float s = wave_sum(valid ? v[f] : 0.0f);
    const float mean = s / nvalid;
    const float d = valid ? v[f] - mean : 0.0f;
    const float M2 = wave_sum(d * d);
    if ((threadIdx.x & 63) == 0) {
      if constexpr (kX) {
        mapx_put(gx + f0 + f, tag, mean);
        mapx_put(gx + nfeat + f0 + f, tag, M2);
      } else {
        part[f0 + f] = mean; part[nfeat + f0 + f] = M2;
      }
    }
  }
}

// BatchNorm1d running-stats update (momentum form of torch's batch_norm)
__device__ __forceinline__ void map_running_update(float* rm, float* rv, long long* nbt, int j, float momentum,
                                                   float mean, float unb) {
  rm[j] = (1.0f - momentum) * rm[j] + momentum * mean;
  rv[j] = (1.0f - momentum) * rv[j] + momentum * unb;
  if (j == 0 && nbt) nbt[0] += 1;
}

// deferred running-stats updates (update_stats == 2) of up to MAPPER_RU_MAX
// forwards, applied in list order: the same arithmetic, in the same order, as
// those forwards updating the buffers themselves one after another
constexpr int MAPPER_RU_MAX = 8;
struct MapperRunningArgs {
  mcaq_mapper_params P;
  const float* rstat[MAPPER_RU_MAX];
  int count;
  float momentum;
};
__device__ __forceinline__ void mapper_running_body(const MapperRunningArgs& A) {
  // per layer: the running buffers and every forward's statistics loaded
  // once, the count updates applied in list order in registers (the values
  // of map_running_update applied one after another), stored once
  const int j = threadIdx.x;
#pragma unroll
  for (int L = 1; L <= 3; ++L) {
    const int N = L == 2 ? 64 : 32;
    if (j < N) {
      const float* g; const float* be; float* rm; float* rv; long long* nbt;
      map_bn(A.P, L, g, be, rm, rv, nbt);
      float mk[MAPPER_RU_MAX], uk[MAPPER_RU_MAX];
#pragma unroll
      for (int k = 0; k < MAPPER_RU_MAX; ++k) {
        const float* r = A.rstat[k < A.count ? k : 0];
        mk[k] = r[(L - 1) * 128 + j];
        uk[k] = r[(L - 1) * 128 + 64 + j];
      }
      float m = rm[j], v = rv[j];
#pragma unroll
      for (int k = 0; k < MAPPER_RU_MAX; ++k) {
        if (k >= A.count) break;
        m = (1.0f - A.momentum) * m + A.momentum * mk[k];
        v = (1.0f - A.momentum) * v + A.momentum * uk[k];
      }
      rm[j] = m;
      rv[j] = v;
      if (j == 0 && nbt) nbt[0] += A.count;
    }
  }
}
__global__ __launch_bounds__(64) void mcaq_mapper_running_kernel(MapperRunningArgs A) { mapper_running_body(A); }

// the quantizers' EMA launch with the mapper's deferred running-statistics
// update as one extra workgroup (threads 0..63): both are a few hundred
// floats, and the EMA launch directly follows the mapper in the train step
struct EmaRunArgs { EmaMulti M; MapperRunningArgs R; int ema_wg; };
__global__ __launch_bounds__(256) void mcaq_ema_running_kernel(EmaRunArgs a) {
  if ((int)blockIdx.x >= a.ema_wg) {
    if (threadIdx.x < 64) mapper_running_body(a.R);
    return;
  }
  ema_multi_body(a.M, (int)blockIdx.x);
}

// the soft-mask pass B launch with the quantizers' EMA and the mapper's
// running-statistics update riding along as workgroups wg0.. (the train
// step's soft-mask planes do not read them; the quantizer launch after does)
static_assert(TILES_THREADS == 256, "the EMA workgroups riding on pass B take 256 channels each");
template <int TS, bool kSmo>
__global__ __launch_bounds__(TILES_THREADS, MCAQ_TILES_MINW) void mcaq_tiles_ema_kernel(MorphArgs a, int wlds,
                                                                                     EmaRunArgs e, int wg0) {
  if ((int)blockIdx.x >= wg0) {
    const int x = (int)blockIdx.x - wg0;
    if (x < e.ema_wg) ema_multi_body(e.M, x);
    else if (e.R.count > 0 && threadIdx.x < 64) mapper_running_body(e.R);
    return;
  }
  tiles_body<TS, kSmo>(a, wlds);
}

// batch statistics of layer L from the forward partials: mean, rstd of every
// feature in LDS (and, once per launch, the running-stats update).  The MW
// waves combine interleaved subsets of the workgroups' partials in parallel
// (Chan), then one thread per feature combines the MW results.
template <int L, bool kX = false>
__device__ void map_stats(const MapperTrainArgs& A, const MapperWork& W, float* s_mean, float* s_rstd, float* s_tmp,
                          unsigned E = 0) {
  constexpr int N = MapL<L>::N;
  const int tid = threadIdx.x, j = tid & 63, part = tid >> 6;
  if (j < N) {
    float n = 0.0f, m = 0.0f, M2 = 0.0f;
    const float* fp = W.fpart(L);
    // one process: this launch's workgroup partials; sharded: every rank's
    const int nsrc = A.gworld > 0 ? A.gworld : A.nwg;
    const bool gs = A.gworld > 0;
    // 4 partials of the wave's share loaded before any is combined (clamped
    // index: no load behind the empty-partial test, which made every
    // partial a round trip of its own), combined in the same order
    for (int w0 = part; w0 < nsrc; w0 += 4 * MW) {
      float nbv[4], mbv[4], m2v[4];
      if constexpr (kX) {
        // fused launch: exchange L's granules (the same values, re-read until published)
        mapx_t* const gx = mapx_region(A, L);
        mapx_t* gp[12];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          mapx_t* const b = gx + (size_t)imin_(w0 + r * MW, nsrc - 1) * MAPX_STRIDE;
          gp[3 * r] = b + 128; gp[3 * r + 1] = b + j; gp[3 * r + 2] = b + N + j;
        }
        float v[12];
        mapx_get<12>(gp, E * 8u + (unsigned)L, v, A.gst);
#pragma unroll
        for (int r = 0; r < 4; ++r) { nbv[r] = v[3 * r]; mbv[r] = v[3 * r + 1]; m2v[r] = v[3 * r + 2]; }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int w = imin_(w0 + r * MW, nsrc - 1);
          nbv[r] = gs ? A.gstat[(size_t)w * RANK_ENT + 128] : W.cnt[w];
          mbv[r] = gs ? A.gstat[(size_t)w * RANK_ENT + j] : fp[(size_t)w * 128 + j];
          m2v[r] = gs ? A.gstat[(size_t)w * RANK_ENT + 64 + j] : fp[(size_t)w * 128 + N + j];
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float nb = w0 + r * MW < nsrc ? nbv[r] : 0.0f;
        if (nb <= 0.0f) continue;
        const float mb = mbv[r], M2b = m2v[r];
        const float nn = n + nb, d = mb - m;
        m = m + d * (nb / nn);
        M2 = M2 + M2b + d * d * (n * nb / nn);
        n = nn;
      }
    }
    s_tmp[part * 192 + j] = n; s_tmp[part * 192 + 64 + j] = m; s_tmp[part * 192 + 128 + j] = M2;
  }
  __syncthreads();
  if (tid < N) {
    float n = 0.0f, m = 0.0f, M2 = 0.0f;
#pragma unroll
    for (int p = 0; p < MW; ++p) {
      const float nb = s_tmp[p * 192 + tid], mb = s_tmp[p * 192 + 64 + tid], M2b = s_tmp[p * 192 + 128 + tid];
      if (nb <= 0.0f) continue;
      const float nn = n + nb, d = mb - m;
      m = m + d * (nb / nn);
      M2 = M2 + M2b + d * d * (n * nb / nn);
      n = nn;
    }
    const float mean = m, var = n > 0.0f ? M2 / n : 0.0f;
    const float rstd = 1.0f / sqrtf(var + 1e-5f);
    s_mean[tid] = mean; s_rstd[tid] = rstd;
    if ((int)blockIdx.x == A.wg0) {
      W.stat[(L - 1) * 128 + tid] = mean;
      W.stat[(L - 1) * 128 + 64 + tid] = rstd;
      if (A.update_stats) {
        const float nf = n;   // the batch's tile count (all ranks' when sharded)
        const float unb = nf > 1.0f ? var * (nf / (nf - 1.0f)) : var;
        if (A.update_stats == 2) {
          // deferred: the caller applies the update later, in its own order
          // (several hook scales on concurrent streams share these buffers)
          W.rstat[(L - 1) * 128 + tid] = mean;
          W.rstat[(L - 1) * 128 + 64 + tid] = unb;
        } else {
          const float* g; const float* be; float* rm; float* rv; long long* nbt;
          map_bn(A.P, L, g, be, rm, rv, nbt);
          map_running_update(rm, rv, nbt, tid, A.momentum, mean, unb);
        }
      }
    }
  }
}

// stage S (1..4) of the train-mode forward
struct MapFwdLds {
  float in[TR_TPB][65];     // this workgroup's tiles' layer inputs
  float mean[64], rstd[64];
  float tmp[MW * 192];
  float w[64 * 34];         // stages 2 / 3: the layer's weights W[f][k] at f * (K + 2) + k (conflict-free MFMA B reads)
};

// kX (fused launch): the moments published as exchange S's granules, the
// previous layer's read from exchange S - 1 (epoch E); the workgroup's own
// activations handed to the next stage in LDS (s_a: [tile][feature]; the
// global copy stays for the backward launch)
template <int S, bool kX = false>
__device__ __forceinline__ void mapper_fwd_stage(const MapperTrainArgs& A, MapFwdLds& L, unsigned E = 0,
                                                 float (*s_a)[65] = nullptr) {
  float (*s_in)[65] = L.in;
  float* s_mean = L.mean;
  float* s_rstd = L.rstd;
  float* s_tmp = L.tmp;
  const MapperWork W = mapper_work(A.work, A.n);
  const mcaq_mapper_params& P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, q = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgi = (int)blockIdx.x - A.wg0;   // workgroup within this segment
  const int t = wgi * TR_TPB + lane;
  const bool valid = t < A.n;
  const int tc = valid ? t : A.n - 1;
  const float nvalid = (float)imin_(TR_TPB, A.n - wgi * TR_TPB);
  if constexpr (S == 2) TSTAMP(50);
  // stages 2 / 3: the layer's weights (K x N = 2048 floats, 4 a thread,
  // coalesced) first, into LDS below - the FMA loop then reads broadcast LDS
  // vectors instead of waiting on ~32 dependent scalar-load batches
  constexpr bool kWL = S == 2 || S == 3;
  constexpr int WN = kWL ? MapL<S>::K * MapL<S>::N : MTH;
  static_assert(WN % MTH == 0 && WN <= 64 * 32, "mapper weight staging");
  float wst[WN / MTH];
  // ... and this lane's biases of the MFMA layer (the accumulators' initial
  // values: loaded where they are used, each MFMA chain waited on them)
  constexpr int FPWB = kWL ? (MapL<S>::N / 16) / 2 : 1;
  float bpre[FPWB];
  if constexpr (kWL) {
    const float* wsrc = S == 2 ? P.w2 : P.w3;
#pragma unroll
    for (int i = 0; i < WN / MTH; ++i) wst[i] = wsrc[tid + i * MTH];
    const float* bsrc = S == 2 ? P.b2 : P.b3;
#pragma unroll
    for (int i = 0; i < FPWB; ++i) bpre[i] = bsrc[((q >> 2) + 2 * i) * 16 + (lane & 15)];
  }
  // this lane's previous-layer activations first: in flight through the
  // batch statistics below
  constexpr int KP = S == 2 ? 32 : (S == 3 ? 64 : 32);
  float apv[S >= 2 ? KP / MW : 1];
  if constexpr (S >= 2) {
    const float* aprev = S == 2 ? W.a1 : (S == 3 ? W.a2 : W.a3);
#pragma unroll
    for (int i = 0; i < KP / MW; ++i)
      apv[i] = kX ? s_a[tc - wgi * TR_TPB][q + i * MW] : aprev[(size_t)(q + i * MW) * A.n + tc];
  }
  if constexpr (S >= 2) map_stats<S - 1, kX>(A, W, s_mean, s_rstd, s_tmp, E);
  if constexpr (S == 2) TSTAMP(51);
  if constexpr (S == 2) TSTAMP(52);
  // ---- layer inputs of this workgroup's tiles -> s_in
  if constexpr (S == 1) {
    if (q == 0) {
      const float c = clampf_(A.c[tc], 0.0f, 1.0f);
      s_in[lane][0] = c; s_in[lane][1] = c * c; s_in[lane][2] = log1pf(c);
    }
  }
  __syncthreads();
  if constexpr (S >= 2) {
    // h = relu(gamma (a - mean) rstd + beta) of the previous layer
    const float* g = S == 2 ? P.g1 : (S == 3 ? P.g2 : P.g3);
    const float* be = S == 2 ? P.be1 : (S == 3 ? P.be2 : P.be3);
#pragma unroll
    for (int i = 0; i < KP / MW; ++i) {
      const int k = q + i * MW;
      const float a = apv[i];
      const float y = g[k] * ((a - s_mean[k]) * s_rstd[k]) + be[k];
      s_in[lane][k] = y > 0.0f ? y : 0.0f;
    }
    if constexpr (kWL) {
      // rows padded to K + 2 floats: the MFMA B reads (16 rows x 2 columns a
      // half-wave) hit 32 different banks
      constexpr int KL = MapL<S>::K;
#pragma unroll
      for (int i = 0; i < WN / MTH; ++i) {
        const int e = tid + i * MTH;
        L.w[(e / KL) * (KL + 2) + (e % KL)] = wst[i];
      }
    }
    __syncthreads();
  }
  if constexpr (S == 2) TSTAMP(53);
  if constexpr (S == 2 || S == 3) {
    // the layer (64 tiles x N) = h (64 x K) W^T (K x N) + b as 16 x 16 blocks
    // on v_mfma_f32_16x16x4_f32 (k in steps of 4, the bias as the initial
    // accumulator): wave q owns tile block q & 3 and feature blocks
    // (q >> 2) + 2 i; a lane holds 4 tiles (rows 4 lk + r) of feature 16 fb + lr.
    // The workgroup moments: sums over a lane's 4 tiles in order, the column's
    // 4 lanes (xor 16, xor 32), the 4 tile blocks in order - mean, then M2
    constexpr int K = MapL<S>::K, N = MapL<S>::N, FPW = (N / 16) / 2;
    const int lr = lane & 15, lk = lane >> 4, mtb = q & 3;
    float* aout = S == 2 ? W.a2 : W.a3;
    float* red1 = s_tmp;                 // [4 tile blocks][64] sums
    float* red2 = s_tmp + 256;           //   ... squared deviations
    static_assert(FPW == FPWB, "bias prefetch");
    float bq[FPW];
#pragma unroll
    for (int i = 0; i < FPW; ++i) bq[i] = bpre[i];
    tr_f4 d[FPW];
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      const int f = ((q >> 2) + 2 * i) * 16 + lr;
      d[i] = tr_f4{bq[i], bq[i], bq[i], bq[i]};
#pragma unroll
      for (int st = 0; st < K / 4; ++st) d[i] = tr_mfma4(s_in[mtb * 16 + lr][4 * st + lk], L.w[f * (K + 2) + 4 * st + lk], d[i]);
      float sm = 0.0f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tg = wgi * TR_TPB + mtb * 16 + 4 * lk + r;
        if (tg < A.n) { aout[(size_t)f * A.n + tg] = d[i][r]; sm += d[i][r]; }
        if constexpr (kX) s_a[mtb * 16 + 4 * lk + r][f] = d[i][r];
      }
      sm += __shfl_xor(sm, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      if (lk == 0) red1[mtb * 64 + f] = sm;
    }
    if constexpr (S == 2) TSTAMP(54);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      const int f = ((q >> 2) + 2 * i) * 16 + lr;
      const float mean = (((red1[f] + red1[64 + f]) + red1[128 + f]) + red1[192 + f]) / nvalid;
      float s2 = 0.0f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tg = wgi * TR_TPB + mtb * 16 + 4 * lk + r;
        const float dv = tg < A.n ? d[i][r] - mean : 0.0f;
        s2 += dv * dv;
      }
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (lk == 0) red2[mtb * 64 + f] = s2;
    }
    __syncthreads();
    if (tid < N) {
      const float pm = (((red1[tid] + red1[64 + tid]) + red1[128 + tid]) + red1[192 + tid]) / nvalid;
      const float p2 = ((red2[tid] + red2[64 + tid]) + red2[128 + tid]) + red2[192 + tid];
      if constexpr (kX) {
        mapx_t* const gx = mapx_region(A, S) + (size_t)wgi * MAPX_STRIDE;
        mapx_put(gx + tid, E * 8u + S, pm);
        mapx_put(gx + N + tid, E * 8u + S, p2);
      } else {
        float* part = W.fpart(S) + (size_t)wgi * 128;
        part[tid] = pm;
        part[N + tid] = p2;
      }
    }
    if (tid == 0) {
      if constexpr (kX) mapx_put(mapx_region(A, S) + (size_t)wgi * MAPX_STRIDE + 128, E * 8u + S, nvalid);
      else W.cnt[wgi] = nvalid;
    }
    if constexpr (S == 2) TSTAMP(55);
  } else if constexpr (S <= 3) {
    constexpr int K = MapL<S>::K, N = MapL<S>::N, NQ = N / MW;
    const float* w = S == 1 ? P.w1 : L.w;
    const float* bb = S == 1 ? P.b1 : (S == 2 ? P.b2 : P.b3);
    float* aout = S == 1 ? W.a1 : (S == 2 ? W.a2 : W.a3);
    float x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = s_in[lane][k];
    // the wave's biases first: inside the loop each load would wait behind
    // the previous output's store (the compiler cannot tell bb from aout)
    float bq[NQ];
#pragma unroll
    for (int f = 0; f < NQ; ++f) bq[f] = bb[q * NQ + f];
    // k outer, the NQ outputs' FMA chains interleaved (each still runs over
    // k in order from its bias)
    float o[NQ];
#pragma unroll
    for (int f = 0; f < NQ; ++f) o[f] = bq[f];
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int f = 0; f < NQ; ++f) o[f] = fmaf(w[(q * NQ + f) * K + k], x[k], o[f]);
    }
#pragma unroll
    for (int f = 0; f < NQ; ++f) {
      if (valid) aout[(size_t)(q * NQ + f) * A.n + t] = o[f];
      if constexpr (kX) s_a[lane][q * NQ + f] = o[f];
    }
    if constexpr (S == 2) TSTAMP(54);
    if constexpr (kX) {
      mapx_t* const gx = mapx_region(A, S) + (size_t)wgi * MAPX_STRIDE;
      wg_moments<NQ, true>(o, valid, nvalid, q * NQ, nullptr, N, gx, E * 8u + S);
      if (tid == 0) mapx_put(gx + 128, E * 8u + S, nvalid);
    } else {
      wg_moments<NQ>(o, valid, nvalid, q * NQ, W.fpart(S) + (size_t)wgi * 128, N);
      if (tid == 0) W.cnt[wgi] = nvalid;
    }
    if constexpr (S == 2) TSTAMP(55);
  } else {
    // last layer + sigmoid + bit range, temperature, clamp (+ round)
    if (q == 0 && valid) {
      float acc = P.b4[0];
#pragma unroll 8
      for (int k = 0; k < 32; ++k) acc = fmaf(P.w4[k], s_in[lane][k], acc);
      const float o = tr_sigmoid(acc);
      W.o[t] = o;
      float bv = A.min_bits + (A.max_bits - A.min_bits) * o;
      if (A.temperature > 0.0f) bv = bv * A.temperature;
      bv = clampf_(bv, A.min_bits, A.max_bits);
      if (A.round_bits) bv = rintf(bv);
      A.bits[t] = bv;
    }
  }
}

template <int S>
__global__ __launch_bounds__(MTH) void mcaq_mapper_fwd_kernel(MapperTrainArgs A) {
  __shared__ MapFwdLds L;
  mapper_fwd_stage<S>(A, L);
}

// grid-wide barrier of a launch whose workgroups are all resident (the mapper
// grids are n / 64 <= a few hundred 512-thread workgroups): every wave
// releases its writes at agent scope, one thread counts in and waits, every
// wave acquires.  `bar` is a persistent zeroed counter the launch leaves
// zeroed (mapper_grid_exit); a bounded spin never hangs the GPU.
__device__ __forceinline__ void mapper_grid_sync(unsigned* bar, unsigned target) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && spins < (1u << 24)) {
      __builtin_amdgcn_s_sleep(1);
      ++spins;
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// the last workgroup out resets the counters for the next launch on the stream
__device__ __forceinline__ void mapper_grid_exit(unsigned* bar, int nwg) {
  if (threadIdx.x == 0) {
    const unsigned out = __hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (out == (unsigned)nwg - 1) {
      __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(bar + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// the four forward stages in one launch, grid barriers between them
__global__ __launch_bounds__(MTH) void mcaq_mapper_fwd_coop_kernel(MapperTrainArgs A, unsigned* bar) {
  __shared__ MapFwdLds L;
  const unsigned n = (unsigned)A.nwg;
  mapper_fwd_stage<1>(A, L);
  mapper_grid_sync(bar, n);
  mapper_fwd_stage<2>(A, L);
  mapper_grid_sync(bar, 2 * n);
  mapper_fwd_stage<3>(A, L);
  mapper_grid_sync(bar, 3 * n);
  mapper_fwd_stage<4>(A, L);
  mapper_grid_exit(bar, A.nwg);
}

// backward stage S (4, 3, 2, 1): gradient of layer S's output activation ->
// (BN S-1 backward inputs, weight partials of layer S)
//   S = 4: g_bits -> g_a4 -> g_h3 -> g_y3 (through ReLU), partials of W4 / b4
//          and of BN3 (sum g_y3, sum g_y3 xhat3)
//   S = 3, 2: g_y(S) + BN(S) sums -> g_a(S) -> W(S) / b(S) / BN(S) gamma-beta
//          partials, g_h(S-1) -> g_y(S-1), BN(S-1) partials
//   S = 1: g_y1 + BN1 sums -> g_a1 -> W1 / b1 partials, g_z -> g_c
struct MapBwdLds {
  float h[TR_TPB][65];     // this layer's input activations h(S-1)
  float g[TR_TPB][65];     // gradient of this layer's pre-activation a(S)
  float mean[64], rstd[64], sg[64], sgx[64];
  float tmp[MW * 128];
  float w[64 * 48];        // stages 3 / 2: the layer's weights W[j][k] at j * (K + 16) + k, for W^T g_a
};

// kX (fused launch): the BN(S-1) sums published as exchange 5 - S's granules,
// the BN(S) sums read from exchange 4 - S (epoch E); g_y handed from stage
// to stage in LDS (s_gy: [tile][feature]) instead of the global scratch
template <int S, bool kX = false>
__device__ __forceinline__ void mapper_bwd_stage(const MapperTrainArgs& A, MapBwdLds& L, unsigned E = 0,
                                                 float (*s_gy)[65] = nullptr) {
  float (*s_h)[65] = L.h;
  float (*s_g)[65] = L.g;
  float* s_mean = L.mean;
  float* s_rstd = L.rstd;
  float* s_sg = L.sg;
  float* s_sgx = L.sgx;
  float* s_tmp = L.tmp;
  const MapperWork W = mapper_work(A.work, A.n);
  const mcaq_mapper_params& P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, q = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgi = (int)blockIdx.x - A.wg0;   // workgroup within this segment
  const int t = wgi * TR_TPB + lane;
  const bool valid = t < A.n;
  const int tc = valid ? t : A.n - 1;
  float* gp = A.gpart + (size_t)wgi * MG_SIZE;
  float* bp = W.bpart_of(S) + (size_t)wgi * 128;   // BN(S-1) partials written here
  if constexpr (S == 3) TSTAMP(56);
  // stages 3 / 2: the layer's weights first (into LDS before the first
  // barrier; W^T g_a reads them as broadcast LDS vectors)
  constexpr bool kWL = S == 2 || S == 3;
  constexpr int WN = kWL ? MapL<S>::K * MapL<S>::N : MTH;
  static_assert(WN % MTH == 0 && WN <= 64 * 32, "mapper weight staging");
  float wst[WN / MTH];
  if constexpr (kWL) {
    const float* wsrc = S == 2 ? P.w2 : P.w3;
#pragma unroll
    for (int i = 0; i < WN / MTH; ++i) wst[i] = wsrc[tid + i * MTH];
  }
  // this lane's per-tile operands first, in flight through the BN sums:
  // g_y(S) and a(S) of step 1, a(S-1) of steps 2 and 4
  constexpr int N1 = S == 4 ? 1 : MapL<S == 4 ? 1 : S>::N;
  constexpr int KI = S == 4 ? 32 : (S == 1 ? 3 : MapL<S>::K);
  float gyp[S <= 3 ? N1 / MW : 1], asp[S <= 3 ? N1 / MW : 1];
  float ap2[S >= 2 ? KI / MW : 1], ap4[S >= 2 ? KI / MW : 1];   // ap4: SQ x SR values (below)
  // ... and BN(S)'s forward statistics and gamma for the BN backward (read
  // after the BN sums, each was one more memory round trip)
  float pmean = 0.0f, prstd = 0.0f, pgam[S <= 3 ? N1 / MW : 1];
  if constexpr (S <= 3) {
    const float* aS = S == 1 ? W.a1 : (S == 2 ? W.a2 : W.a3);
    const float* gS = S == 1 ? P.g1 : (S == 2 ? P.g2 : P.g3);
#pragma unroll
    for (int i = 0; i < N1 / MW; ++i) {
      const int j = q + i * MW;
      gyp[i] = kX ? s_gy[tc - wgi * TR_TPB][j] : W.gy[(size_t)j * A.n + tc];
      asp[i] = aS[(size_t)j * A.n + tc];
      pgam[i] = gS[j];
    }
    if (tid < N1) { pmean = W.stat[(S - 1) * 128 + tid]; prstd = W.stat[(S - 1) * 128 + 64 + tid]; }
  }
  // ... and the BN(S-1) statistics and affine parameters of the step-4
  // columns with that step's a(S-1) values (read after the W^T g_a loop, which
  // did not hide their latency).  Stages 3 / 2 run step 4 on MFMA: wave q
  // owns tile block q & 3 (16 tiles) and column blocks (q >> 2) + 2 i of
  // g_h; a lane holds 4 tiles (rows 4 lk + r) of column 16 kb + lr
  constexpr bool kMF = S == 2 || S == 3;
  constexpr int SQ = kMF ? (KI / 16) / 2 : (KI / MW > 0 ? KI / MW : 1);   // step-4 column sets of this lane
  constexpr int SR = kMF ? 4 : 1;                     // tiles per column set
  const int lr = lane & 15, lk = lane >> 4, mtb = q & 3;
  float smn[SQ], srs[SQ], sgm[SQ], sbe[SQ];
  if constexpr (S >= 2) {
    const float* ap = S == 4 ? W.a3 : (S == 3 ? W.a2 : W.a1);
#pragma unroll
    for (int i = 0; i < KI / MW; ++i) ap2[i] = ap[(size_t)(q + i * MW) * A.n + tc];
    const float* g = S == 4 ? P.g3 : (S == 3 ? P.g2 : P.g1);
    const float* be = S == 4 ? P.be3 : (S == 3 ? P.be2 : P.be1);
    constexpr int Lp = S - 1;
#pragma unroll
    for (int f = 0; f < SQ; ++f) {
      const int k = kMF ? ((q >> 2) + 2 * f) * 16 + lr : q * SQ + f;
#pragma unroll
      for (int r = 0; r < SR; ++r) {
        const int tt = kMF ? imin_(wgi * TR_TPB + mtb * 16 + 4 * lk + r, A.n - 1) : tc;
        ap4[f * SR + r] = ap[(size_t)k * A.n + tt];
      }
      smn[f] = W.stat[(Lp - 1) * 128 + k]; srs[f] = W.stat[(Lp - 1) * 128 + 64 + k];
      sgm[f] = g[k]; sbe[f] = be[k];
    }
  }
  if constexpr (S == 3) TSTAMP(42);
  // ---- 1. gradient of a(S) for this workgroup's tiles -> s_g
  if constexpr (S == 4) {
    if (q == 0) {
      float g = valid ? A.gbits[t] : 0.0f;   // straight-through round / clamp
      if (A.temperature > 0.0f) g = g * A.temperature;
      const float o = W.o[tc];
      s_g[lane][0] = valid ? (A.max_bits - A.min_bits) * g * (o * (1.0f - o)) : 0.0f;
    }
  } else {
    // BN(S) backward: g_a = gamma rstd (g_y - S1/n - xhat S2/n); the BN sums
    // over the workgroups' partials, MW interleaved subsets in parallel
    constexpr int N = MapL<S>::N;
    {
      const int j = tid & 63, part = tid >> 6;
      if (j < N) {
        float s1 = 0.0f, s2 = 0.0f;
        if constexpr (kX) {
          // fused launch: stage S + 1's sums from its granules, the same order
          mapx_t* const gx = mapx_region(A, 4 - S);
          for (int w0 = part; w0 < A.nwg; w0 += 4 * MW) {
            mapx_t* gp[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              mapx_t* const b = gx + (size_t)imin_(w0 + r * MW, A.nwg - 1) * MAPX_STRIDE;
              gp[2 * r] = b + j; gp[2 * r + 1] = b + 64 + j;
            }
            float v[8];
            mapx_get<8>(gp, E * 8u + (unsigned)(4 - S), v, A.gst);
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (w0 + r * MW < A.nwg) { s1 += v[2 * r]; s2 += v[2 * r + 1]; }
          }
        } else {
          const float* bq = W.bpart_of(S + 1);   // written by the previous launch (stage S + 1)
#pragma unroll 4
          for (int w = part; w < A.nwg; w += MW) { s1 += bq[(size_t)w * 128 + j]; s2 += bq[(size_t)w * 128 + 64 + j]; }
        }
        s_tmp[part * 128 + j] = s1; s_tmp[part * 128 + 64 + j] = s2;
      }
    }
    if constexpr (kWL) {
      // rows padded to K + 16 floats: the MFMA B reads (2 rows x 16 columns a
      // half-wave) hit 32 different banks
      constexpr int KL = MapL<S>::K;
#pragma unroll
      for (int i = 0; i < WN / MTH; ++i) {
        const int e = tid + i * MTH;
        L.w[(e / KL) * (KL + 16) + (e % KL)] = wst[i];
      }
    }
    __syncthreads();
    if (tid < N) {
      float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
      for (int p = 0; p < MW; ++p) { s1 += s_tmp[p * 128 + tid]; s2 += s_tmp[p * 128 + 64 + tid]; }
      // sharded: the BN backward takes the sums over every rank's tiles; the
      // gamma / beta gradients below stay this rank's own (summed by the
      // gradient all-reduce)
      s_sg[tid] = A.gworld > 0 ? A.gbsum[tid] : s1;
      s_sgx[tid] = A.gworld > 0 ? A.gbsum[64 + tid] : s2;
      s_mean[tid] = pmean; s_rstd[tid] = prstd;
      // gamma / beta gradients are the BN sums themselves: workgroup 0's
      // partial slot holds them, the others zero
      const int og = S == 1 ? MG_G1 : (S == 2 ? MG_G2 : MG_G3), ob = S == 1 ? MG_BE1 : (S == 2 ? MG_BE2 : MG_BE3);
      gp[og + tid] = wgi == 0 ? s2 : 0.0f;
      gp[ob + tid] = wgi == 0 ? s1 : 0.0f;
    }
    __syncthreads();
    float ntot = (float)A.n;
    if (A.gworld > 0) {
      ntot = 0.0f;
      for (int r = 0; r < A.gworld; ++r) ntot += A.gstat1[(size_t)r * RANK_ENT + 128];
    }
    const float inv_n = 1.0f / ntot;
#pragma unroll
    for (int i = 0; i < N / MW; ++i) {
      const int j = q + i * MW;
      const float gy = gyp[i];
      const float xh = (asp[i] - s_mean[j]) * s_rstd[j];
      s_g[lane][j] = valid ? pgam[i] * s_rstd[j] * (gy - s_sg[j] * inv_n - xh * (s_sgx[j] * inv_n)) : 0.0f;
    }
  }
  if constexpr (S == 3) TSTAMP(43);
  // ---- 2. this layer's input activations h(S-1) -> s_h
  constexpr int K = S == 4 ? 32 : (S == 1 ? 3 : MapL<S>::K);
  if constexpr (S == 1) {
    if (q == 0) {
      const float c = clampf_(A.c[tc], 0.0f, 1.0f);
      s_h[lane][0] = valid ? c : 0.0f; s_h[lane][1] = valid ? c * c : 0.0f; s_h[lane][2] = valid ? log1pf(c) : 0.0f;
    }
  } else {
    const float* g = S == 4 ? P.g3 : (S == 3 ? P.g2 : P.g1);
    const float* be = S == 4 ? P.be3 : (S == 3 ? P.be2 : P.be1);
    const int L = S - 1;
#pragma unroll
    for (int i = 0; i < K / MW; ++i) {
      const int k = q + i * MW;
      const float mean = W.stat[(L - 1) * 128 + k], rstd = W.stat[(L - 1) * 128 + 64 + k];
      const float y = g[k] * ((ap2[i] - mean) * rstd) + be[k];
      s_h[lane][k] = valid && y > 0.0f ? y : 0.0f;
    }
  }
  __syncthreads();
  if constexpr (S == 3) TSTAMP(44);
  // ---- 3. weight / bias partials of layer S: sum over the tiles of g_a (x) h
  {
    constexpr int NO = S == 4 ? 1 : MapL<S>::N;
    const int ow = S == 4 ? MG_W4 : (S == 3 ? MG_W3 : (S == 2 ? MG_W2 : MG_W1));
    const int ob = S == 4 ? MG_B4 : (S == 3 ? MG_B3 : (S == 2 ? MG_B2 : MG_B1));
    if constexpr (NO * K == 4 * MTH) {
      // the NO x K sums over the 64 tiles as one 16 x 16 block per wave on
      // v_mfma_f32_16x16x4_f32: a tile-ordered fp32 FMA chain u = 0..63 (the
      // values of the scalar loop), 2 LDS reads per 4 tiles instead of 5 per tile
      constexpr int TB = K / 16;              // column blocks; (NO / 16) x TB = MW blocks
      static_assert((NO / 16) * TB == MW, "one 16 x 16 block per wave");
      const int jb = q / TB, kb = q - (q / TB) * TB;
      const int lr = lane & 15, lk = lane >> 4;
      tr_f4 d = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int st = 0; st < TR_TPB / 4; ++st)
        d = tr_mfma4(s_g[4 * st + lk][jb * 16 + lr], s_h[4 * st + lk][kb * 16 + lr], d);
#pragma unroll
      for (int r = 0; r < 4; ++r) gp[ow + (jb * 16 + 4 * lk + r) * K + kb * 16 + lr] = d[r];
    } else {
      for (int e = tid; e < NO * K; e += MTH) {
        const int j = e / K, k = e - (e / K) * K;
        float s = 0.0f;
#pragma unroll 8
        for (int u = 0; u < TR_TPB; ++u) s = fmaf(s_g[u][j], s_h[u][k], s);
        gp[ow + e] = s;
      }
    }
    for (int j = tid; j < NO; j += MTH) {
      float s = 0.0f;
#pragma unroll 8
      for (int u = 0; u < TR_TPB; ++u) s += s_g[u][j];
      gp[ob + j] = s;
    }
  }
  if constexpr (S == 3) TSTAMP(45);
  // ---- 4. gradient of the layer input: g_h = W^T g_a, through ReLU / BN(S-1)
  if constexpr (kMF) {
    // g_h (64 tiles x K) = g_a (64 x N) W (N x K) as 16 x 16 blocks on
    // v_mfma_f32_16x16x4_f32 (j in steps of 4 from 0), then per element
    // through ReLU / BN(S-1) as the scalar path below; the BN(S-1) partial
    // sums over the tiles: a lane's 4 tiles in order, the 4 lanes of a column
    // (xor 16, xor 32), the 4 tile blocks in order
    constexpr int NO = MapL<S>::N;
    static_assert(SQ * SR <= KI / MW, "step-4 operands");
    float* red4 = s_tmp;                 // [2][4 tile blocks][64]
#pragma unroll
    for (int f = 0; f < SQ; ++f) {
      const int kb = (q >> 2) + 2 * f, k = kb * 16 + lr;
      tr_f4 d = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int st = 0; st < NO / 4; ++st)
        d = tr_mfma4(s_g[mtb * 16 + lr][4 * st + lk], L.w[(4 * st + lk) * (K + 16) + k], d);
      float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tg = wgi * TR_TPB + mtb * 16 + 4 * lk + r;
        const float xh = (ap4[f * SR + r] - smn[f]) * srs[f];
        const float y = sgm[f] * xh + sbe[f];
        const float gy = (tg < A.n && y > 0.0f) ? d[r] : 0.0f;
        if constexpr (kX) s_gy[mtb * 16 + 4 * lk + r][k] = gy;
        else if (tg < A.n) W.gy[(size_t)k * A.n + tg] = gy;
        s1 += gy; s2 += gy * xh;
      }
      s1 += __shfl_xor(s1, 16, 64); s2 += __shfl_xor(s2, 16, 64);
      s1 += __shfl_xor(s1, 32, 64); s2 += __shfl_xor(s2, 32, 64);
      if (lk == 0) { red4[mtb * 64 + k] = s1; red4[256 + mtb * 64 + k] = s2; }
    }
    if constexpr (S == 3) TSTAMP(48);
    __syncthreads();
    if constexpr (S == 3) TSTAMP(46);
    if (tid < K) {
      const float b1 = ((red4[tid] + red4[64 + tid]) + red4[128 + tid]) + red4[192 + tid];
      const float b2 = ((red4[256 + tid] + red4[320 + tid]) + red4[384 + tid]) + red4[448 + tid];
      if constexpr (kX) {
        mapx_t* const gx = mapx_region(A, 5 - S) + (size_t)wgi * MAPX_STRIDE;
        mapx_put(gx + tid, E * 8u + (5 - S), b1);
        mapx_put(gx + 64 + tid, E * 8u + (5 - S), b2);
      } else {
        bp[tid] = b1;
        bp[64 + tid] = b2;
      }
    }
  } else if constexpr (S >= 2) {
    constexpr int NO = S == 4 ? 1 : MapL<S>::N;
    const float* w = S == 4 ? P.w4 : L.w;
    constexpr int NQ = K / MW;
    static_assert(NQ == KI / MW && NQ == SQ, "step-4 columns");
    float gyv[NQ], xhv[NQ];
    // rows j outer, the wave's NQ consecutive columns inner: one NQ-wide
    // broadcast read of W (LDS, or scalar for the 32-float W4) per row
    // instead of NQ strided ones (each output's sum still runs over j in order);
    // the BN(S-1) statistics / affine parameters (smn, srs, sgm, sbe) were
    // loaded at the top (in the store loop each load would wait behind the
    // previous column's g_y store: W.stat and W.gy share the work buffer)
    float accv[NQ];
#pragma unroll
    for (int f = 0; f < NQ; ++f) accv[f] = 0.0f;
#pragma unroll 8
    for (int j = 0; j < NO; ++j) {
      const float ga = s_g[lane][j];
#pragma unroll
      for (int f = 0; f < NQ; ++f) accv[f] = fmaf(w[j * K + q * NQ + f], ga, accv[f]);
    }
    if constexpr (S == 3) TSTAMP(48);
#pragma unroll
    for (int f = 0; f < NQ; ++f) {
      const int k = q * NQ + f;
      const float acc = accv[f];
      const float xh = (ap4[f] - smn[f]) * srs[f];
      const float y = sgm[f] * xh + sbe[f];
      const float gy = (valid && y > 0.0f) ? acc : 0.0f;
      gyv[f] = gy; xhv[f] = xh;
      if constexpr (kX) s_gy[lane][k] = gy;
      else if (valid) W.gy[(size_t)k * A.n + t] = gy;
    }
    __syncthreads();   // every lane has read its W.gy row of this launch's input (S < 4) before it is overwritten
    if constexpr (S == 3) TSTAMP(46);
    // BN(S-1) partial sums: sum g_y, sum g_y xhat
#pragma unroll
    for (int f = 0; f < NQ; ++f) {
      const float s1 = wave_sum(gyv[f]), s2 = wave_sum(gyv[f] * xhv[f]);
      if (lane == 0) {
        if constexpr (kX) {
          mapx_t* const gx = mapx_region(A, 5 - S) + (size_t)wgi * MAPX_STRIDE;
          mapx_put(gx + q * NQ + f, E * 8u + (5 - S), s1);
          mapx_put(gx + 64 + q * NQ + f, E * 8u + (5 - S), s2);
        } else {
          bp[q * NQ + f] = s1; bp[64 + q * NQ + f] = s2;
        }
      }
    }
  } else {
    // g_z = W1^T g_a1 -> g_c (through the clamp: torch passes the gradient on [0, 1])
    if (q == 0 && valid) {
      float g0 = 0.0f, g1 = 0.0f, g2 = 0.0f;
      for (int j = 0; j < 32; ++j) {
        const float ga = s_g[lane][j];
        g0 = fmaf(P.w1[j * 3 + 0], ga, g0); g1 = fmaf(P.w1[j * 3 + 1], ga, g1); g2 = fmaf(P.w1[j * 3 + 2], ga, g2);
      }
      const float craw = A.c[t];
      const float c = clampf_(craw, 0.0f, 1.0f);
      const float gcv = g0 + 2.0f * c * g1 + g2 / (1.0f + c);
      A.gc[t] = (craw >= 0.0f && craw <= 1.0f) ? gcv : 0.0f;
    }
  }
  if constexpr (S == 3) TSTAMP(47);
}

// sharded mapper: this rank's share of a batch statistic, in workgroup order.
// kind 0: (mean[64], M2[64], n) of layer `layer` from the forward partials
// (Chan's combination, as map_stats); kind 1: the BN sums (S1[64], S2[64])
// of layer `layer` from the backward partials of stage layer + 1
__global__ __launch_bounds__(64) void mcaq_mapper_reduce_kernel(const float* work, int n, int kind, int layer,
                                                                float* out) {
  const MapperWork W = mapper_work(const_cast<float*>(work), n);
  const int j = threadIdx.x;
  const int N = layer == 2 ? 64 : 32;
  if (kind == 0) {
    float c = 0.0f, m = 0.0f, M2 = 0.0f;
    const float* fp = W.fpart(layer);
    for (int w = 0; w < W.nwg; ++w) {
      const float nb = W.cnt[w];
      if (nb <= 0.0f || j >= N) continue;
      const float mb = fp[(size_t)w * 128 + j], M2b = fp[(size_t)w * 128 + N + j];
      const float nn = c + nb, d = mb - m;
      m = m + d * (nb / nn);
      M2 = M2 + M2b + d * d * (c * nb / nn);
      c = nn;
    }
    float cnt = 0.0f;
    for (int w = 0; w < W.nwg; ++w) cnt += W.cnt[w];
    out[j] = j < N ? m : 0.0f;
    out[64 + j] = j < N ? M2 : 0.0f;
    if (j == 0) out[128] = cnt;
  } else {
    const float* bq = W.bpart_of(layer + 1);
    float s1 = 0.0f, s2 = 0.0f;
    if (j < N)
      for (int w = 0; w < W.nwg; ++w) { s1 += bq[(size_t)w * 128 + j]; s2 += bq[(size_t)w * 128 + 64 + j]; }
    out[j] = s1;
    out[64 + j] = s2;
  }
}

template <int S>
__global__ __launch_bounds__(MTH) void mcaq_mapper_bwd_kernel(MapperTrainArgs A) {
  __shared__ MapBwdLds L;
  mapper_bwd_stage<S>(A, L);
}

// the four backward stages and the parameter reduction in one launch
__global__ __launch_bounds__(MTH) void mcaq_mapper_bwd_coop_kernel(MapperTrainArgs A, unsigned* bar, float* gparams,
                                                                   int accumulate) {
  __shared__ MapBwdLds L;
  const unsigned n = (unsigned)A.nwg;
  mapper_bwd_stage<4>(A, L);
  mapper_grid_sync(bar, n);
  mapper_bwd_stage<3>(A, L);
  mapper_grid_sync(bar, 2 * n);
  mapper_bwd_stage<2>(A, L);
  mapper_grid_sync(bar, 3 * n);
  mapper_bwd_stage<1>(A, L);
  mapper_grid_sync(bar, 4 * n);
  // parameter gradients: sum of the workgroups' partials in workgroup order,
  // each workgroup a slice of the flat vector
  for (int e = (int)blockIdx.x * MTH + (int)threadIdx.x; e < MG_SIZE; e += (int)n * MTH) {
    float sum = 0.0f;
    for (int w = 0; w < A.nwg; ++w) sum += A.gpart[(size_t)w * MG_SIZE + e];
    gparams[e] = accumulate ? gparams[e] + sum : sum;
  }
  mapper_grid_exit(bar, A.nwg);
}

// ============================================================================
// analyzer head backward: clamp + bilateral adjoint (per image), complexity
// MLP backward (per tile)
// ============================================================================
// gradient layout: torch parameter order of complexity_mlp
enum : int {
  CG_W1 = 0, CG_B1 = 512, CG_G1 = 576, CG_BE1 = 640, CG_W2 = 704, CG_B2 = 2752, CG_G2 = 2784, CG_BE2 = 2816,
  CG_W3 = 2848, CG_B3 = 2880, CG_SIZE = 2881
};

struct HeadTrainArgs {
  mcaq_cmlp_params P;
  const float* phi;     // (n, 8)
  const float* craw;    // (n) complexity MLP output (before the bilateral)
  const float* gC;      // (n) gradient of C = clamp(bilateral(craw), 0, 1)
  float* gcraw;         // (n) work: gradient of craw
  float* gpart;         // [nwg][CG_SIZE]
  int B, ht, wt, n, nwg;
  int wg0;              // first workgroup of this segment in a multi-segment launch (else 0)
};

// bilateral (morphology.py:309-354, sigma_s 2, sigma_r 0.1, 5x5, replicate):
// C_t = N_t / D_t, N = sum_k w_k p_k, D = sum_k w_k + 1e-8,
// w_k = sp_k exp(-(p_k - c_t)^2 / 0.02), p_k = craw[clamp(t + o_k)].
// One workgroup per image.  Every (tile, tap) pair's weight is evaluated
// once (LDS); the adjoint of tile u gathers, per tap k, the tiles t with
// clamp(t + o_k) == u - one tile for an interior u, a short range at the
// clamped border (tap_range) - in a fixed order (deterministic).
__device__ __forceinline__ void tap_range(int u, int o, int n, int& lo, int& hi) {
  // rows t in [0, n) with clamp(t + o, 0, n - 1) == u
  lo = u == 0 ? 0 : u - o;
  hi = u == n - 1 ? n - 1 : u - o;
  lo = imax_(lo, 0);
  hi = imin_(hi, n - 1);
}

constexpr int BL_TH = 1024;   // threads per bilateral-backward workgroup (one image)
__device__ __forceinline__ void mcaq_bilateral_bwd_body(const HeadTrainArgs& A) {
  TSTAMP(57);
  extern __shared__ float smem_tr[];
  const int b = (int)blockIdx.x - A.wg0, ht = A.ht, wt = A.wt, NT = ht * wt;
  const int tid = threadIdx.x;
  float* cr = smem_tr;            // craw of the image
  float* gd = cr + NT;            // per tile: g_C / D  (0 outside the clamp)
  float* gcen = gd + NT;          // per tile: d/d c_t through its own range weights
  float* wk = gcen + NT;          // [NT][25] range x spatial weights
  float* cf = wk + 25 * NT;       // [NT][25] gd_t * dC_t / dp_k
  const float* crg = A.craw + (size_t)b * NT;
  for (int t = tid; t < NT; t += BL_TH) cr[t] = crg[t];
  __syncthreads();
  for (int e = tid; e < NT * 25; e += BL_TH) {
    const int t = e / 25, k = e - t * 25;
    const int th = t / wt, tw = t - th * wt;
    const int hh = imin_(imax_(th + k / 5 - 2, 0), ht - 1), ww = imin_(imax_(tw + k % 5 - 2, 0), wt - 1);
    const float d = cr[hh * wt + ww] - cr[t];
    wk[e] = bits_as_float(k_bilat_sp_bits[k]) * expf(-(d * d) / 0.02f);
  }
  __syncthreads();
  TSTAMP(58);
  // per tile: forward C, g / D, the centre term
  for (int t = tid; t < NT; t += BL_TH) {
    const int th = t / wt, tw = t - th * wt;
    const float c = cr[t];
    float num = 0.0f, den = 0.0f, sc = 0.0f;
    float pv[25];
#pragma unroll
    for (int k = 0; k < 25; ++k) {
      const int hh = imin_(imax_(th + k / 5 - 2, 0), ht - 1), ww = imin_(imax_(tw + k % 5 - 2, 0), wt - 1);
      pv[k] = cr[hh * wt + ww];
      num = fmaf(wk[t * 25 + k], pv[k], num);
      den += wk[t * 25 + k];
    }
    den += 1e-8f;
    const float Cv = num / den;
    const float g = A.gC[(size_t)b * NT + t];
    const float gdt = (Cv >= 0.0f && Cv <= 1.0f) ? g / den : 0.0f;
#pragma unroll
    for (int k = 0; k < 25; ++k) {
      const float w = wk[t * 25 + k], d = pv[k] - c;
      sc = fmaf((pv[k] - Cv) * w, d / 0.01f, sc);                    // through the range weights, centre
      cf[t * 25 + k] = gdt * (w - (pv[k] - Cv) * w * (d / 0.01f));    // d C_t / d p_k
    }
    gd[t] = gdt;
    gcen[t] = gdt * sc;
  }
  __syncthreads();
  TSTAMP(59);
  // adjoint gather: g_craw[u] = gcen[u] + sum over (k, t) with clamp(t + o_k)
  // = u of cf[t][k].  One item per (tile u, tap k) - the tap's terms, tiles
  // row-major (one term inside the image, up to 9 at a corner) - into the
  // weight array (dead after the per-tile pass), then per tile gcen + the 25
  // tap sums in tap order (one tile-serial chain of 25 variable loops before)
  float* pk = wk;
  for (int e = tid; e < NT * 25; e += BL_TH) {
    const int u = e / 25, k = e - u * 25;
    const int uh = u / wt, uw = u - uh * wt;
    int h0, h1, w0, w1;
    tap_range(uh, k / 5 - 2, ht, h0, h1);
    tap_range(uw, k % 5 - 2, wt, w0, w1);
    float s = 0.0f;
    for (int th = h0; th <= h1; ++th)
      for (int tw = w0; tw <= w1; ++tw) s += cf[(th * wt + tw) * 25 + k];
    pk[e] = s;
  }
  __syncthreads();
  for (int u = tid; u < NT; u += BL_TH) {
    float v[25];
#pragma unroll
    for (int k = 0; k < 25; ++k) v[k] = pk[u * 25 + k];
    float s = gcen[u];
#pragma unroll
    for (int k = 0; k < 25; ++k) s += v[k];
    A.gcraw[(size_t)b * NT + u] = s;
  }
  TSTAMP(60);
}
__global__ __launch_bounds__(BL_TH) void mcaq_bilateral_bwd_kernel(HeadTrainArgs A) { mcaq_bilateral_bwd_body(A); }

// complexity MLP backward (Linear(8,64)-LN-ReLU-Linear(64,32)-LN-ReLU-
// Linear(32,1)-sigmoid, recomputed): 64 tiles per workgroup, one per lane;
// the CB_NW waves split each layer's features (wave q: 1 / CB_NW of them) and
// meet in LDS for the LayerNorm sums.  Weight partials: sums over the
// workgroup's tiles in tile order (W2 in 1 x 4 register blocks).
constexpr int CB_NW = 8;                              // waves per workgroup
constexpr int CB_ST = 8 + 64 * 4 + 32 * 4 + 1 + 4;   // per-tile LDS vector (floats, padded odd)
enum : int { CB_PHI = 0, CB_R1 = 8, CB_GA1 = 72, CB_GY1 = 136, CB_GYX1 = 200, CB_R2 = 264, CB_GA2 = 296,
             CB_GY2 = 328, CB_GYX2 = 360, CB_GA3 = 392 };

// kX (fused launch, mcaq_cmlp_bwd_fused_kernel): the weight partials
// published as granules of gx (this workgroup's CG_SIZE slots) with `tag`
template <bool kX = false>
__device__ __forceinline__ void mcaq_cmlp_bwd_body(const HeadTrainArgs& A, mapx_t* gx = nullptr, unsigned tag = 0) {
  constexpr int NW = CB_NW, F1 = 64 / NW, F2 = 32 / NW, NTH = 64 * NW;
  extern __shared__ float smem_tr[];
  float* sv = smem_tr;                       // [TR_TPB][CB_ST]
  float* red = sv + TR_TPB * CB_ST;          // [NW][TR_TPB] cross-wave partial sums
  float* w2s = red + NW * TR_TPB;            // W2 (32 x 64), read as broadcast LDS vectors
  float* w2t = w2s + 2048;                   // W2 transposed (64 x 32): a wave's 4 layer-2 outputs of one k in one 16-byte read
  const mcaq_cmlp_params& P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, q = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wgi = (int)blockIdx.x - A.wg0;   // workgroup within this segment
  const int t = wgi * TR_TPB + lane;
  const bool valid = t < A.n;
  const int tc = valid ? t : A.n - 1;
  float* v = sv + lane * CB_ST;
  // cross-wave sum of one value per tile (every wave gets the total, in wave order)
  auto xsum = [&](float x) {
    red[q * TR_TPB + lane] = x;
    __syncthreads();
    float r = red[lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) r += red[w * TR_TPB + lane];
    __syncthreads();
    return r;
  };
  TSTAMP(16);
  // W2 into LDS (4 floats a thread; published by the first cross-wave sum's barrier)
#pragma unroll
  for (int i = 0; i < 2048 / NTH; ++i) {
    const int e = tid + i * NTH;
    const float wv = P.w2[e];
    w2s[e] = wv;
    w2t[(e & 63) * 32 + (e >> 6)] = wv;
  }
  float ph[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) ph[k] = A.phi[(size_t)tc * 8 + k];
  if (q == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[CB_PHI + k] = ph[k];
  }
  // ---- forward recompute: layer 1 (wave q: outputs F1 q .. F1 q + F1 - 1)
  float x1[F1];
  float s = 0.0f;
#pragma unroll
  for (int f = 0; f < F1; ++f) x1[f] = P.b1[q * F1 + f];
#pragma unroll
  for (int k = 0; k < 8; ++k) {      // k outer: the F1 chains interleaved, each over k in order
#pragma unroll
    for (int f = 0; f < F1; ++f) x1[f] = fmaf(P.w1[(q * F1 + f) * 8 + k], ph[k], x1[f]);
  }
#pragma unroll
  for (int f = 0; f < F1; ++f) s += x1[f];
  const float mu1 = xsum(s) / 64.0f;
  s = 0.0f;
#pragma unroll
  for (int f = 0; f < F1; ++f) { const float d = x1[f] - mu1; s = fmaf(d, d, s); }
  const float rs1 = 1.0f / sqrtf(xsum(s) / 64.0f + 1e-5f);
#pragma unroll
  for (int f = 0; f < F1; ++f) {
    const int j = q * F1 + f;
    x1[f] = (x1[f] - mu1) * rs1;                       // xhat1
    const float y = P.g1[j] * x1[f] + P.be1[j];
    v[CB_R1 + j] = y > 0.0f ? y : 0.0f;
  }
  __syncthreads();
  TSTAMP(17);
  // layer 2 (wave q: outputs F2 q ..)
  float x2[F2];
  s = 0.0f;
#pragma unroll
  for (int f = 0; f < F2; ++f) x2[f] = P.b2[q * F2 + f];
  static_assert(F2 == 4, "one float4 of W2^T per k");
#pragma unroll 16
  for (int k = 0; k < 64; ++k) {     // k outer: the F2 chains interleaved, each over k in order
    const float r = v[CB_R1 + k];
    const float4 w4 = *reinterpret_cast<const float4*>(w2t + k * 32 + q * F2);
    x2[0] = fmaf(w4.x, r, x2[0]); x2[1] = fmaf(w4.y, r, x2[1]);
    x2[2] = fmaf(w4.z, r, x2[2]); x2[3] = fmaf(w4.w, r, x2[3]);
  }
#pragma unroll
  for (int f = 0; f < F2; ++f) s += x2[f];
  const float mu2 = xsum(s) / 32.0f;
  s = 0.0f;
#pragma unroll
  for (int f = 0; f < F2; ++f) { const float d = x2[f] - mu2; s = fmaf(d, d, s); }
  const float rs2 = 1.0f / sqrtf(xsum(s) / 32.0f + 1e-5f);
  float a3p = 0.0f;
#pragma unroll
  for (int f = 0; f < F2; ++f) {
    const int j = q * F2 + f;
    x2[f] = (x2[f] - mu2) * rs2;                       // xhat2
    const float y = P.g2[j] * x2[f] + P.be2[j];
    const float r = y > 0.0f ? y : 0.0f;
    v[CB_R2 + j] = r;
    a3p = fmaf(P.w3[j], r, a3p);
  }
  const float a3 = xsum(a3p) + P.b3[0];
  const float cv = tr_sigmoid(a3);
  TSTAMP(18);
  // ---- backward: sigmoid, layer 3, LN2
  const float g3 = valid ? A.gcraw[t] * (cv * (1.0f - cv)) : 0.0f;
  if (q == 0) v[CB_GA3] = g3;
  float gx2[F2];
  float m1 = 0.0f, m2 = 0.0f;
#pragma unroll
  for (int f = 0; f < F2; ++f) {
    const int j = q * F2 + f;
    const float y = P.g2[j] * x2[f] + P.be2[j];
    const float gy = y > 0.0f ? P.w3[j] * g3 : 0.0f;
    v[CB_GY2 + j] = gy; v[CB_GYX2 + j] = gy * x2[f];
    gx2[f] = gy * P.g2[j];
    m1 += gx2[f]; m2 = fmaf(gx2[f], x2[f], m2);
  }
  m1 = xsum(m1) / 32.0f; m2 = xsum(m2) / 32.0f;
#pragma unroll
  for (int f = 0; f < F2; ++f) v[CB_GA2 + q * F2 + f] = rs2 * (gx2[f] - m1 - x2[f] * m2);
  __syncthreads();
  TSTAMP(19);
  // layer 2 transpose, LN1 (wave q: inputs F1 q ..)
  float gx1[F1];
  m1 = 0.0f; m2 = 0.0f;
  // rows j outer, the wave's F1 consecutive columns inner: one F1-wide scalar
  // load of W2 per row instead of F1 strided ones (each sum still over j in order)
  float accv[F1];
#pragma unroll
  for (int f = 0; f < F1; ++f) accv[f] = 0.0f;
#pragma unroll 8
  for (int j = 0; j < 32; ++j) {
    const float ga = v[CB_GA2 + j];
#pragma unroll
    for (int f = 0; f < F1; ++f) accv[f] = fmaf(w2s[j * 64 + q * F1 + f], ga, accv[f]);
  }
#pragma unroll
  for (int f = 0; f < F1; ++f) {
    const int k = q * F1 + f;
    const float acc = accv[f];
    const float y = P.g1[k] * x1[f] + P.be1[k];
    const float gy = y > 0.0f ? acc : 0.0f;
    v[CB_GY1 + k] = gy; v[CB_GYX1 + k] = gy * x1[f];
    gx1[f] = gy * P.g1[k];
    m1 += gx1[f]; m2 = fmaf(gx1[f], x1[f], m2);
  }
  m1 = xsum(m1) / 64.0f; m2 = xsum(m2) / 64.0f;
#pragma unroll
  for (int f = 0; f < F1; ++f) v[CB_GA1 + q * F1 + f] = rs1 * (gx1[f] - m1 - x1[f] * m2);
  __syncthreads();
  TSTAMP(20);
  // ---- weight partials over the workgroup's tiles (invalid lanes carry zero
  // gradients).  W2 (32 x 64): thread = one row x 4 columns.
  float* gp = A.gpart + (size_t)wgi * CG_SIZE;
  auto put = [&](int e, float x) {
    if constexpr (kX) mapx_put(gx + e, tag, x);
    else gp[e] = x;
  };
  auto tvec = [&](int u) { return sv + u * CB_ST; };
  {
    // one 16 x 16 block of W2 per wave on v_mfma_f32_16x16x4_f32: a
    // tile-ordered fp32 FMA chain u = 0..63 (the scalar loop's values)
    static_assert(NW == 8, "2 x 4 blocks of 16 x 16");
    const int jb = q >> 2, kb = q & 3, lr = lane & 15, lk = lane >> 4;
    tr_f4 d = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int st = 0; st < TR_TPB / 4; ++st) {
      const float* w = tvec(4 * st + lk);
      d = tr_mfma4(w[CB_GA2 + jb * 16 + lr], w[CB_R1 + kb * 16 + lr], d);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) put(CG_W2 + (jb * 16 + 4 * lk + r) * 64 + kb * 16 + lr, d[r]);
  }
  TSTAMP(21);
  // W1 (64 x 8) on MFMA as well: waves 0..3, one 16-row block each, the
  // B columns 8..15 zero (the same tile-ordered FMA chains)
  if (q < 4) {
    const int lr = lane & 15, lk = lane >> 4;
    tr_f4 d = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int st = 0; st < TR_TPB / 4; ++st) {
      const float* w = tvec(4 * st + lk);
      const float ph_k = w[CB_PHI + (lr & 7)];
      d = tr_mfma4(w[CB_GA1 + q * 16 + lr], lr < 8 ? ph_k : 0.0f, d);
    }
    if (lr < 8) {
#pragma unroll
      for (int r = 0; r < 4; ++r) put(CG_W1 + (q * 16 + 4 * lk + r) * 8 + lr, d[r]);
    }
  }
  // the other sums over the tiles - b1 / LN1 (192) and b2 / LN2 / W3 / b3
  // (129) - one element a thread, waves 4..7 first
  {
    const int r = (tid + NTH / 2) % NTH;
    if (r < 321) {
      const int e = r < 192 ? CG_B1 + r : CG_B2 + (r - 192);
      // every element's term is one FMA A(u) B(u) + a - the bias / LN sums
      // with B = 1 (exactly their adds), W3 ga3 * r2 - as one loop: a wave
      // holding two element types no longer runs two loops one after another
      int oa, ob = -1;
      if (e < CG_G1) oa = CB_GA1 + e - CG_B1;            // b1
      else if (e < CG_BE1) oa = CB_GYX1 + e - CG_G1;     // LN1 gamma
      else if (e < CG_W2) oa = CB_GY1 + e - CG_BE1;      // LN1 beta
      else if (e < CG_G2) oa = CB_GA2 + e - CG_B2;       // b2
      else if (e < CG_BE2) oa = CB_GYX2 + e - CG_G2;     // LN2 gamma
      else if (e < CG_W3) oa = CB_GY2 + e - CG_BE2;      // LN2 beta
      else if (e < CG_B3) { oa = CB_GA3; ob = CB_R2 + e - CG_W3; }   // W3: ga3 * r2
      else oa = CB_GA3;                                  // b3
      const int obc = ob >= 0 ? ob : 0;
      float a = 0.0f;
#pragma unroll 8
      for (int u = 0; u < TR_TPB; ++u) {
        const float* w = tvec(u);
        const float bv = w[obc];
        a = fmaf(w[oa], ob >= 0 ? bv : 1.0f, a);
      }
      put(e, a);
    }
  }
  TSTAMP(22);
}
__global__ __launch_bounds__(64 * CB_NW) void mcaq_cmlp_bwd_kernel(HeadTrainArgs A) { mcaq_cmlp_bwd_body(A); }

// ============================================================================
// soft mask backward (one workgroup per image)
// ============================================================================
// gradient layout: net.0.weight (8,2,3,3), net.0.bias, net.2.weight (2,8,1,1), net.2.bias
enum : int { SG_W1 = 0, SG_B1 = 144, SG_W2 = 152, SG_B2 = 168, SG_SIZE = 170 };

struct MaskTrainArgs {
  mcaq_smask_params P;
  const float* bits;     // (B, ht, wt)
  const float* absmean;  // (B, H, W)
  const float* gm;       // (B, H, W) gradient of m(p)
  float* gbits;          // (B, ht, wt) gradient of the bit map (accumulated if accumulate)
  float* gpart;          // [B][SG_SIZE]
  int B, H, W, ht, wt, accumulate;
  int wg0;               // first workgroup of this segment in a multi-segment launch (else 0)
  int stage;             // 1: |x| mean and m-gradient planes staged in LDS (smask_lds_bytes)
  // fold mode (qwork set, gm NULL): the quantizer backward's per-32-channel-
  // slice partials (mcaq_qat_backward with gm = gb = NULL) are folded here -
  // grad m(p) straight into the staged plane, the quantizer's grad_bits in
  // the fold kernel's order - and gbits = (c + grad_bits(quantizer)) +
  // grad_bits(soft mask), c the bit-budget gradient per tile (bb)
  const float* qwork;
  int qC;
  mcaq_bit_budget bb;
  float rn;              // 1 / (B * ht * wt) of this scale
};

// LDS bytes of the soft-mask backward of one (H, W, ht, wt) image; stage: + the
// staging plane (16-byte aligned)
constexpr int SM_PCH = 6;      // tile chunks of the parameter partials (SM_PCH x SG_SIZE <= threads)
constexpr int SM_HS = 9;       // LDS floats per tile of the 8-wide hidden-layer rows
constexpr int SM_WS = 176;     // LDS floats of the staged soft-mask parameters
inline size_t smask_lds_bytes(int H, int W, int ht, int wt, bool stage, bool fold = false) {
  const size_t base = ((size_t)(4 + 2 * SM_HS) * ht * wt + 64 + 1024 + SM_WS + (size_t)H * wt + (size_t)H * W) * sizeof(float) +
                      (size_t)2 * (ht + wt) * sizeof(int);
  const size_t st = stage ? ((base / 4 + 3) & ~(size_t)3) * 4 + (size_t)H * W * sizeof(float) : base;
  // fold mode: + the grad_bits pixel plane [H][W], band-column sums [ht][W], per-tile sums [NT]
  return fold ? st + ((size_t)H * W + (size_t)ht * W + (size_t)ht * wt) * sizeof(float) : st;
}
// staging applies when it fits and the planes are 16-byte aligned rows of 4
inline bool smask_stage_ok(const float* absmean, const float* gm, int H, int W, int ht, int wt) {
  return ((H * W) & 3) == 0 && (((uintptr_t)absmean | (uintptr_t)gm) & 15) == 0 &&
         smask_lds_bytes(H, W, ht, wt, true) <= 160 * 1024 - 1024;
}

constexpr int SM_TH = 1024;   // threads per soft-mask backward workgroup (one image)


// s + r[a] + ... + r[b - 1] in order, for 16-byte rows (r + a 16-byte
// aligned, b - a a multiple of 4): float4 LDS reads, two in flight.  The
// scalar reads of a tile row hit 4 banks across a wave (tile origins are
// multiples of 8 floats, every lane at the same column offset: 16-way
// conflicts); a float4 read per lane spreads them
__device__ __forceinline__ float smask_row_sum4(const float* r, int a, int b, float s) {
  const float4* r4 = reinterpret_cast<const float4*>(r + a);
  const int n4 = (b - a) >> 2;
  for (int c = 0; c < n4; c += 2) {
    const float4 x = r4[c], y = r4[imin_(c + 1, n4 - 1)];
    s = s + x.x; s = s + x.y; s = s + x.z; s = s + x.w;
    if (c + 1 < n4) { s = s + y.x; s = s + y.y; s = s + y.z; s = s + y.w; }
  }
  return s;
}

// an [n] fp32 plane (16-byte aligned, n % 4 == 0 when staged) into LDS: two
// 16-byte groups per thread per round, both loads issued before either store
__device__ __forceinline__ void smask_copy_plane(float* dst, const float* src, int n, int tid) {
  const int n4 = n >> 2;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  for (int e = tid; e < n4; e += 2 * SM_TH) {
    const int e2 = imin_(e + SM_TH, n4 - 1);
    const float4 a = s4[e], c = s4[e2];
    reinterpret_cast<float4*>(dst)[e] = a;
    if (e + SM_TH < n4) reinterpret_cast<float4*>(dst)[e2] = c;
  }
  for (int e = (n4 << 2) + tid; e < n; e += SM_TH) dst[e] = src[e];
}

__device__ __forceinline__ void mcaq_smask_bwd_body(const MaskTrainArgs& A) {
  extern __shared__ float smem_tr[];
  const int b = (int)blockIdx.x - A.wg0, H = A.H, W = A.W, ht = A.ht, wt = A.wt, NT = ht * wt;
  const int tid = threadIdx.x;
  float* f0 = smem_tr;               // bits feature, clamp((b - 2) / 6, 0, 1)
  float* f1 = f0 + NT;               // activation feature
  float* gl = f1 + NT;               // per tile: gradient of logit 0 (logit 1 gets -gl)
  // per-tile rows of 8 at a stride of SM_HS = 9 floats: a wave's per-tile
  // reads of one hidden unit then hit 32 banks (at stride 8 they hit 4)
  float* gpre = gl + NT;             // per tile x 8: gradient of the hidden pre-activation
  float* rel = gpre + SM_HS * NT;    // per tile x 8: relu(hidden)
  float* red = rel + SM_HS * NT;     // 64 reduction slots
  float* gmt = red + 64;             // per tile: gradient of m(tile)
  float* psc = gmt + NT;             // [SM_PCH][SG_SIZE] parameter partials of tile chunks
  float* wsm = psc + SM_TH;          // the soft-mask net's parameters (SG_SIZE floats, padded)
  int* hlo = (int*)(wsm + SM_WS);    // rows / columns of every tile's nearest-upsample block
  int* hhi = hlo + ht;
  int* wlo = hhi + ht;
  int* whi = wlo + wt;
  float* part = (float*)(whi + wt);  // [H][wt] row partials of the upsample adjoint
  float* tv = part + H * wt;         // [H][W] vertical pass of the smoothing adjoint
  // A.stage: the image's |x| mean plane, then its m(p) gradient plane, are
  // first copied into LDS ([H][W] after tv) with every load issued at once, so
  // the per-tile pooling sums and the 5-tap adjoint read LDS instead of
  // chaining dependent global loads (same values, same order)
  float* stg = smem_tr + ((int)(tv + H * W - smem_tr) + 3 & ~3);   // 16-byte aligned
  const bool fold = A.qwork != nullptr;
  float* fpix = stg + H * W;          // fold mode: grad_bits partial sums per pixel
  float* fcol = fpix + H * W;         //   per (tile row, column)
  float* fgb = fcol + ht * W;         //   per tile: c + the quantizer's grad_bits
  const float* am = A.absmean + (size_t)b * H * W;
  const float* gm = fold ? nullptr : A.gm + (size_t)b * H * W;
  TSTAMP(32);
  // the net's parameters into LDS: W1 (8,2,3,3) | b1 (8) | W2 (2,8) | b2 (2)
  if (tid < SG_SIZE) {
    wsm[tid] = tid < SG_B1 ? A.P.w1[tid] : tid < SG_W2 ? A.P.b1[tid - SG_B1]
                                     : tid < SG_B2 ? A.P.w2[tid - SG_W2] : A.P.b2[tid - SG_B2];
  }
  if (tid == SM_TH - 1) red[63] = 1.0f;   // the constant operand of the bias partials
  if (A.stage) {
    smask_copy_plane(stg, am, H * W, tid);
    __syncthreads();
    am = stg;
  }
  const float sch = (float)ht / (float)H, scw = (float)wt / (float)W;
  // the 5x5 smoothing kernel is the outer product of the 1-D Gaussian
  // (quantization.py:207-209: g1 g1^T): g_d = sqrt(k_dd)
  float g1[5];
#pragma unroll
  for (int d = 0; d < 5; ++d) g1[d] = sqrtf(bits_as_float(k_smooth5_bits[d * 6]));
  for (int i = tid; i < ht; i += SM_TH) { hlo[i] = H; hhi[i] = -1; }
  for (int j = tid; j < wt; j += SM_TH) { wlo[j] = W; whi[j] = -1; }
  __syncthreads();
  // nearest source row / column (floor(o * in / out), clamped) is monotone:
  // every tile's block is a contiguous range
  for (int h = tid; h < H; h += SM_TH) {
    const int i = imin_((int)floorf((float)h * sch), ht - 1);
    if (h == 0 || imin_((int)floorf((float)(h - 1) * sch), ht - 1) != i) hlo[i] = h;
    if (h == H - 1 || imin_((int)floorf((float)(h + 1) * sch), ht - 1) != i) hhi[i] = h;
  }
  for (int w = tid; w < W; w += SM_TH) {
    const int j = imin_((int)floorf((float)w * scw), wt - 1);
    if (w == 0 || imin_((int)floorf((float)(w - 1) * scw), wt - 1) != j) wlo[j] = w;
    if (w == W - 1 || imin_((int)floorf((float)(w + 1) * scw), wt - 1) != j) whi[j] = w;
  }
  TSTAMP(33);
  // ---- forward recompute: per-tile activation (adaptive_avg_pool2d), amax
  float lmx = -3.402823466e38f;
  for (int t = tid; t < NT; t += SM_TH) {
    const float bv = A.bits[(size_t)b * NT + t];   // issued first: in flight through the pooling sums
    const int i = t / wt, j = t - i * wt;
    const int ha = (i * H) / ht, hb = ((i + 1) * H + ht - 1) / ht;
    const int wa = (j * W) / wt, wb = ((j + 1) * W + wt - 1) / wt;
    // h-major, w ascending (adaptive_avg_pool2d's order), each row's values
    // loaded 8 at a time before they are added (clamped index)
    float s = 0.0f;
    if (A.stage && ((W | wa | (wb - wa)) & 3) == 0) {
      for (int h = ha; h < hb; ++h) s = smask_row_sum4(am + h * W, wa, wb, s);
    } else {
      for (int h = ha; h < hb; ++h) {
        const float* r = am + h * W;
        for (int w0 = wa; w0 < wb; w0 += 8) {
          float v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = r[imin_(w0 + k, wb - 1)];
#pragma unroll
          for (int k = 0; k < 8; ++k) s = w0 + k < wb ? s + v[k] : s;
        }
      }
    }
    const float a = (s / (float)(hb - ha)) / (float)(wb - wa);
    f1[t] = a;
    lmx = fmax_(lmx, a);
    f0[t] = clampf_((bv - 2.0f) / 6.0f, 0.0f, 1.0f);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lmx = fmax_(lmx, __shfl_xor(lmx, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = lmx;
  __syncthreads();
  float amax = red[0];
#pragma unroll
  for (int w = 1; w < SM_TH / 64; ++w) amax = fmax_(amax, red[w]);
  const float den = amax + 1e-8f;
  for (int t = tid; t < NT; t += SM_TH) f1[t] = f1[t] / den;
  TSTAMP(34);
  if (fold) {
    // the quantizer backward's fold (qat_fold_band's values): per pixel the
    // slice partials in slice order -> grad m(p) (into the staged plane) and
    // the grad_bits pixel sum; per (tile row, column) the band's rows in
    // order; per tile its columns in order
    __syncthreads();   // every pooling read of the staged |x| plane is done
    const int nsl = (A.qC + 31) / 32;
    const size_t plane = (size_t)A.B * H * W;
    const float* pm = A.qwork + (size_t)b * H * W;
    const float* pf = A.qwork + (size_t)nsl * plane + (size_t)b * H * W;
    // 16-byte groups, two per thread per round, every slice partial of a
    // round loaded before the first sum (slices KC at a time, the index
    // clamped: no load behind a branch); summed in slice order as before
    const bool v4 = ((H * W) & 3) == 0 && (plane & 3) == 0 && ((((uintptr_t)pm) | (uintptr_t)pf) & 15) == 0;
    const int n4 = v4 ? (H * W) >> 2 : 0;
    {
      constexpr int KC = 4;
      const size_t plane4 = plane >> 2;
      const float4* pm4 = reinterpret_cast<const float4*>(pm);
      const float4* pf4 = reinterpret_cast<const float4*>(pf);
      for (int e4 = tid; e4 < n4; e4 += 2 * SM_TH) {
        const int e4b = imin_(e4 + SM_TH, n4 - 1);
        float4 vm = make_float4(0.f, 0.f, 0.f, 0.f), vf = vm, wm = vm, wf = vm;
        for (int k0 = 0; k0 < nsl; k0 += KC) {
          float4 lm[KC], lf[KC], km[KC], kf[KC];
#pragma unroll
          for (int q = 0; q < KC; ++q) {
            const size_t o = (size_t)imin_(k0 + q, nsl - 1) * plane4;
            lm[q] = pm4[o + e4]; lf[q] = pf4[o + e4];
            km[q] = pm4[o + e4b]; kf[q] = pf4[o + e4b];
          }
#pragma unroll
          for (int q = 0; q < KC; ++q) {
            if (k0 + q >= nsl) break;
            if (k0 + q == 0) {
              vm = lm[0]; vf = lf[0]; wm = km[0]; wf = kf[0];
            } else {
              vm.x = vm.x + lm[q].x; vm.y = vm.y + lm[q].y; vm.z = vm.z + lm[q].z; vm.w = vm.w + lm[q].w;
              vf.x = vf.x + lf[q].x; vf.y = vf.y + lf[q].y; vf.z = vf.z + lf[q].z; vf.w = vf.w + lf[q].w;
              wm.x = wm.x + km[q].x; wm.y = wm.y + km[q].y; wm.z = wm.z + km[q].z; wm.w = wm.w + km[q].w;
              wf.x = wf.x + kf[q].x; wf.y = wf.y + kf[q].y; wf.z = wf.z + kf[q].z; wf.w = wf.w + kf[q].w;
            }
          }
        }
        reinterpret_cast<float4*>(stg)[e4] = vm;
        reinterpret_cast<float4*>(fpix)[e4] = vf;
        if (e4 + SM_TH < n4) {
          reinterpret_cast<float4*>(stg)[e4b] = wm;
          reinterpret_cast<float4*>(fpix)[e4b] = wf;
        }
      }
    }
    for (int e = (n4 << 2) + tid; e < H * W; e += SM_TH) {
      float vm = pm[e], vf = pf[e];
      for (int k = 1; k < nsl; ++k) { vm = vm + pm[(size_t)k * plane + e]; vf = vf + pf[(size_t)k * plane + e]; }
      stg[e] = vm;
      fpix[e] = vf;
    }
    __syncthreads();
    gm = stg;
    TSTAMP(41);
    for (int it = tid; it < ht * W; it += SM_TH) {
      const int th = it / W, w = it - th * W;
      float t = 0.0f;
      for (int h = hlo[th]; h <= hhi[th]; ++h) t += fpix[h * W + w];
      fcol[it] = t;
    }
    // the bit-budget gradient of every tile of this scale:
    // d L / d avg = g_avg + g_loss * 2 (avg - target), through mean(stack(means))
    float c = 0.0f;
    const bool has_c = A.bb.g_avg || A.bb.g_loss;
    if (has_c) {
      float dA = A.bb.g_avg ? A.bb.g_avg[0] : 0.0f;
      if (A.bb.g_loss) dA = dA + A.bb.g_loss[0] * (2.0f * (A.bb.avg[0] - A.bb.target));
      c = (dA * (1.0f / (float)A.bb.nscales)) * A.rn;
    }
    __syncthreads();
    for (int t = tid; t < NT; t += SM_TH) {
      const int i = t / wt, j = t - i * wt;
      float g = 0.0f;
      if ((((H * W) | W | wlo[j] | (whi[j] + 1 - wlo[j])) & 3) == 0)
        g = smask_row_sum4(fcol + i * W, wlo[j], whi[j] + 1, 0.0f);   // 16-byte rows
      else
        for (int w = wlo[j]; w <= whi[j]; ++w) g += fcol[i * W + w];
      fgb[t] = has_c ? c + g : g;
    }
  } else if (A.stage) {
    __syncthreads();   // every pooling read of the staged |x| plane is done
    smask_copy_plane(stg, gm, H * W, tid);
    __syncthreads();
    gm = stg;
  }
  TSTAMP(35);
  // adjoint of the smoothing (replicate pad), vertical pass:
  // tv(q, w) = sum_d g_d sum_{p: clamp(p + d - 2) = q} g_m(p, w)
  for (int e = tid; e < H * W; e += SM_TH) {
    const int q = e / W, w = e - q * W;
    float acc = 0.0f;
    if (q >= 2 && q <= H - 3) {
#pragma unroll
      for (int d = 0; d < 5; ++d) acc = fmaf(g1[d], gm[(q - d + 2) * W + w], acc);
    } else {
#pragma unroll
      for (int d = 0; d < 5; ++d) {
        int p0, p1;
        tap_range(q, d - 2, H, p0, p1);
        float r = 0.0f;
        for (int p = p0; p <= p1; ++p) r += gm[p * W + w];
        acc = fmaf(g1[d], r, acc);
      }
    }
    tv[e] = acc;
  }
  __syncthreads();
  TSTAMP(36);

  // horizontal pass + the nearest-upsample adjoint: part[h][j] = the sum,
  // over the columns q of tile column j in order, of the 5-tap value g(q) of
  // row h.  Staged: g(q) of every pixel first (one item per pixel, into the
  // staged plane, dead after the vertical pass), then the column sums;
  // otherwise one item per (row, tile column).  The same values either way.
  auto htap = [&](const float* row, int q) {
    float g = 0.0f;
    if (q >= 2 && q <= W - 3) {
#pragma unroll
      for (int d = 0; d < 5; ++d) g = fmaf(g1[d], row[q - d + 2], g);
    } else {
#pragma unroll
      for (int d = 0; d < 5; ++d) {
        int p0, p1;
        tap_range(q, d - 2, W, p0, p1);
        float r = 0.0f;
        for (int p = p0; p <= p1; ++p) r += row[p];
        g = fmaf(g1[d], r, g);
      }
    }
    return g;
  };
  if (A.stage && W >= 8 && H * W <= (1 << 20)) {
    float* gq = stg;
    // interior columns 2 .. W-3 (the 5 taps, no branch), then the 4 edge
    // columns of every row (the replicate-pad ranges) as items of their own,
    // so no wave runs both paths
    const int WI = W - 4;
    const float rWI = 1.0f / (float)WI;   // floor((e + 0.5) / WI) is exact for e < 2^20
    for (int e = tid; e < H * WI; e += SM_TH) {
      const int h = (int)(((float)e + 0.5f) * rWI), q = 2 + e - h * WI;
      const float* row = tv + h * W;
      float g = 0.0f;
#pragma unroll
      for (int d = 0; d < 5; ++d) g = fmaf(g1[d], row[q - d + 2], g);
      gq[h * W + q] = g;
    }
    for (int e = tid; e < H * 4; e += SM_TH) {
      const int h = e >> 2, k = e & 3, q = k < 2 ? k : W - 4 + k;
      gq[h * W + q] = htap(tv + h * W, q);
    }
    __syncthreads();
    for (int it = tid; it < H * wt; it += SM_TH) {
      const int h = it / wt, j = it - h * wt;
      const float* r = gq + h * W;
      const int q1 = whi[j];
      if (((W | wlo[j] | (q1 + 1 - wlo[j])) & 3) == 0) {
        part[it] = smask_row_sum4(r, wlo[j], q1 + 1, 0.0f);
        continue;
      }
      float acc = 0.0f;
      for (int q0 = wlo[j]; q0 <= q1; q0 += 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = r[imin_(q0 + k, q1)];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = q0 + k <= q1 ? acc + v[k] : acc;
      }
      part[it] = acc;
    }
  } else {
    for (int it = tid; it < H * wt; it += SM_TH) {
      const int h = it / wt, j = it - h * wt;
      const float* row = tv + h * W;
      float acc = 0.0f;
      for (int q = wlo[j]; q <= whi[j]; ++q) acc += htap(row, q);
      part[it] = acc;
    }
  }
  __syncthreads();
  for (int t = tid; t < NT; t += SM_TH) {
    const int i = t / wt, j = t - i * wt;
    float g = 0.0f;
    for (int h = hlo[i]; h <= hhi[i]; ++h) g += part[h * wt + j];
    gmt[t] = g;
  }
  __syncthreads();
  TSTAMP(37);
  // ---- per tile: hidden layer (one item per (tile, hidden unit)), then
  // logits, m(tile), gradients of the logits (one item per tile)
  const float rwt = 1.0f / (float)wt;   // tile row of t: floor((t + 0.5) / wt) is exact for t < 2^14
  for (int u = tid; u < NT * 8; u += SM_TH) {
    const int t = u >> 3, oc = u & 7;
    const int i = (int)(((float)t + 0.5f) * rwt), j = t - i * wt;
    float acc = wsm[SG_B1 + oc];
#pragma unroll
    for (int qq = 0; qq < 9; ++qq) {
      const int ii = i + qq / 3 - 1, jj = j + qq % 3 - 1;
      if (ii < 0 || ii >= ht || jj < 0 || jj >= wt) continue;
      const int s = ii * wt + jj;
      acc = fmaf(wsm[(oc * 2 + 0) * 9 + qq], f0[s], acc);
      acc = fmaf(wsm[(oc * 2 + 1) * 9 + qq], f1[s], acc);
    }
    gpre[t * SM_HS + oc] = acc;       // the pre-activation until its gradient replaces it
    rel[t * SM_HS + oc] = acc > 0.0f ? acc : 0.0f;
  }
  __syncthreads();
  for (int t = tid; t < NT; t += SM_TH) {
    float l0 = wsm[SG_B2], l1 = wsm[SG_B2 + 1];
#pragma unroll
    for (int ic = 0; ic < 8; ++ic) {
      l0 = fmaf(wsm[SG_W2 + ic], rel[t * SM_HS + ic], l0);
      l1 = fmaf(wsm[SG_W2 + 8 + ic], rel[t * SM_HS + ic], l1);
    }
    const float mt = 1.0f / (1.0f + expf(l1 - l0));
    // softmax (2 classes): d m / d l0 = m (1 - m) = -d m / d l1
    const float g0 = gmt[t] * (mt * (1.0f - mt));
    gl[t] = g0;
#pragma unroll
    for (int ic = 0; ic < 8; ++ic) {
      const float gr = wsm[SG_W2 + ic] * g0 - wsm[SG_W2 + 8 + ic] * g0;
      gpre[t * SM_HS + ic] = gpre[t * SM_HS + ic] > 0.0f ? gr : 0.0f;
    }
  }
  __syncthreads();
  TSTAMP(38);
  // ---- gradient of the bits feature: 3x3 transposed conv of gpre, then
  // through the clamp and the affine map
  for (int u = tid; u < NT; u += SM_TH) {
    const int i = u / wt, j = u - i * wt;
    float s = 0.0f;
#pragma unroll
    for (int qq = 0; qq < 9; ++qq) {
      const int ti = i - (qq / 3 - 1), tj = j - (qq % 3 - 1);   // tile whose tap qq lands on u
      if (ti < 0 || ti >= ht || tj < 0 || tj >= wt) continue;
      const int t = ti * wt + tj;
#pragma unroll
      for (int oc = 0; oc < 8; ++oc) s = fmaf(wsm[(oc * 2 + 0) * 9 + qq], gpre[t * SM_HS + oc], s);
    }
    const float bv = A.bits[(size_t)b * NT + u];
    const float f = (bv - 2.0f) / 6.0f;
    const float gb = (f >= 0.0f && f <= 1.0f) ? s / 6.0f : 0.0f;
    float* dst = A.gbits + (size_t)b * NT + u;
    *dst = fold ? fgb[u] + gb : (A.accumulate ? *dst + gb : gb);
  }
  TSTAMP(39);
  // ---- parameter partials of this image: thread (chunk c, element e) sums
  // e's terms over the tiles of chunk c in tile order; the SM_PCH chunk sums
  // of each element are then added in chunk order (deterministic).  Every
  // element's term is one FMA a(t) b(t) (+ s): W1 gpre(t, oc) f(neighbour),
  // b1 gpre(t, oc) x 1, W2 (+-gl(t)) rel(t, ic), b2 (+-gl(t)) x 1 - exactly
  // the sums / FMAs of the per-type loops, as one branch-free loop (a wave
  // holds several element types; per-type loops ran one after another)
  static_assert(SM_PCH * SG_SIZE <= SM_TH, "soft-mask partial chunks exceed the workgroup");
  float* gp = A.gpart + (size_t)b * SG_SIZE;
  if (tid < SM_PCH * SG_SIZE) {
    const int c = tid / SG_SIZE, e = tid - c * SG_SIZE;
    const int t0 = (c * NT) / SM_PCH, t1 = ((c + 1) * NT) / SM_PCH;
    const bool w1 = e < SG_B1;
    // a(t) = sa * pa[t * da]; b(t) = pb[t * db] (W1: a neighbour tap of f0 / f1,
    // masked outside the tile grid; b1 / b2: the constant 1 in red[63])
    const float* pa; const float* pb;
    int da, db, di = 0, dj = 0;
    float sa = 1.0f;
    if (w1) {
      const int oc = e / 18, ic = (e / 9) & 1, qq = e % 9;
      di = qq / 3 - 1; dj = qq % 3 - 1;
      pa = gpre + oc; da = SM_HS;
      pb = (ic == 0 ? f0 : f1) + di * wt + dj; db = 1;
    } else if (e < SG_W2) {
      pa = gpre + (e - SG_B1); da = SM_HS; pb = red + 63; db = 0;
    } else if (e < SG_B2) {
      const int o = (e - SG_W2) >> 3, ic = (e - SG_W2) & 7;
      pa = gl; da = 1; sa = o == 0 ? 1.0f : -1.0f; pb = rel + ic; db = SM_HS;
    } else {
      pa = gl; da = 1; sa = e == SG_B2 ? 1.0f : -1.0f; pb = red + 63; db = 0;
    }
    int i = (int)(((float)t0 + 0.5f) * rwt), j = t0 - i * wt;   // walked forward with t
    float s = 0.0f;
#pragma unroll 4
    for (int t = t0; t < t1; ++t) {
      const bool ok = !w1 || (i + di >= 0 && i + di < ht && j + dj >= 0 && j + dj < wt);
      const float av = sa * pa[t * da];
      const float bv = ok ? pb[t * db] : 0.0f;
      const float v = fmaf(av, bv, s);
      s = ok ? v : s;
      if (++j == wt) { j = 0; ++i; }
    }
    psc[tid] = s;
  }
  __syncthreads();
  if (tid < SG_SIZE) {
    float s = psc[tid];
#pragma unroll
    for (int c = 1; c < SM_PCH; ++c) s += psc[c * SG_SIZE + tid];
    gp[tid] = s;
  }
  TSTAMP(40);
}
__global__ __launch_bounds__(SM_TH) void mcaq_smask_bwd_kernel(MaskTrainArgs A) { mcaq_smask_bwd_body(A); }

// ---- device packing of parameter blobs --------------------------------------
// out[seg.dst + i] for every segment: mode 0 copies n floats from src; mode 1
// writes the v_mfma_f32_16x16x4_f32 A operands of an (n, k) row-major weight
// ([block][step][lane]: lane l of block b, step s holds W[16 b + (l & 15)]
// [4 s + (l >> 4)], zero outside the weight); positions no segment covers
// (tail padding) are zero.  One launch replaces the torch cat / zeros / index
// sequence that re-packs a blob after every optimizer step.
struct PackArgs {
  mcaq_pack_seg seg[MCAQ_PACK_MAXSEG];
  int nseg, total;
};

__device__ __forceinline__ void pack_elem(const PackArgs& a, float* __restrict__ out, int e) {
  if (e >= a.total) return;
  float v = 0.0f;
  for (int i = 0; i < a.nseg; ++i) {
    const mcaq_pack_seg& g = a.seg[i];
    const int kp = (g.k + 3) & ~3, nb = (g.n + 15) >> 4;
    const int len = g.mode == 0 ? g.n : nb * (kp >> 2) * 64;
    const int u = e - g.dst;
    if (u < 0 || u >= len) continue;
    if (g.mode == 0) {
      v = g.src[u];
    } else {
      const int lane = u & 63, st = (u >> 6) % (kp >> 2), b = (u >> 6) / (kp >> 2);
      const int row = 16 * b + (lane & 15), col = 4 * st + (lane >> 4);
      v = (row < g.n && col < g.k) ? g.src[(size_t)row * g.k + col] : 0.0f;
    }
  }
  out[e] = v;
}
__global__ __launch_bounds__(256) void mcaq_pack_kernel(PackArgs a, float* __restrict__ out) {
  pack_elem(a, out, blockIdx.x * 256 + threadIdx.x);
}

// the train step's blob pack riding on its pass-1 launch as workgroups
// units_total.. (pass 1 reads no blob; the morph launch that follows does)
template <bool kVec>
__global__ __launch_bounds__(256, MCAQ_STATS_MINW) void mcaq_stats_pack_kernel(StatsArgs a, PackArgs p,
                                                                             float* __restrict__ out) {
  __shared__ float lds[ST_LDS];
  if ((int)blockIdx.x >= a.units_total) {
    pack_elem(p, out, ((int)blockIdx.x - a.units_total) * 256 + (int)threadIdx.x);
    return;
  }
  stats_dispatch<kVec>(a, lds, (int)blockIdx.x);
}

}  // namespace mcaq

// ============================================================================
// C ABI
// ============================================================================
// ============================================================================
// multi-segment launches: the hook scales of one train step (each its own
// tensors, the same parameters) in ONE launch per stage.  A segment is the
// single-scale launch's argument block with wg0 = its first workgroup; every
// workgroup runs the single-scale body of its segment, so the values are those
// of the per-scale launches.  Single-stream HIP graphs of the QAT step then
// carry a third of the kernel nodes (graph replay issues a multi-stream graph
// node by node: tools/probe/graph_replay_probe.py).
// ============================================================================
constexpr int TR_MAXSEG = 3;
template <typename T> struct TrMulti { T s[TR_MAXSEG]; int nseg; };
template <typename T>
__device__ __forceinline__ const T& tr_seg(const TrMulti<T>& M) {
  const int x = (int)blockIdx.x;
  return (M.nseg > 2 && x >= M.s[2].wg0) ? M.s[2] : ((M.nseg > 1 && x >= M.s[1].wg0) ? M.s[1] : M.s[0]);
}

template <int S>
__global__ __launch_bounds__(MTH) void mcaq_mapper_fwd_multi_kernel(TrMulti<MapperTrainArgs> M) {
  __shared__ MapFwdLds L;
  mapper_fwd_stage<S>(tr_seg(M), L);
}
template <int S>
__global__ __launch_bounds__(MTH) void mcaq_mapper_bwd_multi_kernel(TrMulti<MapperTrainArgs> M) {
  __shared__ MapBwdLds L;
  mapper_bwd_stage<S>(tr_seg(M), L);
}
__global__ __launch_bounds__(BL_TH) void mcaq_bilateral_bwd_multi_kernel(TrMulti<HeadTrainArgs> M) {
  mcaq_bilateral_bwd_body(tr_seg(M));
}
// the complexity MLP's backward of every segment with its parameter
// reduction in the same launch: every workgroup publishes its CG_SIZE weight
// partials as granules (mapx_*: write-through, the epoch tag in each), then
// sums a slice of the elements over every workgroup's partials - the chain
// of mcaq_tr_reduce_multi (segments last scale first, each in workgroup
// order, accumulate / scale as tr_chain_elem), so the values are identical.
// Sync buffer (mcaq_head_sync_bytes): word 0 the epoch, word 1 the status,
// granules from byte 256, [workgroup][CG_SIZE].  Every workgroup must be
// resident at once (at most MAPPER_COOP_MAX_WG).
struct CmlpRed {
  unsigned* sync;
  float* out;
  int accumulate;
  float scale;
  int nwg;             // workgroups of the launch (every segment's)
};
__global__ __launch_bounds__(64 * CB_NW) void mcaq_cmlp_bwd_fused_kernel(TrMulti<HeadTrainArgs> M, CmlpRed R) {
  extern __shared__ float smem_tr[];
  const HeadTrainArgs& A = tr_seg(M);
  mapx_t* const gran = reinterpret_cast<mapx_t*>(R.sync + MAPX_HDR);
  const unsigned tag = __builtin_amdgcn_readfirstlane(
                           __hip_atomic_load(R.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  mcaq_cmlp_bwd_body<true>(A, gran + (size_t)blockIdx.x * CG_SIZE, tag);
  __syncthreads();
  // this workgroup's slice of the elements, every workgroup's partial of each
  // into LDS (one granule load per thread per pass, all in flight), then one
  // thread per element sums them in the chain's order
  const int W = R.nwg, per = (CG_SIZE + W - 1) / W;
  const int e0 = (int)blockIdx.x * per, ne = imin_(per, CG_SIZE - e0);
  float* buf = smem_tr;                       // [ne][W]
  const int tid = (int)threadIdx.x;
  constexpr int NTH = 64 * CB_NW;
  for (int i0 = 0; i0 < ne * W; i0 += 4 * NTH) {
    mapx_t* gp[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = imin_(i0 + r * NTH + tid, ne * W - 1);
      const int el = i / W, w = i - el * W;
      gp[r] = gran + (size_t)w * CG_SIZE + e0 + el;
    }
    float v[4];
    if (ne > 0) mapx_get<4>(gp, tag, v, R.sync + 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + r * NTH + tid;
      if (i < ne * W) buf[i] = v[r];
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid == 0)   // every workgroup published (slice 0 read them all): next epoch
    __hip_atomic_fetch_add(R.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int el = tid; el < ne; el += NTH) {   // a slice can exceed the workgroup (few workgroups)
    const int e = e0 + el;
    const float* row = buf + (size_t)el * W;
    const bool sc = R.scale != 0.0f && R.scale != 1.0f;
    float acc = 0.0f;
    for (int c = 0; c < M.nseg; ++c) {
      const HeadTrainArgs& G = M.s[M.nseg - 1 - c];   // the chain: last segment first
      float sum = 0.0f;
      for (int w = 0; w < G.nwg; ++w) sum = sum + row[G.wg0 + w];
      acc = c == 0 ? ((R.accumulate && !sc) ? R.out[e] + sum : sum) : acc + sum;
    }
    if (sc) acc = R.accumulate ? R.out[e] + acc * R.scale : acc * R.scale;
    R.out[e] = acc;
  }
}

__global__ __launch_bounds__(64 * CB_NW) void mcaq_cmlp_bwd_multi_kernel(TrMulti<HeadTrainArgs> M) {
  mcaq_cmlp_bwd_body(tr_seg(M));
}
__global__ __launch_bounds__(SM_TH) void mcaq_smask_bwd_multi_kernel(TrMulti<MaskTrainArgs> M) {
  mcaq_smask_bwd_body(tr_seg(M));
}

// bit budget forward: per segment the mean of its bits (a fixed-order tree:
// per thread a strided sum, then the block's halving tree), their mean, and
// (avg - target)^2 - deterministic; ATen's CUDA mean reduces in another order
// (fp32 rounding apart)
struct BitBudgetArgs { const float* bits[TR_MAXSEG]; int n[TR_MAXSEG]; int nseg; float target; float* avg; float* loss; };
__global__ __launch_bounds__(1024) void mcaq_bit_budget_kernel(BitBudgetArgs a) {
  __shared__ float red[1024];
  const int tid = (int)threadIdx.x;
  float total = 0.0f;
  for (int k = 0; k < a.nseg; ++k) {
    float s = 0.0f;
    for (int i = tid; i < a.n[k]; i += 1024) s += a.bits[k][i];
    red[tid] = s;
    __syncthreads();
    for (int h = 512; h > 0; h >>= 1) {
      if (tid < h) red[tid] = red[tid] + red[tid + h];
      __syncthreads();
    }
    total = total + red[0] * (1.0f / (float)a.n[k]);
    __syncthreads();
  }
  if (tid == 0) {
    const float avg = total * (1.0f / (float)a.nseg);
    a.avg[0] = avg;
    if (a.loss) a.loss[0] = (avg - a.target) * (avg - a.target);
  }
}

// parameter-gradient reductions of several segments.  chain = 0: segment k
// (blockIdx.y) reduces its partials into its own output, as
// mcaq_tr_reduce_kernel; chain = 1: every segment into segment 0's output, in
// segment order - v = s0 (+ out if accumulate), v += s1, v += s2 - the values
// one reduction launch per segment leaves (the first with `accumulate`, the
// others accumulating)
struct TrReduceSeg { const float* part; float* out; int nwg, stride, count, accumulate; float scale; };
// chain mode: element e of segment 0's output = s_0 (+ out) + s_1 + s_2
// (a variant walking all segments' partials as one 16-deep load list was
// slower: 5.9 -> 10.7 us for the complexity-MLP chain, r05)
__device__ __forceinline__ void tr_chain_elem(const TrMulti<TrReduceSeg>& M, int e) {
  const TrReduceSeg& s0 = M.s[0];
  if (e >= s0.count) return;
  float v = 0.0f;
  const bool sc = s0.scale != 0.0f && s0.scale != 1.0f;
  for (int k = 0; k < M.nseg; ++k) {
    const TrReduceSeg& g = k == 0 ? M.s[0] : (k == 1 ? M.s[1] : M.s[2]);
    const float sum = tr_ordered_sum(g.part, g.nwg, g.stride, e);
    v = k == 0 ? ((s0.accumulate && !sc) ? s0.out[e] + sum : sum) : v + sum;
  }
  // scaled (a data-parallel rank's share of a gradient it computed whole):
  // this launch's sum times the scale, then accumulated
  if (sc) v = s0.accumulate ? s0.out[e] + v * s0.scale : v * s0.scale;
  s0.out[e] = v;
}
__global__ __launch_bounds__(256) void mcaq_tr_reduce_multi_kernel(TrMulti<TrReduceSeg> M, int chain) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (chain) {
    tr_chain_elem(M, e);
  } else {
    const int k = blockIdx.y;
    const TrReduceSeg& g = k == 0 ? M.s[0] : (k == 1 ? M.s[1] : M.s[2]);
    if (k >= M.nseg || e >= g.count) return;
    float sum = tr_ordered_sum(g.part, g.nwg, g.stride, e);
    if (g.scale != 0.0f) sum = sum * g.scale;
    g.out[e] = g.accumulate ? g.out[e] + sum : sum;
  }
}

// per-segment mode as one flat index: element i = (segment i / count, e = i %
// count) of segments of equal count, each into its own output
__device__ __forceinline__ void tr_seg_elem(const TrMulti<TrReduceSeg>& M, int i) {
  const int cnt = M.s[0].count, k = i / cnt, e = i - k * cnt;
  if (k >= M.nseg) return;
  const TrReduceSeg& g = k == 0 ? M.s[0] : (k == 1 ? M.s[1] : M.s[2]);
  float sum = tr_ordered_sum(g.part, g.nwg, g.stride, e);
  if (g.scale != 0.0f) sum = sum * g.scale;
  g.out[e] = g.accumulate ? g.out[e] + sum : sum;
}

// the mapper's first backward stage with per-segment reductions riding along
// as workgroups rwg0.. (MTH elements each): the soft masks' parameter
// gradients, whose partials the soft-mask backward launch before it left
// (train_step._MaskQuantMulti -> _MapperMulti)
template <int S>
__global__ __launch_bounds__(MTH) void mcaq_mapper_bwd_ride_kernel(TrMulti<MapperTrainArgs> M, TrMulti<TrReduceSeg> R,
                                                                   int rwg0) {
  __shared__ MapBwdLds L;
  if ((int)blockIdx.x >= rwg0) {
    tr_seg_elem(R, ((int)blockIdx.x - rwg0) * MTH + (int)threadIdx.x);
    return;
  }
  mapper_bwd_stage<S>(tr_seg(M), L);
}

// the four forward stages of every segment in ONE launch, the batch
// statistics exchanged as granules between them (mapx_*; the arithmetic and
// its order are the staged launches', so the results are bit-identical).
// Every workgroup must be resident at once: the launcher admits at most
// MAPPER_COOP_MAX_WG workgroups (one 512-thread workgroup per CU is enough).
__global__ __launch_bounds__(MTH) void mcaq_mapper_fwd_fused_kernel(TrMulti<MapperTrainArgs> M) {
  __shared__ MapFwdLds L;
  __shared__ float s_a[TR_TPB][65];
  const MapperTrainArgs& A = tr_seg(M);
  const unsigned E = mapx_epoch(A);
  TSTAMP(23);
#if defined(MCAQ_STAMPS_WG) && defined(__HIP_DEVICE_COMPILE__)
  // diagnostic build only: workgroups 0..31's start and end of stage 1 (the
  // global 100 MHz clock), tools/probe/mapx_skew.py
  if (threadIdx.x == 0 && blockIdx.x < 32) g_mapx_wg[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
  mapper_fwd_stage<1, true>(A, L, E, s_a);
  __syncthreads();
#if defined(MCAQ_STAMPS_WG) && defined(__HIP_DEVICE_COMPILE__)
  if (threadIdx.x == 0 && blockIdx.x < 32) g_mapx_wg[32 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
  TSTAMP(24);
  mapper_fwd_stage<2, true>(A, L, E, s_a);
  __syncthreads();
  TSTAMP(25);
  mapper_fwd_stage<3, true>(A, L, E, s_a);
  __syncthreads();
  TSTAMP(26);
  mapper_fwd_stage<4, true>(A, L, E, s_a);
  TSTAMP(27);
  // stage 4 read exchange 3, which every workgroup of the segment published
  // after reading E: the segment's next launch may take the next epoch
  if ((int)blockIdx.x == A.wg0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(A.gep, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the four backward stages in ONE launch (granule exchanges as the forward),
// with per-segment reductions riding along as workgroups rwg0.. (the soft
// masks' parameter gradients: mcaq_mapper_bwd_ride_kernel)
__global__ __launch_bounds__(MTH) void mcaq_mapper_bwd_fused_kernel(TrMulti<MapperTrainArgs> M, TrMulti<TrReduceSeg> R,
                                                                    int rwg0) {
  __shared__ MapBwdLds L;
  __shared__ float s_gy[TR_TPB][65];
  if ((int)blockIdx.x >= rwg0) {
    tr_seg_elem(R, ((int)blockIdx.x - rwg0) * MTH + (int)threadIdx.x);
    return;
  }
  const MapperTrainArgs& A = tr_seg(M);
  const unsigned E = mapx_epoch(A);
  TSTAMP(28);
  mapper_bwd_stage<4, true>(A, L, E, s_gy);
  __syncthreads();
  TSTAMP(29);
  mapper_bwd_stage<3, true>(A, L, E, s_gy);
  __syncthreads();
  TSTAMP(30);
  mapper_bwd_stage<2, true>(A, L, E, s_gy);
  __syncthreads();
  TSTAMP(31);
  mapper_bwd_stage<1, true>(A, L, E, s_gy);
  TSTAMP(49);
  if ((int)blockIdx.x == A.wg0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(A.gep, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the bilateral backward launch with a chain reduction riding along as
// workgroups rwg0.. (BL_TH elements each): the bit mapper's parameter
// gradients, whose partials the mapper's last backward stage left, summed
// while the analyzer head's backward runs (train_step._HeadMulti)
__global__ __launch_bounds__(BL_TH) void mcaq_bilateral_bwd_ride_kernel(TrMulti<HeadTrainArgs> M, TrMulti<TrReduceSeg> R,
                                                                       int rwg0) {
  if ((int)blockIdx.x >= rwg0) {
    tr_chain_elem(R, ((int)blockIdx.x - rwg0) * BL_TH + (int)threadIdx.x);
    return;
  }
  mcaq_bilateral_bwd_body(tr_seg(M));
}

extern "C" {

size_t mcaq_mapper_work_floats(int n) { return mcaq::mapper_work_floats(n); }

int mcaq_mapper_train_forward(const mcaq_mapper_params* P, const float* c, int n, float min_bits, float max_bits,
                              float temperature, float momentum, int round_bits, int update_stats, float* bits,
                              float* work, unsigned* grid_sync, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !c || !bits || !work || n < 1) return (int)hipErrorInvalidValue;
  MapperTrainArgs A{};
  A.P = *P; A.c = c; A.bits = bits; A.work = work; A.n = n; A.nwg = (n + TR_TPB - 1) / TR_TPB;
  A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature; A.momentum = momentum;
  A.round_bits = round_bits; A.update_stats = update_stats;
  const dim3 g(A.nwg), t(MTH);
  if (grid_sync && A.nwg <= MAPPER_COOP_MAX_WG) {
    hipLaunchKernelGGL(mcaq_mapper_fwd_coop_kernel, g, t, 0, stream, A, grid_sync);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<1>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<2>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<3>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<4>, g, t, 0, stream, A);
  return (int)hipGetLastError();
}

int mcaq_mapper_train_backward(const mcaq_mapper_params* P, const float* c, int n, const float* gbits,
                               float min_bits, float max_bits, float temperature, float* work, float* gc,
                               float* gparams, float* gpart, int accumulate, unsigned* grid_sync,
                               hipStream_t stream) {
  using namespace mcaq;
  if (!P || !c || !gbits || !gc || !gpart || !work || n < 1 || (!gparams && grid_sync)) return (int)hipErrorInvalidValue;
  MapperTrainArgs A{};
  A.P = *P; A.c = c; A.gbits = gbits; A.gc = gc; A.work = work; A.gpart = gpart; A.n = n;
  A.nwg = (n + TR_TPB - 1) / TR_TPB;
  A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature;
  const dim3 g(A.nwg), t(MTH);
  if (grid_sync && A.nwg <= MAPPER_COOP_MAX_WG) {
    hipLaunchKernelGGL(mcaq_mapper_bwd_coop_kernel, g, t, 0, stream, A, grid_sync, gparams, accumulate ? 1 : 0);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<4>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<3>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<2>, g, t, 0, stream, A);
  hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<1>, g, t, 0, stream, A);
  if (gparams)   // NULL: the caller reduces gpart (mcaq_mapper_train_grad_reduce)
    hipLaunchKernelGGL(mcaq_tr_reduce_kernel, dim3((MG_SIZE + 255) / 256), dim3(256), 0, stream, (const float*)gpart,
                       A.nwg, (int)MG_SIZE, (int)MG_SIZE, gparams, accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

int mcaq_mapper_running_update(const mcaq_mapper_params* P, const float* const* works, const int* ns, int count,
                               float momentum, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !works || !ns || count < 1 || count > MAPPER_RU_MAX) return (int)hipErrorInvalidValue;
  MapperRunningArgs A{};
  A.P = *P; A.count = count; A.momentum = momentum;
  for (int k = 0; k < count; ++k) {
    if (!works[k] || ns[k] < 1) return (int)hipErrorInvalidValue;
    A.rstat[k] = mapper_work(const_cast<float*>(works[k]), ns[k]).rstat;
  }
  hipLaunchKernelGGL(mcaq_mapper_running_kernel, dim3(1), dim3(64), 0, stream, A);
  return (int)hipGetLastError();
}

int mcaq_ema_stats_multi_running(const mcaq_ema_seg* segs, int nseg, const mcaq_mapper_params* P,
                                 const float* const* works, const int* ns, int count, float momentum,
                                 hipStream_t stream) {
  using namespace mcaq;
  if (!segs || nseg < 1 || nseg > 3 || !P || !works || !ns || count < 1 || count > MAPPER_RU_MAX)
    return (int)hipErrorInvalidValue;
  EmaRunArgs a{};
  const int wg = ema_multi_args(segs, nseg, a.M);
  if (wg < 0) return (int)hipErrorInvalidValue;
  a.R.P = *P; a.R.count = count; a.R.momentum = momentum;
  for (int k = 0; k < count; ++k) {
    if (!works[k] || ns[k] < 1) return (int)hipErrorInvalidValue;
    a.R.rstat[k] = mapper_work(const_cast<float*>(works[k]), ns[k]).rstat;
  }
  a.ema_wg = wg;
  hipLaunchKernelGGL(mcaq_ema_running_kernel, dim3(wg + 1), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

int mcaq_morph_ema(const mcaq_morph_scale* scales, int nscales, const mcaq_ema_seg* esegs, int ne,
                   const mcaq_mapper_params* P, const float* const* works, const int* ns, int count, float momentum,
                   hipStream_t stream) {
  using namespace mcaq;
  if (!esegs || ne < 1 || ne > 3 || count < 0 || count > MAPPER_RU_MAX || (count > 0 && (!P || !works || !ns)))
    return (int)hipErrorInvalidValue;
  MorphLaunch L;
  int e = morph_launch_config(scales, nscales, nullptr, 0, L);
  if (e) return e;
  EmaRunArgs r{};
  const int wg = ema_multi_args(esegs, ne, r.M);
  if (wg < 0) return (int)hipErrorInvalidValue;
  if (count > 0) {
    r.R.P = *P; r.R.count = count; r.R.momentum = momentum;
    for (int k = 0; k < count; ++k) {
      if (!works[k] || ns[k] < 1) return (int)hipErrorInvalidValue;
      r.R.rstat[k] = mapper_work(const_cast<float*>(works[k]), ns[k]).rstat;
    }
  }
  r.ema_wg = wg;
  if (L.grid_a > 0 || L.band || L.tb || L.grid_b <= 0) {
    // no lone pass-B launch to ride on: the morph launch, then the EMA launch
    e = morph_launch(L, 3, stream);
    if (e) return e;
    return count > 0 ? mcaq_ema_stats_multi_running(esegs, ne, P, works, ns, count, momentum, stream)
                     : mcaq_ema_stats_multi(esegs, ne, stream);
  }
  // soft-mask only (the train step's m planes): the tile loads issued up front
  bool smo = true;
  for (int i = 0; i < L.a.nscales; ++i) {
    const MorphScale& S = L.a.s[i];
    smo = smo && (S.flags & (F_PHI | F_CMLP | F_MAPPER | F_SOFTMASK)) == F_SOFTMASK && S.bits_in && S.absmean &&
          S.ht * S.wt <= TILES_THREADS / L.a.tipw[i];
  }
  static int set_te = 0;
  const int lim = MCAQ_MORPH_LDS_LIMIT - 1024;
  if ((int)L.dyn_b > set_te) {
    const void* ks[4] = {(const void*)mcaq_tiles_ema_kernel<TILE_FLOATS_PAD, false>,
                         (const void*)mcaq_tiles_ema_kernel<TILE_FLOATS, false>,
                         (const void*)mcaq_tiles_ema_kernel<TILE_FLOATS_PAD, true>,
                         (const void*)mcaq_tiles_ema_kernel<TILE_FLOATS, true>};
    for (const void* k : ks) {
      const hipError_t ae = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
      if (ae != hipSuccess) return (int)ae;
    }
    set_te = lim;
  }
  const dim3 g(L.grid_b + wg + (count > 0 ? 1 : 0)), t(TILES_THREADS);
  if (L.ts == TILE_FLOATS_PAD) {
    if (smo) hipLaunchKernelGGL((mcaq_tiles_ema_kernel<TILE_FLOATS_PAD, true>), g, t, L.dyn_b, stream, L.a, L.wlds, r, L.grid_b);
    else hipLaunchKernelGGL((mcaq_tiles_ema_kernel<TILE_FLOATS_PAD, false>), g, t, L.dyn_b, stream, L.a, L.wlds, r, L.grid_b);
  } else {
    if (smo) hipLaunchKernelGGL((mcaq_tiles_ema_kernel<TILE_FLOATS, true>), g, t, L.dyn_b, stream, L.a, L.wlds, r, L.grid_b);
    else hipLaunchKernelGGL((mcaq_tiles_ema_kernel<TILE_FLOATS, false>), g, t, L.dyn_b, stream, L.a, L.wlds, r, L.grid_b);
  }
  return (int)hipGetLastError();
}

int mcaq_mapper_train_forward_stage(const mcaq_mapper_params* P, const float* c, int n, float min_bits,
                                    float max_bits, float temperature, float momentum, int round_bits,
                                    int update_stats, float* bits, float* work, int stage, const float* gathered,
                                    int world, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !c || !bits || !work || n < 1 || stage < 1 || stage > 4 || world < 1 || (stage >= 2 && !gathered))
    return (int)hipErrorInvalidValue;
  MapperTrainArgs A{};
  A.P = *P; A.c = c; A.bits = bits; A.work = work; A.n = n; A.nwg = (n + TR_TPB - 1) / TR_TPB;
  A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature; A.momentum = momentum;
  A.round_bits = round_bits; A.update_stats = update_stats;
  A.gstat = gathered; A.gworld = stage >= 2 ? world : 0;
  const dim3 g(A.nwg), t(MTH);
  switch (stage) {
    case 1: hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<1>, g, t, 0, stream, A); break;
    case 2: hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<2>, g, t, 0, stream, A); break;
    case 3: hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<3>, g, t, 0, stream, A); break;
    default: hipLaunchKernelGGL(mcaq_mapper_fwd_kernel<4>, g, t, 0, stream, A); break;
  }
  return (int)hipGetLastError();
}

int mcaq_mapper_train_backward_stage(const mcaq_mapper_params* P, const float* c, int n, const float* gbits,
                                     float min_bits, float max_bits, float temperature, float* work, float* gc,
                                     float* gpart, int stage, const float* gsums, const float* gathered1, int world,
                                     hipStream_t stream) {
  using namespace mcaq;
  if (!P || !c || !gbits || !gc || !gpart || !work || n < 1 || stage < 1 || stage > 4 || world < 1 ||
      (stage <= 3 && (!gsums || !gathered1)))
    return (int)hipErrorInvalidValue;
  MapperTrainArgs A{};
  A.P = *P; A.c = c; A.gbits = gbits; A.gc = gc; A.work = work; A.gpart = gpart; A.n = n;
  A.nwg = (n + TR_TPB - 1) / TR_TPB;
  A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature;
  A.gbsum = gsums; A.gstat1 = gathered1; A.gworld = stage <= 3 ? world : 0;
  const dim3 g(A.nwg), t(MTH);
  switch (stage) {
    case 4: hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<4>, g, t, 0, stream, A); break;
    case 3: hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<3>, g, t, 0, stream, A); break;
    case 2: hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<2>, g, t, 0, stream, A); break;
    default: hipLaunchKernelGGL(mcaq_mapper_bwd_kernel<1>, g, t, 0, stream, A); break;
  }
  return (int)hipGetLastError();
}

int mcaq_mapper_train_reduce(const float* work, int n, int kind, int layer, float* out, hipStream_t stream) {
  using namespace mcaq;
  if (!work || !out || n < 1 || kind < 0 || kind > 1 || layer < 1 || layer > 3) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mcaq_mapper_reduce_kernel, dim3(1), dim3(64), 0, stream, work, n, kind, layer, out);
  return (int)hipGetLastError();
}

int mcaq_mapper_train_grad_reduce(int n, const float* gpart, float* gparams, int accumulate, hipStream_t stream) {
  using namespace mcaq;
  if (!gpart || !gparams || n < 1) return (int)hipErrorInvalidValue;
  const int nwg = (n + TR_TPB - 1) / TR_TPB;
  hipLaunchKernelGGL(mcaq_tr_reduce_kernel, dim3((MG_SIZE + 255) / 256), dim3(256), 0, stream, gpart, nwg,
                     (int)MG_SIZE, (int)MG_SIZE, gparams, accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

size_t mcaq_mapper_gpart_floats(int n) { return (size_t)((n + mcaq::TR_TPB - 1) / mcaq::TR_TPB) * mcaq::MG_SIZE; }

size_t mcaq_head_gpart_floats(int n) { return (size_t)((n + mcaq::TR_TPB - 1) / mcaq::TR_TPB) * mcaq::CG_SIZE; }

int mcaq_head_train_backward(const mcaq_cmlp_params* P, const float* phi, const float* craw, const float* gC, int B,
                             int ht, int wt, float* gcraw, float* gparams, float* gpart, int accumulate,
                             hipStream_t stream) {
  using namespace mcaq;
  if (!P || !phi || !craw || !gC || !gcraw || !gpart || B < 1 || ht < 1 || wt < 1)
    return (int)hipErrorInvalidValue;
  HeadTrainArgs A{};
  A.P = *P; A.phi = phi; A.craw = craw; A.gC = gC; A.gcraw = gcraw; A.gpart = gpart;
  A.B = B; A.ht = ht; A.wt = wt; A.n = B * ht * wt; A.nwg = (A.n + TR_TPB - 1) / TR_TPB;
  const size_t lb = (size_t)53 * ht * wt * sizeof(float);
  if (lb > 160 * 1024 - 1024) return (int)hipErrorInvalidValue;
  const size_t lc = (size_t)(TR_TPB * CB_ST + CB_NW * TR_TPB + 4096) * sizeof(float);
  static int set = 0;
  if (!set) {
    hipError_t e = hipFuncSetAttribute((const void*)mcaq_cmlp_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lc);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)mcaq_bilateral_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 1024);
    if (e != hipSuccess) return (int)e;
    set = 1;
  }
  hipLaunchKernelGGL(mcaq_bilateral_bwd_kernel, dim3(B), dim3(BL_TH), lb, stream, A);
  hipLaunchKernelGGL(mcaq_cmlp_bwd_kernel, dim3(A.nwg), dim3(64 * CB_NW), lc, stream, A);
  if (gparams)   // NULL: the caller reduces gpart (mcaq_head_train_grad_reduce)
    hipLaunchKernelGGL(mcaq_tr_reduce_kernel, dim3((CG_SIZE + 255) / 256), dim3(256), 0, stream, (const float*)gpart,
                       A.nwg, (int)CG_SIZE, (int)CG_SIZE, gparams, accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

int mcaq_mapper_train_forward_multi(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                    float min_bits, float max_bits, float temperature, float momentum,
                                    int round_bits, int update_stats, hipStream_t stream) {
  using namespace mcaq;
  // one launch per stage for every segment: several segments updating the
  // shared running statistics in-kernel would race (update_stats 1)
  if (!P || !segs || nseg < 1 || nseg > TR_MAXSEG || (nseg > 1 && update_stats == 1)) return (int)hipErrorInvalidValue;
  TrMulti<MapperTrainArgs> M{};
  int wg = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_mapper_seg& g = segs[k];
    if (!g.c || !g.bits || !g.work || g.n < 1) return (int)hipErrorInvalidValue;
    MapperTrainArgs& A = M.s[k];
    A.P = *P; A.c = g.c; A.bits = g.bits; A.work = g.work; A.n = g.n; A.nwg = (g.n + TR_TPB - 1) / TR_TPB;
    A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature; A.momentum = momentum;
    A.round_bits = round_bits; A.update_stats = update_stats; A.wg0 = wg;
    wg += A.nwg;
  }
  M.nseg = nseg;
  const dim3 g(wg), t(MTH);
  hipLaunchKernelGGL(mcaq_mapper_fwd_multi_kernel<1>, g, t, 0, stream, M);
  hipLaunchKernelGGL(mcaq_mapper_fwd_multi_kernel<2>, g, t, 0, stream, M);
  hipLaunchKernelGGL(mcaq_mapper_fwd_multi_kernel<3>, g, t, 0, stream, M);
  hipLaunchKernelGGL(mcaq_mapper_fwd_multi_kernel<4>, g, t, 0, stream, M);
  return (int)hipGetLastError();
}

int mcaq_mapper_train_forward_stage_multi(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                          float min_bits, float max_bits, float temperature, float momentum,
                                          int round_bits, int update_stats, int stage, const float* const* gathered,
                                          int world, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !segs || nseg < 1 || nseg > TR_MAXSEG || (nseg > 1 && update_stats == 1) || stage < 1 || stage > 4 ||
      world < 1 || (stage >= 2 && !gathered))
    return (int)hipErrorInvalidValue;
  TrMulti<MapperTrainArgs> M{};
  int wg = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_mapper_seg& g = segs[k];
    if (!g.c || !g.bits || !g.work || g.n < 1 || (stage >= 2 && !gathered[k])) return (int)hipErrorInvalidValue;
    MapperTrainArgs& A = M.s[k];
    A.P = *P; A.c = g.c; A.bits = g.bits; A.work = g.work; A.n = g.n; A.nwg = (g.n + TR_TPB - 1) / TR_TPB;
    A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature; A.momentum = momentum;
    A.round_bits = round_bits; A.update_stats = update_stats; A.wg0 = wg;
    A.gstat = stage >= 2 ? gathered[k] : nullptr; A.gworld = stage >= 2 ? world : 0;
    wg += A.nwg;
  }
  M.nseg = nseg;
  const dim3 g(wg), t(MTH);
  switch (stage) {
    case 1: hipLaunchKernelGGL(mcaq_mapper_fwd_multi_kernel<1>, g, t, 0, stream, M); break;
    case 2: hipLaunchKernelGGL(mcaq_mapper_fwd_multi_kernel<2>, g, t, 0, stream, M); break;
    case 3: hipLaunchKernelGGL(mcaq_mapper_fwd_multi_kernel<3>, g, t, 0, stream, M); break;
    default: hipLaunchKernelGGL(mcaq_mapper_fwd_multi_kernel<4>, g, t, 0, stream, M); break;
  }
  return (int)hipGetLastError();
}

int mcaq_mapper_train_backward_stage_multi(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                           float min_bits, float max_bits, float temperature, int stage,
                                           const float* const* gsums, const float* const* gathered1, int world,
                                           hipStream_t stream) {
  using namespace mcaq;
  if (!P || !segs || nseg < 1 || nseg > TR_MAXSEG || stage < 1 || stage > 4 || world < 1 ||
      (stage <= 3 && (!gsums || !gathered1)))
    return (int)hipErrorInvalidValue;
  TrMulti<MapperTrainArgs> M{};
  int wg = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_mapper_seg& g = segs[k];
    if (!g.c || !g.gbits || !g.gc || !g.gpart || !g.work || g.n < 1 || (stage <= 3 && (!gsums[k] || !gathered1[k])))
      return (int)hipErrorInvalidValue;
    MapperTrainArgs& A = M.s[k];
    A.P = *P; A.c = g.c; A.gbits = g.gbits; A.gc = g.gc; A.work = g.work; A.gpart = g.gpart; A.n = g.n;
    A.nwg = (g.n + TR_TPB - 1) / TR_TPB;
    A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature; A.wg0 = wg;
    A.gbsum = stage <= 3 ? gsums[k] : nullptr; A.gstat1 = stage <= 3 ? gathered1[k] : nullptr;
    A.gworld = stage <= 3 ? world : 0;
    wg += A.nwg;
  }
  M.nseg = nseg;
  const dim3 g(wg), t(MTH);
  switch (stage) {
    case 4: hipLaunchKernelGGL(mcaq_mapper_bwd_multi_kernel<4>, g, t, 0, stream, M); break;
    case 3: hipLaunchKernelGGL(mcaq_mapper_bwd_multi_kernel<3>, g, t, 0, stream, M); break;
    case 2: hipLaunchKernelGGL(mcaq_mapper_bwd_multi_kernel<2>, g, t, 0, stream, M); break;
    default: hipLaunchKernelGGL(mcaq_mapper_bwd_multi_kernel<1>, g, t, 0, stream, M); break;
  }
  return (int)hipGetLastError();
}

int mcaq_mapper_train_backward_multi_ride(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                          float min_bits, float max_bits, float temperature,
                                          const mcaq_reduce_seg* rsegs, int nr, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !segs || nseg < 1 || nseg > TR_MAXSEG || nr < 0 || nr > TR_MAXSEG || (nr > 0 && !rsegs))
    return (int)hipErrorInvalidValue;
  TrMulti<TrReduceSeg> R{};
  for (int k = 0; k < nr; ++k) {
    const mcaq_reduce_seg& g = rsegs[k];
    if (!g.part || !g.out || g.nparts < 1 || g.stride < g.count || g.count < 1 || g.count != rsegs[0].count)
      return (int)hipErrorInvalidValue;
    R.s[k] = TrReduceSeg{g.part, g.out, g.nparts, g.stride, g.count, g.accumulate, g.scale};
  }
  R.nseg = nr;
  TrMulti<MapperTrainArgs> M{};
  int wg = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_mapper_seg& g = segs[k];
    if (!g.c || !g.gbits || !g.gc || !g.gpart || !g.work || g.n < 1) return (int)hipErrorInvalidValue;
    MapperTrainArgs& A = M.s[k];
    A.P = *P; A.c = g.c; A.gbits = g.gbits; A.gc = g.gc; A.work = g.work; A.gpart = g.gpart; A.n = g.n;
    A.nwg = (g.n + TR_TPB - 1) / TR_TPB;
    A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature; A.wg0 = wg;
    wg += A.nwg;
  }
  M.nseg = nseg;
  const dim3 g(wg), t(MTH);
  if (nr > 0)
    hipLaunchKernelGGL(mcaq_mapper_bwd_ride_kernel<4>, dim3(wg + (nr * R.s[0].count + MTH - 1) / MTH), t, 0, stream,
                       M, R, wg);
  else
    hipLaunchKernelGGL(mcaq_mapper_bwd_multi_kernel<4>, g, t, 0, stream, M);
  hipLaunchKernelGGL(mcaq_mapper_bwd_multi_kernel<3>, g, t, 0, stream, M);
  hipLaunchKernelGGL(mcaq_mapper_bwd_multi_kernel<2>, g, t, 0, stream, M);
  hipLaunchKernelGGL(mcaq_mapper_bwd_multi_kernel<1>, g, t, 0, stream, M);
  return (int)hipGetLastError();
}

int mcaq_mapper_train_backward_multi(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                     float min_bits, float max_bits, float temperature, hipStream_t stream) {
  return mcaq_mapper_train_backward_multi_ride(P, segs, nseg, min_bits, max_bits, temperature, nullptr, 0, stream);
}

#if defined(MCAQ_STAMPS_WG)
int mcaq_read_wg_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(mcaq::g_mapx_wg), sizeof(mcaq::g_mapx_wg));
}
#endif

size_t mcaq_mapper_sync_bytes(int total_wg) {
  using namespace mcaq;
  return total_wg < 1 ? 0 : (size_t)MAPX_HDR * 4 + (size_t)3 * MAPX_STRIDE * 8 * total_wg;
}

int mcaq_mapper_fused_max_wg(void) { return mcaq::MAPPER_COOP_MAX_WG; }

}  // extern "C"

namespace mcaq {
// segments of a fused launch over the sync buffer (mcaq_mapper_sync_bytes of
// the total workgroup count): header words, then per segment 3 exchange
// regions of nwg x MAPX_STRIDE granules, segments in order
static int mapx_layout(TrMulti<MapperTrainArgs>& M, int wg, void* sync, size_t sync_bytes) {
  if (!sync || wg > MAPPER_COOP_MAX_WG || sync_bytes < mcaq_mapper_sync_bytes(wg) ||
      ((uintptr_t)sync & 7) != 0)
    return (int)hipErrorInvalidValue;
  unsigned* hdr = static_cast<unsigned*>(sync);
  mapx_t* gran = reinterpret_cast<mapx_t*>(hdr + MAPX_HDR);
  for (int k = 0; k < M.nseg; ++k) {
    MapperTrainArgs& A = M.s[k];
    A.gx = gran + (size_t)3 * MAPX_STRIDE * A.wg0;
    A.gep = hdr + k;
    A.gst = hdr + MAPX_STATUS;
  }
  return 0;
}
}  // namespace mcaq

extern "C" {

int mcaq_mapper_train_forward_fused(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                    float min_bits, float max_bits, float temperature, float momentum,
                                    int round_bits, int update_stats, void* sync, size_t sync_bytes,
                                    hipStream_t stream) {
  using namespace mcaq;
  if (!P || !segs || nseg < 1 || nseg > TR_MAXSEG || (nseg > 1 && update_stats == 1)) return (int)hipErrorInvalidValue;
  TrMulti<MapperTrainArgs> M{};
  int wg = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_mapper_seg& g = segs[k];
    if (!g.c || !g.bits || !g.work || g.n < 1) return (int)hipErrorInvalidValue;
    MapperTrainArgs& A = M.s[k];
    A.P = *P; A.c = g.c; A.bits = g.bits; A.work = g.work; A.n = g.n; A.nwg = (g.n + TR_TPB - 1) / TR_TPB;
    A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature; A.momentum = momentum;
    A.round_bits = round_bits; A.update_stats = update_stats; A.wg0 = wg;
    wg += A.nwg;
  }
  M.nseg = nseg;
  const int le = mapx_layout(M, wg, sync, sync_bytes);
  if (le) return le;
  hipLaunchKernelGGL(mcaq_mapper_fwd_fused_kernel, dim3(wg), dim3(MTH), 0, stream, M);
  return (int)hipGetLastError();
}

int mcaq_mapper_train_backward_fused(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                     float min_bits, float max_bits, float temperature,
                                     const mcaq_reduce_seg* rsegs, int nr, void* sync, size_t sync_bytes,
                                     hipStream_t stream) {
  using namespace mcaq;
  if (!P || !segs || nseg < 1 || nseg > TR_MAXSEG || nr < 0 || nr > TR_MAXSEG || (nr > 0 && !rsegs))
    return (int)hipErrorInvalidValue;
  TrMulti<TrReduceSeg> R{};
  for (int k = 0; k < nr; ++k) {
    const mcaq_reduce_seg& g = rsegs[k];
    if (!g.part || !g.out || g.nparts < 1 || g.stride < g.count || g.count < 1 || g.count != rsegs[0].count)
      return (int)hipErrorInvalidValue;
    R.s[k] = TrReduceSeg{g.part, g.out, g.nparts, g.stride, g.count, g.accumulate, g.scale};
  }
  R.nseg = nr;
  TrMulti<MapperTrainArgs> M{};
  int wg = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_mapper_seg& g = segs[k];
    if (!g.c || !g.gbits || !g.gc || !g.gpart || !g.work || g.n < 1) return (int)hipErrorInvalidValue;
    MapperTrainArgs& A = M.s[k];
    A.P = *P; A.c = g.c; A.gbits = g.gbits; A.gc = g.gc; A.work = g.work; A.gpart = g.gpart; A.n = g.n;
    A.nwg = (g.n + TR_TPB - 1) / TR_TPB;
    A.min_bits = min_bits; A.max_bits = max_bits; A.temperature = temperature; A.wg0 = wg;
    wg += A.nwg;
  }
  M.nseg = nseg;
  const int le = mapx_layout(M, wg, sync, sync_bytes);
  if (le) return le;
  const int rwg = nr > 0 ? (nr * R.s[0].count + MTH - 1) / MTH : 0;
  hipLaunchKernelGGL(mcaq_mapper_bwd_fused_kernel, dim3(wg + rwg), dim3(MTH), 0, stream, M, R, wg);
  return (int)hipGetLastError();
}

int mcaq_head_train_backward_multi_ride(const mcaq_cmlp_params* P, const mcaq_head_seg* segs, int nseg,
                                        const mcaq_reduce_seg* rsegs, int nr, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !segs || nseg < 1 || nseg > TR_MAXSEG || nr < 0 || nr > TR_MAXSEG || (nr > 0 && !rsegs))
    return (int)hipErrorInvalidValue;
  TrMulti<TrReduceSeg> R{};
  for (int k = 0; k < nr; ++k) {
    const mcaq_reduce_seg& g = rsegs[k];
    if (!g.part || (!g.out && k == 0) || g.nparts < 1 || g.stride < g.count || g.count < 1 || g.count != rsegs[0].count)
      return (int)hipErrorInvalidValue;
    R.s[k] = TrReduceSeg{g.part, g.out, g.nparts, g.stride, g.count, g.accumulate, g.scale};
  }
  R.nseg = nr;
  TrMulti<HeadTrainArgs> Mb{}, Mc{};
  int wb = 0, wc = 0;
  size_t lb = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_head_seg& g = segs[k];
    if (!g.phi || !g.craw || !g.gC || !g.gcraw || !g.gpart || g.B < 1 || g.ht < 1 || g.wt < 1)
      return (int)hipErrorInvalidValue;
    HeadTrainArgs A{};
    A.P = *P; A.phi = g.phi; A.craw = g.craw; A.gC = g.gC; A.gcraw = g.gcraw; A.gpart = g.gpart;
    A.B = g.B; A.ht = g.ht; A.wt = g.wt; A.n = g.B * g.ht * g.wt; A.nwg = (A.n + TR_TPB - 1) / TR_TPB;
    const size_t l = (size_t)53 * g.ht * g.wt * sizeof(float);
    if (l > 160 * 1024 - 1024) return (int)hipErrorInvalidValue;
    lb = l > lb ? l : lb;
    Mb.s[k] = A; Mb.s[k].wg0 = wb; wb += A.B;      // bilateral: one workgroup per image
    Mc.s[k] = A; Mc.s[k].wg0 = wc; wc += A.nwg;    // MLP: 64 tiles per workgroup
  }
  Mb.nseg = Mc.nseg = nseg;
  const size_t lc = (size_t)(TR_TPB * CB_ST + CB_NW * TR_TPB + 4096) * sizeof(float);
  static int set = 0;
  if (!set) {
    hipError_t e = hipFuncSetAttribute((const void*)mcaq_cmlp_bwd_multi_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lc);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)mcaq_bilateral_bwd_multi_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 1024);
    if (e != hipSuccess) return (int)e;
    set = 1;
  }
  if (nr > 0) {
    static int set_r = 0;
    if (!set_r) {
      const hipError_t e = hipFuncSetAttribute((const void*)mcaq_bilateral_bwd_ride_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);
      if (e != hipSuccess) return (int)e;
      set_r = 1;
    }
    const int rw = (R.s[0].count + BL_TH - 1) / BL_TH;
    hipLaunchKernelGGL(mcaq_bilateral_bwd_ride_kernel, dim3(wb + rw), dim3(BL_TH), lb, stream, Mb, R, wb);
  } else {
    hipLaunchKernelGGL(mcaq_bilateral_bwd_multi_kernel, dim3(wb), dim3(BL_TH), lb, stream, Mb);
  }
  hipLaunchKernelGGL(mcaq_cmlp_bwd_multi_kernel, dim3(wc), dim3(64 * CB_NW), lc, stream, Mc);
  return (int)hipGetLastError();
}

int mcaq_head_train_backward_multi(const mcaq_cmlp_params* P, const mcaq_head_seg* segs, int nseg, hipStream_t stream) {
  return mcaq_head_train_backward_multi_ride(P, segs, nseg, nullptr, 0, stream);
}

size_t mcaq_head_sync_bytes(int total_wg) {
  using namespace mcaq;
  return total_wg < 1 ? 0 : (size_t)MAPX_HDR * 4 + (size_t)total_wg * CG_SIZE * 8;
}

int mcaq_head_train_backward_fused(const mcaq_cmlp_params* P, const mcaq_head_seg* segs, int nseg,
                                   const mcaq_reduce_seg* rsegs, int nr, float* out, int accumulate, float scale,
                                   void* sync, size_t sync_bytes, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !segs || nseg < 1 || nseg > TR_MAXSEG || nr < 0 || nr > TR_MAXSEG || (nr > 0 && !rsegs) || !out ||
      !sync || ((uintptr_t)sync & 7) != 0)
    return (int)hipErrorInvalidValue;
  TrMulti<TrReduceSeg> R{};
  for (int k = 0; k < nr; ++k) {
    const mcaq_reduce_seg& g = rsegs[k];
    if (!g.part || (!g.out && k == 0) || g.nparts < 1 || g.stride < g.count || g.count < 1 || g.count != rsegs[0].count)
      return (int)hipErrorInvalidValue;
    R.s[k] = TrReduceSeg{g.part, g.out, g.nparts, g.stride, g.count, g.accumulate, g.scale};
  }
  R.nseg = nr;
  TrMulti<HeadTrainArgs> Mb{}, Mc{};
  int wb = 0, wc = 0;
  size_t lb = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_head_seg& g = segs[k];
    if (!g.phi || !g.craw || !g.gC || !g.gcraw || !g.gpart || g.B < 1 || g.ht < 1 || g.wt < 1)
      return (int)hipErrorInvalidValue;
    HeadTrainArgs A{};
    A.P = *P; A.phi = g.phi; A.craw = g.craw; A.gC = g.gC; A.gcraw = g.gcraw; A.gpart = g.gpart;
    A.B = g.B; A.ht = g.ht; A.wt = g.wt; A.n = g.B * g.ht * g.wt; A.nwg = (A.n + TR_TPB - 1) / TR_TPB;
    const size_t l = (size_t)53 * g.ht * g.wt * sizeof(float);
    if (l > 160 * 1024 - 1024) return (int)hipErrorInvalidValue;
    lb = l > lb ? l : lb;
    Mb.s[k] = A; Mb.s[k].wg0 = wb; wb += A.B;
    Mc.s[k] = A; Mc.s[k].wg0 = wc; wc += A.nwg;
  }
  Mb.nseg = Mc.nseg = nseg;
  if (wc > MAPPER_COOP_MAX_WG || sync_bytes < mcaq_head_sync_bytes(wc)) return (int)hipErrorInvalidValue;
  const size_t lc = (size_t)(TR_TPB * CB_ST + CB_NW * TR_TPB + 4096) * sizeof(float);
  static_assert((size_t)TR_TPB * CB_ST >= (size_t)CG_SIZE + MAPPER_COOP_MAX_WG, "slice buffer in the tile vectors");
  static int set = 0;
  if (!set) {
    hipError_t e = hipFuncSetAttribute((const void*)mcaq_cmlp_bwd_fused_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lc);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)mcaq_bilateral_bwd_multi_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 1024);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)mcaq_bilateral_bwd_ride_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 1024);
    if (e != hipSuccess) return (int)e;
    set = 1;
  }
  if (nr > 0) {
    const int rw = (R.s[0].count + BL_TH - 1) / BL_TH;
    hipLaunchKernelGGL(mcaq_bilateral_bwd_ride_kernel, dim3(wb + rw), dim3(BL_TH), lb, stream, Mb, R, wb);
  } else {
    hipLaunchKernelGGL(mcaq_bilateral_bwd_multi_kernel, dim3(wb), dim3(BL_TH), lb, stream, Mb);
  }
  const CmlpRed cr{static_cast<unsigned*>(sync), out, accumulate, scale, wc};
  hipLaunchKernelGGL(mcaq_cmlp_bwd_fused_kernel, dim3(wc), dim3(64 * CB_NW), lc, stream, Mc, cr);
  return (int)hipGetLastError();
}

int mcaq_smask_train_backward_multi(const mcaq_smask_seg* segs, int nseg, hipStream_t stream) {
  using namespace mcaq;
  if (!segs || nseg < 1 || nseg > TR_MAXSEG) return (int)hipErrorInvalidValue;
  TrMulti<MaskTrainArgs> M{};
  int wg = 0;
  size_t lb = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_smask_seg& g = segs[k];
    if (!g.bits || !g.absmean || !g.gm || !g.gbits || !g.gpart || g.B < 1 || g.ht < 1 || g.wt < 1 || g.H < g.ht ||
        g.W < g.wt)
      return (int)hipErrorInvalidValue;
    MaskTrainArgs& A = M.s[k];
    A.P = g.P; A.bits = g.bits; A.absmean = g.absmean; A.gm = g.gm; A.gbits = g.gbits; A.gpart = g.gpart;
    A.B = g.B; A.H = g.H; A.W = g.W; A.ht = g.ht; A.wt = g.wt; A.accumulate = g.accumulate; A.wg0 = wg;
    A.stage = smask_stage_ok(g.absmean, g.gm, g.H, g.W, g.ht, g.wt) ? 1 : 0;
    wg += g.B;
    const size_t l = smask_lds_bytes(g.H, g.W, g.ht, g.wt, A.stage != 0);
    if (l > 160 * 1024 - 1024) return (int)hipErrorInvalidValue;
    lb = l > lb ? l : lb;
  }
  M.nseg = nseg;
  static int set = 0;
  if (!set) {
    const hipError_t e = hipFuncSetAttribute((const void*)mcaq_smask_bwd_multi_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);
    if (e != hipSuccess) return (int)e;
    set = 1;
  }
  hipLaunchKernelGGL(mcaq_smask_bwd_multi_kernel, dim3(wg), dim3(SM_TH), lb, stream, M);
  return (int)hipGetLastError();
}

int mcaq_qat_smask_backward_multi(const mcaq_qat_smask_seg* segs, int nseg, const mcaq_bit_budget* bb,
                                  hipStream_t stream) {
  using namespace mcaq;
  if (!segs || !bb || nseg < 1 || nseg > TR_MAXSEG || bb->nscales < 1 ||
      ((bb->g_avg || bb->g_loss) && !bb->avg))
    return (int)hipErrorInvalidValue;
  TrMulti<MaskTrainArgs> M{};
  int wg = 0;
  size_t lb = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_qat_smask_seg& g = segs[k];
    if (!g.bits || !g.absmean || !g.qat_work || !g.gbits || !g.gpart || g.B < 1 || g.C < 1 || g.ht < 1 ||
        g.wt < 1 || g.H < g.ht || g.W < g.wt)
      return (int)hipErrorInvalidValue;
    MaskTrainArgs& A = M.s[k];
    A.P = g.P; A.bits = g.bits; A.absmean = g.absmean; A.gm = nullptr; A.gbits = g.gbits; A.gpart = g.gpart;
    A.B = g.B; A.H = g.H; A.W = g.W; A.ht = g.ht; A.wt = g.wt; A.accumulate = 0; A.wg0 = wg;
    A.qwork = g.qat_work; A.qC = g.C; A.bb = *bb;
    A.rn = 1.0f / (float)(g.B * g.ht * g.wt);
    // the |x| plane staged when it fits (16-byte rows of 4); the fold planes always in LDS
    A.stage = (((g.H * g.W) & 3) == 0 && ((uintptr_t)g.absmean & 15) == 0) ? 1 : 0;
    wg += g.B;
    const size_t l = smask_lds_bytes(g.H, g.W, g.ht, g.wt, true, true);
    if (l > 160 * 1024 - 1024) return (int)hipErrorInvalidValue;
    lb = l > lb ? l : lb;
  }
  M.nseg = nseg;
  static int set = 0;
  if (!set) {
    const hipError_t e = hipFuncSetAttribute((const void*)mcaq_smask_bwd_multi_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);
    if (e != hipSuccess) return (int)e;
    set = 1;
  }
  hipLaunchKernelGGL(mcaq_smask_bwd_multi_kernel, dim3(wg), dim3(SM_TH), lb, stream, M);
  return (int)hipGetLastError();
}

int mcaq_bit_budget_forward(const float* const* bits, const int* n, int nseg, float target, float* avg, float* loss,
                            hipStream_t stream) {
  using namespace mcaq;
  if (!bits || !n || !avg || nseg < 1 || nseg > TR_MAXSEG) return (int)hipErrorInvalidValue;
  BitBudgetArgs a{};
  for (int k = 0; k < nseg; ++k) {
    if (!bits[k] || n[k] < 1) return (int)hipErrorInvalidValue;
    a.bits[k] = bits[k]; a.n[k] = n[k];
  }
  a.nseg = nseg; a.target = target; a.avg = avg; a.loss = loss;
  hipLaunchKernelGGL(mcaq_bit_budget_kernel, dim3(1), dim3(1024), 0, stream, a);
  return (int)hipGetLastError();
}

int mcaq_train_reduce_multi(const mcaq_reduce_seg* segs, int nseg, int chain, hipStream_t stream) {
  using namespace mcaq;
  if (!segs || nseg < 1 || nseg > TR_MAXSEG) return (int)hipErrorInvalidValue;
  TrMulti<TrReduceSeg> M{};
  int cmax = 0;
  for (int k = 0; k < nseg; ++k) {
    const mcaq_reduce_seg& g = segs[k];
    if (!g.part || (!g.out && !(chain && k > 0)) || g.nparts < 1 || g.stride < g.count || g.count < 1)
      return (int)hipErrorInvalidValue;
    if (chain && g.count != segs[0].count) return (int)hipErrorInvalidValue;
    M.s[k] = TrReduceSeg{g.part, g.out, g.nparts, g.stride, g.count, g.accumulate, g.scale};
    cmax = g.count > cmax ? g.count : cmax;
  }
  M.nseg = nseg;
  hipLaunchKernelGGL(mcaq_tr_reduce_multi_kernel, dim3((cmax + 255) / 256, chain ? 1 : nseg), dim3(256), 0, stream, M,
                     chain ? 1 : 0);
  return (int)hipGetLastError();
}

int mcaq_head_train_grad_reduce(int n, const float* gpart, float* gparams, int accumulate, hipStream_t stream) {
  using namespace mcaq;
  if (!gpart || !gparams || n < 1) return (int)hipErrorInvalidValue;
  const int nwg = (n + TR_TPB - 1) / TR_TPB;
  hipLaunchKernelGGL(mcaq_tr_reduce_kernel, dim3((CG_SIZE + 255) / 256), dim3(256), 0, stream, gpart, nwg,
                     (int)CG_SIZE, (int)CG_SIZE, gparams, accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

size_t mcaq_smask_gpart_floats(int B) { return (size_t)B * mcaq::SG_SIZE; }

static int pack_args(const mcaq_pack_seg* segs, int nseg, float* out, int total, mcaq::PackArgs& a) {
  if (!segs || !out || nseg < 1 || nseg > MCAQ_PACK_MAXSEG || total < 1) return (int)hipErrorInvalidValue;
  for (int i = 0; i < nseg; ++i) {
    const mcaq_pack_seg& g = segs[i];
    if (!g.src || g.n < 1 || g.dst < 0 || (g.mode != 0 && (g.mode != 1 || g.k < 1))) return (int)hipErrorInvalidValue;
    const int len = g.mode == 0 ? g.n : ((g.n + 15) >> 4) * (((g.k + 3) & ~3) >> 2) * 64;
    if (g.dst + len > total) return (int)hipErrorInvalidValue;
    a.seg[i] = g;
  }
  a.nseg = nseg; a.total = total;
  return 0;
}

int mcaq_pack(const mcaq_pack_seg* segs, int nseg, float* out, int total, hipStream_t stream) {
  using namespace mcaq;
  PackArgs a{};
  const int e = pack_args(segs, nseg, out, total, a);
  if (e) return e;
  hipLaunchKernelGGL(mcaq_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, a, out);
  return (int)hipGetLastError();
}

int mcaq_stats_pack(const mcaq_stats_scale* scales, int nscales, const mcaq_pack_seg* segs, int nseg, float* out,
                    int total, hipStream_t stream) {
  using namespace mcaq;
  StatsArgs a;
  bool vec;
  const int e = stats_args(scales, nscales, a, vec);
  if (e) return e;
  if (scales[0].dtype != MCAQ_DTYPE_F32) return (int)hipErrorNotSupported;   // the train step's x is fp32
  PackArgs p{};
  const int pe = pack_args(segs, nseg, out, total, p);
  if (pe) return pe;
  const dim3 g(a.units_total + (total + 255) / 256);
  if (vec)
    launch_k(mcaq_stats_pack_kernel<true>, g, dim3(256), 0, stream, a, p, out);
  else
    launch_k(mcaq_stats_pack_kernel<false>, g, dim3(256), 0, stream, a, p, out);
  return (int)hipGetLastError();
}

int mcaq_smask_train_backward(const mcaq_smask_params* P, const float* bits, const float* absmean, const float* gm,
                              int B, int H, int W, int ht, int wt, float* gbits, int accumulate, float* gparams,
                              float* gpart, hipStream_t stream) {
  using namespace mcaq;
  if (!P || !bits || !absmean || !gm || !gbits || !gparams || !gpart || B < 1 || ht < 1 || wt < 1 || H < ht || W < wt)
    return (int)hipErrorInvalidValue;
  MaskTrainArgs A{};
  A.P = *P; A.bits = bits; A.absmean = absmean; A.gm = gm; A.gbits = gbits; A.gpart = gpart;
  A.B = B; A.H = H; A.W = W; A.ht = ht; A.wt = wt; A.accumulate = accumulate;
  A.stage = smask_stage_ok(absmean, gm, H, W, ht, wt) ? 1 : 0;
  const size_t lb = smask_lds_bytes(H, W, ht, wt, A.stage != 0);
  if (lb > 160 * 1024 - 1024) return (int)hipErrorInvalidValue;   // m(p) gradient of one image staged in LDS
  static int set = 0;
  if ((int)lb > set) {
    const hipError_t e = hipFuncSetAttribute((const void*)mcaq_smask_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             160 * 1024 - 1024);
    if (e != hipSuccess) return (int)e;
    set = 160 * 1024 - 1024;
  }
  hipLaunchKernelGGL(mcaq_smask_bwd_kernel, dim3(B), dim3(SM_TH), lb, stream, A);
  hipLaunchKernelGGL(mcaq_tr_reduce_kernel, dim3(1), dim3(256), 0, stream, (const float*)gpart, B, (int)SG_SIZE,
                     (int)SG_SIZE, gparams, 0);
  return (int)hipGetLastError();
}

}  // extern "C"
