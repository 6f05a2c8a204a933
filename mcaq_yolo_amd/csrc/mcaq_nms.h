// mcaq_nms.h - gfx950 batched non-maximum suppression of YOLOv8 Detect
// outputs: the postprocess of Predictor.predict / predict_batch
// (mcaq_yolo/inference.py:213-219, 410-417), which calls ultralytics
// `non_max_suppression(preds, conf_thres, iou_thres, max_det)` (ultralytics
// 8.4.63, requirements-lock.txt:13; not vendored) whose suppression step is
// torchvision's CPU `nms` kernel.  Restated from their published algorithm:
//
//   per image: candidates = anchors with max class score > conf_thres
//              (score = max, cls = first argmax); box xywh -> xyxy
//              (xy -/+ wh/2); order by score descending (stable: anchor
//              index ascending on ties); keep the first max_nms;
//              boxes offset by cls * max_wh (0 when agnostic);
//              greedy: a candidate is kept unless IoU(kept, cand) > iou_thres
//              for an earlier kept box, IoU = inter / (area_k + area_c - inter)
//              in fp32, compared in double; the first max_det kept boxes.
//
// Two launches.  The scan kernel spreads the (4+nc, N) slab of every image
// over B x ceil(N/256) workgroups (one anchor per thread, class rows read
// coalesced over anchors): the best class score and first argmax per anchor,
// candidates (score > conf) compacted per image with one atomic per wave into
// a 64-bit key array (ordered-score << 32 | anchor) in the workspace, each
// candidate's class recorded.  The NMS kernel (one 1024-thread workgroup per
// image) then sorts the image's keys - in LDS up to NMS_LDS_KEYS candidates,
// in the global key array beyond (large inputs, e.g. 1280x1280 = 33,600
// anchors at a low threshold) - and walks them in chunks of 256: every
// candidate is tested against the boxes kept so far (4 threads per
// candidate), a 256 x 256 chunk-local suppression bit matrix is built (one
// 64-bit word per thread), then one lane resolves the chunk sequentially with
// bit operations - exactly the greedy order of the CPU kernel.
#pragma once

namespace mcaq {

constexpr int NMS_THREADS = 1024;
constexpr int NMS_LDS_KEYS = 8192;       // LDS key array (64 KiB); more candidates sort in global memory
constexpr int NMS_LDS_KEPT = 1024;       // kept boxes cached in LDS (more: read from the workspace)
constexpr int NMS_CHUNK = 256;

struct NmsArgs {
  const float* pred;   // (B, no, N)
  float* out;          // (B, max_det, 6)
  int* counts;         // (B)
  float* kept;         // (B, max_det, 8) workspace: offset box + area
  int* cls;            // (B, N) workspace: class of each candidate anchor
  int* ncand;          // (B) candidate counts (zeroed before the scan)
  unsigned long long* gkeys;   // (B, pow2(N)) candidate keys
  int B, no, N, np2N, nc, max_det, max_nms, agnostic;
  float conf, max_wh;
  double iou;
};

// order-preserving map of a float to uint32, inverted: ascending key order =
// descending score
__device__ __forceinline__ unsigned int nms_score_key(float s) {
  const unsigned int u = __float_as_uint(s);
  const unsigned int o = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ~o;
}
__device__ __forceinline__ float nms_key_score(unsigned int k) {
  const unsigned int o = ~k;
  const unsigned int u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}

// torchvision nms_kernel.cpp: i = the earlier (kept) box, j = the later one
__device__ __forceinline__ bool nms_iou_gt(float4 bi, float ai, float4 bj, float aj, double thr) {
  const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
  const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
  const float w = fmaxf(0.0f, __fsub_rn(xx2, xx1)), h = fmaxf(0.0f, __fsub_rn(yy2, yy1));
  const float inter = __fmul_rn(w, h);
  const float ovr = __fdiv_rn(inter, __fsub_rn(__fadd_rn(ai, aj), inter));
  return (double)ovr > thr;
}

template <class KeyT>
__device__ __forceinline__ void nms_bitonic(KeyT* keys, int np2, int tid) {
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < np2; i += NMS_THREADS) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long x = keys[i], y = keys[ixj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { keys[i] = y; keys[ixj] = x; }
        }
      }
      __syncthreads();
    }
  }
}

constexpr int NMS_SCAN_THREADS = 256;

__global__ __launch_bounds__(NMS_SCAN_THREADS) void mcaq_nms_scan_kernel(NmsArgs a) {
  const int b = blockIdx.y;
  const int N = a.N;
  const int ai = blockIdx.x * NMS_SCAN_THREADS + threadIdx.x;
  const float* P = a.pred + (size_t)b * a.no * N;
  bool cand = false;
  float best = 0.0f;
  int bj = 0;
  if (ai < N) {
    best = P[(size_t)4 * N + ai];
    int c = 1;
    for (; c + 8 <= a.nc; c += 8) {      // 8 class rows in flight, compared in class order
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = P[(size_t)(4 + c + k) * N + ai];
#pragma unroll
      for (int k = 0; k < 8; ++k) if (v[k] > best) { best = v[k]; bj = c + k; }
    }
    for (; c < a.nc; ++c) {
      const float v = P[(size_t)(4 + c) * N + ai];
      if (v > best) { best = v; bj = c; }
    }
    cand = best > a.conf;
  }
  // one atomic per wave: slots in lane order
  const unsigned long long mask = __ballot(cand);
  if (!mask) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)mask) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(a.ncand + b, __popcll(mask));
  base = __shfl(base, leader);
  if (cand) {
    const int slot = base + __popcll(mask & ((1ull << lane) - 1));
    a.gkeys[(size_t)b * a.np2N + slot] = ((unsigned long long)nms_score_key(best) << 32) | (unsigned int)ai;
    a.cls[(size_t)b * N + ai] = bj;
  }
}

__global__ __launch_bounds__(NMS_THREADS) void mcaq_nms_kernel(NmsArgs a) {
  __shared__ unsigned long long lkeys[NMS_LDS_KEYS];
  __shared__ float4 cbox[NMS_CHUNK];        // offset boxes of the chunk
  __shared__ float4 craw[NMS_CHUNK];        // xyxy boxes (output)
  __shared__ float carea[NMS_CHUNK], cscore[NMS_CHUNK], ccls[NMS_CHUNK];
  __shared__ int csup[NMS_CHUNK];
  __shared__ unsigned long long cmask[NMS_CHUNK][4];
  __shared__ float4 kbox[NMS_LDS_KEPT];     // offset boxes kept so far (first NMS_LDS_KEPT)
  __shared__ float karea[NMS_LDS_KEPT];
  __shared__ unsigned long long alive0[4];
  __shared__ int s_K;

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int N = a.N;
  const float* P = a.pred + (size_t)b * a.no * N;
  float* kept = a.kept + (size_t)b * a.max_det * 8;
  float* out = a.out + (size_t)b * a.max_det * 6;
  const int* ccl = a.cls + (size_t)b * N;
  unsigned long long* gk = a.gkeys + (size_t)b * a.np2N;
  const int n = a.ncand[b];
  if (tid == 0) s_K = 0;
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  const bool inlds = n <= NMS_LDS_KEYS;

  // ---- bitonic sort of the scan's keys (ascending key = score desc, anchor asc)
  if (inlds) {
    for (int i = tid; i < np2; i += NMS_THREADS) lkeys[i] = i < n ? gk[i] : ~0ull;
    __syncthreads();
    nms_bitonic(lkeys, np2, tid);
  } else {
    for (int i = n + tid; i < np2; i += NMS_THREADS) gk[i] = ~0ull;
    __syncthreads();
    nms_bitonic(gk, np2, tid);
  }

  // ---- phase 3: greedy suppression in chunks of 256 sorted candidates
  const int nproc = n < a.max_nms ? n : a.max_nms;
  for (int base = 0; base < nproc; base += NMS_CHUNK) {
    const int cn = (nproc - base) < NMS_CHUNK ? (nproc - base) : NMS_CHUNK;
    if (tid < cn) {
      const unsigned long long key = inlds ? lkeys[base + tid] : gk[base + tid];
      const int ai = (int)(unsigned int)key;
      const int cls = ccl[ai];
      const float x = P[ai], y = P[(size_t)N + ai], w = P[(size_t)2 * N + ai], h = P[(size_t)3 * N + ai];
      const float hw = __fdiv_rn(w, 2.0f), hh = __fdiv_rn(h, 2.0f);   // xywh2xyxy
      const float4 r = make_float4(__fsub_rn(x, hw), __fsub_rn(y, hh), __fadd_rn(x, hw), __fadd_rn(y, hh));
      const float fc = (float)cls;
      const float off = a.agnostic ? 0.0f : __fmul_rn(fc, a.max_wh);
      const float4 o = make_float4(__fadd_rn(r.x, off), __fadd_rn(r.y, off), __fadd_rn(r.z, off), __fadd_rn(r.w, off));
      craw[tid] = r;
      cbox[tid] = o;
      carea[tid] = __fmul_rn(__fsub_rn(o.z, o.x), __fsub_rn(o.w, o.y));
      cscore[tid] = nms_key_score((unsigned int)(key >> 32));
      ccls[tid] = fc;
      csup[tid] = 0;
    }
    __syncthreads();
    const int K = s_K;
    // candidates vs the boxes kept by earlier chunks: 4 threads per candidate
    {
      const int t = tid & (NMS_CHUNK - 1), g = tid >> 8;
      if (t < cn && K > 0) {
        const float4 bj = cbox[t];
        const float aj = carea[t];
        bool s = false;
        const int KL = K < NMS_LDS_KEPT ? K : NMS_LDS_KEPT;
        for (int k = g; k < KL && !s; k += 4) s = nms_iou_gt(kbox[k], karea[k], bj, aj, a.iou);
        for (int k = KL + g; k < K && !s; k += 4) {
          const float4 bk = *reinterpret_cast<const float4*>(kept + (size_t)k * 8);
          const float ak = kept[(size_t)k * 8 + 4];
          s = nms_iou_gt(bk, ak, bj, aj, a.iou);
        }
        if (s) csup[t] = 1;
      }
    }
    __syncthreads();
    // the chunk's survivors of the kept boxes as bit words (wave 0, one ballot per word)
    if (tid < 64) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int t = w * 64 + tid;
        const unsigned long long m = __ballot(t < cn && !csup[t]);
        if (tid == 0) alive0[w] = m;
      }
    }
    // chunk-local matrix: row r, word w covers columns 64w..64w+63 (> r);
    // rows and columns already suppressed by a kept box are never consulted
    {
      const int r = tid >> 2, w = tid & 3;
      unsigned long long bits = 0;
      if (r < cn && !csup[r]) {
        const float4 br = cbox[r];
        const float ar = carea[r];
        const int c0 = w * 64;
        for (int q = 0; q < 64; ++q) {
          const int c = c0 + q;
          if (c > r && c < cn && !csup[c] && nms_iou_gt(br, ar, cbox[c], carea[c], a.iou)) bits |= 1ull << q;
        }
      }
      cmask[r][w] = bits;
    }
    __syncthreads();
    if (tid == 0) {
      // greedy in candidate order, visiting only live candidates: alive =
      // not suppressed by a kept box nor by an earlier kept one of the chunk
      unsigned long long rm[4] = {0ull, 0ull, 0ull, 0ull};
      int Kc = K;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        unsigned long long live = alive0[w] & ~rm[w];
        while (live && Kc < a.max_det) {
          const int q = __ffsll((long long)live) - 1;
          const int r = w * 64 + q;
          const float4 o = cbox[r];
          if (Kc < NMS_LDS_KEPT) {
            kbox[Kc] = o;
            karea[Kc] = carea[r];
          } else {
            float* kp = kept + (size_t)Kc * 8;
            kp[0] = o.x; kp[1] = o.y; kp[2] = o.z; kp[3] = o.w; kp[4] = carea[r];
          }
          const float4 rr = craw[r];
          float* op = out + (size_t)Kc * 6;
          op[0] = rr.x; op[1] = rr.y; op[2] = rr.z; op[3] = rr.w; op[4] = cscore[r]; op[5] = ccls[r];
          ++Kc;
#pragma unroll
          for (int j = 0; j < 4; ++j) rm[j] |= cmask[r][j];
          live = alive0[w] & ~rm[w] & ~((2ull << q) - 1ull);   // bits above q (q = 63: none)
        }
      }
      s_K = Kc;
    }
    __syncthreads();
    if (s_K >= a.max_det) break;
  }
  __syncthreads();
  const int Kf = s_K;
  for (int i = Kf * 6 + tid; i < a.max_det * 6; i += NMS_THREADS) out[i] = 0.0f;
  if (tid == 0) a.counts[b] = Kf;
}

}  // namespace mcaq

extern "C" {

static size_t nms_np2(int N) {
  size_t p = 1;
  while (p < (size_t)N) p <<= 1;
  return p;
}

size_t mcaq_nms_work_floats(int B, int N, int max_det) {
  if (B <= 0 || N < 0 || max_det <= 0) return 0;
  // kept boxes + candidate classes + counts, then the pow2(N) key arrays (u64)
  return (size_t)B * ((size_t)max_det * 8 + (size_t)N + 1) + 2 + (size_t)B * 2 * nms_np2(N);
}

int mcaq_nms(const float* pred, int B, int no, int N, int nc, float conf_thres, double iou_thres, int max_det,
             int max_nms, float max_wh, int agnostic, float* out, int* counts, float* work, hipStream_t stream) {
  if (B < 0 || nc < 1 || no != 4 + nc || N < 0 || N > (1 << 30) || max_det < 1 || max_nms < 1)
    return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  if (!pred || !out || !counts || !work) return (int)hipErrorInvalidValue;
  mcaq::NmsArgs a;
  a.pred = pred; a.out = out; a.counts = counts; a.kept = work;
  a.cls = reinterpret_cast<int*>(work + (size_t)B * max_det * 8);
  a.ncand = a.cls + (size_t)B * N;
  {
    const uintptr_t g = reinterpret_cast<uintptr_t>(a.ncand + B);
    a.gkeys = reinterpret_cast<unsigned long long*>((g + 7) & ~(uintptr_t)7);
  }
  a.np2N = (int)nms_np2(N);
  a.B = B; a.no = no; a.N = N; a.nc = nc; a.max_det = max_det; a.max_nms = max_nms;
  a.agnostic = agnostic ? 1 : 0; a.conf = conf_thres; a.max_wh = max_wh; a.iou = iou_thres;
  hipError_t e = hipMemsetAsync(a.ncand, 0, sizeof(int) * (size_t)B, stream);
  if (e != hipSuccess) return (int)e;
  if (N > 0) {
    hipLaunchKernelGGL(mcaq::mcaq_nms_scan_kernel, dim3((N + mcaq::NMS_SCAN_THREADS - 1) / mcaq::NMS_SCAN_THREADS, B),
                       dim3(mcaq::NMS_SCAN_THREADS), 0, stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(mcaq::mcaq_nms_kernel, dim3(B), dim3(mcaq::NMS_THREADS), 0, stream, a);
  return (int)hipGetLastError();
}

}  // extern "C"
