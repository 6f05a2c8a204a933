/* mcaq_hip.h - C ABI of the MI355X (gfx950) MCAQ spatial-adaptive-quantization
 * hook path.  Plain pointers (device memory) and sizes; every launcher is
 * asynchronous on the given HIP stream and returns a hipError_t value.
 *
 * Reference interfaces replaced (yooooonjae/mcaq-yolo):
 *   mcaq_launch_spatial_quantization  <- launch_spatial_quantization
 *       (mcaq_yolo/ops/src/mcaq_kernel.cu:102-123, declared with C++ linkage
 *        in mcaq_yolo/ops/src/mcaq_ops.cpp:7-16 and
 *        mcaq_yolo/engine/MCAQPlugin.cpp:14-24; called by
 *        MCAQPlugin::enqueue, MCAQPlugin.cpp:43-71)
 *   mcaq_stats / mcaq_finalize / mcaq_morph / mcaq_quant
 *       <- the per-scale hook body MCAQYOLO._make_mcaq_hook.hook
 *          (mcaq_yolo/models/mcaq_yolo.py:409-455): analyzer
 *          (core/morphology.py:939-973), bit mapper (core/bit_allocation.py:
 *          42-80, 218-280), quantizer (core/quantization.py:604-746), split
 *          into the three HBM passes of the fused design.
 *   mcaq_qat_forward / mcaq_qat_backward / mcaq_ema_stats
 *       <- SpatialAdaptiveQuantization training branch + StraightThroughEstimator
 *          + update_running_stats (mcaq_yolo/core/quantization.py:699-727,
 *          69-118, 319-353): the QAT quantizer of BASELINE config 5.
 *   mcaq_nms
 *       <- ultralytics non_max_suppression + torchvision nms as called by
 *          Predictor.postprocess / predict_batch (mcaq_yolo/inference.py:
 *          213-219, 410-417): the detection postprocess of the e2e path.
 * One launch processes up to MCAQ_MAX_SEGMENTS segments; a segment is one hook
 * scale (C3/C4/C5) of one batch, each with its own tensors and statistics, so
 * a launch serves the three scales of one batch or of up to three
 * independent batches (a "launch set").
 */
#ifndef MCAQ_HIP_H_
#define MCAQ_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef MCAQ_NO_HIP
typedef void* hipStream_t;
typedef void* hipEvent_t;
#else
#include <hip/hip_runtime_api.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define MCAQ_ABI_VERSION 28
/* feature-map element types (mcaq_stats_scale.dtype, mcaq_quant_scale.dtype) */
#define MCAQ_DTYPE_F32 0
#define MCAQ_DTYPE_F16 1
#define MCAQ_DTYPE_BF16 2
/* segments (hook scale x batch) per mcaq_stats / mcaq_finalize /
 * mcaq_morph* / mcaq_quant launch */
#define MCAQ_MAX_SEGMENTS 9
/* largest dynamic LDS request of the morph kernel (gfx950: 160 KiB per CU) */
#define MCAQ_MORPH_LDS_LIMIT 163840

/* ---- reference-compatible operator ----------------------------------------
 * Same argument order as launch_spatial_quantization (mcaq_kernel.cu:102-111)
 * with hipStream_t; output[n,c,h,w] = dequant(quant_b(input)) * mask[n,h,w]
 * where b = clamp(rint(bit_map[n, min(h/tile_h, Ht-1), min(w/tile_w, Wt-1)]),
 * 2, 8) and per-channel scale/zero-point come from min_vals/max_vals (C
 * entries).  Rounding is half-to-even (torch.round), unlike the reference
 * kernel's roundf; mask may be NULL.  Returns hipErrorInvalidValue on bad
 * sizes.  No workspace. */
int mcaq_launch_spatial_quantization(const float* input, const float* bit_map,
                                     const float* min_vals, const float* max_vals,
                                     const float* mask, float* output,
                                     int N, int C, int H, int W, int tile_h, int tile_w,
                                     int n_tiles_h, int n_tiles_w, hipStream_t stream);

/* ---- pass 1: one streaming read of x ---------------------------------------
 * gray[b,h,w]    = mean_c x[b,c,h,w] over the crop h<Hc, w<Wc, in CPU-ATen
 *                  summation order (NULL to skip)
 * absmean[b,h,w] = mean_c |x[b,c,h,w]| over the full map (NULL to skip)
 * pmin/pmax      = per-(unit, channel) min/max partials, unit = 64, 128 or 256
 *                  pixels of one image: mcaq_stats_units(B,C,H,W) x C floats
 *                  each (NULL to skip). */
typedef struct {
  const float* x;  /* (B, C, H, W) contiguous, of element type `dtype` */
  float* gray;     /* (B, Hc, Wc) */
  float* absmean;  /* (B, H, W) */
  float* pmin;
  float* pmax;
  int B, C, H, W, Hc, Wc;
  int unit_begin;  /* set by the launcher */
  int dtype;       /* element type of x: MCAQ_DTYPE_F32 / _F16 / _BF16 (one per launch);
                      fp16 / bf16 widen exactly, every sum stays fp32 */
} mcaq_stats_scale;
int mcaq_stats(const mcaq_stats_scale* scales, int nscales, hipStream_t stream);
int mcaq_stats_units(int B, int C, int H, int W);

/* ---- channel min/max over the batch (quantization.py:650-654) -------------- */
typedef struct {
  const float* pmin; /* partials from mcaq_stats (or NULL: copy min_in/max_in) */
  const float* pmax;
  const float* min_in;
  const float* max_in;
  float* min_out;    /* (C) */
  float* max_out;    /* (C) */
  int C, nunits, min_stride;
  int block_begin;   /* set by the launcher */
  int per_tensor;    /* 1: ONE min/max over every channel, broadcast to the C
                        outputs (per_channel=False, quantization.py:655-661) */
  int neg_min;       /* 1: min_out receives -min (so [-min, max] of every
                        segment can be combined across ranks by ONE MAX
                        all-reduce in place; mcaq_quant_scale.neg_min reads it
                        back) */
} mcaq_finalize_scale;
int mcaq_finalize(const mcaq_finalize_scale* scales, int nscales, hipStream_t stream);

/* ---- morph: one workgroup per image --------------------------------------
 * flags: 1 phi, 2 complexity MLP + bilateral, 4 mapper, 8 soft mask,
 * 16 continuous bits, 32 temperature given, 64 normalise C, 128 linear mapper,
 * 256 Otsu binarize, 512 no Euler correction, 1024 legacy Canny, 2048 per-image
 * pass B, 4096 every image its own batch of one (batch_offset / batch_total
 * ignored: the reference's batch-1 calls, as compute_dataset_complexity
 * makes them - one launch scores many images).  Parameter blobs are the packed
 * reference state_dict tensors (mcaq_yolo_amd/params.py), 16-byte aligned and
 * zero-padded to a multiple of 4 floats (they are staged with 16-byte loads). */
typedef struct {
  const float* gray;
  const float* absmean;
  const float* cmlp;
  const float* mapper;
  const float* smask;
  const float* c_in;
  const float* bits_in;
  float* phi_out;
  float* cmlp_out;
  float* c_out;
  float* bits_out;
  float* m_out;      /* (B, H, W) m plane, or NULL */
  float* mt_out;     /* (B, ht, wt) soft-mask tile values m(tile), or NULL */
  uint8_t* edge_out;
  uint8_t* bin_out;
  float* gscratch;   /* mcaq_morph_scratch_bytes() bytes, or NULL when 0 */
  float* tile_tmp;   /* (B, ht*wt, 32) per-tile partial quantities, needed with
                        flag 1: written by the edge / mask workgroups of the
                        pixel pass, read by the tile pass */
  int B, H, W, Hc, Wc, tile, ht, wt;
  int batch_offset, batch_total;
  int flags, hyst_iters;
  float temperature, min_bits, max_bits;
  int block_begin;   /* set by the launcher */
  int softmax_threads; /* torch.get_num_threads() of the reference CPU run the
                          soft mask's channel softmax reproduces (its exp per
                          tile depends on ATen's thread partition); <1 = 1 */
  float* pwork;      /* mcaq_morph_work_bytes() bytes, or NULL: pixel-pass
                        workspace of the band / edge kernels (NMS value plane
                        + per-band Otsu histograms).  When every scale of a
                        launch has one and is eligible (default Canny,
                        adaptive binarize, tile 4/8/16, map <= 128 x 128), pass
                        A runs as one workgroup per 16-row band + one per
                        image instead of one whole-CU workgroup per image. */
} mcaq_morph_scale;
int mcaq_morph(const mcaq_morph_scale* scales, int nscales, hipStream_t stream);
/* mcaq_morph + mcaq_finalize in one launch: the channel min/max reduction
 * runs as extra workgroups beside the per-image ones (fscales may be NULL). */
int mcaq_morph_finalize(const mcaq_morph_scale* scales, int nscales,
                        const mcaq_finalize_scale* fscales, int nfscales, hipStream_t stream);
size_t mcaq_morph_scratch_bytes(int B, int Hc, int Wc, int ht, int wt);
/* Global plane scratch of one scale when a launch runs with planes in global
 * memory (the mode is common to a launch's scales: every scale needs this
 * buffer as soon as one scale's mcaq_morph_scratch_bytes is non-zero). */
size_t mcaq_morph_scratch_bytes_global(int B, int Hc, int Wc);
/* pwork bytes of one scale (0: the scale cannot take the band path) */
size_t mcaq_morph_work_bytes(int B, int Hc, int Wc, int tile);

/* ---- pass 2: y = dequant(quant_b(x)) * m ----------------------------------- */
typedef struct {
  const float* x;      /* (B, C, H, W), element type `dtype` */
  float* y;            /* (B, C, H, W), element type `ydtype` */
  const float* bits;   /* (B, ht, wt) integer-valued */
  const float* m;      /* (B, H, W) or NULL */
  const float* mt;     /* (B, ht, wt) soft-mask tile values: when set, m(p) is
                          generated per pixel (nearest upsample + 5x5 Gaussian,
                          replicate pad, quantization.py:235-238) and m is
                          ignored */
  const float* xmin;   /* (C) */
  const float* xmax;   /* (C) */
  int B, C, H, W, ht, wt;
  int bits_lo, nbits;  /* supported widths [bits_lo, bits_lo + nbits - 1] */
  int compat_tile_h, compat_tile_w; /* >0: spatial_quantize tile indexing */
  int unit_begin;      /* set by the launcher */
  int stats_cover_x;   /* 1: xmin / xmax are the min / max of this x itself (the
                          batch statistics of pass 1, all-reduced or not):
                          channels whose statistics are finite hold only
                          finite x and take the shorter arithmetic; 0: any x
                          (frozen / external statistics) */
  int neg_min;         /* 1: xmin holds -min (mcaq_finalize_scale.neg_min) */
  int dtype;           /* element type of x (MCAQ_DTYPE_*, one per launch): fp16 / bf16
                          maps widen exactly and the arithmetic is fp32; they take
                          the tile-aligned kernel only (otherwise hipErrorNotSupported) */
  int ydtype;          /* element type of y: dtype, or MCAQ_DTYPE_F32 (the reference's
                          promotion: an fp16 map times the fp32 soft mask is fp32,
                          quantization.py:742-744); rounded to nearest even */
} mcaq_quant_scale;
int mcaq_quant(const mcaq_quant_scale* scales, int nscales, hipStream_t stream);

/* mcaq_morph_finalize with a choice of passes: bit 0 = pass A (the per-image
 * pixel chain -> tile partials, + the channel min/max workgroups), bit 1 =
 * pass B (tile chain: phi, complexity MLP, bilateral, mapper, soft mask).
 * Pass B reads what pass A wrote (tile_tmp). */
int mcaq_morph_pass(const mcaq_morph_scale* scales, int nscales,
                    const mcaq_finalize_scale* fscales, int nfscales, int passes, hipStream_t stream);

/* Measurement: the calling thread's NEXT mcaq_stats / mcaq_quant launch is
 * issued through hipExtLaunchKernel with these start/stop events (either may
 * be NULL), which the runtime stamps at that dispatch's own start and end -
 * the interval a rocprofv3 kernel trace reports.  Not for graph capture. */
int mcaq_time_next_launch(hipEvent_t start, hipEvent_t stop);
/* the same for the launch after `skip` others of this thread (pass 1, pass 2,
 * the QAT kernels: e.g. skip = 1 times the fold launch of mcaq_qat_backward) */
int mcaq_time_launch(int skip, hipEvent_t start, hipEvent_t stop);

/* ---- QAT quantizer (training branch) --------------------------------------
 * forward:  y = ((1-f) Q_lo(x) + f Q_hi(x)) * m, lo = floor(b), f = b - lo,
 *           Q_hi = Q_lo when lo = 8 (quantization.py:699-727, 733-737); b is
 *           the nearest-upsampled CONTINUOUS tile bit map, Q_k the
 *           per-channel k-bit quant/dequant with xmin/xmax (running stats).
 * backward: gx = gm(1-f) + gm f with gm = g m (straight-through,
 *           quantization.py:94-118); gm_out(p) = sum_c g xq (NULL: skip);
 *           gb(t) = sum over tile t's pixels of sum_c (gm Q_hi - gm Q_lo)
 *           (NULL: skip).  work: mcaq_qat_work_floats(B,C,H,W) floats of
 *           device scratch (per-32-channel-slice partials of both sums). */
typedef struct {
  const float* x;      /* (B, C, H, W) */
  const float* g;      /* (B, C, H, W) upstream gradient (backward) */
  float* y;            /* (B, C, H, W) forward output */
  float* gx;           /* (B, C, H, W) backward output */
  float* gm;           /* (B, H, W) grad of m, or NULL */
  float* gb;           /* (B, ht, wt) grad of the bit map, or NULL */
  float* work;         /* backward scratch */
  const float* bits;   /* (B, ht, wt) continuous bits */
  const float* m;      /* (B, H, W) soft mask, or NULL */
  const float* xmin;   /* (C) */
  const float* xmax;   /* (C) */
  int B, C, H, W, ht, wt;
  int unit_begin, block_begin;  /* set by the launcher */
  int* arrive;         /* (B, ht) zero-initialised arrival counters (left
                          zeroed), 16 <= W <= 512: the last backward unit to
                          finish a (image, tile row) band folds that band's
                          partials into gm / gb inside the same launch;
                          NULL: a separate fold kernel does it */
} mcaq_qat_scale;
int mcaq_qat_forward(const mcaq_qat_scale* scales, int nscales, hipStream_t stream);
int mcaq_qat_backward(const mcaq_qat_scale* scales, int nscales, hipStream_t stream);
/* mcaq_qat_forward plus the train step's bit budget as one extra workgroup of
 * the same launch: avg = mean_k mean(bits[k][0 .. n[k])) over nseg <= 3 bit
 * maps (models/mcaq_yolo.py:572-577) and loss = (avg - target)^2 (NULL: not
 * written; MCAQLoss.compute_bit_budget_loss, :110-118). */
int mcaq_qat_forward_budget(const mcaq_qat_scale* scales, int nscales, const float* const* bits, const int* n,
                            int nseg, float target, float* avg, float* loss, hipStream_t stream);
size_t mcaq_qat_work_floats(int B, int C, int H, int W);
/* running <- fp32(momentum) running + fp32(1 - momentum) batch, per channel
 * (first != 0: running <- batch), in place. */
int mcaq_ema_stats(const float* batch_min, const float* batch_max, float* running_min, float* running_max,
                   int C, double momentum, int first, hipStream_t stream);
/* The same, plus copies of the updated statistics (copy_min / copy_max, the
 * values this step's quantizer uses, or NULL) and num_batches_tracked += 1
 * (num_batches, int64, or NULL) in the same launch. */
int mcaq_ema_stats_ex(const float* batch_min, const float* batch_max, float* running_min, float* running_max,
                      int C, double momentum, int first, float* copy_min, float* copy_max, long long* num_batches,
                      hipStream_t stream);
/* mcaq_ema_stats_ex of several quantizers (one per hook scale, <= 3) in ONE
 * launch: segment k is the argument set of one call. */
typedef struct {
  const float* batch_min; const float* batch_max;
  float* running_min; float* running_max;
  float* copy_min; float* copy_max;   /* or NULL */
  int64_t* num_batches;                /* or NULL */
  int C, first;
  double momentum;
} mcaq_ema_seg;
int mcaq_ema_stats_multi(const mcaq_ema_seg* segs, int nseg, hipStream_t stream);

/* ---- batched NMS of YOLOv8 Detect outputs ----------------------------------
 * pred (B, no, N) fp32 with no = 4 + nc rows (cx, cy, w, h, class scores);
 * per image: candidates with max class score > conf_thres, xyxy boxes,
 * stable score-descending order, first max_nms, class offset cls*max_wh
 * (agnostic: none), greedy IoU > iou_thres suppression (torchvision CPU
 * arithmetic), first max_det kept.  out (B, max_det, 6) = x1 y1 x2 y2 conf
 * cls (rows past counts[b] zeroed), counts (B) int32.  work:
 * mcaq_nms_work_floats(B, N, max_det) floats (kept boxes, candidate classes,
 * candidate counts and a pow2(N) key array per image).  Two kernels and a
 * 4*B-byte memset: a scan over B x ceil(N/256) workgroups, then one
 * workgroup per image. */
int mcaq_nms(const float* pred, int B, int no, int N, int nc, float conf_thres, double iou_thres, int max_det,
             int max_nms, float max_wh, int agnostic, float* out, int* counts, float* work, hipStream_t stream);
size_t mcaq_nms_work_floats(int B, int N, int max_det);

/* ---- train-mode (QAT) tile networks: fused forward / backward ------------
 * Replace the autograd glue of the train-mode hook (DESIGN s.8): the bit
 * mapper with batch-statistics BatchNorm (bit_allocation.py:218-280,
 * 120-130), the analyzer head (complexity MLP + bilateral + clamp,
 * morphology.py:81-97, 309-354, 959-968) and the soft-mask net
 * (quantization.py:213-239).  Parameters are the modules' own fp32 tensors
 * (torch layouts); gradients come back as one flat vector in the modules'
 * parameters() order.  gpart: per-workgroup partial sums (sizes below). */
typedef struct {
  const float *w1, *b1, *g1, *be1;   /* Linear(3,32), BatchNorm1d(32) */
  float *rm1, *rv1;                  /* running mean / var (updated by the forward) */
  long long* nbt1;                   /* num_batches_tracked, or NULL */
  const float *w2, *b2, *g2, *be2;   /* Linear(32,64), BatchNorm1d(64) */
  float *rm2, *rv2;
  long long* nbt2;
  const float *w3, *b3, *g3, *be3;   /* Linear(64,32), BatchNorm1d(32) */
  float *rm3, *rv3;
  long long* nbt3;
  const float *w4, *b4;              /* Linear(32,1) */
} mcaq_mapper_params;
typedef struct {
  const float *w1, *b1, *g1, *be1;   /* Linear(8,64), LayerNorm(64) */
  const float *w2, *b2, *g2, *be2;   /* Linear(64,32), LayerNorm(32) */
  const float *w3, *b3;              /* Linear(32,1) */
} mcaq_cmlp_params;
typedef struct {
  const float *w1, *b1;              /* Conv2d(2,8,3,pad 1) */
  const float *w2, *b2;              /* Conv2d(8,2,1) */
} mcaq_smask_params;

/* bits (n) = train-mode mapper of c (n): 4 launches; work keeps the
 * activations and batch statistics for the backward (temperature <= 0:
 * none; round_bits: straight-through round; update_stats 1: BN running stats
 * with `momentum`, num_batches_tracked += 1; update_stats 2: the update is
 * deferred - its batch mean / unbiased variance stay in `work` for
 * mcaq_mapper_running_update) */
size_t mcaq_mapper_work_floats(int n);
int mcaq_mapper_train_forward(const mcaq_mapper_params* P, const float* c, int n, float min_bits, float max_bits,
                              float temperature, float momentum, int round_bits, int update_stats, float* bits,
                              float* work, unsigned* grid_sync, hipStream_t stream);
/* gc (n), gparams (4609: mapping_network parameters() order); 5 launches */
size_t mcaq_mapper_gpart_floats(int n);
int mcaq_mapper_train_backward(const mcaq_mapper_params* P, const float* c, int n, const float* gbits,
                               float min_bits, float max_bits, float temperature, float* work, float* gc,
                               float* gparams, float* gpart, int accumulate, unsigned* grid_sync,
                               hipStream_t stream);
/* Batch sharded over `world` ranks with process-group BatchNorm (the train-
 * mode mapper of a DDP QAT step, dist.GroupBatchNorm1d semantics): the same
 * kernels one stage per call, the caller's collectives between them.
 *   forward  stage 1..4; before stage s >= 2: every rank's
 *            mcaq_mapper_train_reduce(kind 0, layer s - 1) output (129 floats)
 *            all-gathered in rank order -> `gathered` (world x 129)
 *   backward stage 4..1; before stage s <= 3: mcaq_mapper_train_reduce
 *            (kind 1, layer s) summed over the ranks -> `gsums` (128 floats);
 *            gathered1 = the forward's gathered layer-1 entries (tile counts);
 *            then mcaq_mapper_train_grad_reduce: this rank's parameter
 *            gradients (the caller all-reduces them as DDP does).
 * Replaces the autograd through GroupBatchNorm1d's all-reduces (dist.py). */
int mcaq_mapper_train_forward_stage(const mcaq_mapper_params* P, const float* c, int n, float min_bits,
                                    float max_bits, float temperature, float momentum, int round_bits,
                                    int update_stats, float* bits, float* work, int stage, const float* gathered,
                                    int world, hipStream_t stream);
int mcaq_mapper_train_backward_stage(const mcaq_mapper_params* P, const float* c, int n, const float* gbits,
                                     float min_bits, float max_bits, float temperature, float* work, float* gc,
                                     float* gpart, int stage, const float* gsums, const float* gathered1, int world,
                                     hipStream_t stream);
/* kind 0: this rank's (mean[64], M2[64], n) of layer 1..3 (forward);
 * kind 1: this rank's BN sums (S1[64], S2[64]) of layer 1..3 (backward) */
int mcaq_mapper_train_reduce(const float* work, int n, int kind, int layer, float* out, hipStream_t stream);
int mcaq_mapper_train_grad_reduce(int n, const float* gpart, float* gparams, int accumulate, hipStream_t stream);
/* The deferred running-stats updates of `count` (<= 8) forwards run with
 * update_stats 2 (works[k] of ns[k] tiles), applied in list order - the
 * values those forwards would have left with update_stats 1 one after
 * another.  For hook scales whose train-mode mappers run concurrently on
 * several streams (the running buffers are shared).  1 launch. */
int mcaq_mapper_running_update(const mcaq_mapper_params* P, const float* const* works, const int* ns, int count,
                               float momentum, hipStream_t stream);
/* mcaq_ema_stats_multi(segs, nseg) plus mcaq_mapper_running_update(P, works,
 * ns, count, momentum) as one extra workgroup of the same launch: the train
 * step's deferred BatchNorm running-statistics update of the bit mapper rides
 * on the quantizers' EMA launch that follows it. */
int mcaq_ema_stats_multi_running(const mcaq_ema_seg* segs, int nseg, const mcaq_mapper_params* P,
                                 const float* const* works, const int* ns, int count, float momentum,
                                 hipStream_t stream);
/* mcaq_morph(scales) of a pass-B-only launch (the train step's soft-mask
 * planes) with the quantizers' EMA (esegs, as mcaq_ema_stats_multi) and,
 * count > 0, the mapper's running-statistics update riding along as extra
 * workgroups; any other morph launch runs first, then the EMA launch. */
int mcaq_morph_ema(const mcaq_morph_scale* scales, int nscales, const mcaq_ema_seg* esegs, int ne,
                   const mcaq_mapper_params* P, const float* const* works, const int* ns, int count, float momentum,
                   hipStream_t stream);
/* grid_sync: NULL (one launch per batch-statistics barrier), or 2 zeroed
 * uint32 that launches on one stream share (each launch leaves them zeroed):
 * forward and backward then run as ONE launch each, with grid-wide barriers
 * between the stages (n <= 256 * 64 tiles). */
/* analyzer head: gC (B, ht, wt) -> gcraw (B, ht, wt) work, gparams (2881:
 * complexity_mlp parameters() order); phi (B*ht*wt, 8), craw = the MLP output
 * before the bilateral; 3 launches (2 with gparams NULL: the caller then
 * reduces gpart with mcaq_head_train_grad_reduce) */
size_t mcaq_head_gpart_floats(int n);
int mcaq_head_train_backward(const mcaq_cmlp_params* P, const float* phi, const float* craw, const float* gC, int B,
                             int ht, int wt, float* gcraw, float* gparams, float* gpart, int accumulate,
                             hipStream_t stream);
int mcaq_head_train_grad_reduce(int n, const float* gpart, float* gparams, int accumulate, hipStream_t stream);
/* soft mask: gm (B, H, W) -> gbits (B, ht, wt) (accumulate != 0: added),
 * gparams (170: net parameters() order); 2 launches */
size_t mcaq_smask_gpart_floats(int B);
int mcaq_smask_train_backward(const mcaq_smask_params* P, const float* bits, const float* absmean, const float* gm,
                              int B, int H, int W, int ht, int wt, float* gbits, int accumulate, float* gparams,
                              float* gpart, hipStream_t stream);
/* ---- multi-segment train launches: the hook scales of one QAT step (each
 * scale its own tensors, the same module parameters) in ONE launch per stage
 * instead of one per scale and stage - the values of the per-scale launches.
 * At most MCAQ_TRAIN_MAXSEG segments.  Parameter gradients stay per-segment
 * partials (gpart, as the single-scale launchers' sizes) for
 * mcaq_train_reduce_multi. */
#define MCAQ_TRAIN_MAXSEG 3
typedef struct {
  const float* c;        /* (n) complexity */
  float* bits;           /* (n) forward output */
  float* work;           /* mcaq_mapper_work_floats(n) */
  const float* gbits;    /* (n) backward: upstream gradient */
  float* gc;             /* (n) backward: gradient of c */
  float* gpart;          /* backward: mcaq_mapper_gpart_floats(n) */
  int n;
} mcaq_mapper_seg;
/* 4 launches; update_stats 0 or 2 (deferred, then mcaq_mapper_running_update
 * in segment order) when nseg > 1 */
int mcaq_mapper_train_forward_multi(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                    float min_bits, float max_bits, float temperature, float momentum,
                                    int round_bits, int update_stats, hipStream_t stream);
/* Batch sharded over `world` ranks (process-group BatchNorm): one stage of
 * every segment per call, as mcaq_mapper_train_forward_stage /
 * _backward_stage; gathered / gsums / gathered1 hold one pointer per segment
 * (each that segment's world x 129 gathered entries / 128 summed floats). */
int mcaq_mapper_train_forward_stage_multi(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                          float min_bits, float max_bits, float temperature, float momentum,
                                          int round_bits, int update_stats, int stage, const float* const* gathered,
                                          int world, hipStream_t stream);
int mcaq_mapper_train_backward_stage_multi(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                           float min_bits, float max_bits, float temperature, int stage,
                                           const float* const* gsums, const float* const* gathered1, int world,
                                           hipStream_t stream);
/* 4 launches (no parameter reduction) */
int mcaq_mapper_train_backward_multi(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                     float min_bits, float max_bits, float temperature, hipStream_t stream);
typedef struct {
  const float* phi; const float* craw; const float* gC;
  float* gcraw;          /* (B*ht*wt) work */
  float* gpart;          /* mcaq_head_gpart_floats(B*ht*wt) */
  int B, ht, wt;
} mcaq_head_seg;
/* 2 launches (bilateral adjoint, complexity MLP backward; no reduction) */
int mcaq_head_train_backward_multi(const mcaq_cmlp_params* P, const mcaq_head_seg* segs, int nseg, hipStream_t stream);
typedef struct {
  mcaq_smask_params P;   /* each segment its own soft-mask net (one per quantizer) */
  const float* bits; const float* absmean; const float* gm;
  float* gbits;          /* (B, ht, wt), added to when accumulate */
  float* gpart;          /* mcaq_smask_gpart_floats(B) */
  int B, H, W, ht, wt, accumulate;
} mcaq_smask_seg;
/* 1 launch (no reduction) */
int mcaq_smask_train_backward_multi(const mcaq_smask_seg* segs, int nseg, hipStream_t stream);
/* The bit budget of a QAT step: avg_bits = mean over the segments of
 * mean(bits_k) (models/mcaq_yolo.py:572-577) and loss = (avg_bits - target)^2
 * (MCAQLoss.compute_bit_budget_loss, :110-118), one workgroup. */
int mcaq_bit_budget_forward(const float* const* bits, const int* n, int nseg, float target, float* avg, float* loss,
                            hipStream_t stream);
typedef struct {
  const float* avg;      /* the forward's avg_bits (device scalar) */
  const float* g_avg;    /* dL / d avg_bits, or NULL */
  const float* g_loss;   /* dL / d loss, or NULL */
  float target;
  int nscales;           /* scales averaged by avg_bits */
} mcaq_bit_budget;
/* The quantizer's fold + the soft-mask backward + the bit-budget gradient of
 * every scale in ONE launch (one workgroup per image): from the per-slice
 * partials of mcaq_qat_backward (launched with gm = gb = NULL) grad m(p) and
 * the quantizer's grad_bits in the fold kernel's order, then gbits =
 * (c + grad_bits(quantizer)) + grad_bits(soft mask) per tile, c = dL/d avg
 * / (nscales * B ht wt) - the order autograd adds the three contributions in
 * the per-scale step.  gpart: the soft-mask parameter partials, as
 * mcaq_smask_train_backward_multi. */
typedef struct {
  mcaq_smask_params P;
  const float* bits; const float* absmean;
  const float* qat_work; /* mcaq_qat_work_floats(B, C, H, W) partials of this scale */
  float* gbits;          /* (B, ht, wt) */
  float* gpart;          /* mcaq_smask_gpart_floats(B) */
  int B, C, H, W, ht, wt;
} mcaq_qat_smask_seg;
int mcaq_qat_smask_backward_multi(const mcaq_qat_smask_seg* segs, int nseg, const mcaq_bit_budget* bb,
                                  hipStream_t stream);
typedef struct {
  const float* part;     /* [nparts][stride] partial sums */
  float* out;            /* count floats (chain: segment 0's only) */
  int nparts, stride, count, accumulate;
  float scale;           /* 0 or 1: none; else the launch's sum times scale, then
                            accumulated (chain: segment 0's applies) - a data-parallel
                            rank's 1 / world share of a gradient it computed whole */
} mcaq_reduce_seg;
/* chain 0: out_k (+)= sum of segment k's partials; chain 1: segment 0's out
 * = s_0 (+ out if accumulate) + s_1 + s_2 in segment order (the values of
 * one reduction per segment, the later ones accumulating).  1 launch. */
int mcaq_train_reduce_multi(const mcaq_reduce_seg* segs, int nseg, int chain, hipStream_t stream);
/* mcaq_head_train_backward_multi with a chain reduction (as
 * mcaq_train_reduce_multi with chain 1: nr segments into rsegs[0].out)
 * riding on the bilateral launch as extra workgroups - the bit mapper's
 * parameter gradients summed beside the head's backward instead of in a
 * launch of their own (nr = 0: none). */
int mcaq_head_train_backward_multi_ride(const mcaq_cmlp_params* P, const mcaq_head_seg* segs, int nseg,
                                        const mcaq_reduce_seg* rsegs, int nr, hipStream_t stream);
/* mcaq_head_train_backward_multi_ride with the complexity MLP's parameter
 * reduction inside its launch (round 6): out (+)= the chain sum of every
 * segment's partials, last segment first (as mcaq_train_reduce_multi with
 * chain 1 over the segments' gpart, accumulate / scale as there), through
 * `sync` (mcaq_head_sync_bytes(total MLP workgroups = sum of ceil(B ht wt /
 * 64)), zeroed before first use and whenever the layout changes, one launch
 * at a time; word 1 nonzero after a timed-out exchange).  Bit-identical to
 * the separate reduction; gpart is not written.  hipErrorInvalidValue above
 * mcaq_mapper_fused_max_wg() workgroups. */
size_t mcaq_head_sync_bytes(int total_wg);
int mcaq_head_train_backward_fused(const mcaq_cmlp_params* P, const mcaq_head_seg* segs, int nseg,
                                   const mcaq_reduce_seg* rsegs, int nr, float* out, int accumulate, float scale,
                                   void* sync, size_t sync_bytes, hipStream_t stream);
/* mcaq_mapper_train_backward_multi with per-segment reductions (as
 * mcaq_train_reduce_multi with chain 0, segments of equal count) riding on
 * its first (output-layer) stage launch as extra workgroups - the soft masks'
 * parameter gradients summed beside the mapper's backward (nr = 0: none). */
int mcaq_mapper_train_backward_multi_ride(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                          float min_bits, float max_bits, float temperature,
                                          const mcaq_reduce_seg* rsegs, int nr, hipStream_t stream);
/* The mapper's train-mode forward / backward of every segment as ONE launch
 * each (round 6): the batch statistics between the stages are exchanged
 * inside the launch through `sync`, a device buffer of
 * mcaq_mapper_sync_bytes(total workgroups) bytes (workgroups = sum over the
 * segments of ceil(n / 64), at most mcaq_mapper_fused_max_wg()), zeroed
 * before its first use and whenever the segments' sizes change, and not used
 * by two launches at once (one buffer per mapper and layout; forward and
 * backward of the same segments share it).  Results are bit-identical to
 * mcaq_mapper_train_forward_multi / _backward_multi_ride.  Word 32 of the
 * buffer (uint32) is a status word: nonzero after an exchange timed out
 * (results then invalid).  hipErrorInvalidValue when the buffer is missing or
 * too small or the workgroups exceed the maximum (use the staged calls). */
size_t mcaq_mapper_sync_bytes(int total_wg);
int mcaq_mapper_fused_max_wg(void);
int mcaq_mapper_train_forward_fused(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                    float min_bits, float max_bits, float temperature, float momentum,
                                    int round_bits, int update_stats, void* sync, size_t sync_bytes,
                                    hipStream_t stream);
int mcaq_mapper_train_backward_fused(const mcaq_mapper_params* P, const mcaq_mapper_seg* segs, int nseg,
                                     float min_bits, float max_bits, float temperature,
                                     const mcaq_reduce_seg* rsegs, int nr, void* sync, size_t sync_bytes,
                                     hipStream_t stream);

/* gparams of the mapper / head backward: accumulate != 0 adds to gparams
 * (the parameters' persistent gradient storage), 0 overwrites it; NULL
 * (without grid_sync): no reduction launch - the partials stay in gpart for
 * the matching *_grad_reduce call, which a caller with several streams
 * orders itself. */

/* ---- device packing of parameter blobs (the kernels' weight layouts) -------
 * Segment i fills out[dst .. dst + len): mode 0 copies n floats from src;
 * mode 1 writes the v_mfma_f32_16x16x4_f32 A operands of an (n, k) row-major
 * weight (ceil(n/16) blocks x ceil(k/4) steps x 64 lanes, zero padded);
 * out[0 .. total) not covered by a segment is zeroed.  One launch. */
#define MCAQ_PACK_MAXSEG 24
typedef struct {
  const float* src;
  int n, k, mode, dst;
} mcaq_pack_seg;
int mcaq_pack(const mcaq_pack_seg* segs, int nseg, float* out, int total, hipStream_t stream);
/* mcaq_stats(scales, nscales) with mcaq_pack(segs, nseg, out, total) riding
 * on the same launch as extra workgroups (the train step re-packs its blobs
 * beside pass 1, which reads none of them). */
int mcaq_stats_pack(const mcaq_stats_scale* scales, int nscales, const mcaq_pack_seg* segs, int nseg, float* out,
                    int total, hipStream_t stream);

/* ---- the optimizer end of a QAT step in two launches ----------------------
 * torch.nn.utils.clip_grad_norm_(max_norm) over every segment's gradient
 * (the norm of the per-tensor 2-norms; .grad scaled in place), then
 * torch.optim.AdamW (decoupled weight decay, the fused kernel's update
 * order; each segment's steps[step_idx] += 1 first, as a capturable AdamW's
 * per-parameter step tensors: a parameter without a gradient this step is
 * not a segment and keeps its count) and, for
 * segments with project_abs, p <- |p| (the bit mapper's Eq. 18 projection,
 * bit_allocation.py:186-197) - train.py:626-641.  max_norm <= 0: no clip;
 * total_norm (1 float) receives the pre-clip norm, or NULL.  work:
 * mcaq_clip_adamw_work_floats(total elements) floats of device scratch.  Two
 * launches over 1,024-element chunks (per-chunk squared-norm partials, then
 * norm + update); capturable. */
#define MCAQ_OPT_MAXSEG 64
#define MCAQ_OPT_MAXGROUPS 4
typedef struct {
  float* param; float* grad; float* exp_avg; float* exp_avg_sq;
  int n, project_abs, group;   /* group: row of the hyper-parameter table */
  int step_idx;                /* this parameter's entry of `steps` (distinct per segment) */
} mcaq_adamw_seg;
typedef struct {
  double lr, weight_decay, beta1, beta2, eps;   /* doubles, as torch's fused AdamW takes them */
} mcaq_adamw_group;
/* groups: DEVICE table of ngroups rows, read when the kernels run - a
 * captured step uses the values last written there (an lr schedule writes
 * the table between replays); steps: device float counters. */
size_t mcaq_clip_adamw_work_floats(int total);
int mcaq_clip_adamw(const mcaq_adamw_seg* segs, int nseg, const mcaq_adamw_group* groups, int ngroups,
                    float* steps, float max_norm, float* total_norm, float* work, hipStream_t stream);
/* The same step as ONE launch (round 6; clipping only, max_norm > 0): the
 * chunks' squared-norm partials exchanged inside the launch through `sync`
 * (mcaq_clip_adamw_sync_bytes(total elements, nseg) bytes, zeroed before its
 * first use and whenever the segments change; word 1 (uint32) is nonzero
 * after a timed-out exchange).  Bit-identical to mcaq_clip_adamw.
 * hipErrorInvalidValue when max_norm <= 0, the buffer is missing or short, or
 * the step has more than 256 chunks of 1,024 elements (use mcaq_clip_adamw). */
size_t mcaq_clip_adamw_sync_bytes(int total, int nseg);
int mcaq_clip_adamw_fused(const mcaq_adamw_seg* segs, int nseg, const mcaq_adamw_group* groups, int ngroups,
                          float* steps, float max_norm, float* total_norm, void* sync, size_t sync_bytes,
                          hipStream_t stream);

/* ---- data-parallel QAT step: unpack one all-gather ------------------------
 * g: every rank's send buffer back to back, [world][stride] floats
 * (all_gather_into_tensor).  Segment i, mode 0: out[r * n + j] =
 * g[r * stride + off + j] for every rank r (one hook scale's global batch in
 * rank order = image order); mode 1 / 2: out[j] = min / max over the ranks
 * of g[r * stride + off + j] (NaN propagating).  One launch (csrc/mcaq_dp.h,
 * dist.shard_hooks: the train-mode bit mapper on the global batch). */
#define MCAQ_DP_MAXSEG 16
typedef struct {
  float* out;
  int off, n, mode;
} mcaq_dp_seg;
int mcaq_dp_unpack(const float* g, int world, int stride, const mcaq_dp_seg* segs, int nseg, hipStream_t stream);

int mcaq_abi_version(void);

#ifdef __cplusplus
}

/* C++-linkage entry with the reference's exact declaration
 * (mcaq_yolo/engine/MCAQPlugin.cpp:15-23, mcaq_yolo/ops/src/mcaq_ops.cpp:7-16;
 * cudaStream_t -> hipStream_t): a plugin or extension compiled against that
 * declaration links against libmcaq_hip.so unchanged.  Errors are left for
 * hipGetLastError(), as the reference's void launcher leaves them for
 * cudaGetLastError(). */
void launch_spatial_quantization(const float* input, const float* bit_map,
                                 const float* min_vals, const float* max_vals,
                                 const float* mask, float* output,
                                 int N, int C, int H, int W, int tile_h, int tile_w,
                                 int n_tiles_h, int n_tiles_w, hipStream_t stream);
#endif
#endif /* MCAQ_HIP_H_ */
