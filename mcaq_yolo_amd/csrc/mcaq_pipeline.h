// mcaq_pipeline.h - software-pipelined schedule of the hook path for batched
// throughput (included by mcaq_kernels.hip; C ABI in include/mcaq_hip.h).
//
// One step i issues four independent pieces of four different batches:
//
//   stream 0 (streaming)   pass 1 of batch i, then pass 2 of batch i-3
//   stream 1 (pixel chain) morph pass A (+ channel min/max) of batch i-1
//   stream 2 (tile chain)  morph pass B of batch i-2
//
// Each piece depends only on pieces of the PREVIOUS step (pass A(i-1) on
// pass 1(i-1), pass B(i-2) on pass A(i-2), pass 2(i-3) on pass B(i-3)), so
// within a step the latency-bound morphology runs beside the HBM passes
// instead of in front of them, and a step takes max(streaming, pass A,
// pass B) rather than their sum.  The cross-stream edges are two events per
// stream, alternating by step parity (a wait always refers to the previous
// step's record).  Optional CU masks keep the morphology's workgroups and
// the streaming workgroups on disjoint CUs.
//
// Buffer reuse: a batch's buffers are touched by steps i .. i+3, so callers
// cycle at least four independent buffer sets (HookPlan); with four, every
// reuse hazard is ordered through the events (stream 0 at step i waits for
// stream 2 of step i-1, which waited for stream 1 of step i-2, which waited
// for pass 1 of step i-3, which stream 0 issued after the pass 2 of step
// i-4).
#pragma once

struct mcaq_pipeline {
  hipStream_t s[3];
  hipEvent_t ev[3][2];
  hipEvent_t ev_st[2];     // stream 0 after pass 1 (pass A waits for this, not for pass 2)
  hipEvent_t join[3];
  long long step;
};

extern "C" {

int mcaq_pipeline_create(const uint32_t* cu_masks, int mask_words, mcaq_pipeline** out) {
  if (!out) return (int)hipErrorInvalidValue;
  *out = nullptr;
  mcaq_pipeline* p = new mcaq_pipeline();
  p->step = 0;
  for (int k = 0; k < 3; ++k) {
    hipError_t e;
    const uint32_t* m = cu_masks ? cu_masks + (size_t)k * mask_words : nullptr;
    bool any = false;
    for (int w = 0; m && w < mask_words; ++w) any = any || m[w] != 0;
    if (any)
      e = hipExtStreamCreateWithCUMask(&p->s[k], (uint32_t)mask_words, m);
    else
      e = hipStreamCreateWithFlags(&p->s[k], hipStreamNonBlocking);
    if (e != hipSuccess) { delete p; return (int)e; }
    for (int j = 0; j < 2; ++j) {
      e = hipEventCreateWithFlags(&p->ev[k][j], hipEventDisableTiming);
      if (e != hipSuccess) { delete p; return (int)e; }
    }
    e = hipEventCreateWithFlags(&p->join[k], hipEventDisableTiming);
    if (e != hipSuccess) { delete p; return (int)e; }
  }
  for (int j = 0; j < 2; ++j) {
    const hipError_t e = hipEventCreateWithFlags(&p->ev_st[j], hipEventDisableTiming);
    if (e != hipSuccess) { delete p; return (int)e; }
  }
  *out = p;
  return 0;
}

int mcaq_pipeline_destroy(mcaq_pipeline* p) {
  if (!p) return 0;
  for (int k = 0; k < 3; ++k) (void)hipStreamSynchronize(p->s[k]);
  for (int k = 0; k < 3; ++k) {
    for (int j = 0; j < 2; ++j) (void)hipEventDestroy(p->ev[k][j]);
    (void)hipEventDestroy(p->join[k]);
    (void)hipStreamDestroy(p->s[k]);
  }
  for (int j = 0; j < 2; ++j) (void)hipEventDestroy(p->ev_st[j]);
  delete p;
  return 0;
}

void* mcaq_pipeline_stream(mcaq_pipeline* p, int k) { return (p && k >= 0 && k < 3) ? (void*)p->s[k] : nullptr; }

// One step.  Any piece may be absent (n == 0: pipeline fill / drain).
// hold_a != 0: stream 1's end-of-step event is not recorded; the caller
// enqueues more work on stream 1 (the RCCL min/max all-reduce of batch i-1
// for N > 1, on mcaq_pipeline_stream(p, 1)) and then calls
// mcaq_pipeline_release_a.
int mcaq_pipeline_step(mcaq_pipeline* p,
                       const mcaq_stats_scale* st, int nst,
                       const mcaq_morph_scale* ma, int nma, const mcaq_finalize_scale* fz, int nfz,
                       const mcaq_morph_scale* mb, int nmb,
                       const mcaq_quant_scale* qs, int nq, int hold_a) {
  if (!p) return (int)hipErrorInvalidValue;
  const int cur = (int)(p->step & 1), prev = cur ^ 1;
  const bool first = p->step == 0;
  hipError_t e;
  // resolve the morph launch configurations before enqueueing anything
  MorphLaunch LA, LB;
  if (nma > 0) { const int r = morph_launch_config(ma, nma, fz, nfz, LA); if (r) return r; }
  if (nmb > 0) { const int r = morph_launch_config(mb, nmb, nullptr, 0, LB); if (r) return r; }
  // stream 0: pass 1 (i), pass 2 (i-3) after pass B (i-3) of the previous step
  if (!first && (e = hipStreamWaitEvent(p->s[0], p->ev[2][prev], 0)) != hipSuccess) return (int)e;
  if (nst > 0) { const int r = mcaq_stats(st, nst, p->s[0]); if (r) return r; }
  if ((e = hipEventRecord(p->ev_st[cur], p->s[0])) != hipSuccess) return (int)e;
  if (nq > 0) { const int r = mcaq_quant(qs, nq, p->s[0]); if (r) return r; }
  if ((e = hipEventRecord(p->ev[0][cur], p->s[0])) != hipSuccess) return (int)e;
  // stream 1: pass A (i-1) after pass 1 (i-1) (not after the pass 2 that
  // follows it on stream 0)
  if (!first && (e = hipStreamWaitEvent(p->s[1], p->ev_st[prev], 0)) != hipSuccess) return (int)e;
  if (nma > 0) { const int r = morph_launch(LA, 1, p->s[1]); if (r) return r; }
  if (!hold_a && (e = hipEventRecord(p->ev[1][cur], p->s[1])) != hipSuccess) return (int)e;
  // stream 2: pass B (i-2) after pass A (i-2)
  if (!first && (e = hipStreamWaitEvent(p->s[2], p->ev[1][prev], 0)) != hipSuccess) return (int)e;
  if (nmb > 0) { const int r = morph_launch(LB, 2, p->s[2]); if (r) return r; }
  if ((e = hipEventRecord(p->ev[2][cur], p->s[2])) != hipSuccess) return (int)e;
  p->step++;
  return 0;
}

int mcaq_pipeline_release_a(mcaq_pipeline* p) {
  if (!p || p->step == 0) return (int)hipErrorInvalidValue;
  return (int)hipEventRecord(p->ev[1][(int)((p->step - 1) & 1)], p->s[1]);
}

// Make `stream` wait for everything the pipeline has issued so far.
int mcaq_pipeline_join(mcaq_pipeline* p, hipStream_t stream) {
  if (!p) return (int)hipErrorInvalidValue;
  for (int k = 0; k < 3; ++k) {
    hipError_t e = hipEventRecord(p->join[k], p->s[k]);
    if (e != hipSuccess) return (int)e;
    if ((e = hipStreamWaitEvent(stream, p->join[k], 0)) != hipSuccess) return (int)e;
  }
  return 0;
}

}  // extern "C"
