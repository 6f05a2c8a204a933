// mcaq_pipeline.h - software-pipelined schedule of the hook path for batched
// throughput (included by mcaq_kernels.hip; C ABI in include/mcaq_hip.h).
//
// One step i issues four independent pieces of four different batches, each
// on its own HIP stream:
//
//   stream 0  pass 1 of batch i            (HBM: read x)
//   stream 1  morph pass A (+ channel min/max) of batch i-1   (pixel chain)
//   stream 2  morph pass B of batch i-2    (tile chain)
//   stream 3  pass 2 of batch i-3          (HBM: read x, write y)
//
// Each piece depends only on pieces of EARLIER steps (pass A(i-1) on pass
// 1(i-1), pass B(i-2) on pass A(i-2), pass 2(i-3) on pass B(i-3)), so the two
// latency-bound morphology passes run beside the two HBM passes, and the two
// HBM passes of different batches run beside each other: a step takes
// max(pass 1 | pass 2 | pass A | pass B sharing the chip), not their sum.
//
// Buffer reuse: batch j uses buffer set j % NP (NP >= 4 HookPlans).  Set j%NP
// was last used by batch j-NP, whose pieces ran at steps j-NP .. j-NP+3; the
// stage of batch j that first WRITES each buffer waits for the stream-3 event
// of step j-NP+3 (pass 2 of batch j-NP, which itself waited for that batch's
// pass B, which waited for its pass A, which waited for its pass 1):
//   pass 1 (j)  at step j    writes gray / absmean / min-max partials (and
//               the caller may rewrite x on stream 0 before it)
//   pass A (j)  at step j+1  writes tile partials, xmin / xmax
//   pass B (j)  at step j+2  writes phi / C / bits / mt (ordered after pass A)
//   pass 2 (j)  at step j+3  writes y (ordered after pass B)
// so stream 0 waits for stream 3 of step i-NP+3 (clamped to the event ring:
// waiting for a LATER event of the same stream is stronger) - enqueued at the
// end of step i-1, so a caller's input write on stream 0 is ordered too - and
// every later stage of batch j is ordered after pass 1 (j) through the
// chain's own waits.
// The events live in a ring of RING steps per stream.
//
// Graph capture (mcaq_pipeline_fork): a graph of G steps starts with every
// stream forked from the capture stream and ends with a join; replays on one
// stream are then ordered after each other, so inside the graph the waits on
// steps before the fork are dropped (they completed before the replay began).
#pragma once

#define MCAQ_PIPE_STREAMS 4
#define MCAQ_PIPE_RING 8

struct mcaq_pipeline {
  hipStream_t s[MCAQ_PIPE_STREAMS];
  hipEvent_t ev[MCAQ_PIPE_STREAMS][MCAQ_PIPE_RING];
  hipEvent_t fork;
  hipEvent_t join[MCAQ_PIPE_STREAMS];
  long long step;
  long long base;      // waits on steps < base are dropped (see mcaq_pipeline_fork)
  int nplans;
  int held;            // stream 1's end-of-step event not recorded yet (hold_a)
};

static inline int pipe_wait(mcaq_pipeline* p, int k, int src, long long step) {
  if (step < p->base || step < 0) return 0;
  if (step >= p->step) return (int)hipErrorInvalidValue;   // never wait on the future
  return (int)hipStreamWaitEvent(p->s[k], p->ev[src][step % MCAQ_PIPE_RING], 0);
}

extern "C" {

int mcaq_pipeline_create(const uint32_t* cu_masks, int mask_words, int nplans, mcaq_pipeline** out) {
  if (!out || nplans < 4) return (int)hipErrorInvalidValue;
  *out = nullptr;
  mcaq_pipeline* p = new mcaq_pipeline();
  p->step = 0;
  p->base = 0;
  p->nplans = nplans;
  p->held = 0;
  int created = 0;
  hipError_t e = hipSuccess;
  for (int k = 0; k < MCAQ_PIPE_STREAMS && e == hipSuccess; ++k) {
    const uint32_t* m = cu_masks ? cu_masks + (size_t)k * mask_words : nullptr;
    bool any = false;
    for (int w = 0; m && w < mask_words; ++w) any = any || m[w] != 0;
    e = any ? hipExtStreamCreateWithCUMask(&p->s[k], (uint32_t)mask_words, m)
            : hipStreamCreateWithFlags(&p->s[k], hipStreamNonBlocking);
    if (e != hipSuccess) break;
    created = k + 1;
    for (int j = 0; j < MCAQ_PIPE_RING && e == hipSuccess; ++j)
      e = hipEventCreateWithFlags(&p->ev[k][j], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->join[k], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&p->fork, hipEventDisableTiming);
  if (e != hipSuccess) {
    for (int k = 0; k < created; ++k) (void)hipStreamDestroy(p->s[k]);
    delete p;      // events of a failed create are leaked (creation failures are fatal anyway)
    return (int)e;
  }
  *out = p;
  return 0;
}

int mcaq_pipeline_destroy(mcaq_pipeline* p) {
  if (!p) return 0;
  for (int k = 0; k < MCAQ_PIPE_STREAMS; ++k) (void)hipStreamSynchronize(p->s[k]);
  for (int k = 0; k < MCAQ_PIPE_STREAMS; ++k) {
    for (int j = 0; j < MCAQ_PIPE_RING; ++j) (void)hipEventDestroy(p->ev[k][j]);
    (void)hipEventDestroy(p->join[k]);
    (void)hipStreamDestroy(p->s[k]);
  }
  (void)hipEventDestroy(p->fork);
  delete p;
  return 0;
}

void* mcaq_pipeline_stream(mcaq_pipeline* p, int k) {
  return (p && k >= 0 && k < MCAQ_PIPE_STREAMS) ? (void*)p->s[k] : nullptr;
}

long long mcaq_pipeline_get_step(mcaq_pipeline* p) { return p ? p->step : -1; }

int mcaq_pipeline_set_step(mcaq_pipeline* p, long long step) {
  if (!p || step < 0 || p->held) return (int)hipErrorInvalidValue;
  p->step = step;
  p->base = step;     // events of the skipped range were never recorded (graph replays)
  return 0;
}

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
  if (!p || p->held) return (int)hipErrorInvalidValue;
  const long long i = p->step;
  const int r = (int)(i % MCAQ_PIPE_RING);
  const int back = p->nplans - 3 < MCAQ_PIPE_RING - 1 ? p->nplans - 3 : MCAQ_PIPE_RING - 1;
  int e;
  // resolve the morph launch configurations before enqueueing anything
  MorphLaunch LA, LB;
  if (nma > 0 && (e = morph_launch_config(ma, nma, fz, nfz, LA))) return e;
  if (nmb > 0 && (e = morph_launch_config(mb, nmb, nullptr, 0, LB))) return e;
  // stream 0: pass 1 (i); the wait for batch i-NP to be through pass 2 (its
  // buffer set) was enqueued at the end of the previous step
  if (nst > 0 && (e = mcaq_stats(st, nst, p->s[0]))) return e;
  if ((e = (int)hipEventRecord(p->ev[0][r], p->s[0]))) return e;
  // stream 1: pass A (i-1) after pass 1 (i-1) (which waited for pass 2 of
  // batch i-1-NP, the last reader of the xmin / xmax pass A rewrites)
  if ((e = pipe_wait(p, 1, 0, i - 1))) return e;
  if (nma > 0 && (e = morph_launch(LA, 1, p->s[1]))) return e;
  // stream 2: pass B (i-2) after pass A (i-2)
  if ((e = pipe_wait(p, 2, 1, i - 1))) return e;
  if (nmb > 0 && (e = morph_launch(LB, 2, p->s[2]))) return e;
  if ((e = (int)hipEventRecord(p->ev[2][r], p->s[2]))) return e;
  // stream 3: pass 2 (i-3) after pass B (i-3)
  if ((e = pipe_wait(p, 3, 2, i - 1))) return e;
  if (nq > 0 && (e = mcaq_quant(qs, nq, p->s[3]))) return e;
  if ((e = (int)hipEventRecord(p->ev[3][r], p->s[3]))) return e;
  p->step++;
  // stream 0 for step i+1: wait until batch i+1-NP is through pass 2, so what
  // the caller enqueues on stream 0 before that step (its input x) and pass 1
  // (i+1) itself find the buffer set free
  if ((e = pipe_wait(p, 0, 3, i + 1 - back))) return e;
  if (hold_a) {
    p->held = 1;
    return 0;
  }
  return (int)hipEventRecord(p->ev[1][r], p->s[1]);
}

int mcaq_pipeline_release_a(mcaq_pipeline* p) {
  if (!p || !p->held) return (int)hipErrorInvalidValue;
  p->held = 0;
  return (int)hipEventRecord(p->ev[1][(int)((p->step - 1) % MCAQ_PIPE_RING)], p->s[1]);
}

// Fork: every pipeline stream waits for `stream`'s current position, and the
// waits of later steps on steps issued before this call are dropped.  The
// CALLER guarantees that everything issued through the pipeline so far is
// complete before that position: a graph captured as fork, G steps, join and
// replayed on one stream (the previous replay, or a join of the eager steps
// before the first replay, precedes it there).
int mcaq_pipeline_fork(mcaq_pipeline* p, hipStream_t stream) {
  if (!p || p->held) return (int)hipErrorInvalidValue;
  hipError_t e = hipEventRecord(p->fork, stream);
  for (int k = 0; k < MCAQ_PIPE_STREAMS && e == hipSuccess; ++k) e = hipStreamWaitEvent(p->s[k], p->fork, 0);
  if (e == hipSuccess) p->base = p->step;
  return (int)e;
}

// Make `stream` wait for everything the pipeline has issued so far.
int mcaq_pipeline_join(mcaq_pipeline* p, hipStream_t stream) {
  if (!p || p->held) return (int)hipErrorInvalidValue;
  for (int k = 0; k < MCAQ_PIPE_STREAMS; ++k) {
    hipError_t e = hipEventRecord(p->join[k], p->s[k]);
    if (e != hipSuccess) return (int)e;
    if ((e = hipStreamWaitEvent(stream, p->join[k], 0)) != hipSuccess) return (int)e;
  }
  return 0;
}

}  // extern "C"
