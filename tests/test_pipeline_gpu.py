"""The software-pipelined hook path (engine.HookPipeline, mcaq_pipeline.h)
on the GPU: distinct batches streamed through cycled buffer sets with the
four streams running asynchronously must give, batch by batch, exactly the
bits, complexity and y of the plain single-stream launch of the same batch
(which the other GPU tests pin to the oracle and the reference fixtures).
Every batch's input is written into its buffer set on the pipeline's input
stream right before its pass 1 and its outputs are copied out on the output
stream right after its pass 2, so a missing cross-stream edge (a stage
reading a buffer another batch is still using) shows up as a mismatch.  The
same holds for steps captured as one HIP graph and replayed."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
SHAPES = ((2, 16, 80, 80), (2, 32, 40, 40), (2, 64, 20, 20))
NB = 12


def _blobs():
    import os
    from conftest import GOLDEN
    from mcaq_yolo_amd import params
    w = np.load(os.path.join(GOLDEN, "weights.npz"))
    sd = {k: w[k] for k in w.files}
    cm = torch.from_numpy(params.pack_complexity_mlp(params.sub(sd, "complexity_analyzer."))).to(DEV)
    mm = torch.from_numpy(params.pack_mapper_mlp(params.sub(sd, "bit_mapper."))).to(DEV)
    sm = torch.from_numpy(params.pack_soft_mask(params.sub(sd, "soft_mask."))).to(DEV)
    return cm, mm, sm


def _batch(j):
    g = torch.Generator().manual_seed(100 + j)
    out = []
    for (B, C, H, W) in SHAPES:
        lo = torch.randn(B, C, H // 8, W // 8, generator=g)
        hi = torch.randn(B, C, H, W, generator=g)
        up = torch.nn.functional.interpolate(lo, size=(H, W), mode="bilinear", align_corners=False)
        out.append(torch.nn.functional.silu(1.5 * hi + 2.0 * up * (1 + 0.1 * j)).contiguous().to(DEV))
    return out


def _reference(geoms, batches, cm, mm, sm):
    from mcaq_yolo_amd.engine import HookPlan
    from oracle.mcaq_oracle import REF_THREADS
    ref = []
    rp = HookPlan(geoms, DEV)
    for x in batches:
        out = rp.run(x, cm, mm, [sm] * 3, softmax_threads=REF_THREADS)
        ref.append([(b["y"].clone(), b["bits"].clone(), b["complexity"].clone()) for b in out])
    torch.cuda.synchronize()
    return ref


def _plans(geoms, n, cm, mm, sm):
    from mcaq_yolo_amd.engine import HookPlan
    from oracle.mcaq_oracle import REF_THREADS
    feats = [[torch.empty(s, device=DEV) for s in SHAPES] for _ in range(n)]
    plans = []
    for p in range(n):
        plan = HookPlan(geoms, DEV)
        plan.prepare(feats[p], cm, mm, [sm] * 3, softmax_threads=REF_THREADS)
        plans.append(plan)
    torch.cuda.synchronize()
    return feats, plans


def _check(got, ref):
    for j, r in ref.items():
        for s, ((y, bits, c), (ry, rbits, rc)) in enumerate(zip(got[j], r)):
            assert torch.equal(bits, rbits), (j, s)
            assert torch.equal(c, rc), (j, s)
            assert torch.equal(y, ry), (j, s)


@pytest.mark.parametrize("nplans,masks", [(4, False), (4, True), (5, False)])
def test_pipeline_equals_single_stream(nplans, masks):
    from mcaq_yolo_amd.engine import HookPipeline, ScaleGeom
    cm, mm, sm = _blobs()
    geoms = [ScaleGeom(B, C, H, W, 8) for (B, C, H, W) in SHAPES]
    batches = [_batch(j) for j in range(NB)]
    ref = _reference(geoms, batches, cm, mm, sm)
    feats, plans = _plans(geoms, nplans, cm, mm, sm)
    cu = None
    if masks:
        morph = list(range(0, 256, 4))
        stream = [c for c in range(256) if c % 4]
        cu = [stream, morph, morph, stream]
    pipe = HookPipeline(plans, cu_masks=cu)
    got = {}
    for i in range(NB + 3):
        if i < NB:
            with torch.cuda.stream(pipe.in_stream):
                for f, x in zip(feats[i % nplans], batches[i]):
                    f.copy_(x)
        elif pipe.last is None:
            pipe.last = NB
        done = pipe.submit()
        j = i - 3
        if j >= 0:
            assert done is plans[j % nplans]
            with torch.cuda.stream(pipe.out_stream):
                got[j] = [(b["y"].clone(), b["bits"].clone(), b["complexity"].clone()) for b in done.bufs]
    pipe.join(torch.cuda.current_stream())
    torch.cuda.synchronize()
    pipe.close()
    _check(got, dict(enumerate(ref)))


def test_pipeline_graph_replay_equals_single_stream():
    """Steps captured as HIP graphs (fork, 2 steps, join) with the input
    writes and output copies captured on the pipeline's streams, replayed
    twice around: batch j reads input bank j % 12 through buffer set j % 6,
    so consecutive users of a buffer set see different data (one graph per
    step index mod 12)."""
    from mcaq_yolo_amd.engine import HookPipeline, ScaleGeom
    NP, G, NBANK = 6, 2, 12
    cm, mm, sm = _blobs()
    geoms = [ScaleGeom(B, C, H, W, 8) for (B, C, H, W) in SHAPES]
    bank = [_batch(j) for j in range(NBANK)]
    ref = _reference(geoms, bank, cm, mm, sm)
    feats, plans = _plans(geoms, NP, cm, mm, sm)
    out = [[(torch.empty_like(b["y"]), torch.empty_like(b["bits"]), torch.empty_like(b["complexity"]))
            for b in plans[0].bufs] for _ in range(NBANK)]
    pipe = HookPipeline(plans)

    def pre(i):
        with torch.cuda.stream(pipe.in_stream):
            for f, x in zip(feats[i % NP], bank[i % NBANK]):
                f.copy_(x)

    def post(i, done):
        if done is None:
            return
        with torch.cuda.stream(pipe.out_stream):
            for (y, bits, c), b in zip(out[(i - 3) % NBANK], done.bufs):
                y.copy_(b["y"]); bits.copy_(b["bits"]); c.copy_(b["complexity"])

    for _ in range(NBANK):                # fill eagerly (batches 0..11 started)
        pre(pipe.i)
        post(pipe.i, pipe.submit())
    st = torch.cuda.Stream()
    i0 = pipe.i
    graphs = [pipe.capture(G, st, at=i0 + k, pre=pre, post=post) for k in range(0, NBANK, G)]
    pipe.join(st)
    for _ in range(2):
        for g in graphs:
            pipe.replay(g, st)
    pipe.resync(st)
    for _ in range(3):                    # drain the last replays' batches eagerly
        if pipe.last is None:
            pipe.last = pipe.i
        post(pipe.i, pipe.submit())
    pipe.join(torch.cuda.current_stream())
    torch.cuda.synchronize()
    pipe.close()
    _check({k: out[k] for k in range(NBANK)}, dict(enumerate(ref)))
