"""The software-pipelined hook path (engine.HookPipeline, mcaq_pipeline.h)
on the GPU: 12 distinct batches streamed through 4 cycled buffer sets with
the three streams running asynchronously must give, batch by batch, exactly
the bits, complexity and y of the plain single-stream launch of the same
batch (which the other GPU tests pin to the oracle and the reference
fixtures).  Every batch's input is written into its buffer set on the
streaming stream right before its pass 1 and its outputs are copied out on
the streaming stream right after its pass 2, so a missing cross-stream edge
(a stage reading a buffer another batch is still using) shows up as a
mismatch."""
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


@pytest.mark.parametrize("masks", [False, True])
def test_pipeline_equals_single_stream(masks):
    from mcaq_yolo_amd.engine import HookPipeline, HookPlan, ScaleGeom
    from oracle.mcaq_oracle import REF_THREADS
    cm, mm, sm = _blobs()
    geoms = [ScaleGeom(B, C, H, W, 8) for (B, C, H, W) in SHAPES]
    batches = [_batch(j) for j in range(NB)]
    # reference: the plain launch sequence of each batch on one stream
    ref = []
    rp = HookPlan(geoms, DEV)
    for j in range(NB):
        out = rp.run(batches[j], cm, mm, [sm] * 3, softmax_threads=REF_THREADS)
        ref.append([(b["y"].clone(), b["bits"].clone(), b["complexity"].clone()) for b in out])
    torch.cuda.synchronize()
    # pipeline: 4 buffer sets, inputs written / outputs read on the streaming stream
    feats = [[torch.empty(s, device=DEV) for s in SHAPES] for _ in range(4)]
    plans = []
    for p in range(4):
        plan = HookPlan(geoms, DEV)
        plan.prepare(feats[p], cm, mm, [sm] * 3, softmax_threads=REF_THREADS)
        plans.append(plan)
    torch.cuda.synchronize()
    cu = None
    if masks:
        morph = list(range(0, 256, 4))
        cu = [[c for c in range(256) if c % 4], morph, morph]
    pipe = HookPipeline(plans, cu_masks=cu)
    s0 = torch.cuda.ExternalStream(pipe.lib.mcaq_pipeline_stream(pipe.handle, 0))
    got = {}
    for i in range(NB + 3):
        if i < NB:
            with torch.cuda.stream(s0):
                for f, x in zip(feats[i % 4], batches[i]):
                    f.copy_(x)
            done = pipe.submit()
        else:
            if pipe.last is None:
                pipe.last = NB
            done = pipe.submit()
        j = i - 3
        if j >= 0:
            assert done is plans[j % 4]
            with torch.cuda.stream(s0):
                got[j] = [(b["y"].clone(), b["bits"].clone(), b["complexity"].clone()) for b in done.bufs]
    pipe.join(torch.cuda.current_stream())
    torch.cuda.synchronize()
    pipe.close()
    for j in range(NB):
        for s, ((y, bits, c), (ry, rbits, rc)) in enumerate(zip(got[j], ref[j])):
            assert torch.equal(bits, rbits), (j, s)
            assert torch.equal(c, rc), (j, s)
            assert torch.equal(y, ry), (j, s)

