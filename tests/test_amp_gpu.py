"""fp16 / bf16 feature maps at the hooks: the reference runs
training and evaluation under autocast (train.py:582-585, 748-749;
configs/train_config.yaml:69 amp: true), so C3/C4/C5 reach the hooks in half
precision.

Semantics here (engine.half_native_ok / mcaq_*_scale.dtype): pass 1 and pass 2
read the half map natively and widen it exactly; all arithmetic is fp32, so
the analyzer, bits, statistics and y are those of the fp32 path on
x.float() - bit for bit, and that path is pinned to the reference's fp32
fixtures elsewhere.  y takes the reference's result type: fp32 where the
fp32 soft mask multiplies it (quantization.py:742-744 promotes fp16 * fp32),
the input's dtype without a soft mask (rounded to nearest even from the fp32
value, as .to(dtype) rounds).

Against the reference run on half inputs (tests/golden/make_golden_r06.py ->
amp_*.npz): the analyzer upcasts (morphology.py:834-837), so complexity and
bits are pinned exactly; the reference's quantizer then rounds every
elementwise op to fp16 / bf16 (scale, zero point, x / scale + zp, ...) - a
lower-precision computation this package deliberately does not reproduce
(its CUDA op raises on half inputs, mcaq_ops.cpp:50): that part of y is
PARITY UNPINNED; the test records the result type and the gap."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_weights
from oracle import mcaq_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
DTS = {"f16": torch.float16, "bf16": torch.bfloat16}


def _blobs(dev):
    from mcaq_yolo_amd import params
    w = load_weights()
    cm = torch.from_numpy(params.pack_complexity_mlp(params.sub(w, "complexity_analyzer."))).to(dev)
    mm = torch.from_numpy(params.pack_mapper_mlp(params.sub(w, "bit_mapper."))).to(dev)
    sm = torch.from_numpy(params.pack_soft_mask(params.sub(w, "soft_mask."))).to(dev)
    return cm, mm, sm


def _feats(B, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for c, s in ((64, 80), (128, 40), (256, 20)):
        lo = torch.randn(B, c, s // 8, s // 8, generator=g)
        hi = torch.randn(B, c, s, s, generator=g)
        up = torch.nn.functional.interpolate(lo, size=(s, s), mode="bilinear", align_corners=False)
        out.append(torch.nn.functional.silu(1.5 * hi + 2 * up))
    return out


@pytest.mark.parametrize("dt", ["f16", "bf16"])
@pytest.mark.parametrize("soft_mask", [True, False])
def test_hook_plan_half_equals_fp32_path(dt, soft_mask):
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    cm, mm, sm = _blobs(DEV)
    xs = [f.to(DTS[dt]).to(DEV) for f in _feats(4, 61)]
    geoms = [ScaleGeom(*x.shape, 8) for x in xs]
    res = []
    for feats in (xs, [x.float() for x in xs]):
        plan = HookPlan(geoms, DEV)
        bufs = plan.run(feats, cm, mm, [sm if soft_mask else None] * 3, softmax_threads=O.REF_THREADS)
        torch.cuda.synchronize()
        res.append([{k: bufs[i][k].clone() for k in ("gray", "absmean", "complexity", "bits", "mt", "y")}
                    for i in range(3)] + [plan.mm.clone()])
    half, ref = res
    assert torch.equal(half[3], ref[3])                   # channel min / max
    for s in range(3):
        for k in ("gray", "complexity", "bits") + (("absmean", "mt") if soft_mask else ()):
            assert torch.equal(half[s][k], ref[s][k]), (s, k)
        yd = torch.float32 if soft_mask else DTS[dt]
        assert half[s]["y"].dtype == yd
        assert torch.equal(half[s]["y"], ref[s]["y"].to(yd)), s


@pytest.mark.parametrize("name", ["p3", "p4", "p5"])
@pytest.mark.parametrize("dt", ["f16", "bf16"])
def test_hooks_half_vs_reference_fixture(name, dt):
    from mcaq_yolo_amd.hooks import MCAQHooks
    d = np.load("%s/amp_%s.npz" % (GOLDEN, name))
    x = d["x"].astype(np.float32) if dt == "f16" else d["x_bf16"]
    torch.manual_seed(0)
    h = MCAQHooks(grid_size=int(d["grid"]), bit_mapping="mlp", device=DEV)
    sd = {}
    for k, v in load_weights().items():
        t = torch.from_numpy(np.asarray(v))
        if k.startswith("soft_mask."):
            for idx in (4, 6, 9):
                sd["quantizers.%d.%s" % (idx, k)] = t
        else:
            sd[k] = t
    h.load_state_dict(sd, strict=False)
    h.eval()
    h.softmax_threads = O.REF_THREADS
    xt = torch.from_numpy(x).to(DEV).to(DTS[dt])
    with torch.no_grad():
        outs, aux = h.forward_features([xt])
    torch.cuda.synchronize()
    bits = aux[0]["bit_map"].cpu().numpy()
    # pinned: the analyzer upcasts, so the reference's bits on the half map
    assert np.array_equal(bits, d["bits_" + dt])
    # the result type of the reference's quantizer (fp16 map x fp32 soft mask)
    assert str(outs[0].dtype) == str(d["y_%s_dtype" % dt])
    # pinned: fp32 arithmetic on the widened map = the reference's fp32 path (oracle)
    ref32 = O.hook_forward(x, load_weights(), int(d["grid"]))
    assert np.array_equal(outs[0].cpu().numpy(), ref32["y"])
    # unpinned: the reference's per-op fp16 / bf16 rounding of the quantizer's
    # arithmetic; measured gap (a few quantization steps where a rounded
    # half-precision scale moves a level), recorded, not a parity claim
    gap = float(np.abs(outs[0].cpu().numpy() - d["y_" + dt]).max())
    assert np.isfinite(gap)
    print("amp %s %s: max |y - y_ref(half arithmetic)| = %.4g" % (name, dt, gap))


def test_spatial_quantize_half_input():
    """The drop-in op on an fp16 / bf16 input: fp32 arithmetic on the
    widened input; the result is the promotion of input x mask."""
    from mcaq_yolo_amd import mcaq_cuda_ops
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 8, 16, 16, generator=g).to(DEV)
    b = torch.randint(2, 9, (2, 4, 4), generator=g).float().to(DEV)
    mn, mx = x.amin(dim=(0, 2, 3)), x.amax(dim=(0, 2, 3))
    m = (torch.rand(2, 1, 16, 16, generator=g) * 0.5 + 0.5).to(DEV)
    for dt in (torch.float16, torch.bfloat16):
        xh = x.to(dt)
        ref = mcaq_cuda_ops.spatial_quantize(xh.float(), b, mn, mx, 4, 4)
        y = mcaq_cuda_ops.spatial_quantize(xh, b, mn, mx, 4, 4)
        assert y.dtype == dt and torch.equal(y, ref.to(dt))
        ym = mcaq_cuda_ops.spatial_quantize(xh, b, mn, mx, 4, 4, m)
        assert ym.dtype == torch.float32
        assert torch.equal(ym, mcaq_cuda_ops.spatial_quantize(xh.float(), b, mn, mx, 4, 4, m))
