"""QAT quantizer (training branch; BASELINE config 5) on the
GPU through the C ABI: EMA running statistics, fractional-bit forward and
straight-through backward against the reference's own train-mode fixtures
(tests/golden/qat_*.npz) and the oracle (oracle/mcaq_oracle.py qat_*).

Tolerances: y, grad_x and the running statistics are bit-exact; the two
channel/tile sums (grad of m, grad of the bit map) are fp32 sums in a
different order from ATen's, compared within 1e-4 of the largest magnitude."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_weights
from oracle import mcaq_oracle as O

pytestmark = pytest.mark.gpu
f32 = np.float32
DEV = "cuda"
QAT_CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("qat_") and f.endswith(".npz"))


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=f32)).to(DEV)


def N(t):
    return t.detach().cpu().numpy()


def close_sum(got, ref, tol=1e-4):
    ref = np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-30)
    err = np.abs(np.asarray(got, np.float64) - ref).max()
    assert err <= tol * scale, "max err %g vs scale %g" % (err, scale)


def ema(x, r0min, r0max):
    from mcaq_yolo_amd import abi, core
    xmin, xmax = core._channel_minmax(T(x))
    rmin, rmax = T(r0min).clone(), T(r0max).clone()
    abi.check(abi.lib().mcaq_ema_stats(core._p(xmin), core._p(xmax), core._p(rmin), core._p(rmax), rmin.numel(),
                                       0.99, 0, core._stream()), "ema")
    return rmin, rmax


@pytest.mark.parametrize("name", QAT_CASES)
def test_qat_kernels_vs_reference_fixture(name):
    from mcaq_yolo_amd import core
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    x, bits, g = d["x"], d["bits"], d["g"]
    rmin, rmax = ema(x, d["r0min"], d["r0max"])
    assert np.array_equal(N(rmin), d["rmin"]) and np.array_equal(N(rmax), d["rmax"]), "EMA"
    smooth = bool(d["smooth"])
    m = T(d["m"]) if smooth else None
    y = core.qat_quantize(T(x), T(bits), m, rmin, rmax)
    assert np.array_equal(N(y), d["y"]), "forward"
    gx, gb, gm = core.qat_quantize_backward(T(g), T(x), T(bits), m, rmin, rmax)
    assert np.array_equal(N(gx), d["gx"]), "grad x"
    ogx, ogb, ogm = O.qat_backward(g, x, bits, d["rmin"], d["rmax"], d["m"] if smooth else None)
    close_sum(N(gb), ogb)
    if smooth:
        close_sum(N(gm), ogm)
    else:
        assert gm is None
        close_sum(N(gb), d["gbits"])


@pytest.mark.parametrize("shape", [(2, 64, 80, 80, 10, 10), (3, 40, 13, 17, 3, 4), (1, 33, 20, 20, 5, 5),
                                   (2, 256, 20, 20, 5, 5)])
def test_qat_kernels_vs_oracle(shape):
    """Seeded random shapes incl. ragged H*W (not a multiple of 4), a partial
    channel slice (C = 33, 40) and both ends of the bit range."""
    from mcaq_yolo_amd import core
    B, C, H, W, ht, wt = shape
    rng = np.random.default_rng(sum(shape))
    x = (rng.standard_normal((B, C, H, W)) * 1.5).astype(f32)
    bits = rng.uniform(2.0, 8.0, (B, ht, wt)).astype(f32)
    bits.reshape(-1)[:3] = [2.0, 8.0, 7.5]
    m = rng.uniform(0.5, 1.0, (B, H, W)).astype(f32)
    g = rng.standard_normal((B, C, H, W)).astype(f32)
    mn, mx = x.min(axis=(0, 2, 3)), x.max(axis=(0, 2, 3))
    for mm in (None, m):
        y = core.qat_quantize(T(x), T(bits), None if mm is None else T(mm), T(mn), T(mx))
        ref, _ = O.qat_forward(x, bits, mn, mx, mm)
        assert np.array_equal(N(y), ref)
        gx, gb, gm = core.qat_quantize_backward(T(g), T(x), T(bits), None if mm is None else T(mm), T(mn), T(mx))
        ogx, ogb, ogm = O.qat_backward(g, x, bits, mn, mx, mm)
        assert np.array_equal(N(gx), ogx)
        close_sum(N(gb), ogb)
        if mm is not None:
            close_sum(N(gm), ogm)


def test_qat_integer_bits_equal_inference_kernel():
    """f = 0 everywhere: the QAT forward equals the pass-2 inference kernel,
    at the full P3 shape of config 2 (yolov8n, bs 8 here)."""
    from mcaq_yolo_amd import abi, core
    B, C, H, W, ht, wt = 8, 64, 80, 80, 10, 10
    gen = torch.Generator(device="cpu").manual_seed(11)
    x = (torch.randn(B, C, H, W, generator=gen) * 2).to(DEV)
    bits = torch.randint(2, 9, (B, ht, wt), generator=gen).float().to(DEV)
    m = torch.rand(B, H, W, generator=gen).to(DEV)
    xmin, xmax = core._channel_minmax(x)
    y = core.qat_quantize(x, bits, m, xmin, xmax)
    y2 = torch.empty_like(x)
    q = abi.QuantScale()
    q.x, q.y, q.bits, q.m, q.xmin, q.xmax = core._p(x), core._p(y2), core._p(bits), core._p(m), core._p(xmin), \
        core._p(xmax)
    q.B, q.C, q.H, q.W, q.ht, q.wt, q.bits_lo, q.nbits = B, C, H, W, ht, wt, 2, 7
    abi.check(abi.lib().mcaq_quant(abi.ctypes.byref(q), 1, core._stream()), "mcaq_quant")
    assert torch.equal(y, y2)


@pytest.mark.parametrize("name", ["qat_p4_plain", "qat_p4_smooth", "qat_p5_smooth"])
def test_quantizer_module_train_mode(name):
    """SpatialAdaptiveQuantization in train mode (the reference module's
    forward + autograd): running stats bit-exact, y and grads vs the
    reference's own train-mode outputs."""
    from mcaq_yolo_amd import core
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    smooth = bool(d["smooth"])
    q = core.SpatialAdaptiveQuantization(smooth_transitions=smooth).to(DEV)
    if smooth:
        W = load_weights()
        q.soft_mask.load_state_dict({k[len("soft_mask."):]: torch.from_numpy(np.asarray(v))
                                     for k, v in W.items() if k.startswith("soft_mask.")})
    q.running_min = T(d["r0min"]).view(1, -1, 1, 1)
    q.running_max = T(d["r0max"]).view(1, -1, 1, 1)
    q.train()
    x = T(d["x"]).requires_grad_(True)
    b = T(d["bits"]).requires_grad_(True)
    y = q(x, b, training=True)
    assert np.array_equal(N(q.running_min).reshape(-1), d["rmin"])
    assert np.array_equal(N(q.running_max).reshape(-1), d["rmax"])
    if smooth:   # m from the HIP soft mask (oracle-exact) vs the reference's CPU m: ulps apart
        np.testing.assert_allclose(N(y), d["y"], rtol=1e-5, atol=1e-6)
    else:
        assert np.array_equal(N(y), d["y"])
    y.backward(T(d["g"]))
    if smooth:
        np.testing.assert_allclose(N(x.grad), d["gx"], rtol=1e-5, atol=1e-6)
    else:
        assert np.array_equal(N(x.grad), d["gx"])
    close_sum(N(b.grad), d["gbits"], tol=1e-3 if smooth else 1e-4)


def test_hook_train_step_gradients():
    """MCAQHooks in train mode: one QAT step over the three hook scales reaches
    the complexity MLP, the bit mapper and the soft masks with finite grads."""
    from mcaq_yolo_amd.hooks import MCAQHooks
    torch.manual_seed(0)
    h = MCAQHooks(device=DEV).train()
    gen = torch.Generator(device="cpu").manual_seed(5)
    feats = [torch.nn.functional.silu(1.5 * torch.randn(4, c, s, s, generator=gen)).to(DEV).requires_grad_(True)
             for c, s in ((64, 80), (128, 40), (256, 20))]
    outs, aux = h.forward_features(feats, temperature=1.0)
    assert len(aux) == 3
    for a in aux:
        bm = a["bit_map"]
        assert float(bm.min()) >= 2.0 and float(bm.max()) <= 8.0
    loss = sum((o * o).mean() for o in outs) + 0.01 * torch.stack([a["bit_map"].mean() for a in aux]).mean()
    loss.backward()
    for f in feats:
        assert f.grad is not None and torch.isfinite(f.grad).all()
    named = dict(h.named_parameters())
    for k in ("complexity_analyzer.complexity_mlp.0.weight", "bit_mapper.mapping_network.0.weight",
              "quantizers.4.soft_mask.net.0.weight"):
        gp = named[k].grad
        assert gp is not None and torch.isfinite(gp).all() and float(gp.abs().sum()) > 0, k
    assert all(q.running_min is not None for q in h.quantizers.values())


def test_hook_train_step_linear_mapper_gradients():
    """with bit_mapping='linear' the bit map stays differentiable on
    the GPU path too (bit_allocation.py:42-80): the quantizer's and the bit
    loss's gradients reach the complexity MLP."""
    from mcaq_yolo_amd.hooks import MCAQHooks
    torch.manual_seed(0)
    h = MCAQHooks(device=DEV, bit_mapping="linear").train()
    gen = torch.Generator(device="cpu").manual_seed(6)
    feats = [torch.nn.functional.silu(1.5 * torch.randn(2, c, s, s, generator=gen)).to(DEV).requires_grad_(True)
             for c, s in ((64, 80), (128, 40), (256, 20))]
    outs, aux = h.forward_features(feats, temperature=1.0)
    loss = sum((o * o).mean() for o in outs) + (MCAQHooks.avg_bits(aux) - 4.0) ** 2
    loss.backward()
    gp = dict(h.named_parameters())["complexity_analyzer.complexity_mlp.0.weight"].grad
    assert gp is not None and torch.isfinite(gp).all() and float(gp.abs().sum()) > 0


def test_qat_misaligned_views_match_aligned():
    """contiguous views whose storage offset is not a multiple of 16
    bytes take the scalar kernels (the float4 ones need aligned x/y/g/gx);
    results equal the aligned run."""
    from mcaq_yolo_amd import core
    B, C, H, W, ht, wt = 2, 40, 20, 20, 5, 5
    gen = torch.Generator(device="cpu").manual_seed(12)
    n = B * C * H * W
    xs = torch.randn(n + 1, generator=gen).to(DEV)[1:].view(B, C, H, W)      # 4-byte offset
    gs = torch.randn(n + 1, generator=gen).to(DEV)[1:].view(B, C, H, W)
    assert xs.is_contiguous() and xs.data_ptr() % 16 != 0
    bits = (torch.rand(B, ht, wt, generator=gen) * 6 + 2).to(DEV)
    m = torch.rand(B, H, W, generator=gen).to(DEV)
    mn, mx = core._channel_minmax(xs.clone())
    y1 = core.qat_quantize(xs, bits, m, mn, mx)
    y2 = core.qat_quantize(xs.clone(), bits, m, mn, mx)
    assert torch.equal(y1, y2)
    g1 = core.qat_quantize_backward(gs, xs, bits, m, mn, mx)
    g2 = core.qat_quantize_backward(gs.clone(), xs.clone(), bits, m, mn, mx)
    for a, b in zip(g1, g2):
        assert torch.equal(a, b)


def test_spatial_quantize_misaligned_view():
    from mcaq_yolo_amd import mcaq_cuda_ops
    B, C, H, W = 2, 16, 16, 16
    gen = torch.Generator(device="cpu").manual_seed(13)
    xs = torch.randn(B * C * H * W + 3, generator=gen).to(DEV)[3:].view(B, C, H, W)
    assert xs.data_ptr() % 16 != 0
    bits = torch.randint(2, 9, (B, 4, 4), generator=gen).float().to(DEV)
    mn, mx = xs.amin(dim=(0, 2, 3)), xs.amax(dim=(0, 2, 3))
    y1 = mcaq_cuda_ops.spatial_quantize(xs, bits, mn, mx, 4, 4)
    y2 = mcaq_cuda_ops.spatial_quantize(xs.clone(), bits, mn, mx, 4, 4)
    assert torch.equal(y1, y2)


def _allclose_rel(got, ref, rtol, floor=1e-30):
    """max |got - ref| <= rtol * max(|ref|, floor).  `floor` covers gradients
    that are zero in exact arithmetic (a Linear bias feeding a train-mode
    BatchNorm), whose reference values are rounding noise."""
    ref = np.asarray(ref, np.float64)
    err = np.abs(np.asarray(got, np.float64) - ref).max()
    scale = max(np.abs(ref).max(), floor)
    assert err <= rtol * scale, "max err %g vs scale %g" % (err, scale)


def test_analyzer_train_mode_vs_reference():
    """Train-mode analyzer (phi on the morph kernel, complexity MLP + bilateral
    with autograd) against the reference's own train-mode C and MLP grads
    (tests/golden/train_analyzer.npz; GPU GEMM/LayerNorm ulps: 1e-5 / 1e-4)."""
    from mcaq_yolo_amd import core
    d = np.load(os.path.join(GOLDEN, "train_analyzer.npz"))
    W = load_weights()
    a = core.MorphologicalComplexityAnalyzer(device=DEV)
    a.load_state_dict({k[len("complexity_analyzer."):]: torch.from_numpy(np.asarray(v))
                       for k, v in W.items() if k.startswith("complexity_analyzer.")})
    a.train()
    c = a(T(d["x"]))
    _allclose_rel(N(c), d["c"], 1e-5)
    c.backward(T(d["gc"]))
    gmax = max(np.abs(d[k]).max() for k in d.files if k.startswith("grad."))
    for n, p in a.complexity_mlp.named_parameters():
        _allclose_rel(N(p.grad), d["grad.complexity_mlp." + n], 1e-4, floor=1e-2 * gmax)


@pytest.mark.parametrize("temp", [1, 3])
def test_mapper_train_mode_vs_reference(temp):
    """Train-mode bit mapper (batch-statistics BatchNorm, straight-through
    clamp) against the reference: continuous bits, grads, BN running stats."""
    from mcaq_yolo_amd import core
    d = np.load(os.path.join(GOLDEN, "train_mapper.npz"))
    W = load_weights()
    t = "t%d" % temp
    m = core.ComplexityToBitMappingNetwork().to(DEV)
    m.load_state_dict({k[len("bit_mapper."):]: torch.from_numpy(np.asarray(v))
                       for k, v in W.items() if k.startswith("bit_mapper.")})
    m.train()
    c = T(d[t + ".c"]).requires_grad_(True)
    bits = m(c, float(temp), return_continuous=True)
    _allclose_rel(N(bits), d[t + ".bits"], 1e-5)
    bits.backward(T(d[t + ".gb"]))
    _allclose_rel(N(c.grad), d[t + ".grad_c"], 1e-4)
    gmax = max(np.abs(d[k]).max() for k in d.files if k.startswith(t + ".grad.mapping_network."))
    for n, p in m.mapping_network.named_parameters():
        ref = d[t + ".grad.mapping_network." + n]
        if n in ("0.bias", "3.bias", "6.bias"):
            # a Linear bias feeding a train-mode BatchNorm: zero in exact
            # arithmetic, rounding noise in both implementations
            assert np.abs(N(p.grad)).max() <= 1e-6 * np.abs(d[t + ".grad_c"]).max()
            continue
        _allclose_rel(N(p.grad), ref, 1e-4, floor=1e-2 * gmax)
    for n, b in m.mapping_network.named_buffers():
        if b.dtype.is_floating_point:
            _allclose_rel(N(b), d[t + ".buf.mapping_network." + n], 1e-5)


@pytest.mark.parametrize("shape", [(16, 64, 80, 80, 10, 10), (3, 40, 19, 17, 3, 4), (2, 256, 20, 20, 5, 5),
                                   (2, 32, 44, 52, 11, 13)])
def test_qat_fold_in_launch_equals_fold_kernel(shape):
    """The backward's in-launch fold (last unit of each image, arrival
    counters) gives grad_m / grad_bits bit-identical to the separate fold
    kernel (same summation order), leaves the counters zeroed, and repeated
    launches (three scales in one launch, replayed) give the same bits."""
    from mcaq_yolo_amd import abi, core
    B, C, H, W, ht, wt = shape
    rng = np.random.default_rng(7 + sum(shape))
    x = T((rng.standard_normal((B, C, H, W)) * 1.5).astype(f32))
    g = T(rng.standard_normal((B, C, H, W)).astype(f32))
    bits = T(rng.uniform(2.0, 8.0, (B, ht, wt)).astype(f32))
    m = T(rng.uniform(0.5, 1.0, (B, H, W)).astype(f32))
    mn, mx = core._channel_minmax(x)
    L = abi.lib()
    outs = {}
    arrive = torch.zeros(B * ht, dtype=torch.int32, device=DEV)
    for fused in (False, True, True):
        gx = torch.empty_like(x)
        gm = torch.empty(B, H, W, device=DEV)
        gb = torch.empty(B, ht, wt, device=DEV)
        work = torch.full((L.mcaq_qat_work_floats(B, C, H, W),), float("nan"), device=DEV)
        q = core._qat_struct(x, bits, m, mn, mx)
        q.g, q.gx, q.gm, q.gb, q.work = core._p(g), core._p(gx), core._p(gm), core._p(gb), core._p(work)
        if fused:
            q.arrive = core._p(arrive)
        abi.check(L.mcaq_qat_backward(abi.ctypes.byref(q), 1, core._stream()), "mcaq_qat_backward")
        torch.cuda.synchronize()
        outs.setdefault(fused, []).append((N(gx), N(gm), N(gb)))
    assert int(arrive.abs().sum()) == 0
    ref = outs[False][0]
    for got in outs[True]:
        for a, b in zip(got, ref):
            assert np.array_equal(a, b)
