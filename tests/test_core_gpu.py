"""The drop-in module layer on the GPU: the reference's own smoke tests
(mcaq_yolo/tests/test_smoke.py) restated against mcaq_yolo_amd.core, plus
bit-exact parity of every module against the oracle / golden fixtures."""
import numpy as np
import pytest
import torch

from conftest import load_case, load_weights
from oracle import mcaq_oracle as O

pytestmark = pytest.mark.gpu
f32 = np.float32
DEV = "cuda"


def _sd(prefix):
    W = load_weights()
    return {k[len(prefix):]: torch.from_numpy(np.asarray(v)) for k, v in W.items() if k.startswith(prefix)}


@pytest.fixture(scope="module")
def mods():
    from mcaq_yolo_amd import core
    a = core.MorphologicalComplexityAnalyzer(device=DEV)
    a.load_state_dict(_sd("complexity_analyzer."))
    m = core.ComplexityToBitMappingNetwork().to(DEV)
    m.load_state_dict(_sd("bit_mapper."))
    q = core.SpatialAdaptiveQuantization().to(DEV)
    q.soft_mask.load_state_dict(_sd("soft_mask."))
    return a.eval(), m.eval(), q.eval()


# ---- test_smoke.py restated -------------------------------------------------
@pytest.mark.parametrize("H", [1024, 640, 80, 40, 20])
def test_phi_tiles_shapes(H):
    """test_smoke.py:33-47"""
    from mcaq_yolo_amd.core import MorphologicalComplexityAnalyzer
    a = MorphologicalComplexityAnalyzer(device=DEV)
    x = torch.rand(2, 3, H, H, device=DEV)
    phi, detailed = a.compute_phi_tiles(x)
    tile = a._tile_size(H)
    ht = H // tile
    assert phi.shape == (2, ht, ht, 8), phi.shape
    assert set(detailed) == {"fractal", "texture", "gradient", "edge", "contour"}
    assert tile >= 4 and (tile & (tile - 1)) == 0
    assert float(phi.min()) >= 0.0 and float(phi.max()) <= 1.0 + 1e-5


def test_analyzer_tile128_vs_reference(mods):
    """1024^2 image at grid 8 -> tile 128 (curriculum scoring of large
    inputs): phi bit-exact, C within 1e-6 and bits exact vs the reference
    fixture case_t128_c1."""
    a, m, _ = mods
    d = load_case("t128_c1")
    x = torch.from_numpy(d["x"].astype(f32)).to(DEV)
    with torch.no_grad():
        phi, _ = a.compute_phi_tiles(x)
        c = a(x)
        assert np.array_equal(phi.cpu().numpy(), d["phi"])
        cc = c.cpu().numpy()
        assert np.max(np.abs(cc - d["complexity"]) / np.abs(d["complexity"])) < 1e-6
        assert np.array_equal(m(c, 1.0).cpu().numpy(), d["bits_mlp"])


def test_analyzer_forward_range():
    """test_smoke.py:50-59 (inference half; the gradient half is the QAT path)"""
    from mcaq_yolo_amd.core import MorphologicalComplexityAnalyzer
    a = MorphologicalComplexityAnalyzer(device=DEV).eval()
    c = a(torch.rand(2, 16, 80, 80, device=DEV))
    c = c.detach()
    assert c.dim() == 3 and 0.0 <= float(c.min()) and float(c.max()) <= 1.0


def test_bit_mapper_range_and_temperature():
    """test_smoke.py:74-84"""
    from mcaq_yolo_amd.core import ComplexityToBitMappingNetwork
    m = ComplexityToBitMappingNetwork(min_bits=2, max_bits=8).to(DEV).eval()
    c = torch.rand(2, 8, 8, device=DEV)
    b = m(c, temperature=1.0)
    assert b.shape == (2, 8, 8)
    assert float(b.min()) >= 2.0 and float(b.max()) <= 8.0
    assert torch.allclose(b, torch.round(b))
    b10 = m(c, temperature=10.0)
    assert torch.allclose(b10, torch.full_like(b10, 8.0))


def test_learned_soft_mask_near_identity_init():
    """test_smoke.py:115-126 (forward half)"""
    from mcaq_yolo_amd.core import LearnedSoftMask
    mask = LearnedSoftMask().to(DEV)
    x = torch.randn(2, 8, 32, 32, device=DEV)
    m = mask(torch.full((2, 4, 4), 4.0, device=DEV), x)
    assert m.shape == (2, 1, 32, 32)
    assert float(m.min()) > 0.9, float(m.min())


def test_calibration_freeze():
    """test_smoke.py:129-139 via update_running_stats (the EMA of the
    training-mode forward)."""
    from mcaq_yolo_amd.core import SpatialAdaptiveQuantization
    q = SpatialAdaptiveQuantization(smooth_transitions=False).to(DEV)
    x = torch.randn(2, 4, 16, 16, device=DEV)
    q.update_running_stats(x)
    assert q.running_min is not None
    assert torch.equal(q.running_min.reshape(-1), x.amin(dim=(0, 2, 3)))
    x2 = torch.randn(2, 4, 16, 16, device=DEV)
    q.update_running_stats(x2)
    want = 0.99 * x.amin(dim=(0, 2, 3), keepdim=True) + (1 - 0.99) * x2.amin(dim=(0, 2, 3), keepdim=True)
    assert torch.equal(q.running_min, want)
    frozen = q.running_min.clone()
    q.freeze_calibration()
    q.update_running_stats(torch.randn(2, 4, 16, 16, device=DEV) * 100)
    assert torch.allclose(q.running_min, frozen), "stats moved after freeze"


def test_linear_bit_mapper_spatial_variance():
    """test_smoke.py:188-196"""
    from mcaq_yolo_amd.core import LinearBitMapper
    m = LinearBitMapper(min_bits=2, max_bits=8)
    c = (torch.linspace(0, 1, 16).reshape(1, 4, 4) * 0.05 + 0.4).to(DEV)
    b = m(c, temperature=1.0)
    assert float(b.min()) == 2.0 and float(b.max()) == 8.0
    assert torch.unique(b).numel() >= 5


def test_linear_bit_mapper_flat_map_absolute_fallback():
    """test_smoke.py:199-211"""
    from mcaq_yolo_amd.core import LinearBitMapper
    m = LinearBitMapper(min_bits=2, max_bits=8)
    bits = m(torch.full((1, 8, 8), 0.5, device=DEV))
    assert int(bits.min()) == 5 and int(bits.max()) == 5
    assert int(m(torch.full((1, 8, 8), 0.0, device=DEV)).max()) == 2
    assert int(m(torch.full((1, 8, 8), 1.0, device=DEV)).min()) == 8


def test_cuda_kernel_parity():
    """test_smoke.py:226-246: the extension op vs the PyTorch-path semantics
    (here bit-exact vs the oracle, not atol 1e-4), with and without m."""
    from mcaq_yolo_amd import mcaq_cuda_ops
    from mcaq_yolo_amd.core import SpatialAdaptiveQuantization
    torch.manual_seed(0)
    W = load_weights()
    for smooth in (False, True):
        q = SpatialAdaptiveQuantization(smooth_transitions=smooth).to(DEV).eval()
        if smooth:
            q.soft_mask.load_state_dict(_sd("soft_mask."))
        x = torch.randn(2, 8, 32, 32, device=DEV)
        bit_map = torch.randint(2, 9, (2, 4, 4), device=DEV).float()
        y = q(x, bit_map)
        xn, bn = x.cpu().numpy(), bit_map.cpu().numpy()
        m = O.soft_mask(bn, xn, W) if smooth else None
        ref = O.quantize(xn, bn, m)
        assert np.array_equal(y.cpu().numpy(), ref)
        # the reference extension contract: same numbers through spatial_quantize
        mn = x.amin(dim=(0, 2, 3), keepdim=True)
        mx = x.amax(dim=(0, 2, 3), keepdim=True)
        mm = q.soft_mask(bit_map, x) if smooth else None
        y2 = mcaq_cuda_ops.spatial_quantize(x.contiguous(), bit_map, mn, mx, 8, 8, mm)
        assert torch.equal(y, y2)


def test_spatial_quantize_traceable():
    """mcaq_cuda_ops.spatial_quantize is the torch.library op
    mcaq::spatial_quantize: torch.export and torch.compile (aot_eager, no code
    generation) trace a module that calls it into one opaque node, and the
    traced programs give the eager numbers."""
    from mcaq_yolo_amd import mcaq_cuda_ops

    class Q(torch.nn.Module):
        def forward(self, x, bits, mn, mx):
            return mcaq_cuda_ops.spatial_quantize(x, bits, mn, mx, 4, 4) * 2.0

    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 8, 16, 16, generator=g).to(DEV)
    bits = (torch.rand(2, 4, 4, generator=g) * 6 + 2).round().to(DEV)
    mn, mx = x.amin(dim=(0, 2, 3)).contiguous(), x.amax(dim=(0, 2, 3)).contiguous()
    ref = Q()(x, bits, mn, mx)
    ep = torch.export.export(Q(), (x, bits, mn, mx))
    assert any("mcaq.spatial_quantize" in str(n.target) for n in ep.graph.nodes)
    assert torch.equal(ep.module()(x, bits, mn, mx), ref)
    comp = torch.compile(Q(), backend="aot_eager", fullgraph=True)
    assert torch.equal(comp(x, bits, mn, mx), ref)

    # with a soft mask (the wrapper must not touch the mask's data
    # pointer, which a FakeTensor does not have)
    class QM(torch.nn.Module):
        def forward(self, x, bits, mn, mx, m):
            return mcaq_cuda_ops.spatial_quantize(x, bits, mn, mx, 4, 4, m) + 1.0

    m = (torch.rand(2, 1, 16, 16, generator=g) * 0.5 + 0.5).to(DEV)
    refm = QM()(x, bits, mn, mx, m)
    epm = torch.export.export(QM(), (x, bits, mn, mx, m))
    assert torch.equal(epm.module()(x, bits, mn, mx, m), refm)
    compm = torch.compile(QM(), backend="aot_eager", fullgraph=True)
    assert torch.equal(compm(x, bits, mn, mx, m), refm)


def test_spatial_quantize_errors():
    """mcaq_ops.cpp:37-46 checks raise RuntimeError."""
    from mcaq_yolo_amd import mcaq_cuda_ops
    x = torch.randn(1, 4, 8, 8, device=DEV)
    b = torch.full((1, 2, 2), 4.0, device=DEV)
    with pytest.raises(RuntimeError, match="one entry per channel"):
        mcaq_cuda_ops.spatial_quantize(x, b, torch.zeros(3, device=DEV), torch.ones(3, device=DEV), 4, 4)
    with pytest.raises(RuntimeError, match="mask"):
        mcaq_cuda_ops.spatial_quantize(x, b, torch.zeros(4, device=DEV), torch.ones(4, device=DEV), 4, 4,
                                       torch.ones(1, 1, 4, 4, device=DEV))
    with pytest.raises(RuntimeError, match="float32"):     # fp16 / bf16 are taken (test_amp_gpu.py)
        mcaq_cuda_ops.spatial_quantize(x.double(), b, torch.zeros(4, device=DEV), torch.ones(4, device=DEV), 4, 4)


# ---- module-level parity vs the oracle --------------------------------------
@pytest.mark.parametrize("name", ["p3_c16", "p5_c32", "crop_c8", "rect_c8"])
def test_modules_vs_oracle(mods, name):
    a, m, q = mods
    d = load_case(name)
    x = d["x"].astype(f32)
    W = load_weights()
    grid = int(d["grid"]) if "grid" in d.files else 8
    a.grid_size = grid
    try:
        xt = torch.from_numpy(x).to(DEV)
        phi, _ = a.compute_phi_tiles(xt)
        ref_phi = O.phi_tiles(x, grid)
        assert np.array_equal(phi.cpu().numpy(), ref_phi)
        C = a(xt)
        refC, _, _ = O.analyzer_forward(x, W, grid)
        assert np.array_equal(C.detach().cpu().numpy(), refC)
        bits = m(C, temperature=1.0)
        assert np.array_equal(bits.detach().cpu().numpy(), O.mlp_mapper(refC, W, 1.0))
        y = q(xt, bits)
        ref = O.hook_forward(x, W, grid)
        assert np.array_equal(y.detach().cpu().numpy(), ref["y"])
    finally:
        a.grid_size = 8


@pytest.mark.parametrize("name", ["p3_c16", "p5_c32"])
def test_score_image_vs_oracle(mods, name):
    """Curriculum score (morphology.py:923-937) on the morph kernel's phi;
    fp32 dot/mean reduction order differs from the float64 oracle: rtol 1e-5."""
    a, _, _ = mods
    x = load_case(name)["x"].astype(f32)
    s = a.score_image(torch.from_numpy(x).to(DEV))
    ref = O.score_image(x, 8, a.feature_weights.cpu().numpy())
    assert s.shape == (x.shape[0],)
    np.testing.assert_allclose(s.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)
    w0 = a.feature_weights.clone()
    try:
        alpha = a.fit_feature_weights([torch.from_numpy(x)], max_batches=1)
        assert alpha.shape == (5,) and abs(alpha.sum() - 1.0) < 1e-6 and (alpha >= 0).all()
    finally:
        a.feature_weights.copy_(w0)


def test_hooks_forward_features_vs_oracle():
    """The hook protocol end to end (C3/C4/C5 of one batch) == oracle hook."""
    from mcaq_yolo_amd.hooks import MCAQHooks
    h = MCAQHooks(device=DEV).eval()
    W = load_weights()
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in W.items()
          if k.startswith("complexity_analyzer.") or k.startswith("bit_mapper.")}
    for idx in (4, 6, 9):
        for k, v in W.items():
            if k.startswith("soft_mask."):
                sd["quantizers.%d.%s" % (idx, k)] = torch.from_numpy(np.asarray(v))
    h.load_state_dict(sd, strict=False)
    xs = [load_case(n)["x"].astype(f32) for n in ("full_p3", "full_p4", "full_p5")]
    outs, aux = h.forward_features([torch.from_numpy(x).to(DEV) for x in xs], temperature=1.0)
    assert [a_["layer"] for a_ in aux] == [4, 6, 9]
    for x, y, a_ in zip(xs, outs, aux):
        ref = O.hook_forward(x, W, 8)
        assert np.array_equal(a_["bit_map"].cpu().numpy(), ref["bits"])
        assert np.array_equal(y.cpu().numpy(), ref["y"])
    avg = MCAQHooks.avg_bits(aux)
    assert 2.0 <= float(avg) <= 8.0


def test_hook_descriptor_reuse_equals_fresh_plan():
    """Repeated eager hook calls reuse the plan's launch descriptors and only
    rebind x and the fresh outputs: every call's outputs (kept, not copied)
    equal those of a plan built from scratch for that call, and an option
    change (temperature) rebuilds the descriptors."""
    from mcaq_yolo_amd.hooks import MCAQHooks
    torch.manual_seed(1)
    h = MCAQHooks(device=DEV, indices=(4,)).eval()
    xs = [torch.nn.functional.silu(2 * torch.randn(2, 16, 40, 40, device=DEV)) for _ in range(3)]
    calls = [(xs[0], 1.0), (xs[1], 1.0), (xs[2], 1.0), (xs[0], 0.5), (xs[1], 0.5)]
    got, sts = [], []
    for x, T in calls:
        aux = h.begin(temperature=T)
        y = h.run_scale(4, x, h._mcaq_state)
        h.end()
        got.append((y, aux[0]["bit_map"], aux[0]["complexity"]))
        plan, = h._plans.values()
        sts.append(id(plan._st))
    assert sts[0] == sts[1] == sts[2] and sts[3] != sts[2] and sts[3] == sts[4]
    for (x, T), (y, bits, c) in zip(calls, got):
        h._plans = {}
        aux = h.begin(temperature=T)
        ry = h.run_scale(4, x, h._mcaq_state)
        h.end()
        assert torch.equal(bits, aux[0]["bit_map"]) and torch.equal(c, aux[0]["complexity"])
        assert torch.equal(y, ry)


def test_hooks_on_a_module_chain():
    """register_forward_hook wiring: the hooked layer's output is replaced by the
    quantized map only while a forward is open (models/mcaq_yolo.py:409-455)."""
    from mcaq_yolo_amd.hooks import MCAQHooks
    torch.manual_seed(0)
    layers = torch.nn.Sequential(*[torch.nn.Identity() for _ in range(10)]).to(DEV)
    h = MCAQHooks(device=DEV, indices=(4,)).eval().register(layers)
    x = torch.nn.functional.silu(torch.randn(2, 16, 40, 40, device=DEV))
    assert torch.equal(layers(x), x)            # inactive: pass-through
    aux = h.begin(temperature=1.0)
    y = layers(x)
    h.end()
    assert len(aux) == 1 and torch.equal(y, aux[0]["features_q"]) and not torch.equal(y, x)
    h.begin(quantize=False)
    assert torch.equal(layers(x), x)            # quantize=False: aux only
    h.end()
    h.remove()


# ---- eval mode with autograd: kernel values, reference gradients ------------
def test_eval_modules_keep_reference_gradients(mods):
    """bit_allocation.py:42-80 / 218-280 and morphology.py:939-973 stay
    differentiable in eval mode.  The GPU value is the kernel's (identical to
    the no_grad call; the CPU pure-PyTorch path agrees within the MLP's
    LayerNorm / GEMV ulps, 1e-6); the gradient equals the CPU path's gradient
    (torch recomputation, GEMM ulps: rtol 1e-4)."""
    from mcaq_yolo_amd import core
    a, m, _ = mods
    x = torch.from_numpy(load_case("p3_c16")["x"].astype(f32))
    a_cpu = core.MorphologicalComplexityAnalyzer(device="cpu")
    a_cpu.load_state_dict(_sd("complexity_analyzer."))
    m_cpu = core.ComplexityToBitMappingNetwork()
    m_cpu.load_state_dict(_sd("bit_mapper."))
    lin = core.LinearBitMapper()
    a_cpu.eval(), m_cpu.eval()
    for mod in (a, m, a_cpu, m_cpu):
        mod.zero_grad(set_to_none=True)
    c_gpu = a(x.to(DEV))
    c_cpu = a_cpu(x)
    assert c_gpu.requires_grad
    np.testing.assert_allclose(c_gpu.detach().cpu().numpy(), c_cpu.detach().numpy(), rtol=1e-6, atol=1e-7)
    with torch.no_grad():
        assert torch.equal(a(x.to(DEV)), c_gpu.detach())
    cg = c_gpu.detach().clone().requires_grad_(True)
    cc = c_gpu.detach().cpu().clone().requires_grad_(True)
    for mg, mc in ((m, m_cpu), (lin, lin)):
        bg = mg(cg, 1.0, return_continuous=True)
        bc = mc(cc, 1.0, return_continuous=True)
        np.testing.assert_allclose(bg.detach().cpu().numpy(), bc.detach().numpy(), rtol=1e-6, atol=1e-6)
        w = torch.linspace(-1, 1, bg.numel()).view_as(bc)
        (bg * w.to(DEV)).sum().backward()
        (bc * w).sum().backward()
        np.testing.assert_allclose(cg.grad.cpu().numpy(), cc.grad.numpy(), rtol=1e-4, atol=1e-6)
        cg.grad = cc.grad = None
    for (n, pg), (_, pc) in zip(m.mapping_network.named_parameters(), m_cpu.mapping_network.named_parameters()):
        np.testing.assert_allclose(pg.grad.cpu().numpy(), pc.grad.numpy(), rtol=1e-4, atol=1e-6, err_msg=n)
    (c_gpu * torch.linspace(0, 1, c_gpu.numel(), device=DEV).view_as(c_gpu)).sum().backward()
    (c_cpu * torch.linspace(0, 1, c_cpu.numel()).view_as(c_cpu)).sum().backward()
    for (n, pg), (_, pc) in zip(a.complexity_mlp.named_parameters(), a_cpu.complexity_mlp.named_parameters()):
        np.testing.assert_allclose(pg.grad.cpu().numpy(), pc.grad.numpy(), rtol=1e-4, atol=1e-6, err_msg=n)
    for mod in (a, m):
        mod.zero_grad(set_to_none=True)


@pytest.mark.parametrize("name", ["p3_c16", "odd_c20", "g16_c16"])
def test_gpu_equals_cpu_torch_path(mods, name):
    """The HIP path and the package's pure-PyTorch path give the same bits
    and y on the same inputs (C within the MLP's LayerNorm / GEMV ulps)."""
    from mcaq_yolo_amd.hooks import MCAQHooks
    d = load_case(name)
    grid = int(d["grid"])
    x = torch.from_numpy(d["x"].astype(f32))
    res = {}
    for dev in ("cpu", DEV):
        h = MCAQHooks(grid_size=grid, device=dev, indices=(4,))
        sd = {k: v for k, v in _sd("").items() if k.startswith(("complexity_analyzer.", "bit_mapper."))}
        sd.update({"quantizers.4." + k: v for k, v in _sd("").items() if k.startswith("soft_mask.")})
        h.load_state_dict(sd, strict=False)
        h.to(dev).eval()
        with torch.no_grad():
            outs, aux = h.forward_features([x.to(dev)])
        res[dev] = (outs[0].cpu(), aux[0]["bit_map"].cpu(), aux[0]["complexity"].cpu())
    assert torch.equal(res["cpu"][0], res[DEV][0]) and torch.equal(res["cpu"][1], res[DEV][1])
    np.testing.assert_allclose(res["cpu"][2].numpy(), res[DEV][2].numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("name", ["pt_p3", "pt_p5", "pt_odd"])
@pytest.mark.parametrize("mapping", ["mlp", "linear"])
def test_per_tensor_hook_vs_reference(name, mapping):
    """Fused hook with per_channel=False quantizers (the finalize reduces every
    channel's partials to one min/max): bits and y bit-exact vs the reference
    fixture (tests/golden/make_golden_r02.py pertensor)."""
    import os
    from conftest import GOLDEN
    from test_fallback_cpu import hooks_per_tensor
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    h = hooks_per_tensor(DEV, int(d["grid"]), mapping)
    x = torch.from_numpy(d["x"].astype(f32)).to(DEV)
    with torch.no_grad():
        outs, aux = h.forward_features([x])
    key = "mlp" if mapping == "mlp" else "lin"
    assert np.array_equal(aux[0]["bit_map"].cpu().numpy(), d["bits_" + key])
    assert np.array_equal(outs[0].cpu().numpy(), d["y_" + key])


def test_per_tensor_calibrated_frozen_hook_equals_cpu_path():
    """per_channel=False with calibration then freeze_calibration: the fused
    hook reads the scalar running statistics (min_stride 0) and gives the same
    bits and y as the pure-PyTorch CPU path with the same state."""
    import os
    from conftest import GOLDEN
    from test_fallback_cpu import hooks_per_tensor
    d = np.load(os.path.join(GOLDEN, "pt_p5.npz"))
    x = torch.from_numpy(d["x"].astype(f32))
    res = {}
    for dev in ("cpu", DEV):
        h = hooks_per_tensor(dev, int(d["grid"]), "mlp")
        q = h.quantizers["4"]
        with torch.no_grad():
            for k in range(3):      # calibration passes (EMA of the batch min/max)
                h.begin(calibrating=True)
                h.run_scale(4, (x * (1.0 + 0.1 * k)).to(dev), h._mcaq_state)
                h.end()
            q.freeze_calibration()
            assert q.running_min.numel() == 1
            outs, aux = h.forward_features([x.to(dev)])
        res[dev] = (outs[0].cpu().numpy(), aux[0]["bit_map"].cpu().numpy(), float(q.running_min), float(q.running_max))
    assert res["cpu"][2:] == res[DEV][2:]
    assert np.array_equal(res["cpu"][1], res[DEV][1])
    assert np.array_equal(res["cpu"][0], res[DEV][0])


def test_hooks_softmax_threads_pinned():
    """MCAQHooks.softmax_threads pins the ATen thread partition the soft mask
    reproduces: the fused hook at softmax_threads=T equals the oracle at T,
    whatever torch.get_num_threads() is in this process."""
    from mcaq_yolo_amd.hooks import MCAQHooks
    d = load_case("odd_c20")
    x = d["x"].astype(f32)
    W = load_weights()
    h = MCAQHooks(grid_size=int(d["grid"]), device=DEV, indices=(4,))
    sd = {k: v for k, v in _sd("").items() if k.startswith(("complexity_analyzer.", "bit_mapper."))}
    sd.update({"quantizers.4." + k: v for k, v in _sd("").items() if k.startswith("soft_mask.")})
    h.load_state_dict(sd, strict=False)
    h.eval()
    old = torch.get_num_threads()
    try:
        torch.set_num_threads(3)
        for T in (1, 8):
            h.softmax_threads = T
            with torch.no_grad():
                outs, aux = h.forward_features([torch.from_numpy(x).to(DEV)])
            bits = aux[0]["bit_map"].cpu().numpy()
            m = O.soft_mask(bits, x, W, threads=T)
            y = O.quantize(x, bits, m, x.min(axis=(0, 2, 3)), x.max(axis=(0, 2, 3)))
            assert np.array_equal(outs[0].cpu().numpy(), y), T
    finally:
        torch.set_num_threads(old)


@pytest.mark.parametrize("shape", [(2, 24, 40, 40), (3, 20, 13, 11), (2, 256, 20, 20)])
def test_channel_minmax_nonfinite_like_aten(shape):
    """Pass 1 + finalize channel min/max propagate NaN and keep +-inf, as
    ATen's amin/amax (quantization.py:650-654) do."""
    from mcaq_yolo_amd import core
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(*shape, generator=g)
    B, C, H, W = shape
    x[1, 2, H // 2, W // 3] = float("nan")
    x[0, 3, H - 1, W - 1] = float("inf")
    x[-1, 4, 0, 0] = float("-inf")
    x[:, 5] = float("inf")
    x[:, 6] = -0.0
    mn, mx = core._channel_minmax(x.to(DEV))
    rmn, rmx = x.amin(dim=(0, 2, 3)), x.amax(dim=(0, 2, 3))
    torch.testing.assert_close(mn.cpu(), rmn, rtol=0, atol=0, equal_nan=True)
    torch.testing.assert_close(mx.cpu(), rmx, rtol=0, atol=0, equal_nan=True)


@pytest.mark.parametrize("smooth", [False, True])
def test_frozen_quant_nonfinite_like_reference(smooth):
    """Pass 2 with frozen calibration statistics on inputs holding +-inf and
    NaN: +inf -> the qmax level, -inf -> the qmin level, NaN stays NaN, as the
    reference's torch.round / torch.clamp quantizer (quantization.py:592-600)
    gives -- the CPU module (the reference algorithm), the HIP module and the
    extension op agree bit for bit, NaN positions included."""
    from mcaq_yolo_amd import mcaq_cuda_ops
    from mcaq_yolo_amd.core import SpatialAdaptiveQuantization
    g = torch.Generator().manual_seed(11)
    B, C, H, W = 2, 12, 16, 16
    x = torch.randn(B, C, H, W, generator=g)
    rmin, rmax = x.amin(dim=(0, 2, 3), keepdim=True), x.amax(dim=(0, 2, 3), keepdim=True)
    x[0, 1, 3, 4] = float("inf")
    x[1, 2, 5, 6] = float("-inf")
    x[0, 3, 7, 8] = float("nan")
    x[1, 4, :, 0] = float("inf")
    x[0, 5, 0, :] = float("nan")
    bit_map = torch.randint(2, 9, (B, 4, 4), generator=g).float()
    outs = {}
    for dev in ("cpu", DEV):
        q = SpatialAdaptiveQuantization(smooth_transitions=smooth)
        if smooth:
            q.soft_mask.load_state_dict(_sd("soft_mask."))
        q = q.to(dev).eval()
        q.running_min, q.running_max = rmin.to(dev), rmax.to(dev)
        q.freeze_calibration()
        with torch.no_grad():
            outs[dev] = q(x.to(dev), bit_map.to(dev)).cpu()
    torch.testing.assert_close(outs[DEV], outs["cpu"], rtol=0, atol=0, equal_nan=True)
    y = outs[DEV]
    assert torch.isnan(y[0, 3, 7, 8]) and torch.isnan(y[0, 5, 0]).all()
    if not smooth:
        # (with the soft mask, the image's NaN / inf |x| make its m NaN, as in the reference)
        assert torch.isfinite(y[0, 1, 3, 4]) and torch.isfinite(y[1, 2, 5, 6]) and torch.isfinite(y[1, 4, :, 0]).all()
        # extension op, same statistics
        y2 = mcaq_cuda_ops.spatial_quantize(x.to(DEV).contiguous(), bit_map.to(DEV), rmin.to(DEV), rmax.to(DEV), 4, 4)
        torch.testing.assert_close(y2.cpu(), outs["cpu"], rtol=0, atol=0, equal_nan=True)


@pytest.mark.parametrize("name", ["p3", "p5", "odd", "img"])
def test_score_and_fit_vs_reference_fixture(name):
    """Curriculum scoring on the HIP path vs the reference's own outputs
    (tests/golden/score_*.npz, make_golden_r03.py).  phi comes from the
    morph kernel (bit-exact); the 5-term dot and the tile mean run as device
    reductions in another fp32 order than CPU ATen: scores within rtol 1e-6.
    The NNLS target is the complexity MLP on the device (ulps from the CPU
    GEMM order): alpha within 1e-5."""
    from test_score_cpu import analyzer, load
    d, x, fits = load(name)
    a = analyzer(DEV, int(d["grid"]))
    s0 = a.score_image(torch.from_numpy(x).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(s0, d["score0"], rtol=1e-6, atol=1e-7)
    alpha = a.fit_feature_weights(iter(torch.from_numpy(f) for f in fits), max_batches=len(fits))
    np.testing.assert_allclose(alpha, d["alpha"], rtol=0, atol=1e-5)
    s1 = a.score_image(torch.from_numpy(x).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(s1, d["score1"], rtol=1e-5, atol=1e-6)
