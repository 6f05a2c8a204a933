"""Fused train-mode tile networks (csrc/mcaq_train.h) against the torch
autograd restatement of the same modules (core.FUSED_TRAIN = False, the r02
path, itself checked against the reference's train fixtures in
test_qat_gpu.py) and against those fixtures directly.

Tolerances (fp32 sums in other orders than ATen's): values 1e-5 relative,
gradients 1e-3 of the largest magnitude of the reference gradient; the
Linear layers feeding a train-mode BatchNorm (bias gradient zero in exact
arithmetic, weight gradient a cancelling sum) against 1e-4 of the module's
largest gradient."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_weights

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(got, ref, rtol, floor=1e-30):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    err = float((got - ref).abs().max())
    scale = max(float(ref.abs().max()), floor)
    assert err <= rtol * scale, "max err %g vs scale %g" % (err, scale)


def _hooks(mapper="mlp"):
    from mcaq_yolo_amd.hooks import MCAQHooks
    torch.manual_seed(0)
    h = MCAQHooks(device=DEV, bit_mapping=mapper)
    W = load_weights()
    sd = {}
    for k, v in W.items():
        t = torch.from_numpy(np.asarray(v))
        if k.startswith("soft_mask."):
            for idx in (4, 6, 9):
                sd["quantizers.%d.%s" % (idx, k)] = t
        elif mapper == "mlp" or not k.startswith("bit_mapper."):
            sd[k] = t
    h.load_state_dict(sd, strict=False)
    return h.train()


def _step(fused, B=4, seed=5, mapper="mlp", temperature=1.0, shapes=((64, 80), (128, 40), (256, 20))):
    """One train-mode forward + backward of the three hooks; returns outputs,
    aux, feature grads, parameter grads and buffers."""
    from mcaq_yolo_amd import core
    old = core.FUSED_TRAIN
    core.FUSED_TRAIN = fused
    try:
        h = _hooks(mapper)
        gen = torch.Generator(device="cpu").manual_seed(seed)
        feats = []
        for c, s in shapes:
            lo = torch.randn(B, c, s // 8, s // 8, generator=gen)
            hi = torch.randn(B, c, s, s, generator=gen)
            up = torch.nn.functional.interpolate(lo, size=(s, s), mode="bilinear", align_corners=False)
            feats.append(torch.nn.functional.silu(1.5 * hi + 2 * up).to(DEV).requires_grad_(True))
        outs, aux = h.forward_features(feats, temperature=temperature)
        gens = [torch.randn(o.shape, generator=gen).to(DEV) * 1e-3 for o in outs]
        avg = torch.stack([a["bit_map"].float().mean() for a in aux]).mean()
        smooth = sum(((a["bit_map"][:, 1:] - a["bit_map"][:, :-1]) ** 2).mean() for a in aux)
        loss = sum((o * g).sum() for o, g in zip(outs, gens)) + 0.1 * (avg - 4.0) ** 2 + 0.01 * smooth
        loss.backward()
        torch.cuda.synchronize()
        grads = {k: p.grad.detach().clone() for k, p in h.named_parameters() if p.grad is not None}
        bufs = {k: b.detach().clone() for k, b in h.named_buffers() if b is not None}
        return outs, aux, [f.grad.detach().clone() for f in feats], grads, bufs
    finally:
        core.FUSED_TRAIN = old


def _cmp_grads(g1, g0):
    """Parameter gradients of the fused step against the torch path (the
    tolerances of the module docstring)."""
    assert set(g1) == set(g0)
    gmax = {}
    for k in g0:
        mod = k.rsplit(".", 2)[0]
        gmax[mod] = max(gmax.get(mod, 0.0), float(g0[k].abs().max()))
    bad = []
    for k in g0:
        mod = k.rsplit(".", 2)[0]
        err = float((g1[k].double() - g0[k].double()).abs().max())
        if k.startswith("bit_mapper.") and k.endswith(("0.bias", "3.bias", "6.bias", "0.weight", "3.weight",
                                                       "6.weight")):
            # a Linear feeding a train-mode BatchNorm: its bias gradient is zero
            # in exact arithmetic and its weight gradient sum_t g_a(t) z(t)^T
            # cancels to ~1e-2 of its terms (sum_t g_a(t) = 0), so both carry
            # the summation noise of the BN backward (~1e-5 of the module's
            # largest gradient in either implementation): absolute floor
            scale, tol = max(gmax[mod], 1e-30), 1e-4
        else:
            scale, tol = max(float(g0[k].abs().max()), 1e-3 * gmax[mod]), 1e-3
        print("%-60s err %.3g scale %.3g rel %.3g" % (k, err, scale, err / scale))
        if err > tol * scale:
            bad.append(k)
    assert not bad, bad


@pytest.mark.parametrize("temperature", [1.0, 2.5])
def test_fused_train_step_matches_torch_path(temperature):
    _check_step_vs_torch(temperature)


def test_fused_train_step_config5_bs16_matches_torch_path():
    """The whole QAT hook step at BASELINE config 5's per-GPU batch (yolov8n
    bs16, 640x640: C3 64x80x80, C4 128x40x40, C5 256x20x20) - the multi-scale
    launches with the fused soft-mask / quantizer / bit-budget node, as
    bench.py --config 5 runs it - against the reference's per-scale torch
    path, at the tolerances of the B = 4 test."""
    _check_step_vs_torch(1.0, B=16)


def _check_step_vs_torch(temperature, B=4):
    o1, a1, gx1, g1, b1 = _step(True, B=B, temperature=temperature)
    o0, a0, gx0, g0, b0 = _step(False, B=B, temperature=temperature)
    for a, b in zip(a1, a0):
        assert torch.equal(a["complexity"], b["complexity"]), "analyzer forward (morph kernel) differs"
        _rel(a["bit_map"], b["bit_map"], 1e-5)
    for a, b in zip(o1, o0):
        _rel(a, b, 1e-4)
    for a, b in zip(gx1, gx0):
        _rel(a, b, 1e-4)
    _cmp_grads(g1, g0)
    for k in b0:
        if b0[k].dtype.is_floating_point:
            _rel(b1[k], b0[k], 1e-5, floor=1e-6)
        else:
            assert torch.equal(b1[k], b0[k]), k


def test_fused_mapper_vs_reference_fixture():
    """The fused train-mode mapper against the reference's own train-mode
    outputs (tests/golden/train_mapper.npz): bits, grads, running stats."""
    from mcaq_yolo_amd import core
    assert core.FUSED_TRAIN
    d = np.load(os.path.join(GOLDEN, "train_mapper.npz"))
    W = load_weights()
    for temp in (1, 3):
        t = "t%d" % temp
        m = core.ComplexityToBitMappingNetwork().to(DEV)
        m.load_state_dict({k[len("bit_mapper."):]: torch.from_numpy(np.asarray(v))
                           for k, v in W.items() if k.startswith("bit_mapper.")})
        m.train()
        c = torch.from_numpy(d[t + ".c"]).to(DEV).requires_grad_(True)
        bits = m(c, float(temp), return_continuous=True)
        assert bits.grad_fn is not None and "MapperTrain" in type(bits.grad_fn).__name__
        _rel(bits, torch.from_numpy(d[t + ".bits"]), 1e-5)
        bits.backward(torch.from_numpy(d[t + ".gb"]).to(DEV))
        _rel(c.grad, torch.from_numpy(d[t + ".grad_c"]), 1e-4)
        for n, b in m.mapping_network.named_buffers():
            if b.dtype.is_floating_point:
                _rel(b, torch.from_numpy(d[t + ".buf.mapping_network." + n]), 1e-5)
            else:   # num_batches_tracked: the loaded count + one train-mode forward
                assert int(b) == int(np.asarray(W["bit_mapper.mapping_network." + n])) + 1, n


def test_fused_softmask_backward_vs_autograd():
    """LearnedSoftMask backward: the fused kernel vs torch autograd of the
    tile-sized restatement (quantization.py:213-239), ragged grids included."""
    from mcaq_yolo_amd import core
    W = load_weights()
    gen = torch.Generator(device="cpu").manual_seed(9)
    for (B, H, Wd, ht, wt) in ((2, 80, 80, 10, 10), (3, 20, 20, 5, 5), (2, 44, 52, 11, 13), (1, 40, 40, 10, 10)):
        sm = core.LearnedSoftMask().to(DEV)
        sm.load_state_dict({k[len("soft_mask."):]: torch.from_numpy(np.asarray(v))
                            for k, v in W.items() if k.startswith("soft_mask.")})
        bits = (torch.rand(B, ht, wt, generator=gen) * 7 + 1.5).to(DEV)
        absmean = torch.rand(B, H, Wd, generator=gen).to(DEV)
        gm = torch.randn(B, 1, H, Wd, generator=gen).to(DEV)
        b1 = bits.clone().requires_grad_(True)
        m1 = core._SoftMaskFn.apply(b1, absmean, sm, *sm.net.parameters())
        m1.backward(gm)
        g_fused = [p.grad.clone() for p in sm.net.parameters()]
        for p in sm.net.parameters():
            p.grad = None
        b0 = bits.clone().requires_grad_(True)
        m0 = sm._torch_forward(b0, absmean)
        m0.backward(gm)
        _rel(m1, m0, 1e-5)
        _rel(b1.grad, b0.grad, 1e-4)
        for a, p in zip(g_fused, sm.net.parameters()):
            _rel(a, p.grad, 1e-4)


def test_device_pack_equals_torch_pack():
    """mcaq_pack (one launch) builds the complexity-MLP and soft-mask blobs
    bit-identically to the torch packing (cat / zeros / MFMA operand index)
    that the CPU modules use."""
    import copy
    from mcaq_yolo_amd import core
    torch.manual_seed(3)
    an = core.MorphologicalComplexityAnalyzer(device="cpu")
    sm = core.LearnedSoftMask()
    for p in list(an.parameters()) + list(sm.parameters()):
        with torch.no_grad():
            p.add_(0.01 * torch.randn_like(p))
    ref_c = core._pack_cmlp(an.complexity_mlp)
    ref_s = core._pack_softmask(sm.net)
    gpu_c = core._pack_cmlp(copy.deepcopy(an.complexity_mlp).to(DEV))
    gpu_s = core._pack_softmask(copy.deepcopy(sm.net).to(DEV))
    assert gpu_c.is_cuda and gpu_c.shape == ref_c.shape
    assert torch.equal(gpu_c.cpu(), ref_c)
    assert torch.equal(gpu_s.cpu(), ref_s)
    # the mapper (20 tensors + 3 MFMA operand segments) also takes the one-launch
    # device path (MCAQ_PACK_MAXSEG was 16 < 23, so it never did)
    mp = core.ComplexityToBitMappingNetwork()
    for p in mp.parameters():
        with torch.no_grad():
            p.add_(0.01 * torch.randn_like(p))
    ref_m = core._pack_mapper(mp.mapping_network)
    calls = []
    orig = core._device_pack

    def spy(*a, **k):
        r = orig(*a, **k)
        calls.append(r is not None)
        return r
    core._device_pack = spy
    try:
        gpu_m = core._pack_mapper(copy.deepcopy(mp.mapping_network).to(DEV))
    finally:
        core._device_pack = orig
    assert calls == [True], "mapper blob did not take the device pack"
    assert torch.equal(gpu_m.cpu(), ref_m)


def test_direct_grad_accumulation_matches_autograd_return():
    """core.DIRECT_GRAD_ACCUM: the shared modules' gradients of the three
    scales accumulated by the fused kernels into .grad equal the ones
    returned to autograd (and summed by it)."""
    from mcaq_yolo_amd import core
    res = {}
    for direct in (True, False):
        old = core.DIRECT_GRAD_ACCUM
        core.DIRECT_GRAD_ACCUM = direct
        try:
            o, a, gx, g, b = _step(True, B=2, seed=11)
            res[direct] = g
        finally:
            core.DIRECT_GRAD_ACCUM = old
    assert set(res[True]) == set(res[False])
    for k in res[False]:
        _rel(res[True][k], res[False][k], 1e-5, floor=1e-12)


def test_mapper_one_launch_equals_staged_launches():
    """The train-mode mapper as ONE launch per direction (grid barriers
    between the batch-statistics stages) gives the values of the per-stage
    launches: bits, c gradient, parameter gradients and running stats."""
    from mcaq_yolo_amd import core
    W = load_weights()
    g = torch.Generator().manual_seed(21)
    res = {}
    for one in (True, False):
        old = core.MAPPER_ONE_LAUNCH
        core.MAPPER_ONE_LAUNCH = one
        try:
            m = core.ComplexityToBitMappingNetwork().to(DEV)
            m.load_state_dict({k[len("bit_mapper."):]: torch.from_numpy(np.asarray(v))
                               for k, v in W.items() if k.startswith("bit_mapper.")})
            m.train()
            torch.manual_seed(21)
            c = torch.rand(5, 37, 41).to(DEV).requires_grad_(True)     # 7585 tiles: 119 workgroups
            bits = m(c, 2.0, return_continuous=True)
            bits.backward(torch.randn(bits.shape, generator=g.manual_seed(22)).to(DEV))
            torch.cuda.synchronize()
            res[one] = ([bits.detach().clone(), c.grad.clone()] + [p.grad.clone() for p in m.parameters()] +
                        [b.clone() for b in m.buffers()])
        finally:
            core.MAPPER_ONE_LAUNCH = old
    for a, b in zip(res[True], res[False]):
        assert torch.equal(a, b)


def test_pass1_sharing_equals_separate_passes():
    """core.PASS1_SHARE: the quantizer taking the analyzer's |x| means and
    min/max partials of the same read gives exactly the step of separate
    pass-1 launches (outputs, feature gradients, parameter gradients, EMA
    statistics)."""
    from mcaq_yolo_amd import core
    res = {}
    for share in (True, False):
        old = core.PASS1_SHARE
        core.PASS1_SHARE = share
        try:
            res[share] = _step(True, B=2, seed=13)
        finally:
            core.PASS1_SHARE = old
    (o1, a1, gx1, g1, b1), (o0, a0, gx0, g0, b0) = res[True], res[False]
    for x, y in zip(o1 + gx1, o0 + gx0):
        assert torch.equal(x, y)
    for k in g0:
        assert torch.equal(g1[k], g0[k]), k
    for k in b0:
        assert torch.equal(b1[k], b0[k]), k


def test_fused_train_large_map_takes_torch_backward():
    """the fused soft-mask backward stages one image's m(p)
    gradient in LDS and cannot take a 208x208 map (173 KiB); the call takes
    the torch recompute instead of raising, and the step still equals the
    all-torch path.  Host checks of both LDS bounds."""
    from mcaq_yolo_amd import core
    assert not core._smask_bwd_fits(208, 208, 13, 13) and core._smask_bwd_fits(80, 80, 10, 10)
    assert core._head_bwd_fits(10, 10) and not core._head_bwd_fits(32, 32)
    shapes = ((8, 208), (8, 104), (8, 52))
    o1, a1, gx1, g1, b1 = _step(True, B=1, shapes=shapes)
    o0, a0, gx0, g0, b0 = _step(False, B=1, shapes=shapes)
    for x, y in zip(o1, o0):
        _rel(x, y, 1e-5)
    for x, y in zip(gx1, gx0):
        _rel(x, y, 1e-3, floor=1e-12)
    _cmp_grads(g1, g0)
