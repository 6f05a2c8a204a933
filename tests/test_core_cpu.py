"""The drop-in module layer without a GPU: reference constructor / state_dict
compatibility, CPU dispatch to the pure-PyTorch path, loud failure of the
kernel entry points on non-CUDA tensors."""
import numpy as np
import pytest
import torch

from conftest import load_weights
from mcaq_yolo_amd import core, mcaq_cuda_ops
from mcaq_yolo_amd.hooks import MCAQHooks


def _sd(prefix):
    W = load_weights()
    return {k[len(prefix):]: torch.from_numpy(np.asarray(v)) for k, v in W.items() if k.startswith(prefix)}


def test_state_dict_keys_match_reference():
    """Keys (and shapes) of the reference modules, as stored in the fixture
    weights generated from the reference itself (tests/golden/make_golden.py)."""
    a = core.MorphologicalComplexityAnalyzer(device="cpu")
    a.load_state_dict(_sd("complexity_analyzer."), strict=True)
    m = core.ComplexityToBitMappingNetwork()
    m.load_state_dict(_sd("bit_mapper."), strict=True)
    sm = core.LearnedSoftMask()
    sm.load_state_dict(_sd("soft_mask."), strict=True)
    ref_kernel = torch.from_numpy(np.asarray(load_weights()["soft_mask.smooth_kernel"]))
    assert torch.equal(sm.smooth_kernel, ref_kernel)


def test_quantizer_lazy_running_stats_load():
    """quantization.py:297-312: checkpointed running_min/max materialise on load."""
    q = core.SpatialAdaptiveQuantization()
    sd = q.state_dict()
    assert "running_min" not in sd
    sd["running_min"] = torch.zeros(1, 4, 1, 1)
    sd["running_max"] = torch.ones(1, 4, 1, 1)
    sd["stats_frozen"] = torch.tensor(True)
    q.load_state_dict(sd)
    assert q.running_min.shape == (1, 4, 1, 1) and bool(q.stats_frozen)


def test_hooks_state_dict_prefixes():
    h = MCAQHooks(device="cpu")
    keys = set(h.state_dict())
    W = load_weights()
    for k in W:
        if k.startswith("complexity_analyzer.") or k.startswith("bit_mapper."):
            assert k in keys, k
        if k.startswith("soft_mask."):
            for idx in (4, 6, 9):
                assert "quantizers.%d.%s" % (idx, k) in keys


def test_reference_options_rejected_loudly():
    with pytest.raises(NotImplementedError):
        core.MorphologicalComplexityAnalyzer(device="cpu", metric_backend="cv2")
    with pytest.raises(NotImplementedError):
        core.SpatialAdaptiveQuantization(calibration_mode="entropy")


def test_cpu_tensors_take_the_torch_path():
    """CPU tensors run the package's pure-PyTorch path (quantization.py:631-634
    dispatch); the native-op mirror keeps the extension's contract and raises."""
    a = core.MorphologicalComplexityAnalyzer(device="cpu").eval()
    c = a(torch.rand(1, 3, 40, 40))
    assert c.shape == (1, 10, 10)
    m = core.LinearBitMapper()
    assert m(torch.rand(1, 4, 4)).shape == (1, 4, 4)
    q = core.SpatialAdaptiveQuantization().eval()
    assert q(torch.rand(1, 4, 16, 16), torch.full((1, 4, 4), 4.0)).shape == (1, 4, 16, 16)
    with pytest.raises(RuntimeError):
        mcaq_cuda_ops.spatial_quantize(torch.rand(1, 4, 16, 16), torch.full((1, 4, 4), 4.0),
                                       torch.zeros(4), torch.ones(4), 4, 4)


def test_gpu_paths_fail_loudly_without_hip():
    """No silent CPU fallback for CUDA work: the kernel entry points demand
    CUDA tensors (and the library, abi.lib())."""
    with pytest.raises(RuntimeError, match="HIP"):
        core._run_mapper(torch.rand(1, 4, 4), 0, 2, 8, 1.0, False)
    with pytest.raises(RuntimeError, match="HIP"):
        core._need_cuda(torch.rand(1), "x")


def test_enforce_weight_constraints():
    m = core.ComplexityToBitMappingNetwork()
    with torch.no_grad():
        m.mapping_network[0].weight.neg_()
        m.mapping_network[1].weight.fill_(-1.0)
    m.enforce_weight_constraints()
    assert bool((m.mapping_network[0].weight >= 0).all()) and bool((m.mapping_network[1].weight == 1).all())


def test_mfma_operand_packing_matches_host_packer():
    from mcaq_yolo_amd import params
    W = load_weights()
    a = core.MorphologicalComplexityAnalyzer(device="cpu")
    a.load_state_dict(_sd("complexity_analyzer."))
    m = core.ComplexityToBitMappingNetwork()
    m.load_state_dict(_sd("bit_mapper."))
    sm = core.LearnedSoftMask()
    sm.load_state_dict(_sd("soft_mask."))
    assert np.array_equal(a.cmlp_blob().numpy(), params.pack_complexity_mlp(params.sub(W, "complexity_analyzer.")))
    assert np.array_equal(m.mapper_blob().numpy(), params.pack_mapper_mlp(params.sub(W, "bit_mapper.")))
    assert np.array_equal(sm.blob().numpy(), params.pack_soft_mask(params.sub(W, "soft_mask.")))


def test_plan_descriptor_signature():
    """HookPlan._signature (descriptor reuse of eager hook calls): the
    rebound outputs y / complexity / bits and x do not enter it; any other
    buffer, blob, frozen min/max or option does, and a frozen min/max that
    prepare() would copy disables reuse."""
    from mcaq_yolo_amd.engine import HookPlan
    p = HookPlan.__new__(HookPlan)
    p.bufs = [{"y": torch.empty(8), "bits": torch.empty(2), "complexity": torch.empty(2),
               "gray": torch.empty(4), "units": 3, "m": None}]
    cm, mm, sm = torch.empty(5), torch.empty(6), torch.empty(7)
    lo, hi = torch.empty(4), torch.empty(4)
    opts = (1.0, "mlp", False)
    s0 = p._signature(cm, mm, [sm], None, opts)
    keep = [p.bufs[0]["y"], p.bufs[0]["bits"]]
    p.bufs[0]["y"], p.bufs[0]["bits"] = torch.empty(8), torch.empty(2)
    assert p._signature(cm, mm, [sm], None, opts) == s0
    assert p._signature(cm, mm, [sm], None, (0.5, "mlp", False)) != s0
    assert p._signature(cm, mm, [None], None, opts) != s0
    assert p._signature(cm, mm, [sm], [(lo, hi)], opts) != s0
    assert p._signature(cm, mm, [sm], [(lo, hi)], opts) == p._signature(cm, mm, [sm], [(lo, hi)], opts)
    assert p._signature(cm, mm, [sm], [(lo.double(), hi)], opts) is None
    keep.append(p.bufs[0]["gray"])
    p.bufs[0]["gray"] = torch.empty(4)
    assert p._signature(cm, mm, [sm], None, opts) != s0


def test_plan_descriptor_reuse_equals_rebuild(monkeypatch):
    """HookPlan.prepare's reuse path (same blobs / buffers / options, new x
    and new y / complexity / bits) leaves every descriptor field equal to a
    full rebuild's.  Host-side only: plan buffers are CPU tensors, nothing
    is launched."""
    from mcaq_yolo_amd import engine
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    monkeypatch.setattr(engine, "_require_cuda", lambda *ts: None)
    shapes = ((2, 16, 80, 80), (2, 32, 40, 40), (2, 64, 20, 20))
    p = HookPlan.__new__(HookPlan)
    p.geoms = [ScaleGeom(*s, 8) for s in shapes]
    p.scale_geoms, p.batches, p.seg = list(p.geoms), 1, [(i, 0) for i in range(len(shapes))]
    p.device = torch.device("cpu")
    p.lib = None
    p.bufs = []
    for g in p.geoms:
        b = {"units": 7}
        for k in ("gray", "absmean", "pmin", "pmax", "xmin", "xmax", "complexity", "bits", "mt", "y", "phi",
                  "tile_tmp", "cmlp"):
            b[k] = torch.empty(4)
        b["m"] = b["edge"] = b["binmask"] = b["gscratch"] = b["pwork"] = None
        p.bufs.append(b)
    cm, mm, sms = torch.empty(8), torch.empty(8), [torch.empty(8) for _ in shapes]

    def snap():
        out = {}
        for name in ("_st", "_fz", "_mo", "_qs"):
            arr = getattr(p, name)
            for i in range(len(arr)):
                for f, _ in arr[i]._fields_:
                    v = getattr(arr[i], f)
                    out[(name, i, f)] = list(v) if hasattr(v, "__len__") else v
        return out

    def fresh_io():
        feats = [torch.empty(s) for s in shapes]
        for b in p.bufs:
            for k in HookPlan._REBOUND:
                b[k] = torch.empty(4)
        return feats

    keep = []
    for kw in ({}, {"temperature": 0.5, "per_tensor": True}, {"minmax": [(torch.empty(16), torch.empty(16)), None, None]},
               {"shared_stats": True}):
        feats = fresh_io()
        keep.append((feats, [dict(b) for b in p.bufs]))
        p.prepare(feats, cm, mm, sms, **kw)
        st0 = id(p._st)
        feats = fresh_io()
        keep.append((feats, [dict(b) for b in p.bufs]))
        p.prepare(feats, cm, mm, sms, **kw)
        assert id(p._st) == st0                      # reused
        reused = snap()
        p._sig = None
        p.prepare(feats, cm, mm, sms, **kw)          # rebuilt from scratch
        assert id(p._st) != st0
        assert snap() == reused
