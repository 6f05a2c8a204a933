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
