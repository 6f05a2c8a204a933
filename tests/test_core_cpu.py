"""The drop-in module layer without a GPU: reference constructor / state_dict
compatibility, and loud failure on CPU tensors (no CPU fallback)."""
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
        core.MorphologicalComplexityAnalyzer(device="cpu", canny_impl="legacy")
    with pytest.raises(NotImplementedError):
        core.SpatialAdaptiveQuantization(calibration_mode="entropy")


def test_cpu_tensors_raise_no_fallback():
    a = core.MorphologicalComplexityAnalyzer(device="cpu").eval()
    with pytest.raises(RuntimeError, match="HIP"):
        a(torch.rand(1, 3, 40, 40))
    m = core.LinearBitMapper()
    with pytest.raises(RuntimeError, match="HIP"):
        m(torch.rand(1, 4, 4))
    q = core.SpatialAdaptiveQuantization().eval()
    with pytest.raises(RuntimeError, match="HIP"):
        q(torch.rand(1, 4, 16, 16), torch.full((1, 4, 4), 4.0))
    with pytest.raises(RuntimeError):
        mcaq_cuda_ops.spatial_quantize(torch.rand(1, 4, 16, 16), torch.full((1, 4, 4), 4.0),
                                       torch.zeros(4), torch.ones(4), 4, 4)


def test_training_paths_have_no_cpu_fallback():
    """The QAT (train-mode) paths run on the GPU only: CPU tensors raise."""
    m = core.ComplexityToBitMappingNetwork()
    m.train()
    with pytest.raises(RuntimeError, match="HIP"):
        m(torch.rand(1, 4, 4))
    q = core.SpatialAdaptiveQuantization()
    with pytest.raises(RuntimeError, match="HIP"):
        q(torch.rand(1, 4, 16, 16), torch.full((1, 4, 4), 4.0), training=True)


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
