"""The multi-scale QAT step (train_step.py: every stage once for all hook
scales, per-scale segments in one launch) against the per-scale modules on one
stream (hooks.MULTI_SCALE_TRAIN / CONCURRENT_TRAIN_SCALES off).  The segments
run the per-scale kernels' bodies on the same data, the mapper's running
statistics are updated in scale order and the shared parameter gradients are
summed in autograd's per-scale order, so every value is bit-identical:
outputs, complexity / bit maps, feature and parameter gradients, parameters
after SGD steps, every buffer - eager and captured in a HIP graph."""
import pytest
import torch

from test_concurrent_scales_gpu import _close, _feats, _run, _same
from test_train_fused_gpu import _hooks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mapper", ["mlp", "linear"])
def test_multi_scale_step_equals_per_scale_eager(mapper):
    _same(_run(False, mapper=mapper, multi=True), _run(False, mapper=mapper))


@pytest.mark.parametrize("variant", ["normalize", "per_tensor", "no_mask"])
def test_multi_scale_step_equals_per_scale_variants(variant):
    """The module options the multi-segment step keeps per-scale pieces for:
    normalize_complexity (torch quantile ops between analyzer and mapper),
    per-tensor quantizers (their EMA per quantizer), a quantizer without the
    soft mask (its QAT segment without m)."""
    _same(_run(False, multi=True, variant=variant), _run(False, variant=variant))


def test_multi_scale_step_equals_per_scale_graph():
    _same(_run(False, steps=3, graph=True, multi=True), _run(False, steps=4))


def test_multi_scale_step_launches_once_per_stage():
    """One train-mode mapper forward / backward call for all three scales,
    and none of the per-scale Functions."""
    from mcaq_yolo_amd import core, hooks, train_step
    assert hooks.MULTI_SCALE_TRAIN
    h = _hooks()
    feats, gens = _feats()
    calls = {"multi": 0, "per_scale": 0}
    om, op = train_step._MapperMulti.forward, core._MapperTrainFn.forward

    def spy_m(ctx, *a):
        calls["multi"] += 1
        return om(ctx, *a)

    def spy_p(ctx, *a):
        calls["per_scale"] += 1
        return op(ctx, *a)
    train_step._MapperMulti.forward = staticmethod(spy_m)
    core._MapperTrainFn.forward = staticmethod(spy_p)
    try:
        outs, aux = h.forward_features(feats)
        sum((o * g).sum() for o, g in zip(outs, gens)).backward()
        torch.cuda.synchronize()
    finally:
        train_step._MapperMulti.forward = staticmethod(om)
        core._MapperTrainFn.forward = staticmethod(op)
    assert calls == {"multi": 1, "per_scale": 0}
    assert len(aux) == 3 and all(f.grad is not None for f in feats)


def test_multi_scale_step_quantize_off_and_frozen():
    """quantize=False (aux only, inputs returned) and frozen quantizer
    statistics take the same values on both paths."""
    from mcaq_yolo_amd import hooks
    feats, _ = _feats()
    res = []
    for multi in (True, False):
        old = hooks.MULTI_SCALE_TRAIN, hooks.CONCURRENT_TRAIN_SCALES
        hooks.MULTI_SCALE_TRAIN, hooks.CONCURRENT_TRAIN_SCALES = multi, False
        try:
            h = _hooks()
            outs, aux = h.forward_features(feats, quantize=False)
            assert all(o is f for o, f in zip(outs, feats))
            h.forward_features(feats)                  # running stats exist
            for q in h.quantizers.values():
                q.freeze_calibration()
            outs2, aux2 = h.forward_features(feats)
            torch.cuda.synchronize()
            res.append([a["bit_map"].detach().clone() for a in aux] + [o.detach().clone() for o in outs2])
        finally:
            hooks.MULTI_SCALE_TRAIN, hooks.CONCURRENT_TRAIN_SCALES = old
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_frozen_mapper_in_training_hooks_takes_per_scale_path():
    """hooks.train() with the bit mapper frozen by .eval(): the
    multi-scale step must not run the train-mode mapper.  forward_features
    then takes the per-scale modules, which follow the mapper's own flag
    (running-statistics BatchNorm, no running-stat update): the bit maps and
    outputs equal the per-scale path's and running_mean / running_var /
    num_batches_tracked stay untouched."""
    from mcaq_yolo_amd import hooks, train_step
    feats, gens = _feats()
    res = []
    for multi in (True, False):
        old = hooks.MULTI_SCALE_TRAIN, hooks.CONCURRENT_TRAIN_SCALES
        hooks.MULTI_SCALE_TRAIN, hooks.CONCURRENT_TRAIN_SCALES = multi, False
        try:
            h = _hooks()
            h.bit_mapper.eval()
            assert not train_step.multi_ok(h, feats)
            before = {k: v.clone() for k, v in h.bit_mapper.state_dict().items() if "running" in k or "num_batches" in k}
            outs, aux = h.forward_features(feats, temperature=1.0)
            sum((o * g).sum() for o, g in zip(outs, gens)).backward()
            torch.cuda.synchronize()
            after = h.bit_mapper.state_dict()
            for k, v in before.items():
                assert torch.equal(after[k], v), "%s changed with the mapper in eval mode" % k
            res.append([a["bit_map"].detach().clone() for a in aux] + [o.detach().clone() for o in outs] +
                       [f.grad.clone() for f in feats])
            for f in feats:
                f.grad = None
        finally:
            hooks.MULTI_SCALE_TRAIN, hooks.CONCURRENT_TRAIN_SCALES = old
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("budget", [False, True])
def test_fused_mask_quant_budget_step_close_to_per_scale(budget):
    """train_step.FUSED_MASK_QAT (the default): soft masks, quantizers and
    the bit budget of every scale as one autograd node whose backward folds
    the quantizer, the soft mask and the bit-budget gradient into one launch.
    The first forward is bit-identical to the per-scale step; the bit-map
    gradient sums its contributions in another association, so gradients and
    later steps agree within fp32 rounding.  budget: the loss's bit-budget
    term through MCAQHooks.bit_budget_loss (the fused value and gradient on
    the multi path, torch ops on the per-scale path)."""
    a = _run(False, steps=1, multi=True, fused_mq=True, budget=budget)
    b = _run(False, steps=1, budget=budget)
    for k in ("outs", "bits", "cplx"):
        for x, y in zip(a[k], b[k]):
            assert torch.equal(x, y), k
    _close(a, b)
    # (one step only: the biases of the Linear layers that feed train-mode
    # BatchNorm have a mathematically zero gradient, so theirs is rounding
    # noise in either association - 20-40 % apart here - and SGD steps on it
    # move the two runs apart along directions the loss does not see
    # (tools/diag/fused_mq_drift.py); the fused step's determinism is
    # test_fused_mask_quant_budget_graph's exact graph-vs-eager check)


def test_fused_mask_quant_budget_graph():
    """The fused step captured in a HIP graph == the same step eager, bit
    for bit (warm-up step + 3 replays vs 4 eager steps)."""
    _same(_run(False, steps=3, graph=True, multi=True, fused_mq=True, budget=True),
          _run(False, steps=4, multi=True, fused_mq=True, budget=True))


def test_bit_budget_values():
    """avg_bits / bit_budget_loss of the fused step against the torch
    expressions on the same bit maps (fp32 reduction order apart)."""
    from mcaq_yolo_amd import hooks, train_step
    from test_train_fused_gpu import _hooks
    assert train_step.FUSED_MASK_QAT and hooks.MULTI_SCALE_TRAIN
    h = _hooks()
    feats, _ = _feats()
    outs, aux = h.forward_features(feats)
    avg = h.avg_bits(aux)
    ref = torch.stack([a["bit_map"].float().mean() for a in aux]).mean()
    assert aux[0]["_bit_budget"]["avg_bits"] is avg
    assert abs(float(avg) - float(ref)) <= 2e-6 * abs(float(ref))
    lb = h.bit_budget_loss(aux, 4.0)
    assert abs(float(lb) - (float(ref) - 4.0) ** 2) <= 1e-5 * max((float(ref) - 4.0) ** 2, 1e-6)
    lb5 = h.bit_budget_loss(aux, 5.0)          # another target: torch ops on the fused avg
    assert abs(float(lb5) - (float(avg) - 5.0) ** 2) <= 1e-6


@pytest.mark.parametrize("mode", ["ride", "flush", "one_frozen"])
def test_fused_soft_mask_grad_sinks(mode):
    """The soft masks' parameter gradients go straight into per-net gradient
    sinks, reduced as extra workgroups of the mapper's first backward launch
    ("ride"; "flush": analyzer and mapper frozen, so no mapper backward runs
    and the engine callback at the end of backward launches the reduction;
    "one_frozen": one soft mask frozen, so no net takes the sink path and
    none of their .grad may be touched).  Against the same step with the
    gradients returned through autograd (core.DIRECT_GRAD_ACCUM off), bit for
    bit, over two backwards without zero_grad (the sinks' accumulate path)."""
    frozen_head = mode == "flush"
    from mcaq_yolo_amd import core, train_step
    assert train_step.FUSED_MASK_QAT
    feats, gens = _feats()
    res = []
    old = core.DIRECT_GRAD_ACCUM
    for direct in (True, False):
        core.DIRECT_GRAD_ACCUM = direct
        try:
            h = _hooks()
            if frozen_head:
                for p in list(h.complexity_analyzer.parameters()) + list(h.bit_mapper.parameters()):
                    p.requires_grad_(False)
            if mode == "one_frozen":
                for p in h.quantizers["6"].soft_mask.parameters():
                    p.requires_grad_(False)
            for _ in range(2):
                for f in feats:
                    f.grad = None
                outs, aux = h.forward_features(feats, temperature=1.0)
                loss = sum((o * g).sum() for o, g in zip(outs, gens)) + 0.1 * h.bit_budget_loss(aux, 4.0)
                loss.backward()
            torch.cuda.synchronize()
            sm = {n: p.grad.clone() for n, p in h.named_parameters() if "soft_mask" in n and p.requires_grad}
            assert len(sm) == (8 if mode == "one_frozen" else 12) and all(g is not None for g in sm.values())
            res.append((sm, [f.grad.clone() for f in feats]))
        finally:
            core.DIRECT_GRAD_ACCUM = old
    (a, fa), (b, fb) = res
    for n in a:
        assert torch.equal(a[n], b[n]), n
    for x, y in zip(fa, fb):
        assert torch.equal(x, y)
