"""Train-mode hook scales on concurrent streams (hooks.CONCURRENT_TRAIN_SCALES,
core.concurrent_scales) against the same step with the scales one after
another on one stream.  The shared state is ordered explicitly (deferred
mapper running-stat updates in scale order, event-chained gradient
reductions in autograd's order), so every value must be bit-identical:
outputs, complexity / bit maps, feature and parameter gradients, every
buffer (BatchNorm running stats, num_batches_tracked, EMA min/max) - eager
and captured in a HIP graph, over several steps."""
import pytest
import torch

from test_train_fused_gpu import _hooks

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _feats(B=4, seed=5, shapes=((64, 80), (128, 40), (256, 20))):
    gen = torch.Generator(device="cpu").manual_seed(seed)
    feats = []
    for c, s in shapes:
        lo = torch.randn(B, c, s // 8, s // 8, generator=gen)
        hi = torch.randn(B, c, s, s, generator=gen)
        up = torch.nn.functional.interpolate(lo, size=(s, s), mode="bilinear", align_corners=False)
        feats.append(torch.nn.functional.silu(1.5 * hi + 2 * up).to(DEV).requires_grad_(True))
    gens = [(torch.randn(f.shape, generator=gen) * 1e-3).to(DEV) for f in feats]
    return feats, gens


def _run(concurrent, steps=3, graph=False, mapper="mlp", multi=False, variant=None, fused_mq=False, budget=False):
    """concurrent / multi select the train path (hooks.CONCURRENT_TRAIN_SCALES,
    hooks.MULTI_SCALE_TRAIN); both False: per-scale modules on one stream.
    variant: None, "normalize" (normalize_complexity), "per_tensor" (every
    quantizer per_channel=False) or "no_mask" (the C4 quantizer without
    smooth transitions).  fused_mq: train_step.FUSED_MASK_QAT (the soft
    masks, quantizers and bit budget as one node); budget: the bit-budget
    term through MCAQHooks.bit_budget_loss instead of torch ops on the aux
    bit maps."""
    from mcaq_yolo_amd import hooks, train_step
    old = hooks.CONCURRENT_TRAIN_SCALES, hooks.MULTI_SCALE_TRAIN, train_step.FUSED_MASK_QAT
    hooks.CONCURRENT_TRAIN_SCALES, hooks.MULTI_SCALE_TRAIN = concurrent, multi
    train_step.FUSED_MASK_QAT = fused_mq
    try:
        h = _hooks(mapper)
        if variant == "normalize":
            h.normalize_complexity = True
        elif variant == "per_tensor":
            for q in h.quantizers.values():
                q.per_channel = False
        elif variant == "no_mask":
            h.quantizers["6"].smooth_transitions = False
        feats, gens = _feats()
        params = [p for p in h.parameters() if p.requires_grad]
        opt = torch.optim.SGD(params, lr=1e-2, momentum=0.9)
        rec = {}

        def step():
            opt.zero_grad(set_to_none=True)
            for f in feats:
                f.grad = None
            outs, aux = h.forward_features(feats, temperature=1.0)
            if budget:
                lb = h.bit_budget_loss(aux, 4.0)
            else:
                lb = (torch.stack([a["bit_map"].float().mean() for a in aux]).mean() - 4.0) ** 2
            loss = sum((o * g).sum() for o, g in zip(outs, gens)) + 0.1 * lb
            loss.backward()
            rec["outs"] = [o.detach() for o in outs]
            rec["bits"] = [a["bit_map"].detach() for a in aux]
            rec["cplx"] = [a["complexity"].detach() for a in aux]
            opt.step()
            if hasattr(h.bit_mapper, "enforce_weight_constraints"):
                h.bit_mapper.enforce_weight_constraints()

        if graph:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                step()                         # warm-up: lazy buffers, grad sinks
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            opt.zero_grad(set_to_none=True)
            with torch.cuda.graph(g):
                step()
            for _ in range(steps):
                g.replay()
        else:
            for _ in range(steps):
                step()
        torch.cuda.synchronize()
        snap = {k: [t.clone() for t in v] for k, v in rec.items()}
        snap["fgrad"] = [f.grad.detach().clone() for f in feats]
        snap["grads"] = {k: p.grad.detach().clone() for k, p in h.named_parameters() if p.grad is not None}
        snap["params"] = {k: p.detach().clone() for k, p in h.named_parameters()}
        snap["bufs"] = {k: b.detach().clone() for k, b in h.named_buffers() if b is not None}
        return snap
    finally:
        hooks.CONCURRENT_TRAIN_SCALES, hooks.MULTI_SCALE_TRAIN, train_step.FUSED_MASK_QAT = old


def _close(a, b, rtol=1e-5):
    """Within fp32 rounding of the tensor's scale: the fused node sums the
    bit-map gradient contributions (and the bit budget) in another order."""
    for k in ("outs", "bits", "cplx", "fgrad"):
        for i, (x, y) in enumerate(zip(a[k], b[k])):
            err = float((x - y).abs().max())
            assert err <= rtol * max(float(y.abs().max()), 1e-30), "%s[%d]: %g" % (k, i, err)
    # gradients: relative to the module's largest gradient (the Linear layers
    # feeding a train-mode BatchNorm carry cancelling sums: test_dist_qat_gpu)
    gmax = {}
    for n, y in b["grads"].items():
        mod = ".".join(n.split(".")[:2])
        gmax[mod] = max(gmax.get(mod, 0.0), float(y.abs().max()))
    for k in ("grads", "params", "bufs"):
        assert set(a[k]) == set(b[k]), k
        for n in a[k]:
            x, y = a[k][n].float(), b[k][n].float()
            err = float((x - y).abs().max()) if x.numel() else 0.0
            scale = max(float(y.abs().max()) if y.numel() else 0.0, 1e-30)
            if k == "grads":
                scale, tol = max(gmax[".".join(n.split(".")[:2])], 1e-30), 1e-4
            else:
                tol = rtol
            assert err <= tol * scale, "%s %s: %g vs %g" % (k, n, err, scale)


def _same(a, b):
    for k in ("outs", "bits", "cplx", "fgrad"):
        for i, (x, y) in enumerate(zip(a[k], b[k])):
            assert torch.equal(x, y), "%s[%d] differs" % (k, i)
    for k in ("grads", "params", "bufs"):
        assert set(a[k]) == set(b[k]), k
        for n in a[k]:
            assert torch.equal(a[k][n], b[k][n]), "%s %s differs" % (k, n)


@pytest.mark.parametrize("mapper", ["mlp", "linear"])
def test_concurrent_scales_equal_sequential_eager(mapper):
    _same(_run(True, mapper=mapper), _run(False, mapper=mapper))


def test_concurrent_scales_equal_sequential_graph():
    """The concurrent step captured as one HIP graph (fork / join of three
    side streams, event-chained reductions) replayed 3 times vs the
    sequential eager step 4 times (warm-up step + 3)."""
    _same(_run(True, steps=3, graph=True), _run(False, steps=4))


def test_concurrent_scales_runs_on_side_streams():
    """The concurrent path really forks: the scale chains' kernels are issued
    on three streams other than the caller's (the mapper's deferred running
    update is issued on the caller's stream after the join)."""
    from mcaq_yolo_amd import core, hooks
    assert hooks.CONCURRENT_TRAIN_SCALES
    h = _hooks()
    feats, _ = _feats()
    seen = []
    orig = core._MapperTrainFn.forward

    def spy(ctx, *a):
        seen.append(torch.cuda.current_stream().cuda_stream)
        return orig(ctx, *a)
    core._MapperTrainFn.forward = staticmethod(spy)
    old = hooks.MULTI_SCALE_TRAIN
    hooks.MULTI_SCALE_TRAIN = False
    try:
        h.forward_features(feats)
    finally:
        core._MapperTrainFn.forward = staticmethod(orig)
        hooks.MULTI_SCALE_TRAIN = old
    main = torch.cuda.current_stream().cuda_stream
    assert len(seen) == 3 and len(set(seen)) == 3 and main not in seen
