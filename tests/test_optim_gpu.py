"""optim.ClipAdamW (two launches: clip_grad_norm_ + AdamW + |W| projection,
train.py:626-641) against torch's own three steps - clip_grad_norm_(1.0),
torch.optim.AdamW(fused), the mapper's enforce_weight_constraints - over
several steps on the hook parameters with real QAT gradients.  fp32 sums in
other orders (the gradient norm): parameters within rtol 1e-5 of the
largest magnitude per tensor after 5 steps, the clipped gradients and
exp_avg / exp_avg_sq likewise; the total norm within rtol 1e-6."""
import pytest
import torch

from test_concurrent_scales_gpu import _feats
from test_train_fused_gpu import _hooks

pytestmark = pytest.mark.gpu


def _close(a, b, rtol, what):
    scale = max(float(b.abs().max()), 1e-30)
    err = float((a - b).abs().max())
    assert err <= rtol * scale, "%s: max err %g vs scale %g" % (what, err, scale)


@pytest.mark.parametrize("max_norm", [1.0, 1e-4, None])
def test_clip_adamw_matches_torch_steps(max_norm):
    from mcaq_yolo_amd.optim import ClipAdamW
    h0, h1 = _hooks(), _hooks()          # identical (seeded, same fixture weights)
    feats, gens = _feats()
    p0 = [p for p in h0.parameters() if p.requires_grad]
    p1 = [p for p in h1.parameters() if p.requires_grad]
    o0 = torch.optim.AdamW(p0, lr=1e-3, weight_decay=0.05, betas=(0.9, 0.999), fused=True)
    o1 = ClipAdamW(p1, lr=1e-3, weight_decay=0.05, betas=(0.9, 0.999), max_norm=max_norm,
                   project_abs=h1.bit_mapper.constrained_weights())
    for it in range(5):
        for h, o, ps in ((h0, o0, p0), (h1, o1, p1)):
            o.zero_grad(set_to_none=True)
            xs = [f.detach().clone().requires_grad_(True) for f in feats]
            outs, aux = h.forward_features(xs, temperature=1.0)
            avg = torch.stack([a["bit_map"].float().mean() for a in aux]).mean()
            (sum((y * g).sum() for y, g in zip(outs, gens)) + 0.1 * (avg - 4.0) ** 2).backward()
        # the same gradients go into both optimizers (they only differ after step 1)
        for a, b in zip(p0, p1):
            b.grad.copy_(a.grad)
        tn = torch.nn.utils.clip_grad_norm_(p0, max_norm) if max_norm is not None else None
        o0.step()
        h0.bit_mapper.enforce_weight_constraints()
        o1.step()
        torch.cuda.synchronize()
        if max_norm is not None:
            _close(o1.last_total_norm.reshape(()), tn, 1e-6, "total norm step %d" % it)
        for (n, a), b in zip([(n, p) for n, p in h0.named_parameters() if p.requires_grad], p1):
            _close(b.grad, a.grad, 1e-5, "clipped grad %s" % n)
            _close(b, a, 1e-5, "param %s step %d" % (n, it))
            _close(o1.state[b]["exp_avg"], o0.state[a]["exp_avg"], 1e-5, "exp_avg %s" % n)
            _close(o1.state[b]["exp_avg_sq"], o0.state[a]["exp_avg_sq"], 1e-5, "exp_avg_sq %s" % n)
        # copy torch's parameters over so the steps compare one update at a time
        with torch.no_grad():
            for a, b in zip(p0, p1):
                b.copy_(a)
                o1.state[b]["exp_avg"].copy_(o0.state[a]["exp_avg"])
                o1.state[b]["exp_avg_sq"].copy_(o0.state[a]["exp_avg_sq"])
    for w in h1.bit_mapper.constrained_weights():
        assert bool((w >= 0).all())


def test_clip_adamw_state_dict_roundtrip_with_torch_adamw():
    from mcaq_yolo_amd.optim import ClipAdamW
    h = _hooks()
    ps = [p for p in h.parameters() if p.requires_grad]
    o = ClipAdamW(ps, lr=1e-3, weight_decay=0.05, max_norm=1.0)
    for p in ps:
        p.grad = torch.randn_like(p) * 1e-2
    o.step()
    o.step()
    sd = o.state_dict()
    t = torch.optim.AdamW(ps, lr=1e-3, weight_decay=0.05)
    t.load_state_dict(sd)
    assert float(t.state[ps[0]]["step"]) == 2.0
    o2 = ClipAdamW(ps, lr=1e-3, weight_decay=0.05, max_norm=1.0)
    o2.load_state_dict(t.state_dict())
    for p in ps:
        assert torch.equal(o2.state[p]["exp_avg"], o.state[p]["exp_avg"])
        assert torch.equal(o2.state[p]["exp_avg_sq"], o.state[p]["exp_avg_sq"])
    assert float(o2.state[ps[0]]["step"]) == 2.0


def test_clip_adamw_graph_capture():
    """The step captured in a HIP graph (the bench's QAT step) replays the
    same updates as eager steps."""
    from mcaq_yolo_amd.optim import ClipAdamW
    torch.manual_seed(3)
    ps = [torch.randn(n, device="cuda", requires_grad=True) for n in (97, 2048, 5)]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    gs = [torch.randn_like(p) for p in ps]
    oa = ClipAdamW(ps, lr=1e-2, weight_decay=0.05, max_norm=0.5, project_abs=[ps[1]])
    ob = ClipAdamW(qs, lr=1e-2, weight_decay=0.05, max_norm=0.5, project_abs=[qs[1]])
    for p, g in zip(ps, gs):
        p.grad = g.clone()
    for q, g in zip(qs, gs):
        q.grad = g.clone()
    oa.step()
    ob.step()          # warm-up (state allocation) outside capture
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ob.step()
    for _ in range(3):
        for p, g in zip(ps, gs):
            p.grad.copy_(g)
        oa.step()
        for q, g in zip(qs, gs):
            q.grad.copy_(g)
        graph.replay()
    torch.cuda.synchronize()
    for p, q in zip(ps, qs):
        assert torch.equal(p, q)
    assert all(float(oa.state[p]["step"]) == float(ob.state[q]["step"]) == 4.0 for p, q in zip(ps, qs))


def test_clip_adamw_step_reaches_packed_blobs():
    """The kernel writes the parameters through raw pointers; the optimizer
    bumps their version counters, so the hooks' packed weight blobs
    (core._BlobCache) are re-packed and the next eager forward sees the
    update (equal to the same hooks stepped by torch's optimizer)."""
    from mcaq_yolo_amd.optim import ClipAdamW
    feats, gens = _feats()
    res = []
    for fused in (True, False):
        h = _hooks()
        ps = [p for p in h.parameters() if p.requires_grad]
        o = ClipAdamW(ps, lr=1e-2, weight_decay=0.05) if fused else torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.05)
        for it in range(2):
            o.zero_grad(set_to_none=True)
            xs = [f.detach().clone().requires_grad_(True) for f in feats]
            outs, aux = h.forward_features(xs, temperature=1.0)
            sum((y * g).sum() for y, g in zip(outs, gens)).backward()
            o.step()
        with torch.no_grad():
            h.eval()
            outs, aux = h.forward_features([f.detach() for f in feats])
        torch.cuda.synchronize()
        res.append([a["complexity"].clone() for a in aux])
    for a, b in zip(*res):
        err = float((a - b).abs().max())
        assert err <= 1e-4 * float(b.abs().max()), err
    # and not equal to the un-stepped hooks'
    h0 = _hooks().eval()
    with torch.no_grad():
        _, aux0 = h0.forward_features([f.detach() for f in feats])
    assert not torch.equal(aux0[0]["complexity"], res[0][0])


@pytest.mark.parametrize("sizes", [(97, 2048, 5), (97, 20000, 5, 3000)])
def test_clip_adamw_chunked_lists_match_torch(sizes):
    """Parameter lists of 3 and 24 1,024-element chunks (tensors spanning
    chunk boundaries) against torch's clip_grad_norm_ + fused AdamW + abs,
    over 4 steps with fresh gradients, and the device step counter."""
    from mcaq_yolo_amd.optim import ClipAdamW
    torch.manual_seed(11)
    ps = [torch.randn(n, device="cuda", requires_grad=True) for n in sizes]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    o0 = torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.05, betas=(0.9, 0.999), fused=True)
    o1 = ClipAdamW(qs, lr=1e-2, weight_decay=0.05, betas=(0.9, 0.999), max_norm=0.5, project_abs=[qs[1]])
    for it in range(4):
        gs = [torch.randn_like(p) for p in ps]
        for p, q, g in zip(ps, qs, gs):
            p.grad = g.clone()
            q.grad = g.clone()
        tn = torch.nn.utils.clip_grad_norm_(ps, 0.5)
        o0.step()
        with torch.no_grad():
            ps[1].abs_()
        o1.step()
        torch.cuda.synchronize()
        _close(o1.last_total_norm.reshape(()), tn, 1e-6, "total norm step %d" % it)
        for k, (p, q) in enumerate(zip(ps, qs)):
            _close(q.grad, p.grad, 1e-6, "clipped grad %d step %d" % (k, it))
            _close(q, p, 1e-5, "param %d step %d" % (k, it))
            _close(o1.state[q]["exp_avg"], o0.state[p]["exp_avg"], 1e-5, "exp_avg %d" % k)
            _close(o1.state[q]["exp_avg_sq"], o0.state[p]["exp_avg_sq"], 1e-5, "exp_avg_sq %d" % k)
        with torch.no_grad():
            for p, q in zip(ps, qs):
                q.copy_(p)
                o1.state[q]["exp_avg"].copy_(o0.state[p]["exp_avg"])
                o1.state[q]["exp_avg_sq"].copy_(o0.state[p]["exp_avg_sq"])
    assert all(float(o1.state[q]["step"]) == 4.0 for q in qs)


def test_clip_adamw_step_after_load_state_dict_matches_torch():
    """a GPU step after load_state_dict (following earlier steps)
    rebuilds its launch descriptors against the re-homed moment buffers; the
    run step, load, step equals torch's fused AdamW over the same three steps."""
    from mcaq_yolo_amd.optim import ClipAdamW
    torch.manual_seed(5)
    ps = [torch.randn(n, device="cuda", requires_grad=True) for n in (97, 2048, 5)]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    o0 = torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.05, fused=True)
    o1 = ClipAdamW(qs, lr=1e-2, weight_decay=0.05)
    gs = [[torch.randn_like(p) for p in ps] for _ in range(3)]
    for it in range(3):
        for p, q, g in zip(ps, qs, gs[it]):
            p.grad, q.grad = g.clone(), g.clone()
        o0.step()
        o1.step()
        if it == 1:
            o1.load_state_dict(o1.state_dict())
    torch.cuda.synchronize()
    for k, (p, q) in enumerate(zip(ps, qs)):
        _close(q, p, 1e-5, "param %d" % k)
        assert float(o1.state[q]["step"]) == 3.0


def test_clip_adamw_per_parameter_steps_and_lr_table():
    """a parameter without a gradient keeps its step (torch's
    per-parameter counters), and an lr change reaches a captured step through
    the device hyper-parameter table (sync_hyperparameters)."""
    from mcaq_yolo_amd.optim import ClipAdamW
    torch.manual_seed(6)
    ps = [torch.randn(n, device="cuda", requires_grad=True) for n in (33, 700)]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    o0 = torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.05, fused=True)
    o1 = ClipAdamW(qs, lr=1e-2, weight_decay=0.05)
    g = [torch.randn_like(p) for p in ps]
    # step 1: both; step 2: only the second parameter has a gradient
    for p, q, gg in zip(ps, qs, g):
        p.grad, q.grad = gg.clone(), gg.clone()
    o0.step(); o1.step()
    ps[0].grad = qs[0].grad = None
    o0.step(); o1.step()
    torch.cuda.synchronize()
    assert float(o1.state[qs[0]]["step"]) == 1.0 and float(o1.state[qs[1]]["step"]) == 2.0
    for k, (p, q) in enumerate(zip(ps, qs)):
        _close(q, p, 1e-5, "param %d" % k)
    # captured step, then lr halved between replays
    qs[0].grad = g[0].clone()
    ps[0].grad = g[0].clone()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        o1.step()
    for gr in (o0.param_groups[0], o1.param_groups[0]):
        gr["lr"] = 5e-3
    o1.sync_hyperparameters()
    o0.step()
    graph.replay()
    torch.cuda.synchronize()
    for k, (p, q) in enumerate(zip(ps, qs)):
        _close(q, p, 1e-5, "param %d after lr change" % k)


@pytest.mark.parametrize("sizes", [(97, 2048, 5), (4609, 2881, 33, 1, 1024, 3000), (261144, 1000)])
def test_clip_adamw_one_launch_equals_two_launches(sizes):
    """The clipped step as ONE launch (optim.ONE_LAUNCH: the chunks' norm
    partials exchanged inside the launch) against the two launches, bit for
    bit: parameters, clipped gradients, moments, step counts and total norm
    over eager steps (one parameter without a gradient in step 2: its count
    stays) and graph replays; the exchange status word stays clear.  The
    last case is the one-launch maximum: 256 chunks of 1,024 elements."""
    from mcaq_yolo_amd import abi, optim
    from mcaq_yolo_amd.optim import ClipAdamW
    torch.manual_seed(7)
    init = [torch.randn(n, device="cuda") for n in sizes]
    grads = [[torch.randn(n, device="cuda") * (0.1 + it) for n in sizes] for it in range(6)]
    res = {}
    for one in (True, False):
        old = optim.ONE_LAUNCH
        optim.ONE_LAUNCH = one
        try:
            ps = [t.clone().requires_grad_(True) for t in init]
            o = ClipAdamW(ps, lr=1e-2, weight_decay=0.05, max_norm=0.5, project_abs=[ps[1]])
            norms = []
            for it in range(3):
                for p, g in zip(ps, grads[it]):
                    p.grad = g.clone()
                if it == 1:
                    ps[0].grad = None
                o.step()
                norms.append(o.last_total_norm.clone())
            for p, g in zip(ps, grads[3]):
                p.grad = g.clone()
            o.step()                                   # new descriptors (grads reallocated), then capture
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                o.step()
            for it in (4, 5):
                for p, g in zip(ps, grads[it]):
                    p.grad.copy_(g)
                graph.replay()
                norms.append(o.last_total_norm.clone())
            torch.cuda.synchronize()
            if one:
                assert o._sync is not None
                assert int(o._sync.view(torch.int32)[abi.ADAMW_SYNC_STATUS_WORD].item()) == 0
            res[one] = ([p.detach().clone() for p in ps] + [p.grad.clone() for p in ps] +
                        [o.state[p][k].clone() for p in ps for k in ("exp_avg", "exp_avg_sq")] + norms,
                        [float(o.state[p]["step"]) for p in ps])
        finally:
            optim.ONE_LAUNCH = old
    (a, sa), (b, sb) = res[True], res[False]
    assert sa == sb and sa[0] == 5.0 and sa[1] == 6.0
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x, y), i
