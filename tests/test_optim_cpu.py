"""optim.ClipAdamW on CPU parameters (the torch-op path) and its state_dict
against torch.optim.AdamW: every parameter's step is its own
tensor in the state_dict, so an AdamW loading it advances each once per step
(a shared step tensor was advanced once per parameter), and a parameter
without a gradient keeps its step, as in torch."""
import torch


def _params():
    torch.manual_seed(0)
    return [torch.nn.Parameter(torch.randn(n)) for n in (3, 5, 2)]


def test_state_dict_steps_are_per_parameter_for_torch_adamw():
    from mcaq_yolo_amd.optim import ClipAdamW
    ps = _params()
    o = ClipAdamW(ps, lr=1e-2, weight_decay=0.05, max_norm=1.0)
    for p in ps:
        p.grad = torch.ones_like(p)
    o.step()
    t = torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.05)
    t.load_state_dict(o.state_dict())
    t.step()
    assert [float(t.state[p]["step"]) for p in ps] == [2.0, 2.0, 2.0]
    # ClipAdamW's own counters were not touched by torch's step
    assert [float(o.state[p]["step"]) for p in ps] == [1.0, 1.0, 1.0]


def test_matches_torch_adamw_with_unused_parameter():
    from mcaq_yolo_amd.optim import ClipAdamW
    ps, qs = _params(), _params()
    o0 = torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.05, foreach=False)
    o1 = ClipAdamW(qs, lr=1e-2, weight_decay=0.05)
    g = torch.Generator().manual_seed(1)
    for it in range(4):
        gs = [torch.randn(p.shape, generator=g) for p in ps]
        for k, (p, q, gg) in enumerate(zip(ps, qs, gs)):
            use = not (k == 1 and it in (1, 2))         # parameter 1 unused on steps 1 and 2
            p.grad = gg.clone() if use else None
            q.grad = gg.clone() if use else None
        o0.step()
        o1.step()
    for p, q in zip(ps, qs):
        assert torch.allclose(p, q, rtol=1e-6, atol=1e-7)
        assert float(o0.state[p]["step"]) == float(o1.state[q]["step"])
    assert float(o1.state[qs[1]]["step"]) == 2.0


def test_load_state_dict_roundtrip():
    from mcaq_yolo_amd.optim import ClipAdamW
    ps = _params()
    o = ClipAdamW(ps, lr=1e-2)
    for p in ps:
        p.grad = torch.ones_like(p)
    o.step()
    o.step()
    o2 = ClipAdamW(ps, lr=1e-2)
    o2.load_state_dict(o.state_dict())
    for p in ps:
        assert torch.equal(o2.state[p]["exp_avg"], o.state[p]["exp_avg"])
        assert float(o2.state[p]["step"]) == 2.0
