"""Probe: device time of one optim.ClipAdamW step (mcaq_clip_adamw) on the
hook parameters, with and without the clip phase, against torch's clip +
fused AdamW + foreach abs, back to back (events around 200 steps)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_train_fused_gpu import _hooks  # noqa: E402
from mcaq_yolo_amd.optim import ClipAdamW  # noqa: E402

h = _hooks()
ps = [p for p in h.parameters() if p.requires_grad]
for p in ps:
    p.grad = torch.randn_like(p) * 1e-2
print("tensors", len(ps), "elements", sum(p.numel() for p in ps))


def timed(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


for mn in (1.0, None):
    o = ClipAdamW(ps, lr=1e-3, weight_decay=0.05, max_norm=mn, project_abs=h.bit_mapper.constrained_weights())
    print("ClipAdamW max_norm=%s: %.2f us/step" % (mn, timed(o.step)))
t = torch.optim.AdamW(ps, lr=1e-3, weight_decay=0.05, fused=True, capturable=True)


def torch_step():
    torch.nn.utils.clip_grad_norm_(ps, 1.0)
    t.step()
    h.bit_mapper.enforce_weight_constraints()


print("torch clip + fused AdamW + abs: %.2f us/step" % timed(torch_step))


def graph_timed(step):
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            step()
    return timed(g.replay, 20) / 20


for mn in (1.0, None):
    o = ClipAdamW(ps, lr=1e-3, weight_decay=0.05, max_norm=mn, project_abs=h.bit_mapper.constrained_weights())
    print("graph: ClipAdamW max_norm=%s: %.2f us/step" % (mn, graph_timed(o.step)))
print("graph: torch clip + fused AdamW + abs: %.2f us/step" % graph_timed(torch_step))
x = torch.zeros(1, device="cuda")
print("graph: one tiny ATen kernel: %.2f us" % graph_timed(lambda: x.add_(1.0)))
