"""Probe: timing events recorded INSIDE a captured HIP graph (external=True)."""
import torch
x = torch.randn(64 << 20, device="cuda")
y = torch.empty_like(x)
s = torch.cuda.Stream()
evs = [torch.cuda.Event(enable_timing=True, external=True) for _ in range(3)]
with torch.cuda.stream(s):
    y.copy_(x); torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    evs[0].record()
    y.copy_(x)
    evs[1].record()
    y.mul_(2.0)
    evs[2].record()
for it in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("replay", it, "copy %.1f us" % (evs[0].elapsed_time(evs[1]) * 1e3), "mul %.1f us" % (evs[1].elapsed_time(evs[2]) * 1e3))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); y.copy_(x); e1.record(); torch.cuda.synchronize()
print("eager copy %.1f us" % (e0.elapsed_time(e1) * 1e3))
