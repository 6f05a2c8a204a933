"""Probe: host cost of hipGraphLaunch (torch.cuda.CUDAGraph.replay) per kernel
node on this ROCm, for graphs of N tiny kernels: one stream vs the same
kernels in 3 fork/join branches, and the QAT step's own graph shape
(bench --config 5 has ~110 kernel nodes over 4 streams).  Prints host
enqueue time per replay and wall time per replay (back to back)."""
import time

import torch

dev = torch.device("cuda:0")
x = [torch.zeros(256, device=dev) for _ in range(3)]
main = torch.cuda.Stream()
sides = [torch.cuda.Stream() for _ in range(3)]


def body(n, branches):
    if branches == 1:
        for i in range(n):
            x[0].add_(1.0)
        return
    cur = torch.cuda.current_stream()
    for s in sides[:branches]:
        s.wait_stream(cur)
    for b in range(branches):
        with torch.cuda.stream(sides[b]):
            for i in range(n // branches):
                x[b].add_(1.0)
    for s in sides[:branches]:
        cur.wait_stream(s)


def measure(n, branches, reps=50):
    torch.cuda.synchronize()
    with torch.cuda.stream(main):
        body(n, branches)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=main):
        body(n, branches)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    te = time.perf_counter() - t0
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    g.replay()
    t1e = time.perf_counter() - t1
    torch.cuda.synchronize()
    t1w = time.perf_counter() - t1
    print("N=%4d branches=%d: enqueue %7.1f us/replay (%5.2f us/node), wall %7.1f us/replay; single replay "
          "enqueue %7.1f us, latency %7.1f us" % (n, branches, te / reps * 1e6, te / reps / n * 1e6, tw / reps * 1e6,
                                                  t1e * 1e6, t1w * 1e6), flush=True)


for n in (12, 48, 96, 192):
    for br in (1, 3):
        measure(n, br)
