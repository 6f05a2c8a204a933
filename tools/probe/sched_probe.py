"""Probe: a streaming-stream schedule for the pipelined hook step (config 2).
One stream S runs every HBM pass in order - pass 1 of batch j+L, then pass 2
of batch j - and the morphologies run on 3 side streams, joined by events
(pass 1 -> morphology -> pass 2), so the streaming passes follow each other
instead of three chains drifting into their morphology halves together
(profiles/r04_sched/trace_concurrency.txt).  Variants: the default (one graph
per batch on 3 streams), this schedule with eager launches, and with one
single-stream graph per pass; lookahead L = 1 / 2.  us per step."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom  # noqa: E402

dev = torch.device("cuda:0")
name, B, chans, grid, mapper = bench.CONFIGS[2]
cm, mm, sm = bench.load_blobs(dev)
geoms = [ScaleGeom(B, c, h, w, grid) for c, (h, w) in zip(chans, bench.SIZES)]
NP = 4
plans = []
for p in range(NP):
    feats = [bench.synth_features(B, c, h, w, 2000 + i + 104729 * p, dev) for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))]
    plan = HookPlan(geoms, dev)
    plan.prepare(feats, cm, mm, [sm] * 3, mapper_kind=mapper)
    plan.feats = feats
    plans.append(plan)
    plan.launch()
torch.cuda.synchronize()


def capture(fn, st):
    with torch.cuda.stream(st):
        fn(st)
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        fn(st)
    return g


main = [torch.cuda.Stream() for _ in range(3)]
full = [capture(lambda s, pl=pl: pl.launch(s), main[p % 3]) for p, pl in enumerate(plans[:3])]


def step_default(i):
    with torch.cuda.stream(main[i % 3]):
        full[i % 3].replay()


class Sched:
    def __init__(self, L, graphs):
        self.L = L
        self.S = torch.cuda.Stream()
        self.M = [torch.cuda.Stream() for _ in range(3)]
        self.es = [torch.cuda.Event() for _ in range(NP)]
        self.em = [torch.cuda.Event() for _ in range(NP)]
        self.g = None
        if graphs:
            self.g = [(capture(lambda s, pl=pl: pl.launch_stats(s), self.S),
                       capture(lambda s, pl=pl: pl.launch_morph(s), self.M[p % 3]),
                       capture(lambda s, pl=pl: pl.launch_quant(s), self.S)) for p, pl in enumerate(plans)]
        torch.cuda.synchronize()
        self.started = 0

    def _front(self, j):
        p = j % NP
        S, M = self.S, self.M[j % 3]
        with torch.cuda.stream(S):
            if self.g: self.g[p][0].replay()
            else: plans[p].launch_stats(S)
            self.es[p].record(S)
        with torch.cuda.stream(M):
            M.wait_event(self.es[p])
            if self.g: self.g[p][1].replay()
            else: plans[p].launch_morph(M)
            self.em[p].record(M)

    def step(self, i):
        if i == 0:
            for j in range(self.L):
                self._front(j)
        self._front(i + self.L)
        p = i % NP
        S = self.S
        with torch.cuda.stream(S):
            S.wait_event(self.em[p])
            if self.g: self.g[p][2].replay()
            else: plans[p].launch_quant(S)

    def sync(self):
        torch.cuda.synchronize()


def timeit(step, K=300):
    for i in range(K):      # a fresh run: warm-up then the timed steps continue it
        step(i)
        if i == 29:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
    te = time.perf_counter() - t0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (K - 30) * 1e6, te / (K - 30) * 1e6


for rep in range(3):
    out = ["default %.1f (enq %.1f)" % timeit(step_default)]
    for L in (1, 2):
        for gr in (False, True):
            s = Sched(L, gr)
            out.append("S L%d %s %.1f (enq %.1f)" % ((L, "graph" if gr else "eager") + timeit(s.step)))
            del s
    print(" | ".join(out), flush=True)
