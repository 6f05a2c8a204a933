"""Probe: does dispatch priority for the morphology shorten the pipelined step?
Config 2, 3 batches in flight.  Variants (us per step, interleaved repeats):
  graph       one HIP graph per batch on its stream (bench.Runner, the default)
  eager       the same launches without graphs
  split       per batch three single-stream graphs: pass 1 on the batch's main
              stream, morphology (pass A + B + finalize) on a side stream, pass 2
              on the main stream, joined by events; side streams normal priority
  split_hi    the same with the side streams at the highest stream priority
  split_lo    main streams at the highest priority instead (streaming first)
Every batch slot keeps its own streams, so pass 1 of batch i+3 follows pass 2
of batch i on the main stream and its morphology waits for that pass 1."""
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
plans = []
for p in range(3):
    feats = [bench.synth_features(B, c, h, w, 2000 + i + 104729 * p, dev) for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))]
    plan = HookPlan(geoms, dev)
    plan.prepare(feats, cm, mm, [sm] * 3, mapper_kind=mapper)
    plan.feats = feats
    plans.append(plan)
    plan.launch()
torch.cuda.synchronize()
lo_pri, hi_pri = torch.cuda.Stream.priority_range()
print("stream priority range (lowest, highest):", lo_pri, hi_pri, flush=True)

main = [torch.cuda.Stream() for _ in range(3)]


def capture(fn, st):
    with torch.cuda.stream(st):
        fn(st)
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        fn(st)
    return g


full_graphs = [capture(lambda s, pl=pl: pl.launch(s), main[p]) for p, pl in enumerate(plans)]


class Split:
    def __init__(self, main_pri, side_pri):
        self.m = [torch.cuda.Stream(priority=main_pri) for _ in range(3)]
        self.s = [torch.cuda.Stream(priority=side_pri) for _ in range(3)]
        self.g = []
        for p, pl in enumerate(plans):
            self.g.append((capture(lambda s, pl=pl: pl.launch_stats(s), self.m[p]),
                           capture(lambda s, pl=pl: pl.launch_morph(s), self.s[p]),
                           capture(lambda s, pl=pl: pl.launch_quant(s), self.m[p])))
        self.e1 = [torch.cuda.Event() for _ in range(3)]
        self.e2 = [torch.cuda.Event() for _ in range(3)]
        torch.cuda.synchronize()

    def step(self, i):
        p = i % 3
        m, s = self.m[p], self.s[p]
        g1, g2, g3 = self.g[p]
        with torch.cuda.stream(m):
            g1.replay()
            self.e1[p].record(m)
        with torch.cuda.stream(s):
            s.wait_event(self.e1[p])
            g2.replay()
            self.e2[p].record(s)
        with torch.cuda.stream(m):
            m.wait_event(self.e2[p])
            g3.replay()


def step_graph(i):
    with torch.cuda.stream(main[i % 3]):
        full_graphs[i % 3].replay()


def step_eager(i):
    st = main[i % 3]
    with torch.cuda.stream(st):
        plans[i % 3].launch(st)


split = Split(lo_pri, lo_pri)
split_hi = Split(lo_pri, hi_pri)
split_lo = Split(hi_pri, lo_pri)
VARIANTS = {"graph": step_graph, "eager": step_eager, "split": split.step, "split_hi": split_hi.step,
            "split_lo": split_lo.step}


def timeit(fn, K=300):
    for i in range(30):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        fn(i)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e6, t_enq / K * 1e6


for rep in range(3):
    out = []
    for v, fn in VARIANTS.items():
        us, enq = timeit(fn)
        out.append("%s %.1f (enq %.1f)" % (v, us, enq))
    print(" | ".join(out), flush=True)
