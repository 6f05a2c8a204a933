"""Probe: bounds of the pipelined hook step at config 2 (3 launch sets in
flight on 3 streams, one HIP graph per launch set, as bench.Runner; argv[1]
= batches per launch set, default 1): the full chain, the streaming passes
only (pass 1 + pass 2), the morphology only (pass A + B), and pass A / pass B
alone - us per 32-image batch, interleaved repeats."""
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
K = int(sys.argv[1]) if len(sys.argv) > 1 else 1
plans = []
for p in range(3):
    feats = [[bench.synth_features(B, c, h, w, 2000 + i + 104729 * (p * K + k), dev)
              for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))] for k in range(K)]
    plan = HookPlan(geoms, dev, batches=K)
    plan.prepare(feats if K > 1 else feats[0], cm, mm, [sm] * 3, mapper_kind=mapper)
    plan.feats = feats
    plans.append(plan)
    plan.launch()
torch.cuda.synchronize()
L = plans[0].lib


def passA(pl, s):
    L.mcaq_morph_pass(pl._mo, pl._n, pl._fz, pl._n, 1, ctypes.c_void_p(s.cuda_stream))


def passB(pl, s):
    L.mcaq_morph_pass(pl._mo, pl._n, None, 0, 2, ctypes.c_void_p(s.cuda_stream))


import ctypes  # noqa: E402
VARIANTS = {
    "full": lambda pl, s: pl.launch(s),
    "stream_only": lambda pl, s: (pl.launch_stats(s), pl.launch_quant(s)),
    "morph_only": lambda pl, s: pl.launch_morph(s),
    "passA_only": passA,
    "passB_only": passB,
    "stats_only": lambda pl, s: pl.launch_stats(s),
    "quant_only": lambda pl, s: pl.launch_quant(s),
}
streams = [torch.cuda.Stream() for _ in range(3)]
graphs = {}
for v, fn in VARIANTS.items():
    gs = []
    for p, pl in enumerate(plans):
        st = streams[p]
        with torch.cuda.stream(st):
            fn(pl, st)
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            fn(pl, st)
        gs.append(g)
    graphs[v] = gs
torch.cuda.synchronize()


NB = K


def timeit(v, K=300):
    gs = graphs[v]
    for i in range(30):
        with torch.cuda.stream(streams[i % 3]):
            gs[i % 3].replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        with torch.cuda.stream(streams[i % 3]):
            gs[i % 3].replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (K * NB) * 1e6


print("batches per launch set:", NB)
for rep in range(3):
    print(" | ".join("%s %.1f" % (v, timeit(v)) for v in VARIANTS), flush=True)
