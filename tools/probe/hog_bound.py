"""Probe: streaming passes (pass 1 + pass 2, 3 batches in flight, HIP graphs)
while a hog kernel holds K whole CUs (all their LDS) - how the HBM passes
scale with the CUs left to them.  wall_clock64 runs at 100 MHz."""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom  # noqa: E402

hog = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "hog.so"))
hog.hog_launch.argtypes = [ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p]
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
streams = [torch.cuda.Stream() for _ in range(3)]
hs = torch.cuda.Stream()
sink = torch.zeros(1024, dtype=torch.int32, device=dev)


def graphs(fn):
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
    return gs


G = {"stream_only": graphs(lambda pl, s: (pl.launch_stats(s), pl.launch_quant(s))),
     "full": graphs(lambda pl, s: pl.launch(s)),
     "morph_only": graphs(lambda pl, s: pl.launch_morph(s))}
VARIANTS = sys.argv[1].split(",") if len(sys.argv) > 1 else ["stream_only", "full"]
HOGS = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 32, 64, 104, 128, 160]


def run(gs, K):
    for i in range(K):
        with torch.cuda.stream(streams[i % 3]):
            gs[i % 3].replay()


for v in VARIANTS:
    for nh in HOGS:
        run(G[v], 30)
        torch.cuda.synchronize()
        if nh:
            hog.hog_launch(nh, 2_500_000, ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(hs.cuda_stream))  # 25 ms
            time.sleep(0.002)
        t0 = time.perf_counter()
        run(G[v], 250)
        for st in streams:
            st.synchronize()
        dt = (time.perf_counter() - t0) / 250 * 1e6
        torch.cuda.synchronize()
        print("%-12s hog %3d CUs: %.1f us/step" % (v, nh, dt), flush=True)
