"""Probe: the streaming passes (pass 1 + pass 2, 3 batches in flight, HIP
graphs) beside a sleeping hog of K 1024-thread workgroups with a pass-A
footprint (~104 KB LDS) at 128 / 96 / 64 VGPRs per lane - what a pass A with
fewer registers (same latency) would leave to the streaming waves on its CUs.
wall_clock64 runs at 100 MHz."""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom  # noqa: E402

hog = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "hog_regs.so"))
hog.hog_regs_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p,
                                ctypes.c_void_p]
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
gs = []
for p, pl in enumerate(plans):
    st = streams[p]
    with torch.cuda.stream(st):
        pl.launch_stats(st); pl.launch_quant(st)
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        pl.launch_stats(st); pl.launch_quant(st)
    gs.append(g)
torch.cuda.synchronize()


def run(K):
    for i in range(K):
        with torch.cuda.stream(streams[i % 3]):
            gs[i % 3].replay()


LDS = 104 * 1024
CASES = [(0, 0)] + [(n, v) for n in (104, 160) for v in (128, 96, 64)]
for rep in range(2):
    for nh, nv in CASES:
        run(30)
        torch.cuda.synchronize()
        if nh:
            err = hog.hog_regs_launch(nh, nv, LDS, 4_000_000, ctypes.c_void_p(sink.data_ptr()),
                                      ctypes.c_void_p(hs.cuda_stream))   # 40 ms
            assert err == 0, err
            time.sleep(0.002)
        t0 = time.perf_counter()
        run(200)
        for st in streams:
            st.synchronize()
        dt = (time.perf_counter() - t0) / 200 * 1e6
        torch.cuda.synchronize()
        print("stream_only beside hog %3d WGs x %3d VGPRs: %.1f us/step" % (nh, nv, dt), flush=True)
