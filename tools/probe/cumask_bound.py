"""Probe: how the streaming passes (pass 1 + pass 2) and the morphology
(pass A + B) scale with the CUs they may use - eager launches on
CU-masked streams (hipExtStreamCreateWithCUMask), 3 batches in flight,
us per step.  Decides whether a CU-partitioned schedule (morph on M CUs,
streaming on the rest) can beat the shared one."""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
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


def masked_streams(cus, n=3):
    words = 8
    arr = (ctypes.c_uint32 * words)()
    for c in cus:
        arr[c // 32] |= 1 << (c % 32)
    out = []
    for _ in range(n):
        s = ctypes.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, arr) == 0
        out.append(torch.cuda.ExternalStream(s.value))
    return out


def spread(n, ncus=256):
    step = ncus / float(n)
    return sorted({int(k * step) for k in range(n)})


def timeit(fn, streams, K=200):
    for i in range(20):
        fn(plans[i % 3], streams[i % 3])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        fn(plans[i % 3], streams[i % 3])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e6


def stream_only(pl, s):
    pl.launch_stats(s); pl.launch_quant(s)


def morph_only(pl, s):
    pl.launch_morph(s)


for n in (256, 224, 192, 160, 128):
    st = masked_streams(spread(n))
    print("stream_only %3d CUs: %.1f %.1f us/step" % (n, timeit(stream_only, st), timeit(stream_only, st)), flush=True)
for n in (32, 64, 96, 128, 256):
    st = masked_streams(spread(n))
    print("morph_only  %3d CUs: %.1f %.1f us/step" % (n, timeit(morph_only, st), timeit(morph_only, st)), flush=True)
