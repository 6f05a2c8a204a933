"""Probe: pass-1 (mcaq_stats) time per hook scale at BASELINE config 2, and of
all three scales in one launch, each launch timed by its own start/stop events
(mcaq_time_next_launch), launches back to back on one stream; pass 2
(mcaq_quant) alone for comparison.  Run on the GPU box:

    python tools/probe/stats_split.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd import abi  # noqa: E402
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom  # noqa: E402


def timed(L, fn, reps=20):
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        b.record(st)
    fn()
    torch.cuda.synchronize()
    for a, b in ev:
        L.mcaq_time_next_launch(ctypes.c_void_p(a.cuda_event), ctypes.c_void_p(b.cuda_event))
        fn()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) * 1e3 / reps


def main():
    dev = torch.device("cuda:0")
    name, B, chans, grid, mapper = bench.CONFIGS[int(os.environ.get("CFG", "2"))]
    B = int(os.environ.get("BATCH", B))        # e.g. 16: the QAT step's per-GPU batch
    cm, mm, sm = bench.load_blobs(dev)
    geoms = [ScaleGeom(B, c, h, w, grid) for c, (h, w) in zip(chans, bench.SIZES)]
    feats = [bench.synth_features(B, c, h, w, 1000 + i, dev) for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))]
    plan = HookPlan(geoms, dev)
    plan.prepare(feats, cm, mm, [sm] * 3, temperature=1.0, mapper_kind=mapper)
    torch.cuda.synchronize()
    L = plan.lib
    sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    st_arr = plan._st
    size = ctypes.sizeof(abi.StatsScale)
    base = ctypes.addressof(st_arr)
    for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES)):
        one = abi.StatsScale.from_address(base + i * size)
        us = timed(L, lambda: abi.check(L.mcaq_stats(ctypes.byref(one), 1, sh), "stats"))
        mb = B * c * h * w * 4 / 1e6
        print("stats scale %d  C=%3d %dx%d  %6.2f us  %6.1f MB  %6.0f GB/s" % (i, c, h, w, us, mb, mb * 1e3 / us))
    us = timed(L, lambda: abi.check(L.mcaq_stats(st_arr, 3, sh), "stats"))
    mb = sum(B * c * h * w * 4 for c, (h, w) in zip(chans, bench.SIZES)) / 1e6
    print("stats all 3     %6.2f us  %6.1f MB  %6.0f GB/s" % (us, mb, mb * 1e3 / us))
    plan.launch_stats()
    plan.launch_morph()
    torch.cuda.synchronize()
    us = timed(L, lambda: plan.launch_quant())
    print("quant all 3     %6.2f us  %6.1f MB  %6.0f GB/s" % (us, 2 * mb, 2 * mb * 1e3 / us))


if __name__ == "__main__":
    main()
