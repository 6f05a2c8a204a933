"""Diagnostic: per-stage cycles of the band / edge kernels of pass A (band 1
and the edge workgroup of image 0 of each scale, launched alone), from a
-DMCAQ_STAMPS build (python tools/build.py --stamps)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd import abi  # noqa: E402

BAND = ["S0 gray min/max", "S0 G rows", "S1 row pass + blur", "S2 BIN + sobel", "S3 nms/lbp/planes", "S4 tile items"]
EDGE = ["loads (hist + nms)", "otsu", "double threshold", "hysteresis", "tile items"]


def main():
    path = os.path.join(ROOT, "mcaq_yolo_amd", "lib", "libmcaq_hip_stamps.so")
    abi._LIB = abi.load_library(path)
    L = abi._LIB
    L.mcaq_read_stamps.argtypes = [ctypes.c_void_p]
    L.mcaq_reset_stamps.argtypes = []
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    dev = torch.device("cuda:0")
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    name, B, chans, grid, mapper = bench.CONFIGS[cfg]
    feats = [bench.synth_features(B, c, h, w, 1000 * cfg + i, dev) for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))]
    cm, mm, sm = bench.load_blobs(dev)
    plan = HookPlan([ScaleGeom(B, c, h, w, grid) for c, (h, w) in zip(chans, bench.SIZES)], dev)
    plan.prepare(feats, cm, mm, [sm] * 3)
    plan.launch()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 64)()
    st_ = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for i in range(plan._n):
        for _ in range(3):
            L.mcaq_morph_pass(ctypes.byref(plan._mo[i]), 1, None, 0, 1, st_)
        torch.cuda.synchronize()
        L.mcaq_read_stamps(ctypes.cast(buf, ctypes.c_void_p))
        st = list(buf[:64])
        print("scale %d (%dx%d, C=%d): band %d ticks, edge %d ticks"
              % (i, bench.SIZES[i][0], bench.SIZES[i][1], chans[i], st[62] - st[56], st[21] - st[16]))
        for k, nm in enumerate(BAND):
            print("   band %-22s %8d" % (nm, st[57 + k] - st[56 + k]))
        for k, nm in enumerate(EDGE):
            print("   edge %-22s %8d" % (nm, st[17 + k] - st[16 + k]))


if __name__ == "__main__":
    main()
