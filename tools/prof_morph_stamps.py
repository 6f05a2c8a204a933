"""Diagnostic: per-stage cycles of the morph kernel (workgroup 0 of each scale),
from a -DMCAQ_STAMPS build (tools/build.py --stamps writes lib/libmcaq_hip_stamps.so)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd import abi  # noqa: E402

# (stamp slot, next slot, name): pass A edge workgroup 0..9, mask workgroup 16..25,
# pass B (tiles kernel) 10..15
STAGES = [(0, 1, "E gray+norm"), (1, 2, "E blur+hist"), (2, 3, "E otsu"), (3, 4, "E sobel255+dir"),
          (4, 5, "E nms"), (5, 6, "E hysteresis"), (8, 9, "E tile items"),
          (16, 17, "M gray+norm"), (17, 23, "M binarize"), (23, 24, "M sobel+lbp+planes"), (24, 25, "M tile items"),
          (10, 26, "B stage loads"), (26, 27, "B assemble phi"), (27, 28, "B cmlp mfma"), (28, 11, "B cmlp out"), (11, 12, "B bilateral"), (11, 29, "B  bilateral: weights (exp)"), (29, 12, "B  bilateral: 25-tap sums"), (12, 13, "B mapper"), (12, 30, "B  mapper: BN fold"), (30, 13, "B  mapper: MLP + finish"),
          (40, 41, "B  w0 cmlp L1"), (41, 42, "B  w0 cmlp LN1"), (42, 43, "B  w0 cmlp L2"), (43, 44, "B  w0 cmlp LN2"),
          (44, 45, "B  w0 cmlp L3+sigmoid"), (48, 49, "B  w0 map in (log1p)"), (49, 50, "B  w0 map L1+BN"),
          (50, 51, "B  w0 map L2+BN"), (51, 52, "B  w0 map L3+BN"), (52, 53, "B  w0 map L4 dot"), (53, 54, "B  w0 map sigmoid"),
          (13, 14, "B softmask tiles"), (13, 31, "B  softmask: pool |x| + max"), (31, 14, "B  softmask: net + softmax"),
          (14, 15, "B m plane")]


def main():
    path = os.path.join(ROOT, "mcaq_yolo_amd", "lib", "libmcaq_hip_stamps.so")
    abi._LIB = abi.load_library(path)
    L = abi._LIB
    L.mcaq_read_stamps.argtypes = [ctypes.c_void_p]
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
    for i in range(plan._n):
        for _ in range(3):
            L.mcaq_morph(ctypes.byref(plan._mo[i]), 1, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        L.mcaq_read_stamps(ctypes.cast(buf, ctypes.c_void_p))
        st = list(buf[:64])
        ta, tm, tb = st[9] - st[0], st[25] - st[16], st[15] - st[10]
        print("scale %d (%dx%d, C=%d): pass A edge %d / mask %d ticks, pass B %d ticks"
              % (i, bench.SIZES[i][0], bench.SIZES[i][1], chans[i], ta, tm, tb))
        for k, k2, name in STAGES:
            d = st[k2] - st[k]
            print("   %-20s %8d" % (name, d))


if __name__ == "__main__":
    main()
