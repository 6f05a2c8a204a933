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

# (stamp interval, name): pass A (edges kernel) stamps 0..9, pass B (tiles kernel) 10..15
STAGES = [(0, "gray+norm"), (1, "blur"), (2, "otsu"), (3, "sobel255+dir"), (4, "nms"), (5, "hysteresis"),
          (6, "binarize"), (7, "sobel+lbp+planes"), (8, "phi tiles"),
          (10, "phi load+cmlp"), (11, "bilateral"), (12, "mapper"), (13, "softmask tiles"), (14, "m plane")]


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
        st = list(buf[:16])
        ta, tb = st[9] - st[0], st[15] - st[10]
        print("scale %d (%dx%d, C=%d): pass A %d ticks, pass B %d ticks"
              % (i, bench.SIZES[i][0], bench.SIZES[i][1], chans[i], ta, tb))
        for k, name in STAGES:
            d = st[k + 1] - st[k]
            print("   %-18s %8d  %5.1f%%" % (name, d, 100.0 * d / max(ta if k < 9 else tb, 1)))


if __name__ == "__main__":
    main()
