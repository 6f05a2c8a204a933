"""Probe: per-stage cycles of pass A / pass B (scale 0, image 0) alone and
inside the pipelined step (3 batches in flight, HIP graphs, as bench.Runner),
from a -DMCAQ_STAMPS -DMCAQ_STAMPS_ACC build (slot k = cycles from the
previous stamp to stamp k, summed over launches)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd import abi  # noqa: E402

abi._LIB = abi.load_library(sys.argv[1])
L = abi._LIB
L.mcaq_read_stamps.argtypes = [ctypes.c_void_p]
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom  # noqa: E402

NAMES = {1: "E gray+norm", 2: "E blur+hist", 3: "E otsu", 4: "E sobel255+dir", 5: "E nms", 6: "E hysteresis",
         7: "E (7)", 8: "E (8)", 9: "E tile items",
         17: "M gray+norm", 18: "M binarize: row pass", 19: "M binarize: column pass", 20: "M sobel+lbp", 21: "M (21)", 22: "M (22)", 23: "M binarize: exact list",
         24: "M boundary+euler planes", 25: "M tile items",
         10: "B start", 26: "B stage loads", 27: "B assemble phi", 28: "B cmlp mfma", 11: "B cmlp out",
         29: "B bilateral weights", 12: "B bilateral sums", 30: "B mapper BN fold", 13: "B mapper MLP + finish",
         31: "B softmask pool |x| + max", 14: "B softmask net + softmax", 15: "B m plane"}
ORDER = [1, 2, 3, 4, 5, 6, 7, 8, 9, 17, 18, 19, 20, 21, 22, 23, 24, 25, 10, 26, 27, 28, 11, 29, 12, 30, 13, 31, 14, 15]

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


def read(n):
    buf = (ctypes.c_ulonglong * 64)()
    L.mcaq_read_stamps(ctypes.cast(buf, ctypes.c_void_p))
    return [v / n for v in buf[:64]]


res = {}
N = 100
L.mcaq_reset_stamps()
for i in range(N):
    plans[i % 3].launch(torch.cuda.current_stream())
    torch.cuda.synchronize()
res["alone"] = read(N)
runner = bench.Runner(plans, None, True, 3)
runner.run(30)
runner.sync()
torch.cuda.synchronize()
N = 300
L.mcaq_reset_stamps()
runner.run(N)
runner.sync()
torch.cuda.synchronize()
res["pipelined"] = read(N)
print("%-28s %10s %10s %6s" % ("stage (scale 0, image 0)", "alone", "pipelined", "x"))
for k in ORDER:
    a, b = res["alone"][k], res["pipelined"][k]
    if a == 0 and b == 0:
        continue
    print("%-28s %10.0f %10.0f %6.2f" % (NAMES.get(k, str(k)), a, b, b / max(a, 1)))
for nm, sl in (("pass A edge", range(1, 10)), ("pass A mask", range(17, 26)),
               ("pass B", [10, 26, 27, 28, 11, 29, 12, 30, 13, 31, 14, 15])):
    a = sum(res["alone"][k] for k in sl); b = sum(res["pipelined"][k] for k in sl)
    print("%-28s %10.0f %10.0f %6.2f" % (nm + " total", a, b, b / max(a, 1)))
