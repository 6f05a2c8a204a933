"""Diagnostic: stage cycles of the train-step kernels' workgroup 0 (the
soft-mask backward of scale 0's image 0, slots 32..41; the mapper's backward
stage 3 and forward stage 2, slots 42..56) from a -DMCAQ_STAMPS
build (python tools/build.py --stamps -> lib/libmcaq_hip_stamps.so), one QAT
step at config 5 (bench.py --config 5 shapes)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mcaq_yolo_amd import abi  # noqa: E402

abi._LIB = abi.load_library(os.path.join(ROOT, "mcaq_yolo_amd", "lib", "libmcaq_hip_stamps.so"))
L = abi._LIB
L.mcaq_read_stamps.argtypes = [ctypes.c_void_p]
from test_train_fused_gpu import _hooks  # noqa: E402

STAGES = [(32, 33, "stage |x| plane + ranges"), (33, 34, "pool |x| per tile + amax"), (34, 41, "fold: slice loads"),
          (41, 35, "fold: band / tile sums"), (35, 36, "smoothing adjoint, vertical"),
          (36, 37, "horizontal + upsample adjoint"), (37, 38, "per-tile net + logit grads"),
          (38, 39, "bits-feature grad (3x3^T)"), (39, 40, "parameter partials")]


MAPPER_BWD = [(56, 42, "operand loads issued + BN sums"), (42, 43, "g_a(S) (BN backward)"),
              (43, 44, "h(S-1) recompute"), (44, 45, "weight / bias partials"), (45, 48, "W^T g_a (FMA)"), (48, 46, "g_y stores"),
              (46, 47, "BN(S-1) partial sums")]
BILAT = [(57, 58, "range x spatial weights (exp)"), (58, 59, "per tile: C, g / D, centre"),
         (59, 60, "adjoint gather")]
CMLP = [(16, 17, "recompute layer 1 + LN1"), (17, 18, "recompute layer 2 + LN2 + L3"), (18, 19, "sigmoid / L3 / LN2 bwd"),
        (19, 20, "L2^T + LN1 bwd"), (20, 21, "W2 partials (MFMA)"), (21, 22, "other partials")]
MAPPER_FWD = [(50, 51, "batch statistics (map_stats)"), (52, 53, "h(S-1) into LDS"), (53, 54, "layer (FMA)"),
              (54, 55, "workgroup moments")]


def main():
    dev = torch.device("cuda:0")
    h = _hooks()
    gen = torch.Generator(device="cpu").manual_seed(5)
    feats = [torch.randn(16, c, s, s, generator=gen).to(dev).requires_grad_(True)
             for c, s in ((64, 80), (128, 40), (256, 20))]
    for _ in range(3):
        outs, aux = h.forward_features(feats)
        loss = sum(o.sum() for o in outs) * 1e-3 + h.bit_budget_loss(aux, 4.0)
        loss.backward()
        torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 64)()
    L.mcaq_read_stamps(ctypes.cast(buf, ctypes.c_void_p))
    st = list(buf)
    print("soft-mask backward, scale 0 image 0 (80x80, 10x10 tiles): %d s_memtime ticks total"
          % (st[40] - st[32]))
    for a, b, name in STAGES:
        print("   %-34s %8d" % (name, st[b] - st[a]))
    print("mapper backward stage 3, workgroup 0 (64 tiles of scale 0): %d ticks" % (st[47] - st[56]))
    for a, b, name in MAPPER_BWD:
        print("   %-34s %8d" % (name, st[b] - st[a]))
    print("bilateral backward, image 0 of scale 0: %d ticks" % (st[60] - st[57]))
    for a, b, name in BILAT:
        print("   %-34s %8d" % (name, st[b] - st[a]))
    print("complexity-MLP backward, workgroup 0: %d ticks" % (st[22] - st[16]))
    for a, b, name in CMLP:
        print("   %-34s %8d" % (name, st[b] - st[a]))
    print("mapper forward stage 2, workgroup 0: %d ticks" % (st[55] - st[50]))
    for a, b, name in MAPPER_FWD:
        print("   %-34s %8d" % (name, st[b] - st[a]))
    # the fused mapper launches (train_step.MAPPER_FUSED), workgroup 0
    print("mapper forward, one launch: %d ticks" % (st[27] - st[23]))
    for a, b, name in ((23, 24, "stage 1"), (24, 25, "stage 2 (sweep of exchange 1 + layer)"),
                       (25, 26, "stage 3 (sweep of exchange 2 + layer)"), (26, 27, "stage 4 (sweep of exchange 3 + bits)")):
        print("   %-40s %8d" % (name, st[b] - st[a]))
    print("mapper backward, one launch: %d ticks" % (st[49] - st[28]))
    for a, b, name in ((28, 29, "stage 4"), (29, 30, "stage 3 (sweep of exchange 1)"),
                       (30, 31, "stage 2 (sweep of exchange 2)"), (31, 49, "stage 1 (sweep of exchange 3)")):
        print("   %-40s %8d" % (name, st[b] - st[a]))


if __name__ == "__main__":
    main()
