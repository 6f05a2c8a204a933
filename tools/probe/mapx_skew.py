"""Diagnostic: when the fused mapper forward's workgroups 0..31 start and
finish stage 1 (the 100 MHz global clock, a -DMCAQ_STAMPS_WG build:
tools/build_ab.sh wg -DMCAQ_STAMPS_WG, copied over lib/libmcaq_hip.so by the
caller), one multi-scale forward at config 5's shapes.  The exchange after
stage 1 waits for the LAST of them; this prints how late that is."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mcaq_yolo_amd import abi  # noqa: E402
from test_train_fused_gpu import _hooks  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    L = abi.lib()
    L.mcaq_read_wg_stamps.argtypes = [ctypes.c_void_p]
    h = _hooks()
    gen = torch.Generator(device="cpu").manual_seed(5)
    feats = [torch.randn(16, c, s, s, generator=gen).to(dev).requires_grad_(True)
             for c, s in ((64, 80), (128, 40), (256, 20))]
    for it in range(4):
        outs, aux = h.forward_features(feats)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 64)()
        L.mcaq_read_wg_stamps(ctypes.cast(buf, ctypes.c_void_p))
        st = list(buf)
        t0 = min(st[:32])
        starts = [(x - t0) * 10 for x in st[:32]]          # ns
        ends = [(x - t0) * 10 for x in st[32:]]
        dur = [e - s for s, e in zip(starts, ends)]
        print("iter %d: start skew max %d ns; stage-1 end min %d max %d ns; stage-1 duration min %d max %d ns"
              % (it, max(starts), min(ends), max(ends), min(dur), max(dur)))
        if it == 3:
            print("per workgroup (start, end) ns:", list(zip(starts, ends)))


if __name__ == "__main__":
    main()
