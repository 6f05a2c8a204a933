"""Probe: 50 x mcaq_qat_backward at config 5's three scales (bench QAT shapes),
for a rocprofv3 kernel trace of the quantizer + fold dispatches."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mcaq_yolo_amd import abi, core  # noqa: E402

dev = torch.device("cuda:0")
B, chans, SIZES = 16, (64, 128, 256), ((80, 80), (40, 40), (20, 20))
L = abi.lib()
sh = abi.ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
xs = [torch.randn(B, c, h, w, device=dev) for c, (h, w) in zip(chans, SIZES)]
G = [torch.randn_like(x) * 1e-3 for x in xs]
bits = [torch.rand(B, 10 if h > 20 else 5, 10 if h > 20 else 5, device=dev) * 6 + 2 for (h, w) in SIZES]
ms = [torch.rand(B, h, w, device=dev) for (h, w) in SIZES]
mm = [core._channel_minmax(x) for x in xs]
keep = []
arr = (abi.QatScale * 3)()
for i in range(3):
    q = core._qat_struct(xs[i], bits[i], ms[i], mm[i][0], mm[i][1])
    gx, gm, gb = torch.empty_like(xs[i]), torch.empty_like(ms[i]), torch.empty_like(bits[i])
    work = torch.empty(L.mcaq_qat_work_floats(*xs[i].shape), device=dev)
    keep += [gx, gm, gb, work]
    q.g, q.gx, q.gm, q.gb, q.work = core._p(G[i]), core._p(gx), core._p(gm), core._p(gb), core._p(work)
    arr[i] = q
for _ in range(50):
    abi.check(L.mcaq_qat_backward(arr, 3, sh), "bwd")
torch.cuda.synchronize()
print("ok")
