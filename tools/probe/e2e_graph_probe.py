"""Probe: e2e graph replay vs eager (test_mcaq_yolo_graph_capture_and_nms)
with and without the one-launch device blob packing."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_e2e_gpu as T  # noqa: E402
from mcaq_yolo_amd import core  # noqa: E402
from mcaq_yolo_amd.postprocess import nms_padded  # noqa: E402

orig = core._device_pack
for variant in ("device_pack", "torch_pack"):
    core._device_pack = orig if variant == "device_pack" else (lambda *a, **k: None)
    m = T._mcaq_yolo("mlp")
    x = torch.rand(2, 3, 256, 256, generator=torch.Generator().manual_seed(5)).to(T.DEV)

    def step():
        (y, _), aux = m(x)
        out, cnt = nms_padded(y, 0.001, 0.45, 300)
        return y, out, cnt, aux["bit_map"][0], aux["bit_map"][1], aux["bit_map"][2], aux["complexity_map"][0]

    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step(); step()
        torch.cuda.current_stream().wait_stream(s)
        ref = [t.clone() for t in step()]
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            outs = step()
        graph.replay()
        torch.cuda.synchronize()
        again = [t.clone() for t in step()]
    names = ("y", "nms", "cnt", "bits3", "bits4", "bits5", "C3")
    print(variant, {n: (bool(torch.equal(a, b)), bool(torch.equal(a, c))) for n, a, b, c in zip(names, ref, outs, again)},
          flush=True)
