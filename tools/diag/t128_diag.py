"""Dump the hook path's m(p), bits and y for case_t128_c1 (diagnostic)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import test_gpu_parity as P  # noqa: E402
from conftest import load_case  # noqa: E402

d = load_case("t128_c1")
x = d["x"].astype(np.float32)
blobs = P.blobs.__wrapped__("cuda") if hasattr(P.blobs, "__wrapped__") else None
if blobs is None:
    import torch
    from mcaq_yolo_amd import params
    from conftest import load_weights
    W = load_weights()
    blobs = (W, torch.from_numpy(params.pack_complexity_mlp(params.sub(W, "complexity_analyzer."))).cuda(),
             torch.from_numpy(params.pack_mapper_mlp(params.sub(W, "bit_mapper."))).cuda(),
             torch.from_numpy(params.pack_soft_mask(params.sub(W, "soft_mask."))).cuda())
out = P.run_plan("cuda", blobs, [x], 8, "mlp")[0]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "t128_out.npz"), m=out["m"], y=out["y"], bits=out["bits"])
print("saved")
