"""Round-6 golden fixtures: the REFERENCE's hook modules on fp16 / bf16
feature maps (what an autocast region hands the hooks, train.py:582-585,
748-749), CPU, with the committed seeded weights.

The analyzer upcasts (`features.float()`, morphology.py:834-837), so its
complexity and the bits are those of the fp32 map.  The quantizer's
inference branch (_forward_pytorch, quantization.py:729-746) then runs its
elementwise ops in the input's dtype - per-op rounding to fp16 / bf16 of the
scale, zero point, x / scale + zp and the dequantized value - and the fp32
soft mask promotes the product to fp32.  (The reference's CUDA op raises on a
half input: data_ptr<float>, mcaq_ops.cpp:50.)

Run in the build container only (needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r06.py

Writes tests/golden/amp_<shape>.npz: x (the map, fp16-representable values),
complexity, bits_mlp, and for dt in (f16, bf16): y_<dt> (the reference's
output as float32), y_<dt>_dtype (its dtype name).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import synth_features  # noqa: E402
from make_golden_r02 import modules  # noqa: E402   (reference analyzer / mapper / quantizer, seeded)

torch.set_num_threads(8)
SHAPES = {"p3": (2, 16, 80, 80, 8), "p4": (2, 32, 40, 40, 8), "p5": (3, 32, 20, 20, 8)}


def main():
    for si, (name, (B, C, H, W, grid)) in enumerate(SHAPES.items()):
        x = synth_features(B, C, H, W, seed=606000 + si)
        xb = x.to(torch.bfloat16).float()            # bf16-representable copy for the bf16 case
        a, mapper, q = modules({})
        a.grid_size = grid
        out = dict(B=B, C=C, H=H, W=W, grid=grid, x=x.numpy().astype(np.float16),
                   x_bf16=xb.numpy().astype(np.float32))
        with torch.no_grad():
            for dt, xs in (("f16", x.half()), ("bf16", xb.to(torch.bfloat16))):
                comp = a(xs)
                bits = mapper(comp, 1.0)
                y = q(xs, bits, training=False)
                out["complexity_" + dt] = comp.numpy()
                out["bits_" + dt] = bits.numpy()
                out["y_" + dt] = y.float().numpy()
                out["y_%s_dtype" % dt] = np.array(str(y.dtype))
        np.savez_compressed(os.path.join(HERE, "amp_%s.npz" % name), **out)
        print(name, "bits", np.unique(out["bits_f16"]).astype(int).tolist(), "y dtype", out["y_f16_dtype"],
              out["y_bf16_dtype"])


if __name__ == "__main__":
    main()
