"""Diagnose per-tensor hook mismatches on the GPU (pt_*.npz fixtures)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_fallback_cpu import hooks_per_tensor  # noqa: E402
from conftest import GOLDEN  # noqa: E402
for name in ("pt_odd", "pt_p3", "pt_p5"):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    for mapping in ("linear", "mlp"):
        key = "mlp" if mapping == "mlp" else "lin"
        res = {}
        for dev in ("cpu", "cuda"):
            h = hooks_per_tensor(dev, int(d["grid"]), mapping)
            x = torch.from_numpy(d["x"].astype(np.float32)).to(dev)
            with torch.no_grad():
                outs, aux = h.forward_features([x])
            res[dev] = outs[0].cpu().numpy()
            if dev == "cuda":
                b = list(h._plans.values())[0].bufs[0]
                print(name, mapping, "gpu xmin/xmax", b["xmin"][:3].tolist(), b["xmax"][:3].tolist(),
                      "ref", float(d["xmin"]), float(d["xmax"]))
        y = d["y_" + key]
        for dev in ("cpu", "cuda"):
            bad = np.argwhere(res[dev] != y)
            print("  ", dev, "mismatches", len(bad), bad[:5].tolist(),
                  [(float(res[dev][tuple(i)]), float(y[tuple(i)])) for i in bad[:5]])
