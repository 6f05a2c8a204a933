"""Zero-edit drop-in by the reference's module name: a fresh process runs
`import mcaq_cuda_ops` (no install(), only this repository on the Python path,
as the reference's `try: import mcaq_cuda_ops` at quantization.py:14-16 would)
and calls `spatial_quantize` with exactly the arguments the reference's
`SpatialAdaptiveQuantization._forward_cuda` builds (quantization.py:636-679):
(1, C, 1, 1) min / max - per-channel batch statistics, per-tensor ones
expanded to C, frozen running statistics - a float bit map (B, Ht, Wt) and
the (B, 1, H, W) soft mask.  Outputs are compared bit for bit with the
oracle's restatement of that contract (oracle.spatial_quantize_compat)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import mcaq_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, numpy as np, torch
import mcaq_cuda_ops                                   # resolves to the repository's top-level module
assert "mcaq_yolo_amd" in mcaq_cuda_ops.spatial_quantize.__module__
out = {}
g = torch.Generator(device="cpu").manual_seed(5)
for case, (B, C, H, W, Ht, Wt) in enumerate([(2, 16, 40, 40, 5, 5), (3, 24, 42, 37, 5, 4), (1, 64, 80, 80, 10, 10)]):
    x = (1.5 * torch.randn(B, C, H, W, generator=g)).cuda()
    bit_map = (torch.rand(B, Ht, Wt, generator=g) * 7 + 1.6).cuda()      # float, rounded by the op
    m = (0.9 + 0.1 * torch.rand(B, 1, H, W, generator=g)).cuda()
    tile_h, tile_w = H // Ht, W // Wt                                   # quantization.py:640-641
    stats = {
        "per_channel": (x.amin(dim=(0, 2, 3), keepdim=True), x.amax(dim=(0, 2, 3), keepdim=True)),
        "per_tensor": (x.min().reshape(1, 1, 1, 1).expand(1, C, 1, 1), x.max().reshape(1, 1, 1, 1).expand(1, C, 1, 1)),
        "frozen": ((x.amin(dim=(0, 2, 3)) * 0.8).reshape(1, -1, 1, 1), (x.amax(dim=(0, 2, 3)) * 0.8).reshape(1, -1, 1, 1)),
    }
    for name, (x_min, x_max) in stats.items():
        for mask in (m, None):
            y = mcaq_cuda_ops.spatial_quantize(x.contiguous(), bit_map.float().contiguous(),
                                               x_min.float().contiguous(), x_max.float().contiguous(),
                                               tile_h, tile_w, mask)
            key = "%d_%s_%s" % (case, name, "m" if mask is not None else "nom")
            out[key + "_y"] = y.cpu().numpy()
            out[key + "_x"] = x.cpu().numpy()
            out[key + "_b"] = bit_map.cpu().numpy()
            out[key + "_mn"] = x_min.float().contiguous().cpu().numpy()
            out[key + "_mx"] = x_max.float().contiguous().cpu().numpy()
            out[key + "_t"] = np.array([tile_h, tile_w])
            if mask is not None:
                out[key + "_m"] = mask.cpu().numpy()
try:
    mcaq_cuda_ops.spatial_quantize(x, bit_map, x_min[:, :1], x_max, tile_h, tile_w, None)
    raise SystemExit("wrong-size min_vals accepted")
except RuntimeError as e:
    assert "one entry per channel" in str(e)
np.savez(sys.argv[1], **out)
print("child ok", len(out))
'''


def test_import_by_reference_name_fresh_process(tmp_path):
    path = str(tmp_path / "out.npz")
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD, path], cwd=str(tmp_path), env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = np.load(path)
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files})
    assert len(keys) == 18
    for k in keys:
        th, tw = (int(v) for v in d[k + "_t"])
        want = O.spatial_quantize_compat(d[k + "_x"], d[k + "_b"], d[k + "_mn"], d[k + "_mx"], th, tw,
                                         d[k + "_m"] if (k + "_m") in d.files else None)
        assert np.array_equal(d[k + "_y"], want), k
