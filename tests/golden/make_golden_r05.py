"""Round-5 golden fixture: curriculum scores of a small image dataset from the
REFERENCE's own `compute_dataset_complexity` (mcaq_yolo/utils/dataset.py:
276-401), preferred (tensor) path: one image at a time, `/ 255` for images
whose max exceeds 1.5, `analyzer.score_image(x).mean().item()` with the
committed seeded analyzer weights (tests/golden/weights.npz), device "cpu".

utils/dataset.py imports cv2 at module top (:10) for its edge-density
fallback only; the cv2 stub of _refload.py raises on any use, so the
fallback can never produce these values.  Loaded by file path.

Run in the build container only (needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r05.py

Writes tests/golden/dataset_scores.npz: img_<i> (the dataset's images, in
order; shapes and value ranges mixed), scores (the reference's float32
array), saved (np.load of the reference's own save_path file).
"""
import importlib.util
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _refload import _install_stubs, load_reference  # noqa: E402
from make_golden_r03 import analyzer  # noqa: E402   (the reference analyzer, seeded weights)

torch.set_num_threads(8)


def dataset_images():
    g = torch.Generator().manual_seed(505)
    imgs = []
    for _ in range(3):          # [0, 1] images, 128 x 128
        imgs.append((torch.rand(3, 128, 128, generator=g) * 1024).round() / 1024)
    for _ in range(3):          # 0..255 images (divided by 255 inside), 96 x 160
        imgs.append(torch.randint(0, 256, (3, 96, 160), generator=g).float())
    imgs.append((torch.rand(3, 64, 64, generator=g) * 1024).round() / 1024)
    for _ in range(2):          # 128 x 128 again after a shape change
        imgs.append((torch.rand(3, 128, 128, generator=g) * 1024).round() / 1024)
    # a smoothed image (a larger-scale structure than uniform noise)
    lo = torch.rand(1, 3, 16, 16, generator=g)
    imgs.append((torch.nn.functional.interpolate(lo, size=(128, 128), mode="bilinear")[0] * 1024).round() / 1024)
    return imgs


def main():
    load_reference()            # stubs + the morphology module the analyzer comes from
    _install_stubs()
    spec = importlib.util.spec_from_file_location("ref_dataset", "/root/reference/mcaq_yolo/utils/dataset.py")
    ds_mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ds_mod)
    imgs = dataset_images()
    items = [{"img": im, "cls": torch.zeros(0)} for im in imgs]
    a = analyzer(8)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "scores.npy")
        scores = ds_mod.compute_dataset_complexity(items, model=a, device="cpu", save_path=path)
        saved = np.load(path)
    out = {"img_%d" % i: im.numpy() for i, im in enumerate(imgs)}
    out["scores"] = np.asarray(scores, np.float32)
    out["saved"] = saved
    out["grid"] = 8
    np.savez_compressed(os.path.join(HERE, "dataset_scores.npz"), **out)
    print("scores", out["scores"])


if __name__ == "__main__":
    main()
