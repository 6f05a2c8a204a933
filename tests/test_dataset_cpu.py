"""Dataset curriculum scoring: the package's
compute_dataset_complexity against the reference's own
compute_dataset_complexity run on a small image dataset
(tests/golden/dataset_scores.npz, make_golden_r05.py: batch-1 calls, mixed
shapes, [0, 1] and 0..255 images).  The pure-PyTorch path issues the
reference's ATen ops per image and is bit-exact for any batch_size; the
float64 oracle (batch-1 phi) agrees within fp32 reduction-order rounding."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import mcaq_oracle as O
from test_score_cpu import analyzer

D = np.load(os.path.join(GOLDEN, "dataset_scores.npz"))
IMGS = [D["img_%d" % i] for i in range(len([k for k in D.files if k.startswith("img_")]))]


def items():
    return [{"img": torch.from_numpy(im.copy()), "cls": torch.zeros(0)} for im in IMGS]


def test_fixture_self_consistent():
    assert np.array_equal(D["scores"], D["saved"])
    assert D["scores"].dtype == np.float32 and D["scores"].shape == (len(IMGS),)


def test_oracle_batch1_scores_vs_reference():
    got = []
    for im in IMGS:
        x = im[None].astype(np.float32)
        if x.max() > 1.5:
            x = (x / np.float32(255.0)).astype(np.float32)
        got.append(O.score_image(x, int(D["grid"]))[0])
    np.testing.assert_allclose(np.array(got, np.float32), D["scores"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("bs", [1, 4, 32])
def test_compute_dataset_complexity_cpu_bit_exact(tmp_path, bs):
    from mcaq_yolo_amd.dataset import compute_dataset_complexity
    a = analyzer("cpu", int(D["grid"]))
    path = str(tmp_path / "scores.npy")
    out = compute_dataset_complexity(items(), model=a, batch_size=bs, device="cpu", save_path=path, verbose=False)
    assert out.dtype == np.float32
    assert np.array_equal(out, D["scores"])
    assert np.array_equal(np.load(path), out)


def test_compute_dataset_complexity_item_forms():
    """(img, label) tuples and (1, C, H, W) images are taken as the reference
    takes them (dataset.py:337-344); a model object holding the analyzer."""
    from mcaq_yolo_amd.dataset import compute_dataset_complexity

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.complexity_analyzer = analyzer("cpu", int(D["grid"]))
    tup = [(torch.from_numpy(im.copy())[None], None) for im in IMGS[:4]]
    out = compute_dataset_complexity(tup, model=M(), batch_size=3, device="cpu", verbose=False)
    assert np.array_equal(out, D["scores"][:4])


def test_compute_dataset_complexity_without_analyzer_needs_cv2():
    from mcaq_yolo_amd.dataset import compute_dataset_complexity
    with pytest.raises(NotImplementedError):
        compute_dataset_complexity(items(), model=None, device="cpu", verbose=False)
    with pytest.raises(NotImplementedError):
        compute_dataset_complexity([(IMGS[0], None)], model=analyzer("cpu", 8), device="cpu", verbose=False)
