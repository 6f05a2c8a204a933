"""Dataset curriculum scoring on the HIP path against
the reference's own compute_dataset_complexity (tests/golden/
dataset_scores.npz): phi of every image bit-exact vs its batch-1 call (one
launch per batch with the F_IMAGE_BATCH flag) and vs the oracle; scores
within rtol 1e-6 (the 5-term dot and the tile mean are device reductions in
another fp32 order than CPU ATen, as test_core_gpu.test_score_and_fit_vs_
reference_fixture)."""
import numpy as np
import pytest
import torch

from oracle import mcaq_oracle as O
from test_dataset_cpu import D, IMGS, items
from test_score_cpu import analyzer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("bs", [1, 3, 32])
def test_compute_dataset_complexity_hip_vs_reference(tmp_path, bs):
    from mcaq_yolo_amd.dataset import compute_dataset_complexity
    a = analyzer(DEV, int(D["grid"]))
    path = str(tmp_path / "s.npy")
    out = compute_dataset_complexity(items(), model=a, batch_size=bs, device=DEV, save_path=path, verbose=False)
    np.testing.assert_allclose(out, D["scores"], rtol=1e-6, atol=1e-7)
    assert np.array_equal(np.load(path), out)


def test_image_batch_phi_equals_batch1_calls_and_oracle():
    """One launch over a batch with every image as its own batch of one ==
    the per-image calls, bit for bit, and == the oracle's batch-1 phi; the
    plain batch call differs only where the reference's own batch call does
    (the fractal regression's position-dependent reduction order)."""
    a = analyzer(DEV, 8)
    x = np.stack([im for im in IMGS if im.shape == (3, 128, 128)]).astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    phi_b, _ = a.compute_phi_tiles(xd, image_batch=True)
    for i in range(x.shape[0]):
        phi_1, _ = a.compute_phi_tiles(xd[i:i + 1])
        assert torch.equal(phi_b[i:i + 1], phi_1), "image %d" % i
        assert np.array_equal(phi_1.cpu().numpy(), O.phi_tiles(x[i:i + 1], 8))
    phi_all, _ = a.compute_phi_tiles(xd)
    assert np.array_equal(phi_all.cpu().numpy(), O.phi_tiles(x, 8))


def test_dataset_scoring_640_throughput_smoke():
    """640 x 640 images (the metric's resolution: tile 64, planes in global
    scratch) through the batched scorer: finite scores in [0, 1], and the
    first image equal to its batch-1 score."""
    from mcaq_yolo_amd.dataset import score_batch
    a = analyzer(DEV, 8)
    g = torch.Generator(device="cpu").manual_seed(3)
    x = (torch.rand(8, 3, 640, 640, generator=g) * 255).round().to(DEV)
    s = score_batch(a, x)
    s1 = score_batch(a, x[:1])
    torch.cuda.synchronize()
    assert s.shape == (8,) and bool(torch.isfinite(s).all()) and bool(((s >= 0) & (s <= 1)).all())
    np.testing.assert_allclose(s[:1].cpu().numpy(), s1.cpu().numpy(), rtol=1e-6)
