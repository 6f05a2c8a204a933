"""Curriculum scoring (morphology.py:875-937) pinned to the reference's own
outputs (tests/golden/make_golden_r03.py): the package's pure-PyTorch path
issues the reference's ATen ops on the same shapes and is bit-exact for the
scores, and its NNLS alpha equals the reference's; the float64 oracle agrees
within fp32 reduction-order rounding (rtol 1e-6)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_weights
from oracle import mcaq_oracle as O

CASES = sorted(f[6:-4] for f in os.listdir(GOLDEN) if f.startswith("score_") and f.endswith(".npz"))


def analyzer(dev, grid):
    from mcaq_yolo_amd import core
    w = load_weights()
    a = core.MorphologicalComplexityAnalyzer(device=dev, grid_size=grid)
    a.load_state_dict({k[len("complexity_analyzer."):]: torch.from_numpy(np.asarray(v)) for k, v in w.items()
                       if k.startswith("complexity_analyzer.")})
    return a.to(dev).eval()


def load(name):
    d = np.load(os.path.join(GOLDEN, "score_%s.npz" % name))
    fits = [d["fit_%d" % k].astype(np.float32) for k in range(len([f for f in d.files if f.startswith("fit_")]))]
    return d, d["x"].astype(np.float32), fits


@pytest.mark.parametrize("name", CASES)
def test_score_and_fit_cpu_path_bit_exact(name):
    d, x, fits = load(name)
    a = analyzer("cpu", int(d["grid"]))
    s0 = a.score_image(torch.from_numpy(x)).numpy()
    assert np.array_equal(s0, d["score0"])
    alpha = a.fit_feature_weights(iter(torch.from_numpy(f) for f in fits), max_batches=len(fits))
    np.testing.assert_allclose(alpha, d["alpha"], rtol=0, atol=1e-12)
    assert np.array_equal(a.feature_weights.numpy(), d["feature_weights"])
    assert np.array_equal(a.score_image(torch.from_numpy(x)).numpy(), d["score1"])


@pytest.mark.parametrize("name", CASES)
def test_score_oracle_vs_reference(name):
    d, x, _ = load(name)
    np.testing.assert_allclose(O.score_image(x, int(d["grid"])), d["score0"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(O.score_image(x, int(d["grid"]), d["feature_weights"]), d["score1"],
                               rtol=1e-6, atol=1e-7)
