"""Round-3 golden fixtures: curriculum scoring, generated from the REFERENCE
itself (MorphologicalComplexityAnalyzer.score_image, morphology.py:923-937,
and fit_feature_weights, morphology.py:875-921) with the committed seeded
weights (tests/golden/weights.npz).

Run in the build container only (needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r03.py

Files written (DATA only; no reference source is copied):
  score_<name>.npz   x (fp16-representable inputs), grid, score0 (score_image
                     with the initial alpha = 1/5), alpha (fit_feature_weights
                     over the fit batches, float64), score1 (score_image after
                     the fit), fit_<k> (the fit batches)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _refload import load_reference  # noqa: E402
from make_golden import synth_features  # noqa: E402

torch.set_num_threads(8)
morph_mod, _, _ = load_reference()
Analyzer = morph_mod.MorphologicalComplexityAnalyzer

# name -> (B, C, H, W, grid, number of fit batches)
CASES = {"p3": (2, 16, 80, 80, 8, 2), "p5": (3, 32, 20, 20, 8, 2), "odd": (2, 20, 44, 52, 8, 1),
         "img": (2, 3, 128, 128, 8, 2)}


def analyzer(grid):
    w = np.load(os.path.join(HERE, "weights.npz"))
    sd = {k[len("complexity_analyzer."):]: torch.from_numpy(np.array(w[k])) for k in w.files
          if k.startswith("complexity_analyzer.")}
    a = Analyzer(device="cpu", grid_size=grid)
    a.load_state_dict(sd)
    return a.eval()


def make(name, B, C, H, W, grid, nfit, seed):
    if name == "img":
        # image-domain inputs in [0, 1] (score_image sorts the dataset's images)
        g = torch.Generator().manual_seed(seed)
        x = (torch.rand(B, C, H, W, generator=g) * 1024).round() / 1024
        fits = [((torch.rand(B, C, H, W, generator=g) * 1024).round() / 1024) for _ in range(nfit)]
    else:
        x = synth_features(B, C, H, W, seed=seed)
        fits = [synth_features(B, C, H, W, seed=seed + 1 + k) for k in range(nfit)]
    a = analyzer(grid)
    out = dict(grid=grid, x=x.numpy().astype(np.float16))
    for k, f in enumerate(fits):
        out["fit_%d" % k] = f.numpy().astype(np.float16)
    with torch.no_grad():
        out["score0"] = a.score_image(x).numpy()
        alpha = a.fit_feature_weights(iter(fits), max_batches=nfit)
        out["alpha"] = np.asarray(alpha, np.float64)
        out["feature_weights"] = a.feature_weights.numpy().copy()
        out["score1"] = a.score_image(x).numpy()
    assert np.array_equal(out["x"].astype(np.float32), x.numpy())
    np.savez_compressed(os.path.join(HERE, "score_%s.npz" % name), **out)
    print(name, "score0", out["score0"], "alpha", np.round(out["alpha"], 4), "score1", out["score1"])


def main():
    for i, (name, (B, C, H, W, grid, nfit)) in enumerate(CASES.items()):
        make(name, B, C, H, W, grid, nfit, 55000 + 100 * i)


if __name__ == "__main__":
    main()
