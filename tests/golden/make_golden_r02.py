"""Round-2 golden fixtures, generated from the REFERENCE itself with the
committed seeded weights (tests/golden/weights.npz, left unchanged).

Run in the build container only (needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r02.py

Files written (DATA only; no reference source is copied):
  case_m_p3.npz, case_m_p4.npz   yolov8m C3 / C4 shapes (192 x 80^2, 384 x 40^2),
                                 BASELINE config 4's per-GPU slice, same keys as
                                 make_golden.py's large cases (y head + channel sums)
  opt_<variant>_<shape>.npz      the analyzer switches the reference exposes
                                 (morphology.py:29-37): binarize_impl='otsu',
                                 contour_components=False, canny_impl='legacy'
  pt_<shape>.npz                 per_channel=False quantizer (quantization.py:655-661):
                                 one batch min/max over every channel; full y
                                 (`python make_golden_r02.py pertensor` writes only these)
  case_t128_c1.npz               1 x 1 x 1024^2 at grid 8: tile 128, the largest tile the
                                 analyzer kernel takes (`python make_golden_r02.py t128`
                                 writes only this); y as channel sums
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
morph_mod, bits_mod, quant_mod = load_reference()
Analyzer = morph_mod.MorphologicalComplexityAnalyzer
MLPMapper = bits_mod.ComplexityToBitMappingNetwork
LinMapper = bits_mod.LinearBitMapper
SAQ = quant_mod.SpatialAdaptiveQuantization

LARGE = {"m_p3": (2, 192, 80, 80, 8), "m_p4": (2, 384, 40, 40, 8)}
OPT_SHAPES = {"p3": (2, 16, 80, 80, 8), "p5": (3, 32, 20, 20, 8), "odd": (2, 20, 44, 52, 8),
              "g16": (2, 16, 80, 80, 16)}
VARIANTS = {"otsu": {"binarize_impl": "otsu"}, "noeuler": {"contour_components": False},
            "legacy": {"canny_impl": "legacy"}}


def modules(opts, per_channel=True):
    w = np.load(os.path.join(HERE, "weights.npz"))
    sd = {k: torch.from_numpy(np.array(w[k])) for k in w.files}

    def sub(prefix):
        return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}
    a = Analyzer(device="cpu", **opts)
    a.load_state_dict(sub("complexity_analyzer."))
    m = MLPMapper(2, 8)
    m.load_state_dict(sub("bit_mapper."))
    q = SAQ(calibration_mode="minmax", smooth_transitions=True, per_channel=per_channel)
    q.soft_mask.load_state_dict(sub("soft_mask."))
    return a.eval(), m.eval(), q.eval()


def run_case(x, grid, opts, full_y):
    a, mapper, q = modules(opts)
    a.grid_size = grid
    B, C, H, W = x.shape
    tile = a._tile_size(H)
    ht, wt = H // tile, W // tile
    out = dict(B=B, C=C, H=H, W=W, grid=grid, tile=tile, ht=ht, wt=wt, x=x.numpy().astype(np.float16))
    with torch.no_grad():
        gray = a._normalize01(x[:, :, :ht * tile, :wt * tile].mean(dim=1, keepdim=True).float())
        out["edge"] = a._gpu_canny(gray)[:, 0].numpy().astype(np.uint8)
        out["binmask"] = a._binarize(gray)[:, 0].numpy().astype(np.uint8)
        phi, _ = a.compute_phi_tiles(x)
        out["phi"] = phi.numpy()
        comp = a(x)
        out["complexity"] = comp.numpy()
        out["bits_mlp"] = mapper(comp, 1.0).numpy()
        out["bits_lin"] = LinMapper(2, 8)(comp, 1.0).numpy()
        out["xmin"] = x.amin(dim=(0, 2, 3)).numpy()
        out["xmax"] = x.amax(dim=(0, 2, 3)).numpy()
        for kind in ("mlp", "lin") if full_y is not None else ("mlp",):
            bm = torch.from_numpy(out["bits_" + kind])
            if full_y is not None:
                out["m_" + kind] = q.soft_mask(bm, x)[:, 0].numpy()
            y = q(x, bm, training=False)
            if full_y:
                out["y_" + kind] = y.numpy()
            elif full_y is None:
                out["y_%s_sum" % kind] = y.double().sum(dim=(2, 3)).numpy()
            else:
                out["y_%s_head" % kind] = y[:, :2].numpy().copy()
                out["y_%s_sum" % kind] = y.double().sum(dim=(2, 3)).numpy()
    return out


PT_SHAPES = {"p3": (2, 16, 80, 80, 8), "p5": (3, 32, 20, 20, 8), "odd": (2, 20, 44, 52, 8)}


def per_tensor():
    for si, (sname, (B, C, H, W, grid)) in enumerate(PT_SHAPES.items()):
        x = synth_features(B, C, H, W, seed=99000 + si)
        a, mapper, q = modules({}, per_channel=False)
        a.grid_size = grid
        out = dict(B=B, C=C, H=H, W=W, grid=grid, x=x.numpy().astype(np.float16))
        with torch.no_grad():
            comp = a(x)
            out["complexity"] = comp.numpy()
            for kind, mp in (("mlp", mapper), ("lin", LinMapper(2, 8))):
                bm = mp(comp, 1.0)
                out["bits_" + kind] = bm.numpy()
                out["y_" + kind] = q(x, bm, training=False).numpy()
        out["xmin"] = np.array(x.min().item(), np.float32)
        out["xmax"] = np.array(x.max().item(), np.float32)
        np.savez_compressed(os.path.join(HERE, "pt_%s.npz" % sname), **out)
        print("pt", sname, "bits", np.unique(out["bits_mlp"]).astype(int).tolist())


def t128():
    x = synth_features(1, 1, 1024, 1024, seed=66000)
    out = run_case(x, 8, {}, full_y=None)
    np.savez_compressed(os.path.join(HERE, "case_t128_c1.npz"), **out)
    print("t128_c1 tile", out["tile"], "bits", np.unique(out["bits_mlp"]).astype(int).tolist())


def main():
    if sys.argv[1:] == ["pertensor"]:
        return per_tensor()
    if sys.argv[1:] == ["t128"]:
        return t128()
    for i, (name, (B, C, H, W, grid)) in enumerate(LARGE.items()):
        x = synth_features(B, C, H, W, seed=77000 + i)
        out = run_case(x, grid, {}, full_y=False)
        np.savez_compressed(os.path.join(HERE, "case_%s.npz" % name), **out)
        print(name, "bits", np.unique(out["bits_mlp"]).astype(int).tolist())
    for vi, (vname, opts) in enumerate(VARIANTS.items()):
        for si, (sname, (B, C, H, W, grid)) in enumerate(OPT_SHAPES.items()):
            x = synth_features(B, C, H, W, seed=88000 + 10 * vi + si)
            out = run_case(x, grid, opts, full_y=None)   # bits are the point: y as channel sums only
            for k, v in opts.items():
                out["opt_" + k] = np.array(v)
            np.savez_compressed(os.path.join(HERE, "opt_%s_%s.npz" % (vname, sname)), **out)
            print(vname, sname, "bits", np.unique(out["bits_mlp"]).astype(int).tolist())
    per_tensor()
    t128()


if __name__ == "__main__":
    main()
