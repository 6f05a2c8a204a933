"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run in the build container only (needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference's pure-PyTorch tensor path (morphology.py "gpu" backend,
bit_allocation.py, quantization.py `_forward_pytorch`) is executed on CPU
(torch 2.10.0) and its inputs/outputs are written as .npz DATA files.  No
reference source is copied; the GPU box only ever sees the .npz files.

Files written:
  weights.npz    seeded state dicts (reference key names) for the complexity
                 MLP, the bit-mapping MLP (BN running stats calibrated on the
                 fixture complexity maps so bits span 2..8) and the soft mask
  constants.npz  the constant kernels/tables the reference builds at run time
  case_<name>.npz  one file per input case (see CASES)
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _refload import load_reference  # noqa: E402

torch.set_num_threads(8)
morph_mod, bits_mod, quant_mod = load_reference()
Analyzer = morph_mod.MorphologicalComplexityAnalyzer
MLPMapper = bits_mod.ComplexityToBitMappingNetwork
LinMapper = bits_mod.LinearBitMapper
SAQ = quant_mod.SpatialAdaptiveQuantization
SoftMask = quant_mod.LearnedSoftMask

# name: (B, C, H, W, grid_size, store_full_y)
CASES = {
    "p3_c16":   (2, 16, 80, 80, 8, True),     # tile 8, 10x10 grid
    "p4_c32":   (2, 32, 40, 40, 8, True),     # tile 4, 10x10
    "p5_c32":   (3, 32, 20, 20, 8, True),     # tile 4, 5x5 (25 tiles < 32: ATen tail sums)
    "g16_c16":  (2, 16, 80, 80, 16, True),    # tile 4, 20x20 (config-3 grid)
    "crop_c8":  (2, 8, 100, 100, 8, True),    # tile 8, 12x12 grid, 96x96 crop
    "rect_c8":  (2, 8, 64, 96, 8, True),      # H != W: tile from H only
    "t32_c4":   (2, 4, 320, 320, 8, False),   # tile 32: 5 box-count scales
    "t64_c1":   (2, 1, 640, 640, 8, False),   # tile 64 (reference test_phi_tiles_shapes H=640)
    "odd_c20":  (2, 20, 44, 52, 8, True),     # C % 4 != 0, HW % 32 != 0
    "b1_c16":   (1, 16, 40, 40, 8, True),     # batch 1 (CPU conv path differs at B=1)
    "full_p3":  (2, 64, 80, 80, 8, False),    # yolov8n C3 shape
    "full_p4":  (2, 128, 40, 40, 8, False),   # yolov8n C4 shape
    "full_p5":  (2, 256, 20, 20, 8, False),   # yolov8n C5 shape
    "m_p5":     (2, 576, 20, 20, 8, False),   # yolov8m C5 channel count
}


def synth_features(B, C, H, W, seed):
    """silu(1.5*randn + 2*bilinear_up(randn(B,C,H/8,W/8))), rounded to
    fp16-representable fp32 values so the stored fp16 input is exact."""
    g = torch.Generator().manual_seed(seed)
    lo = torch.randn(B, C, max(1, H // 8), max(1, W // 8), generator=g)
    hi = torch.randn(B, C, H, W, generator=g)
    up = F.interpolate(lo, size=(H, W), mode="bilinear", align_corners=False)
    x = F.silu(1.5 * hi + 2.0 * up)
    return x.half().float().contiguous()


def state_np(module, prefix):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def build_weights(sample_complexities):
    torch.manual_seed(1234)
    analyzer = Analyzer(grid_size=8, device="cpu")
    torch.manual_seed(4321)
    mapper = MLPMapper(min_bits=2, max_bits=8)
    # Seeded mapper whose bits span 2..8 on the fixture scales.  A fresh init
    # saturates at 8 bits; instead (1) shift every BN beta to +3 so the ReLUs
    # stay active over the calibration range (the monotone net is then close
    # to linear in C), (2) calibrate BN running stats on C values sampled
    # uniformly over the fixture range, (3) rescale/re-bias the final layer so
    # the sigmoid input has mean 0 and std 3.5 over that range.
    allc = torch.cat([t.reshape(-1) for t in sample_complexities])
    c = torch.linspace(float(allc.min()), float(allc.max()), 4096).reshape(-1, 1, 1)
    for m in mapper.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            m.reset_running_stats()
            m.momentum = None
            with torch.no_grad():
                m.bias.fill_(3.0)
    mapper.train()
    with torch.no_grad():
        mapper(c)
    mapper.eval()
    net = mapper.mapping_network
    feats = {}
    h = net[-2].register_forward_hook(lambda mod, i, o: feats.__setitem__("z", i[0]))
    with torch.no_grad():
        mapper(c)
    h.remove()
    h3 = feats["z"]
    with torch.no_grad():
        z = h3 @ net[-2].weight.t()
        net[-2].weight.mul_(3.5 / float(z.std().clamp(min=1e-6)))
        net[-2].bias.fill_(-float((h3 @ net[-2].weight.t()).mean()))
    torch.manual_seed(99)
    sm = SoftMask()
    with torch.no_grad():  # widen the near-identity init so m(p) varies visibly
        sm.net[-1].weight.normal_(0.0, 0.5)
    return analyzer, mapper, sm


def main():
    os.makedirs(HERE, exist_ok=True)
    # pass 1: inputs + complexity maps with the seeded analyzer
    torch.manual_seed(1234)
    analyzer0 = Analyzer(grid_size=8, device="cpu")
    cmlp_state = {k: v.clone() for k, v in analyzer0.state_dict().items()}
    inputs, comps = {}, []
    for i, (name, (B, C, H, W, grid, _)) in enumerate(CASES.items()):
        x = synth_features(B, C, H, W, seed=1000 * (i + 1) + 4)
        inputs[name] = x
        a = Analyzer(grid_size=grid, device="cpu")
        a.load_state_dict(cmlp_state)
        a.eval()
        with torch.no_grad():
            comps.append(a(x))
    analyzer, mapper, sm = build_weights(comps)
    assert all(torch.equal(analyzer.state_dict()[k], cmlp_state[k]) for k in cmlp_state)

    wts = {}
    wts.update(state_np(analyzer, "complexity_analyzer."))
    wts.update(state_np(mapper, "bit_mapper."))
    wts.update(state_np(sm, "soft_mask."))
    np.savez(os.path.join(HERE, "weights.npz"), **wts)

    # constants the reference builds at run time (CPU values)
    consts = {}
    x1 = torch.arange(5, dtype=torch.float32) - 2
    g1 = torch.exp(-(x1 ** 2) / 2.0)
    g1 = g1 / g1.sum()
    consts["gauss5_canny"] = (g1.unsqueeze(0) * g1.unsqueeze(1)).numpy()
    k = 11
    sigma = 0.3 * ((k - 1) * 0.5 - 1) + 0.8
    xk = torch.arange(k, dtype=torch.float32) - k // 2
    gk = torch.exp(-(xk ** 2) / (2 * sigma ** 2))
    gk = gk / gk.sum()
    consts["gauss11_adaptive"] = (gk.unsqueeze(0) * gk.unsqueeze(1)).numpy()
    consts["smooth5_softmask"] = sm.smooth_kernel.reshape(5, 5).numpy()
    coords = torch.arange(5, dtype=torch.float32) - 2
    yy, xx = torch.meshgrid(coords, coords, indexing="ij")
    consts["bilateral_spatial"] = torch.exp(-(yy ** 2 + xx ** 2) / (2 * 2.0 ** 2)).numpy()
    np.savez(os.path.join(HERE, "constants.npz"), **consts)

    total = 0
    for name, (B, C, H, W, grid, full_y) in CASES.items():
        x = inputs[name]
        a = Analyzer(grid_size=grid, device="cpu")
        a.load_state_dict(analyzer.state_dict())
        a.eval()
        tile = a._tile_size(H)
        ht, wt = H // tile, W // tile
        Hc, Wc = ht * tile, wt * tile
        out = dict(B=B, C=C, H=H, W=W, grid=grid, tile=tile, ht=ht, wt=wt)
        out["x"] = x.numpy().astype(np.float16)
        with torch.no_grad():
            xc = x[:, :, :Hc, :Wc]
            graw = xc.mean(dim=1, keepdim=True).float()
            gray = a._normalize01(graw)
            gx, gy = a._sobel(gray)
            planes = Hc * Wc <= 10000  # float planes only for small maps
            if planes:
                out["gray_raw"] = graw[:, 0].numpy()
                out["gray"] = gray[:, 0].numpy()
                out["gx"] = gx[:, 0].numpy()
                out["gy"] = gy[:, 0].numpy()
            # canny internals (morphology.py:458-509)
            x1 = torch.arange(5, dtype=torch.float32) - 2
            g1 = torch.exp(-(x1 ** 2) / 2.0)
            g1 = g1 / g1.sum()
            g2 = (g1.unsqueeze(0) * g1.unsqueeze(1)).view(1, 1, 5, 5)
            b01 = F.conv2d(gray, g2, padding=2)
            if planes:
                out["blur"] = b01[:, 0].numpy()
            out["otsu_thr"] = a._otsu_threshold(b01).reshape(-1).numpy()
            edge = a._gpu_canny(gray)
            binm = a._binarize(gray)
            out["edge"] = edge[:, 0].numpy().astype(np.uint8)
            out["binmask"] = binm[:, 0].numpy().astype(np.uint8)
            phi, det = a.compute_phi_tiles(x)
            out["phi"] = phi.numpy()
            out["c_mlp"] = a.complexity_mlp(phi.reshape(-1, 8)).reshape(B, ht, wt).numpy()
            comp = a(x)
            out["complexity"] = comp.numpy()
            for T in (1.0, 10.0):
                sfx = "" if T == 1.0 else "_t10"
                out["bits_mlp_cont" + sfx] = mapper(comp, T, return_continuous=True).numpy()
                out["bits_mlp" + sfx] = mapper(comp, T, return_continuous=False).numpy()
            lin = LinMapper(2, 8)
            out["bits_lin_cont"] = lin(comp, 1.0, return_continuous=True).numpy()
            out["bits_lin"] = lin(comp, 1.0, return_continuous=False).numpy()

            q = SAQ(calibration_mode="minmax", smooth_transitions=True, per_channel=True)
            q.soft_mask.load_state_dict(sm.state_dict())
            q.eval()
            out["xmin"] = x.amin(dim=(0, 2, 3)).numpy()
            out["xmax"] = x.amax(dim=(0, 2, 3)).numpy()
            for kind in ("mlp", "lin"):
                bm = torch.from_numpy(out["bits_" + kind])
                m = q.soft_mask(bm, x)
                out["m_" + kind] = m[:, 0].numpy()
                y = q(x, bm, training=False)
                if full_y:
                    out["y_" + kind] = y.numpy()
                else:
                    out["y_%s_head" % kind] = y[:, :2].numpy().copy()
                    out["y_%s_sum" % kind] = y.double().sum(dim=(2, 3)).numpy()
            if full_y:
                q2 = SAQ(smooth_transitions=False)
                q2.eval()
                out["y_nomask"] = q2(x, torch.from_numpy(out["bits_mlp"]), training=False).numpy()
        path = os.path.join(HERE, "case_%s.npz" % name)
        np.savez_compressed(path, **out)
        sz = os.path.getsize(path)
        total += sz
        bl = out["bits_lin"]
        bmv = out["bits_mlp"]
        print("%-9s tile=%2d grid=%2dx%-2d  mlp bits %s  lin bits %s  %.2f MB" % (
            name, tile, ht, wt, np.unique(bmv).astype(int).tolist(),
            np.unique(bl).astype(int).tolist(), sz / 1e6))
    print("total %.2f MB" % (total / 1e6))


if __name__ == "__main__":
    main()
