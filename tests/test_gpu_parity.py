"""GPU parity: the HIP path (through the C ABI) against the golden fixtures and
the oracle.  Bit-exact everywhere the oracle is bit-exact:

  gray, edge map, adaptive mask, phi, complexity, bits, m, channel min/max, y

(the oracle reproduces the reference exactly on the decision path; against the
fixtures themselves complexity is within 1e-6 relative and phi8 within 1 ulp,
see test_oracle_cpu.py).  Tolerances are written where they apply.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, case_names, load_case, load_weights
from oracle import mcaq_oracle as O

pytestmark = pytest.mark.gpu
f32 = np.float32


@pytest.fixture(scope="module")
def dev():
    import torch
    from mcaq_yolo_amd import abi
    abi.lib()   # fails loudly if the library is missing
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def blobs(dev):
    import torch
    from mcaq_yolo_amd import params
    W = load_weights()
    cm = torch.from_numpy(params.pack_complexity_mlp(params.sub(W, "complexity_analyzer."))).to(dev)
    mm = torch.from_numpy(params.pack_mapper_mlp(params.sub(W, "bit_mapper."))).to(dev)
    sm = torch.from_numpy(params.pack_soft_mask(params.sub(W, "soft_mask."))).to(dev)
    return W, cm, mm, sm


def run_plan(dev, blobs, xs, grid, mapper="mlp", T=1.0, **kw):
    import torch
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    W, cm, mm, sm = blobs
    feats = [torch.from_numpy(x).to(dev) for x in xs]
    geoms = [ScaleGeom(*f.shape, grid) for f in feats]
    plan = HookPlan(geoms, dev, want=("phi", "cmlp", "debug"))
    bufs = plan.run(feats, cm, mm, [sm] * len(feats), temperature=T, mapper_kind=mapper, **kw)
    torch.cuda.synchronize()
    return [{k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in b.items()} for b in bufs]


def check_against_oracle(out, x, W, grid, mapper, T=1.0):
    ref = O.hook_forward(x, W, grid, mapper=mapper, temperature=T)
    B, C, H, Wd = x.shape
    tile = O.tile_size(H, grid)
    Hc, Wc = (H // tile) * tile, (Wd // tile) * tile
    _, I = O.phi_tiles(x, grid, internals=True)
    assert np.array_equal(out["gray"], I["gray_raw"]), "gray"
    assert np.array_equal(out["absmean"], O.abs_channel_mean(x)), "absmean"
    assert np.array_equal(out["edge"], I["edge"]), "edge"
    assert np.array_equal(out["binmask"], I["binmask"]), "binmask"
    assert np.array_equal(out["phi"], ref["phi"]), "phi"
    assert np.array_equal(out["cmlp"], ref["c_mlp"]), "complexity MLP"
    assert np.array_equal(out["complexity"], ref["complexity"]), "complexity"
    assert np.array_equal(out["bits"], ref["bits"]), "bits"
    assert np.array_equal(out["xmin"], ref["xmin"]) and np.array_equal(out["xmax"], ref["xmax"]), "minmax"
    assert np.array_equal(out["m"][:, 0], ref["m"]), "soft mask"
    assert np.array_equal(out["y"], ref["y"]), "y"
    return ref


@pytest.mark.parametrize("name", [c for c in case_names() if c not in ("t64_c1", "t128_c1")])
@pytest.mark.parametrize("mapper", ["mlp", "linear"])
def test_golden_case(dev, blobs, name, mapper):
    d = load_case(name)
    x = d["x"].astype(f32)
    grid = int(d["grid"])
    out = run_plan(dev, blobs, [x], grid, mapper)[0]
    key = "mlp" if mapper == "mlp" else "lin"
    # against the reference's own outputs
    if "gray_raw" in d.files:
        assert np.array_equal(out["gray"], d["gray_raw"])
    assert np.array_equal(out["edge"], d["edge"])
    assert np.array_equal(out["binmask"], d["binmask"])
    assert np.array_equal(out["bits"], d["bits_" + key]), "tile bits must be bit-exact vs reference"
    rel = np.abs(out["complexity"] - d["complexity"]) / np.abs(d["complexity"])
    assert rel.max() < 1e-6
    assert np.array_equal(out["xmin"], d["xmin"]) and np.array_equal(out["xmax"], d["xmax"])
    tol_m = 0 if name != "b1_c16" else 1e-6
    assert np.all(np.abs(out["m"][:, 0] - d["m_" + key]) <= tol_m * np.abs(d["m_" + key]))
    if ("y_" + key) in d.files:
        if name != "b1_c16":
            assert np.array_equal(out["y"], d["y_" + key])
        else:
            assert np.allclose(out["y"], d["y_" + key], rtol=1e-4, atol=0)
    # against the oracle: everything bit-exact
    check_against_oracle(out, x, blobs[0], grid, mapper)


def test_three_scales_one_launch(dev, blobs):
    """C3/C4/C5 of one batch in a single set of launches == per-scale oracle."""
    xs = [load_case(n)["x"].astype(f32) for n in ("full_p3", "full_p4", "full_p5")]
    outs = run_plan(dev, blobs, xs, 8, "mlp")
    for o, x in zip(outs, xs):
        check_against_oracle(o, x, blobs[0], 8, "mlp")


@pytest.mark.parametrize("shape,grid", [((3, 24, 48, 48), 8), ((2, 40, 36, 60), 8), ((4, 8, 80, 80), 16),
                                        ((1, 12, 33, 41), 8)])
def test_random_shapes_vs_oracle(dev, blobs, shape, grid):
    rng = np.random.default_rng(sum(shape))
    x = (rng.standard_normal(shape) * 1.5).astype(f32)
    x = np.where(x > 0, x, x * f32(0.1)).astype(f32)
    out = run_plan(dev, blobs, [x], grid, "linear")[0]
    check_against_oracle(out, x, blobs[0], grid, "linear")


def _near_tie_image(H, Wd, step, seed):
    """x (1, 1, H, W) whose pixels on a `step` lattice sit within the adaptive
    threshold's separable-estimate margin (g255 ~ mean(g255) - 2)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(0.2, 0.8, size=(1, 1, H, Wd)).astype(f32)
    x[0, 0, 0, 0], x[0, 0, -1, -1] = 0.0, 1.0          # normalize01 is then the identity
    k = O.K["gauss11_adaptive"].astype(np.float64)
    kc = k[5, 5]
    for _ in range(40 if step < 11 else 1):   # Gauss-Seidel when the windows overlap
        for i, h in enumerate(range(8, H - 8, step)):
            for j, w in enumerate(range(8, Wd - 8, step)):
                g = x[0, 0].astype(np.float64) * 255.0
                others = float((k * g[h - 5:h + 6, w - 5:w + 6]).sum() - kc * g[h, w])
                delta = (-1.5e-3, 0.0, 1.5e-3, 4e-4)[(i + j) % 4]
                x[0, 0, h, w] = f32((others - 2.0 + delta) / (1.0 - kc) / 255.0)
    return x


@pytest.mark.parametrize("H,step", [(64, 12), (80, 4)])
def test_adaptive_threshold_near_ties(dev, blobs, H, step):
    """Pixels within the margin take the exact 121-tap sum (listed, one wave
    per pixel); a few per image and several hundred (more than the
    workgroup's waves) - the mask equals the oracle's bit for bit."""
    x = _near_tie_image(H, H, step, 7 + step)
    gray = O.normalize01(O.channel_mean(x, H, H))
    g255 = (gray * f32(255.0)).astype(f32)
    mean = O.conv2d(g255, O.K["gauss11_adaptive"], pad="replicate")
    marg = float(np.frombuffer(np.uint32(0x3B926590).tobytes(), f32)[0])
    near = int((np.abs(g255 - (mean - f32(2.0))) <= marg).sum())
    assert near >= (4 if step > 4 else 200), near
    out = run_plan(dev, blobs, [x], 8, "mlp")[0]
    assert np.array_equal(out["binmask"], O.adaptive_binarize(gray))
    check_against_oracle(out, x, blobs[0], 8, "mlp")


def test_three_scales_global_planes(dev, blobs):
    """A launch whose largest scale does not fit the LDS (160x160 at grid 8)
    runs every scale with planes in global scratch, each at its own stride."""
    rng = np.random.default_rng(7)
    xs = []
    for (C, S) in ((8, 160), (16, 80), (32, 40)):
        x = (rng.standard_normal((1, C, S, S)) * 1.5).astype(f32)
        xs.append(np.where(x > 0, x, x * f32(0.1)).astype(f32))
    outs = run_plan(dev, blobs, xs, 8, "mlp")
    for o, x in zip(outs, xs):
        check_against_oracle(o, x, blobs[0], 8, "mlp")


def test_large_map_global_planes(dev, blobs):
    """t64_c1 (640x640, tile 64): planes do not fit LDS -> global workspace path."""
    d = load_case("t64_c1")
    x = d["x"].astype(f32)
    out = run_plan(dev, blobs, [x], 8, "linear")[0]
    assert np.array_equal(out["edge"], d["edge"])
    assert np.array_equal(out["binmask"], d["binmask"])
    assert np.array_equal(out["bits"], d["bits_lin"])
    assert np.array_equal(out["y"][:, :2], d["y_lin_head"])


def test_tile128_hook_path(dev, blobs):
    """t128_c1 (1024x1024, tile 128, 8x8 tiles): edge / mask / phi / bits vs
    the reference fixture; m and y bit-exact vs the oracle.  B = 1, so the
    reference's soft-mask convolution takes the CPU MKL batch-1 path (as for
    b1_c16): its y channel sum is matched within 1e-8 relative only."""
    d = load_case("t128_c1")
    x = d["x"].astype(f32)
    out = run_plan(dev, blobs, [x], 8, "mlp")[0]
    assert np.array_equal(out["edge"], d["edge"])
    assert np.array_equal(out["binmask"], d["binmask"])
    assert np.array_equal(out["phi"], d["phi"])
    assert np.array_equal(out["bits"], d["bits_mlp"])
    m = O.soft_mask(d["bits_mlp"], x, blobs[0])
    assert np.array_equal(out["m"][:, 0], m)
    y = O.quantize(x, d["bits_mlp"], m, x.min(axis=(0, 2, 3)), x.max(axis=(0, 2, 3)))
    assert np.array_equal(out["y"], y)
    np.testing.assert_allclose(out["y"].astype(np.float64).sum(axis=(2, 3)), d["y_mlp_sum"], rtol=1e-8)


def test_constant_and_degenerate_inputs(dev, blobs):
    """All-zero map (normalisation denominator 1e-8, flat Otsu), constant
    channels (zero range -> scale clamp), all-positive channels (zp clamp)."""
    x = np.zeros((2, 8, 40, 40), f32)
    x[:, 3] = 1.5
    x[:, 5] = np.linspace(0.1, 2.0, 1600, dtype=f32).reshape(40, 40)
    out = run_plan(dev, blobs, [x], 8, "linear")[0]
    check_against_oracle(out, x, blobs[0], 8, "linear")


def test_options_vs_oracle(dev, blobs):
    """continuous bits / normalize_complexity / temperature / frozen stats."""
    import torch
    d = load_case("p4_c32")
    x = d["x"].astype(f32)
    W = blobs[0]
    out = run_plan(dev, blobs, [x], 8, "mlp", T=0.7, continuous=True, normalize=True)[0]
    C, _, _ = O.analyzer_forward(x, W, 8)
    assert np.array_equal(out["bits"], O.mlp_mapper(O.normalize_complexity(C), W, 0.7, continuous=True))
    out = run_plan(dev, blobs, [x], 8, "mlp", T=10.0)[0]
    assert np.all(out["bits"] == 8.0)
    lo = torch.full((32,), -0.5, device=dev)
    hi = torch.full((32,), 3.0, device=dev)
    out = run_plan(dev, blobs, [x], 8, "linear", minmax=[(lo, hi)])[0]
    ref = O.hook_forward(x, W, 8, mapper="linear", xmin=np.full(32, -0.5, f32), xmax=np.full(32, 3.0, f32))
    assert np.array_equal(out["y"], ref["y"])


def test_spatial_quantize_compat(dev):
    """mcaq_launch_spatial_quantization (the reference kernel contract) vs the
    oracle, divisible and remainder tiles, with and without mask; and the
    reference's own parity test semantics (tests/test_smoke.py:226-246)."""
    import ctypes
    import torch
    from mcaq_yolo_amd import abi
    L = abi.lib()
    rng = np.random.default_rng(7)
    for (N, C, H, W_, Ht, Wt) in ((2, 8, 32, 32, 4, 4), (2, 5, 10, 13, 4, 3), (1, 3, 7, 9, 2, 2)):
        x = rng.standard_normal((N, C, H, W_)).astype(f32)
        bits = rng.integers(1, 10, (N, Ht, Wt)).astype(f32)
        mask = rng.random((N, 1, H, W_)).astype(f32)
        mn, mx = x.min(axis=(0, 2, 3)), x.max(axis=(0, 2, 3))
        th, tw = H // Ht, W_ // Wt
        for m in (None, mask):
            tx, tb = torch.from_numpy(x).cuda(), torch.from_numpy(bits).cuda()
            tmn, tmx = torch.from_numpy(mn).cuda(), torch.from_numpy(mx).cuda()
            tm = torch.from_numpy(m).cuda() if m is not None else None
            y = torch.empty_like(tx)
            p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
            err = L.mcaq_launch_spatial_quantization(p(tx), p(tb), p(tmn), p(tmx), p(tm), p(y), N, C, H, W_,
                                                     th, tw, Ht, Wt,
                                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert err == 0
            torch.cuda.synchronize()
            want = O.spatial_quantize_compat(x, bits, mn, mx, th, tw, m)
            assert np.array_equal(y.cpu().numpy(), want)


def test_bench_config_properties(dev, blobs):
    """yolov8n bs32 640x640 (BASELINE config 2) at full size: determinism,
    bits in [2, 8], per-channel min/max exact vs torch, and the first two
    images bit-exact vs the oracle (batch min/max passed in)."""
    import torch
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    W, cm, mm, sm = blobs
    g = torch.Generator(device="cpu").manual_seed(2)
    shapes = [(32, 64, 80, 80), (32, 128, 40, 40), (32, 256, 20, 20)]
    feats = [torch.nn.functional.silu(1.5 * torch.randn(s, generator=g)).to(dev) for s in shapes]
    plan = HookPlan([ScaleGeom(*s, 8) for s in shapes], dev)
    bufs = plan.run(feats, cm, mm, [sm] * 3)
    y1 = [b["y"].clone() for b in bufs]
    bufs = plan.run(feats, cm, mm, [sm] * 3)
    torch.cuda.synchronize()
    for f, b, yy in zip(feats, bufs, y1):
        assert torch.equal(b["y"], yy), "non-deterministic"
        assert torch.equal(b["xmin"], f.amin(dim=(0, 2, 3))) and torch.equal(b["xmax"], f.amax(dim=(0, 2, 3)))
        bits = b["bits"]
        assert bool(((bits >= 2) & (bits <= 8) & (bits == bits.round())).all())
        assert bool(torch.isfinite(b["y"]).all())
    for f, b in zip(feats, bufs):
        x2 = f[:2].cpu().numpy()
        ref = O.hook_forward(x2, W, 8, xmin=b["xmin"].cpu().numpy(), xmax=b["xmax"].cpu().numpy())
        assert np.array_equal(b["bits"][:2].cpu().numpy(), ref["bits"])
        assert np.array_equal(b["y"][:2].cpu().numpy(), ref["y"])


@pytest.mark.parametrize("shape", [(2, 64, 80, 80), (2, 128, 40, 40), (2, 256, 20, 20), (1, 200, 20, 20),
                                   (1, 576, 20, 20), (1, 1100, 12, 12), (2, 130, 18, 22), (1, 67, 9, 13)])
def test_stats_pass_orders(dev, blobs, shape):
    """Pass 1 across its code paths: 4/2/1 pixels per lane, several channel
    rounds, partial cascade blocks, leftover rows of the row_sum tail order,
    the cooperative tail and the per-pixel tail (C > 1024): gray, |x| mean and
    channel min/max bit-exact vs the oracle."""
    rng = np.random.default_rng(shape[1] * 7 + shape[2])
    x = (rng.standard_normal(shape) * 2.0).astype(f32)
    grid = 8 if shape[2] >= 32 else 4
    out = run_plan(dev, blobs, [x], grid, "linear")[0]
    _, I = O.phi_tiles(x, grid, internals=True)
    assert np.array_equal(out["gray"], I["gray_raw"]), "gray"
    assert np.array_equal(out["absmean"], O.abs_channel_mean(x)), "absmean"
    assert np.array_equal(out["xmin"], x.min(axis=(0, 2, 3))), "min"
    assert np.array_equal(out["xmax"], x.max(axis=(0, 2, 3))), "max"


@pytest.mark.parametrize("shape", [(5, 16, 20, 20), (6, 12, 40, 40), (3, 8, 24, 24)])
def test_packed_workgroups_vs_oracle(dev, blobs, shape):
    """Small images share a workgroup (pass A: up to 8 per 1024 threads, pass B:
    4 per 256); batches that leave a workgroup partly filled (its spare groups
    recompute the last image) stay bit-exact for every image."""
    rng = np.random.default_rng(shape[0] * 31 + shape[2])
    x = (rng.standard_normal(shape) * 1.5).astype(f32)
    x = np.where(x > 0, x, x * f32(0.1)).astype(f32)
    out = run_plan(dev, blobs, [x], 8, "mlp")[0]
    check_against_oracle(out, x, blobs[0], 8, "mlp")


OPT_GPU = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("opt_") and f.endswith(".npz"))


@pytest.mark.parametrize("name", OPT_GPU)
def test_analyzer_switches_vs_reference(dev, blobs, name):
    """binarize_impl='otsu', contour_components=False and canny_impl='legacy' on the morph kernel
    against the reference's own outputs (tests/golden/make_golden_r02.py) and
    the oracle: edge, mask, phi1..7 and bits bit-exact, phi8 within 1 ulp of
    the reference (bit-exact vs the oracle)."""
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    opts = {k[4:]: (str(d[k]) if d[k].dtype.kind == "U" else d[k].item()) for k in d.files if k.startswith("opt_")}
    x = d["x"].astype(f32)
    grid = int(d["grid"])
    out = run_plan(dev, blobs, [x], grid, "mlp", binarize_otsu=opts.get("binarize_impl") == "otsu",
                   contour_components=opts.get("contour_components", True),
                   canny_legacy=opts.get("canny_impl") == "legacy")[0]
    assert np.array_equal(out["edge"], d["edge"])
    assert np.array_equal(out["binmask"], d["binmask"])
    assert np.array_equal(out["phi"][..., :7], d["phi"][..., :7])
    assert np.all(np.abs(out["phi"][..., 7] - d["phi"][..., 7]) <= np.spacing(np.abs(d["phi"][..., 7])))
    assert np.array_equal(out["bits"], d["bits_mlp"])
    ref = O.hook_forward(x, blobs[0], grid, **opts)
    assert np.array_equal(out["phi"], ref["phi"])
    assert np.array_equal(out["complexity"], ref["complexity"])
    assert np.array_equal(out["y"], ref["y"])


def _full_size_properties(dev, blobs, shapes, grid, seed):
    """Determinism, bits in [2, 8] integers, exact channel min/max, finite y,
    and the first two images of every scale bit-exact vs the oracle (with the
    batch min/max the kernel computed) at a BASELINE config's full shapes."""
    import torch
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    W, cm, mm, sm = blobs
    g = torch.Generator(device="cpu").manual_seed(seed)
    feats = [torch.nn.functional.silu(1.5 * torch.randn(s, generator=g) +
                                      torch.nn.functional.interpolate(torch.randn(s[0], s[1], s[2] // 8, s[3] // 8,
                                                                                  generator=g), size=s[2:],
                                                                      mode="bilinear")).to(dev) for s in shapes]
    plan = HookPlan([ScaleGeom(*s, grid) for s in shapes], dev)
    bufs = plan.run(feats, cm, mm, [sm] * len(shapes))
    y1 = [b["y"].clone() for b in bufs]
    bits1 = [b["bits"].clone() for b in bufs]
    bufs = plan.run(feats, cm, mm, [sm] * len(shapes))
    torch.cuda.synchronize()
    seen = set()
    for f, b, yy, bb in zip(feats, bufs, y1, bits1):
        assert torch.equal(b["y"], yy) and torch.equal(b["bits"], bb), "non-deterministic"
        assert torch.equal(b["xmin"], f.amin(dim=(0, 2, 3))) and torch.equal(b["xmax"], f.amax(dim=(0, 2, 3)))
        bits = b["bits"]
        assert bool(((bits >= 2) & (bits <= 8) & (bits == bits.round())).all())
        seen |= set(bits.unique().tolist())
        assert bool(torch.isfinite(b["y"]).all())
    for f, b in zip(feats, bufs):
        x2 = f[:2].cpu().numpy()
        # batch_total: the fractal regression's ATen reduction order follows
        # the tile's column in the whole batch (oracle fractal_tiles)
        ref = O.hook_forward(x2, W, grid, xmin=b["xmin"].cpu().numpy(), xmax=b["xmax"].cpu().numpy(),
                             batch_total=f.shape[0])
        assert np.array_equal(b["bits"][:2].cpu().numpy(), ref["bits"])
        assert np.array_equal(b["y"][:2].cpu().numpy(), ref["y"])
    return seen


def test_config3_yolov8s_bs64_grid16_properties(dev, blobs):
    """BASELINE config 3 (yolov8s bs64, grid 16: P3 tile 4 / 20x20 tiles, the
    LDS-tile stress case) at full size."""
    seen = _full_size_properties(dev, blobs, [(64, 128, 80, 80), (64, 256, 40, 40), (64, 512, 20, 20)], 16, 3)
    assert len(seen) >= 2


def test_config4_yolov8m_slice_properties(dev, blobs):
    """BASELINE config 4's per-GPU slice (yolov8m, 32 images: 192 x 80^2,
    384 x 40^2, 576 x 20^2, grid 8) at full size."""
    seen = _full_size_properties(dev, blobs, [(32, 192, 80, 80), (32, 384, 40, 40), (32, 576, 20, 20)], 8, 4)
    assert len(seen) >= 2


def test_m_plane_option_same_y(dev, blobs):
    """m_plane=True (pass B writes m(p), pass 2 reads it) gives the y of the
    default (pass 2 regenerates m(p) from the tile values): same FMA order."""
    xs = [load_case(n)["x"].astype(f32) for n in ("full_p3", "full_p4", "full_p5")]
    a = run_plan(dev, blobs, xs, 8, "mlp")
    b = run_plan(dev, blobs, xs, 8, "mlp", m_plane=True)
    for oa, ob, x in zip(a, b, xs):
        assert np.array_equal(oa["y"], ob["y"])
        check_against_oracle(ob, x, blobs[0], 8, "mlp")


@pytest.mark.parametrize("cfg", [("c2", [(32, 64, 80, 80), (32, 128, 40, 40), (32, 256, 20, 20)], 8),
                                 ("c3", [(64, 128, 80, 80), (64, 256, 40, 40), (64, 512, 20, 20)], 16)])
def test_band_pass_equals_image_pass_full_size(dev, blobs, cfg):
    """Pass A as band + edge workgroups (round 4, csrc/mcaq_band.h) against the
    per-image pass A on the GPU at BASELINE config 2 / 3 full shapes: every
    debug plane and output bit for bit (tile partials through phi, edge and
    mask planes, complexity, bits, y)."""
    import torch
    from mcaq_yolo_amd import engine
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    name, shapes, grid = cfg
    W, cm, mm, sm = blobs
    g = torch.Generator(device="cpu").manual_seed(41)
    feats = [torch.nn.functional.silu(1.5 * torch.randn(s, generator=g)).to(dev) for s in shapes]
    outs = {}
    for band in (True, False):
        old = engine.BAND_PASS
        engine.BAND_PASS = band
        try:
            plan = HookPlan([ScaleGeom(*s, grid) for s in shapes], dev, want=("phi", "cmlp", "debug"))
            assert all((b["pwork"] is not None) == band for b in plan.bufs)
            bufs = plan.run(feats, cm, mm, [sm] * len(shapes))
            torch.cuda.synchronize()
            outs[band] = [{k: v.clone() for k, v in b.items() if torch.is_tensor(v) and k != "pwork"} for b in bufs]
        finally:
            engine.BAND_PASS = old
    for a, b, s in zip(outs[True], outs[False], shapes):
        T = ScaleGeom(*s, grid).tile
        nit = 20 + (T.bit_length() - 2)      # 20 + number of box-counting scales 2..T
        assert torch.equal(a["tile_tmp"][..., :nit], b["tile_tmp"][..., :nit]), (name, "tile_tmp")
        for k in ("edge", "binmask", "phi", "cmlp", "complexity", "bits", "mt", "m", "y"):
            assert torch.equal(a[k], b[k]), (name, k)


@pytest.mark.parametrize("cfg", [("c2", [(32, 64, 80, 80), (32, 128, 40, 40), (32, 256, 20, 20)], 8, {}),
                                 ("c3", [(64, 128, 80, 80), (64, 256, 40, 40), (64, 512, 20, 20)], 16, {}),
                                 ("c2_T", [(8, 64, 80, 80), (8, 128, 40, 40), (8, 256, 20, 20)], 8,
                                  {"temperature": 0.6, "continuous": True})])
def test_batch_tile_pass_equals_image_pass_full_size(dev, blobs, cfg):
    """Pass B as batch-wide tile kernels (round 4, csrc/mcaq_tiles_batch.h)
    against the per-image pass B on the GPU at BASELINE config 2 / 3 full
    shapes (and a temperature / continuous-bits variant): phi, raw and
    filtered complexity, bits, m(tile), the m(p) plane and y bit for bit."""
    import torch
    from mcaq_yolo_amd import engine
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    name, shapes, grid, kw = cfg
    W, cm, mm, sm = blobs
    g = torch.Generator(device="cpu").manual_seed(43)
    feats = [torch.nn.functional.silu(1.5 * torch.randn(s, generator=g)).to(dev) for s in shapes]
    outs = {}
    for batch in (True, False):
        old = engine.TILES_BATCH
        engine.TILES_BATCH = batch
        try:
            plan = HookPlan([ScaleGeom(*s, grid) for s in shapes], dev, want=("phi", "cmlp", "debug"))
            bufs = plan.run(feats, cm, mm, [sm] * len(shapes), **kw)
            torch.cuda.synchronize()
            outs[batch] = [{k: v.clone() for k, v in b.items() if torch.is_tensor(v)} for b in bufs]
        finally:
            engine.TILES_BATCH = old
    for a, b in zip(outs[True], outs[False]):
        for k in ("phi", "cmlp", "complexity", "bits", "mt", "m", "y"):
            assert torch.equal(a[k], b[k]), (name, k)
