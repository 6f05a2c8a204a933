"""Host emulation of the gfx950 morph kernel (same mcaq_morph.h source, one
thread) against the oracle: every output bit-exact, on every golden case and
both mappers, plus the option flags.  Catches arithmetic-order mistakes in the
kernel source without a GPU."""
import ctypes
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, case_names, load_case, load_weights
from oracle import mcaq_oracle as O

sys.path.insert(0, os.path.join(ROOT, "tests", "emu"))
import build_emu  # noqa: E402

from mcaq_yolo_amd import abi, params  # noqa: E402

f32 = np.float32


@pytest.fixture(scope="module")
def emu():
    lib = ctypes.CDLL(build_emu.build())
    lib.emu_morph.argtypes = [ctypes.POINTER(abi.MorphScale)]
    lib.emu_morph_band.argtypes = [ctypes.POINTER(abi.MorphScale)]
    lib.emu_morph_tb.argtypes = [ctypes.POINTER(abi.MorphScale)]
    W = load_weights()
    blobs = (params.pack_complexity_mlp(params.sub(W, "complexity_analyzer.")),
             params.pack_mapper_mlp(params.sub(W, "bit_mapper.")),
             params.pack_soft_mask(params.sub(W, "soft_mask.")))
    return lib, W, blobs


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def run_emu(emu, x, grid, flags, T=1.0, c_in=None, bits_in=None, band=False, tb=False):
    lib, W, (cm, mm, sm) = emu
    B, C, H, Wd = x.shape
    tile = O.tile_size(H, grid)
    ht, wt = H // tile, Wd // tile
    Hc, Wc = ht * tile, wt * tile
    gray = O.channel_mean(x, Hc, Wc)
    am = O.abs_channel_mean(x)
    out = dict(phi=np.zeros((B, ht, wt, 8), f32), cmlp=np.zeros((B, ht, wt), f32),
               c=np.zeros((B, ht, wt), f32), bits=np.zeros((B, ht, wt), f32),
               m=np.zeros((B, H, Wd), f32), edge=np.zeros((B, Hc, Wc), np.uint8),
               bin=np.zeros((B, Hc, Wc), np.uint8))
    s = abi.MorphScale()
    s.gray, s.absmean, s.cmlp, s.mapper, s.smask = _ptr(gray), _ptr(am), _ptr(cm), _ptr(mm), _ptr(sm)
    s.c_in, s.bits_in = _ptr(c_in), _ptr(bits_in)
    s.phi_out, s.cmlp_out, s.c_out = _ptr(out["phi"]), _ptr(out["cmlp"]), _ptr(out["c"])
    s.bits_out, s.m_out, s.edge_out, s.bin_out = _ptr(out["bits"]), _ptr(out["m"]), _ptr(out["edge"]), _ptr(out["bin"])
    out["tile_tmp"] = np.zeros((B, ht * wt, 32), f32)
    out["mt"] = np.zeros((B, ht, wt), f32)
    s.mt_out = _ptr(out["mt"])
    s.tile_tmp = _ptr(out["tile_tmp"])
    s.B, s.H, s.W, s.Hc, s.Wc, s.tile, s.ht, s.wt = B, H, Wd, Hc, Wc, tile, ht, wt
    s.batch_offset, s.batch_total = 0, B
    s.flags = flags
    s.hyst_iters = 8
    s.softmax_threads = O.REF_THREADS
    s.temperature, s.min_bits, s.max_bits = max(T, 0.1), 2.0, 8.0
    if tb:
        # pass B as the batch-wide tile kernels (mcaq_tiles_batch.h)
        assert lib.emu_morph_tb(ctypes.byref(s)) == 0, "flags not eligible for the batch-wide tile pass"
    elif band:
        # pass A as band + edge workgroups (mcaq_band.h): pwork = NMS plane + band histograms
        nb = -(-Hc // max(tile, 16))
        out["pwork"] = np.zeros(B * Hc * Wc + B * nb * 256, f32)
        s.pwork = _ptr(out["pwork"])
        assert lib.emu_morph_band(ctypes.byref(s)) == 0, "scale not eligible for the band path"
    else:
        lib.emu_morph(ctypes.byref(s))
    return out


ALL = abi.F_PHI | abi.F_CMLP | abi.F_MAPPER | abi.F_SOFTMASK | abi.F_HAS_T
CASES = [c for c in case_names() if c not in ("t64_c1", "t128_c1")]


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("mapper", ["mlp", "linear"])
def test_emu_matches_oracle(emu, name, mapper):
    d = load_case(name)
    x = d["x"].astype(f32)
    grid = int(d["grid"])
    flags = ALL | (abi.F_MAP_LINEAR if mapper == "linear" else 0)
    out = run_emu(emu, x, grid, flags)
    ref = O.hook_forward(x, emu[1], grid, mapper=mapper)
    _, I = O.phi_tiles(x, grid, internals=True)
    assert np.array_equal(out["edge"], I["edge"])
    assert np.array_equal(out["bin"], I["binmask"])
    assert np.array_equal(out["phi"], ref["phi"])
    assert np.array_equal(out["cmlp"], ref["c_mlp"])
    assert np.array_equal(out["c"], ref["complexity"])
    assert np.array_equal(out["bits"], ref["bits"])
    assert np.array_equal(out["m"], ref["m"])
    assert np.array_equal(out["bits"], d["bits_mlp" if mapper == "mlp" else "bits_lin"])


@pytest.mark.parametrize("name", ["t64_c1", "t128_c1"])
@pytest.mark.parametrize("mapper", ["mlp", "linear"])
def test_emu_large_tiles_vs_reference(emu, name, mapper):
    """tile 64 (640^2) and tile 128 (1024^2): the kernel source's edge, mask,
    phi and bits vs the reference fixtures directly (the oracle is slow here)."""
    d = load_case(name)
    x = d["x"].astype(f32)
    out = run_emu(emu, x, 8, ALL | (abi.F_MAP_LINEAR if mapper == "linear" else 0))
    assert np.array_equal(out["edge"], d["edge"])
    assert np.array_equal(out["bin"], d["binmask"])
    assert np.array_equal(out["phi"], d["phi"])
    assert np.max(np.abs(out["c"] - d["complexity"]) / np.abs(d["complexity"])) < 1e-6
    assert np.array_equal(out["bits"], d["bits_mlp" if mapper == "mlp" else "bits_lin"])


def test_emu_options(emu):
    """normalize_complexity, continuous bits, temperature, Otsu binarize,
    no Euler correction, mapper-only and softmask-only stages."""
    d = load_case("p4_c32")
    x = d["x"].astype(f32)
    W = emu[1]
    # continuous + normalize + T=0.7
    out = run_emu(emu, x, 8, ALL | abi.F_CONT | abi.F_NORM_C, T=0.7)
    C, _, _ = O.analyzer_forward(x, W, 8)
    want = O.mlp_mapper(O.normalize_complexity(C), W, 0.7, continuous=True)
    assert np.array_equal(out["bits"], want)
    # mapper-only from given complexity (linear, T=10 -> all 8)
    c_in = d["complexity"].astype(f32).copy()
    out = run_emu(emu, x, 8, abi.F_MAPPER | abi.F_MAP_LINEAR | abi.F_HAS_T, T=10.0, c_in=c_in)
    assert np.all(out["bits"] == 8.0)
    # softmask-only from given bits
    bits_in = d["bits_lin"].astype(f32).copy()
    out = run_emu(emu, x, 8, abi.F_SOFTMASK, bits_in=bits_in)
    assert np.array_equal(out["m"], O.soft_mask(bits_in, x, W))


def test_emu_otsu_binarize_and_no_euler(emu):
    d = load_case("p3_c16")
    x = d["x"].astype(f32)
    out = run_emu(emu, x, 8, abi.F_PHI | abi.F_BIN_OTSU | abi.F_NO_EULER)
    tile = 8
    gray = O.normalize01(O.channel_mean(x, 80, 80))
    thr = O.otsu_threshold(gray)
    binm = (gray > thr[:, None, None]).astype(np.uint8)
    assert np.array_equal(out["bin"], binm)
    assert np.array_equal(out["phi"][..., 4], O.contour_tiles(binm, tile, contour_components=False))


def test_emu_adaptive_threshold_near_ties(emu):
    """Pixels placed within the separable estimate's error margin of the
    adaptive threshold (g255 ~ mean - 2) take the exact 121-tap path; the
    mask must still equal the oracle's bit for bit."""
    rng = np.random.default_rng(7)
    H = Wd = 64
    x = rng.uniform(0.2, 0.8, size=(1, 1, H, Wd)).astype(f32)
    x[0, 0, 0, 0], x[0, 0, -1, -1] = 0.0, 1.0          # normalize01 is then the identity
    k = O.K["gauss11_adaptive"].astype(np.float64)
    kc = k[5, 5]
    marg = float(np.frombuffer(np.uint32(0x3B926590).tobytes(), f32)[0])
    targets = []
    for i, h in enumerate(range(8, H - 8, 12)):
        for j, w in enumerate(range(8, Wd - 8, 12)):
            g = x[0, 0].astype(np.float64) * 255.0
            win = g[h - 5:h + 6, w - 5:w + 6]
            others = float((k * win).sum() - kc * g[h, w])
            delta = (-1.5e-3, 0.0, 1.5e-3, 4e-4)[(i + j) % 4]
            v = (others - 2.0 + delta) / (1.0 - kc)      # g255 = mean(g255) - 2 + delta
            x[0, 0, h, w] = f32(v / 255.0)
            targets.append((h, w))
    gray = O.normalize01(O.channel_mean(x, H, Wd))
    assert np.array_equal(gray, x[:, 0])
    g255 = (gray * f32(255.0)).astype(f32)
    mean = O.conv2d(g255, O.K["gauss11_adaptive"], pad="replicate")
    gap = np.abs(g255 - (mean - f32(2.0)))
    near = sum(gap[0, h, w] <= marg for h, w in targets)
    assert near >= len(targets) // 2, "construction must land inside the margin"
    out = run_emu(emu, x, 8, abi.F_PHI)
    assert np.array_equal(out["bin"], O.adaptive_binarize(gray))


OPT_CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("opt_") and f.endswith(".npz"))


@pytest.mark.parametrize("name", OPT_CASES)
def test_emu_analyzer_switches_vs_reference(emu, name):
    """canny_impl='legacy', binarize_impl='otsu', contour_components=False
    through the kernel source against the reference's own outputs
    (tests/golden/make_golden_r02.py) and the oracle."""
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    opts = {k[4:]: (str(d[k]) if d[k].dtype.kind == "U" else d[k].item()) for k in d.files if k.startswith("opt_")}
    x = d["x"].astype(f32)
    grid = int(d["grid"])
    flags = ALL | (abi.F_BIN_OTSU if opts.get("binarize_impl") == "otsu" else 0) | \
        (0 if opts.get("contour_components", True) else abi.F_NO_EULER) | \
        (abi.F_CANNY_LEGACY if opts.get("canny_impl") == "legacy" else 0)
    out = run_emu(emu, x, grid, flags)
    assert np.array_equal(out["edge"], d["edge"])
    assert np.array_equal(out["bin"], d["binmask"])
    assert np.array_equal(out["phi"][..., :7], d["phi"][..., :7])
    assert np.array_equal(out["bits"], d["bits_mlp"])
    ref = O.hook_forward(x, emu[1], grid, **opts)
    assert np.array_equal(out["phi"], ref["phi"])
    assert np.array_equal(out["c"], ref["complexity"])
    assert np.array_equal(out["m"], ref["m"])


def _band_ok(x, grid, flags):
    tile = O.tile_size(x.shape[2], grid)
    Hc, Wc = (x.shape[2] // tile) * tile, (x.shape[3] // tile) * tile
    return tile in (4, 8, 16) and Hc <= 128 and Wc <= 128 and not flags & (abi.F_CANNY_LEGACY | abi.F_BIN_OTSU)


BAND_KEYS = ("tile_tmp", "edge", "bin", "phi", "cmlp", "c", "bits", "m")


@pytest.mark.parametrize("name", ["case_" + c for c in case_names()] + OPT_CASES)
def test_emu_band_pass_equals_image_pass(emu, name):
    """Pass A as band + edge workgroups (round 4, mcaq_band.h) against the
    per-image pass A of the same source: every per-tile partial, the edge and
    mask planes and everything downstream bit for bit, on every golden case
    whose scale the band path takes (and the option switches it supports)."""
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    x = d["x"].astype(f32)
    grid = int(d["grid"])
    opts = {k[4:]: (str(d[k]) if d[k].dtype.kind == "U" else d[k].item()) for k in d.files if k.startswith("opt_")}
    flags = ALL | (abi.F_BIN_OTSU if opts.get("binarize_impl") == "otsu" else 0) | \
        (0 if opts.get("contour_components", True) else abi.F_NO_EULER) | \
        (abi.F_CANNY_LEGACY if opts.get("canny_impl") == "legacy" else 0)
    if not _band_ok(x, grid, flags):
        pytest.skip("scale not eligible for the band path (kept on the per-image pass A)")
    ref = run_emu(emu, x, grid, flags)
    out = run_emu(emu, x, grid, flags, band=True)
    for k in BAND_KEYS:
        assert np.array_equal(out[k], ref[k]), k
    if "bits_mlp" in d.files:
        assert np.array_equal(out["bits"], d["bits_mlp"])


def test_emu_band_pass_near_ties_and_batch(emu):
    """The adaptive threshold's exact fallback inside band halos, several
    images per launch, and an image whose rows are not a multiple of 16."""
    rng = np.random.default_rng(11)
    for shape, grid in (((3, 4, 48, 40), 8), ((2, 8, 36, 52), 8), ((2, 3, 128, 128), 8), ((1, 2, 64, 64), 4)):
        x = rng.uniform(0.0, 1.0, size=shape).astype(f32)
        x[:, :, ::7, ::5] = 0.5          # plateaus: ties in LBP, NMS and the threshold
        flags = ALL
        if not _band_ok(x, grid, flags):
            continue
        ref = run_emu(emu, x, grid, flags)
        out = run_emu(emu, x, grid, flags, band=True)
        for k in BAND_KEYS:
            assert np.array_equal(out[k], ref[k]), (shape, k)


TB_KEYS = ("phi", "cmlp", "c", "bits", "mt", "m")


@pytest.mark.parametrize("name", ["case_" + c for c in case_names()] + OPT_CASES)
def test_emu_batch_tile_pass_equals_image_pass(emu, name):
    """Pass B as batch-wide tile kernels (round 4, mcaq_tiles_batch.h) against
    the per-image pass B of the same source: phi, raw and filtered complexity,
    bits and the soft-mask tile values bit for bit on every golden case, with
    the option switches and a temperature / continuous bits variant."""
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    x = d["x"].astype(f32)
    grid = int(d["grid"])
    opts = {k[4:]: (str(d[k]) if d[k].dtype.kind == "U" else d[k].item()) for k in d.files if k.startswith("opt_")}
    if opts.get("canny_impl") == "legacy":
        pytest.skip("legacy Canny: the host emulation of the batch path runs the default pass A")
    flags = ALL | (abi.F_BIN_OTSU if opts.get("binarize_impl") == "otsu" else 0) | \
        (0 if opts.get("contour_components", True) else abi.F_NO_EULER)
    for fl, T in ((flags, 1.0), (flags | abi.F_CONT, 0.7)):
        ref = run_emu(emu, x, grid, fl, T=T)
        out = run_emu(emu, x, grid, fl, T=T, tb=True)
        for k in TB_KEYS:
            assert np.array_equal(out[k], ref[k]), (k, fl)
    if "bits_mlp" in d.files:
        assert np.array_equal(out["bits"], ref["bits"])
