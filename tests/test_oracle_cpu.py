"""The CPU oracle against the golden fixtures generated from the reference.

Decision path (gray, Sobel, blur, Otsu, edges, adaptive mask, phi1..phi7) must
be bit-exact; phi8 = sqrt(phi4*phi5 + 1e-12) may differ by 1 ulp (CPU
torch.sqrt is not correctly rounded); complexity within 1e-6 relative; bits
exact; soft mask / y exact except the B=1 case (CPU conv takes an MKL path at
batch 1), where they are within 1e-6 relative.
"""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, case_names, load_case, load_weights
from oracle import mcaq_oracle as O
from oracle.ieee import aten_sum, fma32

FAST = [c for c in case_names() if c not in ("t64_c1", "t32_c4", "t128_c1", "m_p3", "m_p4")]   # m_*: test_option_and_yolov8m_fixtures


def rel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-30)))


def test_constants_match_reference_tensors():
    import os
    from conftest import GOLDEN
    c = np.load(os.path.join(GOLDEN, "constants.npz"))
    for k in c.files:
        assert np.array_equal(c[k], O.K[k]), k


def test_tables_header_matches_oracle():
    import os
    from conftest import ROOT
    src = open(os.path.join(ROOT, "mcaq_yolo_amd", "csrc", "mcaq_tables.h")).read()
    for name, key in (("k_gauss5", "gauss5_canny"), ("k_gauss11", "gauss11_adaptive"),
                      ("k_smooth5", "smooth5_softmask"), ("k_bilat_sp", "bilateral_spatial")):
        words = ", ".join("0x%08Xu" % int(v) for v in O.K[key].reshape(-1).view(np.uint32))
        assert words in src, name


def test_fma32_known_answers():
    a = np.float32(1 + 2 ** -12)
    # (1+2^-12)^2 = 1 + 2^-11 + 2^-24 : exact fp32 midpoint; + tiny decides
    assert fma32(a, a, np.float32(2 ** -60)) == np.float32(1 + 2 ** -11 + 2 ** -23)
    assert fma32(a, a, np.float32(-2 ** -60)) == np.float32(1 + 2 ** -11)
    assert fma32(np.float32(2.0), np.float32(3.0), np.float32(1.0)) == np.float32(7.0)


@pytest.mark.parametrize("C,M", [(3, 25), (17, 100), (64, 6400), (192, 400), (576, 1600)])
def test_aten_sum_matches_torch(C, M):
    torch = pytest.importorskip("torch")
    x = np.random.default_rng(C * M).standard_normal((2, C, M)).astype(np.float32)
    t = torch.from_numpy(x).sum(dim=1).numpy()
    e = np.stack([aten_sum(x[b]) for b in range(2)])
    assert np.array_equal(t, e)


@pytest.mark.parametrize("name", FAST + ["t32_c4"])
def test_phi_path_bit_exact(name):
    d = load_case(name)
    x = d["x"].astype(np.float32)
    phi, I = O.phi_tiles(x, int(d["grid"]), internals=True)
    for k in ("gray_raw", "gray", "blur"):
        if k in d.files:
            assert np.array_equal(I[k], d[k]), k
    if name != "b1_c16":   # B=1 Sobel runs through MKL on the CPU reference
        for k in ("gx", "gy"):
            if k in d.files:
                assert np.array_equal(I[k], d[k]), k
    assert np.array_equal(I["otsu_thr"], d["otsu_thr"])
    assert np.array_equal(I["edge"], d["edge"])
    assert np.array_equal(I["binmask"], d["binmask"])
    exact = range(7) if name != "b1_c16" else (0, 1, 3, 4, 5)
    for k in exact:
        assert np.array_equal(phi[..., k], d["phi"][..., k]), "phi%d" % (k + 1)
    ulp = np.spacing(np.abs(d["phi"][..., 7]).astype(np.float32))
    assert np.all(np.abs(phi[..., 7] - d["phi"][..., 7]) <= ulp)
    if name == "b1_c16":
        assert rel(phi[..., 2], d["phi"][..., 2]) < 1e-6


@pytest.mark.parametrize("name", FAST)
def test_complexity_bits_mask_y(name):
    d = load_case(name)
    W = load_weights()
    x = d["x"].astype(np.float32)
    C, phi, cm = O.analyzer_forward(x, W, int(d["grid"]))
    assert rel(C, d["complexity"]) < 1e-6
    assert np.array_equal(O.mlp_mapper(C, W, 1.0), d["bits_mlp"])
    assert np.array_equal(O.linear_mapper(C, 1.0), d["bits_lin"])
    assert np.array_equal(O.linear_mapper(d["complexity"], 1.0, continuous=True), d["bits_lin_cont"])
    assert np.abs(O.mlp_mapper(d["complexity"], W, 1.0, continuous=True) - d["bits_mlp_cont"]).max() < 1e-5
    assert np.array_equal(O.mlp_mapper(C, W, 10.0), d["bits_mlp_t10"])
    assert np.all(d["bits_mlp_t10"] == 8.0)          # reference test_bit_mapper_range_and_temperature
    m = O.soft_mask(d["bits_mlp"], x, W)
    xmin, xmax = x.min(axis=(0, 2, 3)), x.max(axis=(0, 2, 3))
    assert np.array_equal(xmin, d["xmin"]) and np.array_equal(xmax, d["xmax"])
    if name == "b1_c16":
        assert rel(m, d["m_mlp"]) < 1e-6
    else:
        assert np.array_equal(m, d["m_mlp"])
    y = O.quantize(x, d["bits_mlp"], d["m_mlp"], xmin, xmax)
    if "y_mlp" in d.files:
        assert np.array_equal(y, d["y_mlp"])
        assert np.array_equal(O.quantize(x, d["bits_mlp"], None, xmin, xmax), d["y_nomask"])
        assert np.array_equal(O.quantize(x, d["bits_lin"], d["m_lin"], xmin, xmax), d["y_lin"])
    else:
        assert np.array_equal(y[:, :2], d["y_mlp_head"])
        assert np.allclose(y.astype(np.float64).sum(axis=(2, 3)), d["y_mlp_sum"], rtol=1e-9, atol=1e-6)


def test_tile128_fixture():
    """case_t128_c1 (1x1x1024^2, grid 8 -> tile 128, the largest tile the
    analyzer kernel takes): edge / mask / phi1..phi8 bit-exact, bits exact."""
    d = load_case("t128_c1")
    assert int(d["tile"]) == 128
    x = d["x"].astype(np.float32)
    W = load_weights()
    phi, I = O.phi_tiles(x, 8, internals=True)
    assert np.array_equal(I["edge"], d["edge"]) and np.array_equal(I["binmask"], d["binmask"])
    assert np.array_equal(phi, d["phi"])
    c = O.complexity_mlp(phi.reshape(-1, 8), W).reshape(phi.shape[:3])
    C = np.clip(O.bilateral(c), np.float32(0.0), np.float32(1.0)).astype(np.float32)
    assert rel(C, d["complexity"]) < 1e-6
    assert np.array_equal(O.mlp_mapper(C, W, 1.0), d["bits_mlp"])
    assert np.array_equal(O.linear_mapper(C, 1.0), d["bits_lin"])


# ---- the reference's own known-answer tests (tests/test_smoke.py) ----------

def test_euler_component_kat():
    """test_smoke.py:214-223: one blob -> 1, two blobs -> 2 on a 16x16 map."""
    m = np.zeros((1, 16, 16), np.uint8)
    m[0, 2:6, 2:6] = 1
    assert O.euler_components_tiles(m, 16)[0, 0, 0] == 1.0
    m[0, 10:14, 10:14] = 1
    assert O.euler_components_tiles(m, 16)[0, 0, 0] == 2.0


def test_linear_mapper_kats():
    """test_smoke.py:188-211."""
    c = (np.linspace(0, 1, 16, dtype=np.float32).reshape(1, 4, 4) * np.float32(0.05) + np.float32(0.4)).astype(np.float32)
    b = O.linear_mapper(c, 1.0)
    assert b.min() == 2.0 and b.max() == 8.0 and len(np.unique(b)) >= 5
    for v, want in ((0.5, 5.0), (0.0, 2.0), (1.0, 8.0)):
        bb = O.linear_mapper(np.full((1, 8, 8), v, np.float32), 1.0)
        assert np.all(bb == want)


@pytest.mark.parametrize("H", [640, 80, 40, 20])
def test_tile_size_and_ranges(H):
    """test_smoke.py:33-47: pow2 tiles >= 4 and phi in [0, 1]."""
    t = O.tile_size(H, 8)
    assert t >= 4 and (t & (t - 1)) == 0
    if H <= 80:
        x = np.random.default_rng(H).random((2, 3, H, H)).astype(np.float32)
        phi = O.phi_tiles(x, 8)
        assert phi.shape == (2, H // t, H // t, 8)
        assert phi.min() >= 0.0 and phi.max() <= 1.0 + 1e-5


def test_log2_overrides_match_torch():
    torch = pytest.importorskip("torch")
    for T in (4, 8, 16, 32, 64, 128):
        p = (np.arange(T * T + 1, dtype=np.float32) / np.float32(T * T)).astype(np.float32)
        a = (p + np.float32(1e-10)).astype(np.float32)
        assert np.array_equal(torch.log2(torch.from_numpy(a)).numpy(), O.log2_torch(a))


def test_spatial_quantize_compat_vs_pytorch_semantics():
    """The reference kernel contract (mcaq_kernel.cu) on a divisible grid equals
    the PyTorch quantizer (quantization.py:729-746) with the same min/max."""
    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, 8, 32, 32)).astype(np.float32)
    bits = rng.integers(2, 9, (2, 4, 4)).astype(np.float32)
    mn, mx = x.min(axis=(0, 2, 3)), x.max(axis=(0, 2, 3))
    y1 = O.spatial_quantize_compat(x, bits, mn, mx, 8, 8, None)
    y2 = O.quantize(x, bits, None, mn, mx)
    assert np.array_equal(y1, y2)
    assert math.isfinite(float(y1.sum()))


OPT_CASES = sorted(f[4:-4] for f in os.listdir(GOLDEN) if f.startswith("opt_") and f.endswith(".npz"))


def _opts(d):
    return {k[4:]: (str(d[k]) if d[k].dtype.kind == "U" else d[k].item()) for k in d.files if k.startswith("opt_")}


@pytest.mark.parametrize("name", ["opt_" + c for c in OPT_CASES] + ["case_m_p3", "case_m_p4"])
def test_option_and_yolov8m_fixtures(name):
    """The analyzer switches (binarize_impl='otsu', contour_components=False,
    canny_impl='legacy') and the yolov8m C3/C4 shapes, against the reference's
    own outputs (tests/golden/make_golden_r02.py)."""
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    W = load_weights()
    x = d["x"].astype(np.float32)
    opts = _opts(d)
    phi, I = O.phi_tiles(x, int(d["grid"]), internals=True, **opts)
    assert np.array_equal(I["edge"], d["edge"])
    assert np.array_equal(I["binmask"], d["binmask"])
    assert np.array_equal(phi[..., :7], d["phi"][..., :7])
    assert np.all(np.abs(phi[..., 7] - d["phi"][..., 7]) <= np.spacing(np.abs(d["phi"][..., 7])))
    C, _, _ = O.analyzer_forward(x, W, int(d["grid"]), **opts)
    assert rel(C, d["complexity"]) < 1e-6
    assert np.array_equal(O.mlp_mapper(C, W, 1.0), d["bits_mlp"])
    assert np.array_equal(O.linear_mapper(C, 1.0), d["bits_lin"])


def test_softmax_exp_partition_matches_aten():
    """ATen's dim-1 softmax of (B, 2, ht, wt): SLEEF expf on vectorized lanes,
    glibc on scalar tails, by at::parallel_for's partition for T threads
    (oracle/ieee.py); bit-exact vs torch.softmax for T = 1, 3, 8, 16 on hook
    tile grids.  Plain cr-exp everywhere differs from torch on ~1 % of tiles."""
    import torch
    from oracle.ieee import aten_softmax_vec_lanes, cr32, sleef_expf32
    rng = np.random.default_rng(11)
    old = torch.get_num_threads()
    try:
        for T in (1, 3, 8, 16):
            torch.set_num_threads(T)
            for B, ht, wt in ((1, 10, 10), (3, 11, 13), (32, 10, 10), (32, 5, 5), (16, 20, 20), (2, 37, 41)):
                lg = (rng.standard_normal((B, 2, ht, wt)) * 3).astype(np.float32)
                ref = torch.softmax(torch.from_numpy(lg), 1)[:, 0].numpy()
                vl = aten_softmax_vec_lanes(B, ht * wt, T).reshape(B, ht, wt)
                mx = np.maximum(lg[:, 0], lg[:, 1])
                a0, a1 = (lg[:, 0] - mx).astype(np.float32), (lg[:, 1] - mx).astype(np.float32)
                e0 = np.where(vl, sleef_expf32(a0), cr32(np.exp, a0))
                e1 = np.where(vl, sleef_expf32(a1), cr32(np.exp, a1))
                m = (e0 / (e0 + e1).astype(np.float32)).astype(np.float32)
                assert np.array_equal(m, ref), (T, B, ht, wt, int((m != ref).sum()))
    finally:
        torch.set_num_threads(old)


def test_sleef_expf_restatement():
    """sleef_expf32 on a sweep of arguments: finite, within 1 ulp of the
    correctly rounded exp, exactly 1 at 0, 0 below -104."""
    from oracle.ieee import cr32, sleef_expf32
    x = np.linspace(-103.0, 88.0, 200001).astype(np.float32)
    e = sleef_expf32(x)
    c = cr32(np.exp, x)
    ulp = np.abs(e.view(np.int32).astype(np.int64) - c.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1 and 0.01 < (ulp == 1).mean() < 0.3
    assert sleef_expf32(np.float32(0.0)) == 1.0 and sleef_expf32(np.float32(-105.0)) == 0.0


def test_reciprocal_division_is_correctly_rounded():
    """The kernels' x / s (mcaq_math.h div_by): q0 = RN(x * RN(1/s)),
    r = x - q0 s exactly (FMA), RN(q0 + r RN(1/s)) equals IEEE x / s on
    qparam-shaped scales and on divisors with adversarial mantissas."""
    from oracle.ieee import fma32
    f32 = np.float32
    rng = np.random.default_rng(3)
    n = 400000
    rngv = np.exp(rng.uniform(np.log(1e-8), np.log(50.0), n)).astype(f32)
    s = (rngv / (2.0 ** rng.integers(1, 16, n) - 1).astype(f32)).astype(f32)
    x = (rng.standard_normal(n) * np.exp(rng.uniform(-8, 5, n))).astype(f32)
    mant = np.array([0x7fffff, 0x7ffffe, 0x000001, 0x400000, 0x555555], np.uint32)
    adv = ((np.arange(110, 135, dtype=np.uint32)[:, None] << 23) | mant[None, :]).ravel().view(f32)
    s = np.concatenate([s, np.repeat(adv, 2000)])
    x = np.concatenate([x, rng.uniform(-1000, 1000, adv.size * 2000).astype(f32)])
    y = (f32(1.0) / s).astype(f32)
    q0 = (x * y).astype(f32)
    q1 = fma32(fma32(-q0, s, x), y, q0)
    assert np.array_equal(q1, (x / s).astype(f32))
