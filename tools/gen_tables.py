"""Write mcaq_yolo_amd/csrc/mcaq_tables.h from the oracle's constant kernels.

The values are the CPU values of the reference's run-time constant tensors
(Gaussian kernels, bilateral spatial weights); tests/test_oracle_cpu.py pins
oracle.K against tests/golden/constants.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.ieee import aten_sum, cr32  # noqa: E402
from oracle.mcaq_oracle import K, log2_torch  # noqa: E402

HDR = os.path.join(ROOT, "mcaq_yolo_amd", "csrc", "mcaq_tables.h")


def table(name, arr):
    a = np.asarray(arr, np.float32).reshape(-1)
    words = ", ".join("0x%08Xu" % int(v) for v in a.view(np.uint32))
    return "MCAQ_TABLE uint32_t %s_bits[%d] = {%s};\n" % (name, a.size, words)


def fractal_constants():
    """Box-counting regression terms that depend only on the number of scales
    S = log2(tile) (morphology.py:596-617, oracle.fractal_tiles): x = log(s),
    w = exp(-0.1 i), and per S the scalars w_sum, x_mean, var; S <= 8 (the
    kernel's register arrays), tile <= 128 used."""
    f32 = np.float32
    x = cr32(np.log, np.array([2.0 ** (i + 1) for i in range(8)], f32))
    w = cr32(np.exp, (f32(-0.1) * np.arange(8, dtype=f32)).astype(f32))
    st = np.zeros((9, 4), f32)
    for S in range(2, 9):
        ws, xs = w[:S], x[:S]
        w_sum = aten_sum(ws[:, None])[0]
        x_mean = (aten_sum((ws * xs).astype(f32)[:, None])[0] / w_sum).astype(f32)
        dx = (xs - x_mean).astype(f32)
        var = aten_sum((ws * (dx * dx).astype(f32)).astype(f32)[:, None])[0]
        st[S, :3] = (w_sum, x_mean, var)
    return x, w, st


def separable_g11():
    """1-D factor of the 11x11 adaptive-threshold kernel and a proven bound on
    |separable fp32 estimate - exact oneDNN-order 121-tap fp32 sum| (+ the two
    roundings of `mean - C` and of the comparison difference) for inputs in
    [0, 255] (mcaq_morph.h, binarize)."""
    f32 = np.float32
    k2 = np.asarray(K["gauss11_adaptive"], f32).astype(np.float64)
    k1 = np.sqrt(np.diag(k2)).astype(f32)
    k1d = k1.astype(np.float64)
    u = 2.0 ** -24
    s1 = float(np.abs(k1d).sum())
    s2 = float(np.abs(k2).sum())
    e_exact = 121 * u * 255.0 * max(s2, 1.0)
    e_sep = 22 * u * 255.0 * max(s1, 1.0) ** 2
    e_kern = 255.0 * float(np.abs(np.outer(k1d, k1d) - k2).sum())
    e_sub = 3 * u * 300.0
    margin = 2.0 * (e_exact + e_sep + e_kern + e_sub)
    return k1, np.array([margin], f32)


def lbp_terms(T):
    """p * log2(p + 1e-10) for p = k / T^2, k = 0..T^2 (the per-label entropy
    term of morphology.py:640-650 as oracle.lbp_entropy_tiles computes it)."""
    f32 = np.float32
    p = (np.arange(T * T + 1, dtype=f32) / f32(T * T)).astype(f32)
    return (p * log2_torch((p + f32(1e-10)).astype(f32))).astype(f32)


def box_logs(n):
    """fp32 log(k + 1), k = 0..n (box-count regression ordinates, oracle.fractal_tiles)."""
    f32 = np.float32
    return cr32(np.log, (np.arange(n + 1, dtype=f32) + f32(1.0)).astype(f32))


def main():
    fx, fw, fst = fractal_constants()
    k1, marg = separable_g11()
    body = "".join(table(n, K[k]) for n, k in (
        ("k_gauss5", "gauss5_canny"), ("k_gauss11", "gauss11_adaptive"),
        ("k_smooth5", "smooth5_softmask"), ("k_bilat_sp", "bilateral_spatial")))
    body += table("k_frac_x", fx) + table("k_frac_w", fw) + table("k_frac_st", fst)
    body += table("k_g11_sep", k1) + table("k_g11_margin", marg)
    body += table("k_lbp_t4", lbp_terms(4)) + table("k_lbp_t8", lbp_terms(8)) + table("k_lbp_t16", lbp_terms(16))
    body += table("k_lognp1", box_logs(64))
    src = open(HDR).read()
    a = src.index("// @@TABLES@@")
    b = src.index("}  // namespace mcaq")
    src = src[:a] + "// @@TABLES@@\n" + body + src[b:]
    open(HDR, "w").write(src)
    print("wrote", HDR)


if __name__ == "__main__":
    main()
