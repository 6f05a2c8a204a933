"""CPU oracle for the MCAQ spatial-adaptive-quantization inference path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker / the timed
CPU baseline.  The product (mcaq_yolo_amd/) never imports it and never falls
back to it.

This is a from-scratch numpy restatement of the reference's pure-PyTorch hot
path (yooooonjae/mcaq-yolo, files under mcaq_yolo/), written as an explicit
sequence of IEEE fp32 operations so that it is machine independent and so that
it is the exact arithmetic specification the HIP kernels implement:

  * the decision path (channel mean, normalisation, Sobel/Gaussian/adaptive
    convolutions, Otsu, NMS, hysteresis, LBP, box counts, Euler numbers, tile
    sums, quantile, quant/dequant) follows the CPU ATen order of the reference
    run and is pinned bit-for-bit against golden
    fixtures generated from the reference itself (tests/golden/);
  * transcendentals (exp, log, log2, log1p, atan2) are correctly rounded fp32
    values (float64 libm, one rounding); the reference's SLEEF/glibc results
    agree except at rare 1-ulp points - except the soft mask's channel
    softmax, where the 1-ulp points were seen to reach the output: there the
    exp is SLEEF expf_u10 (ieee.sleef_expf32) on the lanes ATen vectorizes
    and glibc on its scalar tails, by ATen's thread partition (REF_THREADS);
  * LayerNorm / BatchNorm / softmax / the N=1 GEMV use a fixed, documented
    order (ATen's internal order there is not reproduced: those values are
    continuous, compared against the fixtures within tolerance).

Layout conventions: x is (B, C, H, W) float32; per-image planes are (B, H, W);
tile maps are (B, ht, wt).
"""
import math

import numpy as np

from .ieee import aten_softmax_vec_lanes, aten_sum, cr32, f32, f64, fma32, rint32, seq_sum, sleef_expf32

# torch.get_num_threads() of the process that generated tests/golden (make_golden*.py
# set 8): the soft mask's softmax exp per tile depends on it (aten_softmax_vec_lanes)
REF_THREADS = 8

F32 = f32

# ---------------------------------------------------------------------------
# constants (values of the reference's run-time constant tensors on CPU)
# ---------------------------------------------------------------------------


def _gauss1d(k, sigma2x2):
    """exp(-(x^2)/(2 sigma^2)) normalised by its torch sum (5 or 11 taps).

    morphology.py:485-488 (Canny blur) and :566-570 (adaptive threshold).  The
    vector is short, so ATen sums it in row_sum order (tail columns)."""
    x = (np.arange(k, dtype=f32) - f32(k // 2)).astype(f32)
    g = cr32(np.exp, -(x * x) / f32(sigma2x2))
    s = aten_sum(g[:, None])[0]
    return (g / s).astype(f32)


def gaussian_kernels():
    """Returns dict of fp32 constant kernels used on the path."""
    g5 = _gauss1d(5, 2.0)                               # morphology.py:485-488
    sig = 0.3 * ((11 - 1) * 0.5 - 1) + 0.8               # morphology.py:566
    g11 = _gauss1d(11, 2 * sig ** 2)
    sm_sig = 5 / 3.0                                     # quantization.py:205-209
    g5s = _gauss1d(5, 2 * sm_sig ** 2)
    c = (np.arange(5, dtype=f32) - f32(2)).astype(f32)
    r2 = (c[:, None] * c[:, None] + c[None, :] * c[None, :]).astype(f32)
    spatial = cr32(np.exp, -r2 / f32(2 * 2.0 ** 2))      # morphology.py:346
    return {
        "gauss5_canny": (g5[None, :] * g5[:, None]).astype(f32),
        "gauss11_adaptive": (g11[None, :] * g11[:, None]).astype(f32),
        "smooth5_softmask": (g5s[None, :] * g5s[:, None]).astype(f32),
        "bilateral_spatial": spatial.astype(f32),
    }


K = gaussian_kernels()

# ---------------------------------------------------------------------------
# small building blocks
# ---------------------------------------------------------------------------


def tile_size(H, grid_size):
    """morphology.py:359-376: largest power of two <= max(4, H // grid)."""
    raw = max(4, H // grid_size)
    return 1 << (raw.bit_length() - 1)


def channel_mean(x, Hc, Wc):
    """gray = x[:, :, :Hc, :Wc].mean(1) (morphology.py:837) in ATen CPU order.

    Contiguous input: cascade outer reduction over C with HW columns.  A cropped
    (non-contiguous) view is reduced by ATen's elementwise path instead, i.e. a
    plain sequential sum over C.  mean = sum / C."""
    B, C, H, W = x.shape
    out = np.empty((B, Hc, Wc), f32)
    for b in range(B):
        if Hc == H and Wc == W:
            s = aten_sum(x[b].reshape(C, H * W)).reshape(H, W)
        else:
            s = seq_sum(x[b, :, :Hc, :Wc])
        out[b] = s / f32(C)
    return out


def abs_channel_mean(x):
    """x.abs().mean(1) over the full map (quantization.py:224)."""
    B, C, H, W = x.shape
    out = np.empty((B, H, W), f32)
    for b in range(B):
        out[b] = (aten_sum(np.abs(x[b]).reshape(C, H * W)) / f32(C)).reshape(H, W)
    return out


def normalize01(g):
    """morphology.py:379-383, per image: (x - min) / (max - min + 1e-8)."""
    mn = g.min(axis=(1, 2), keepdims=True)
    mx = g.max(axis=(1, 2), keepdims=True)
    return ((g - mn) / ((mx - mn) + f32(1e-8))).astype(f32)


def conv2d(img, k, pad="zero"):
    """Single-channel 'same' convolution in oneDNN order: taps row-major
    (kh outer, kw inner), fp32 FMA accumulation from 0.
    Zero-padded taps are exact no-ops and are skipped; replicate padding clamps
    the source coordinate."""
    B, H, W = img.shape
    kh, kw = k.shape
    ph, pw = kh // 2, kw // 2
    acc = np.zeros((B, H, W), f32)
    if pad == "replicate":
        src = img[:, np.clip(np.arange(-ph, H + ph), 0, H - 1)][:, :, np.clip(np.arange(-pw, W + pw), 0, W - 1)]
    else:
        src = np.zeros((B, H + 2 * ph, W + 2 * pw), f32)
        src[:, ph:ph + H, pw:pw + W] = img
    for i in range(kh):
        for j in range(kw):
            if k[i, j] == 0 and pad != "replicate":
                continue  # fma(0, v, acc) == acc exactly (acc is never -0)
            acc = fma32(k[i, j], src[:, i:i + H, j:j + W], acc)
    return acc


SOBEL_X = np.array([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]], f32)
SOBEL_Y = np.array([[-1, -2, -1], [0, 0, 0], [1, 2, 1]], f32)


def sobel(g):
    """morphology.py:386-395 (zero padding 1)."""
    return conv2d(g, SOBEL_X), conv2d(g, SOBEL_Y)


def otsu_threshold(v):
    """morphology.py:398-418 per image; v (B, H, W) in [0,1] -> thr (B,) fp32.

    histc ignores values outside [0,1]; bin = int(x*256) with 1.0 -> 255.
    cumsum accumulates in double and casts each prefix to fp32."""
    B = v.shape[0]
    centers = ((np.arange(256, dtype=f32) + f32(0.5)) / f32(256)).astype(f32)
    thr = np.empty(B, f32)
    for b in range(B):
        x = v[b].reshape(-1)
        x = x[(x >= 0) & (x <= 1)]
        idx = np.minimum((x * f32(256)).astype(np.int64), 255)
        hist = np.bincount(idx, minlength=256).astype(f32)
        p = (hist / max(f32(hist.sum()), f32(1.0))).astype(f32)
        omega = np.cumsum(p.astype(f64)).astype(f32)
        mu = np.cumsum((p * centers).astype(f32).astype(f64)).astype(f32)
        mu_t = mu[-1]
        num = (mu_t * omega - mu).astype(f32)
        num = (num * num).astype(f32)
        den = ((omega * (f32(1.0) - omega)).astype(f32) + f32(1e-12)).astype(f32)
        sb = (num / den).astype(f32)
        thr[b] = centers[int(np.argmax(sb))]
    return thr


def _shift_rep(t, dy, dx):
    B, H, W = t.shape
    return t[:, np.clip(np.arange(H) + dy, 0, H - 1)][:, :, np.clip(np.arange(W) + dx, 0, W - 1)]


def _max3x3(t, fill):
    """3x3 max pool, stride 1, padding 1 with `fill` outside the image."""
    B, H, W = t.shape
    p = np.full((B, H + 2, W + 2), fill, t.dtype)
    p[:, 1:-1, 1:-1] = t
    out = p[:, 0:H, 0:W].copy()
    for dy in range(3):
        for dx in range(3):
            out = np.maximum(out, p[:, dy:dy + H, dx:dx + W])
    return out


def nms_direction(gx, gy):
    """Direction bin 0..3 of morphology.py:430-444 (atan2 in degrees, folded
    to [0,180), bins at 22.5/67.5/112.5/157.5)."""
    ang = (cr32(np.arctan2, gy, gx) * f32(180.0 / math.pi)).astype(f32)
    ang = np.where(ang < 0, (ang + f32(180.0)).astype(f32), ang)
    d = np.zeros(ang.shape, np.int8)
    d[(ang >= f32(22.5)) & (ang < f32(67.5))] = 1
    d[(ang >= f32(67.5)) & (ang < f32(112.5))] = 2
    d[(ang >= f32(112.5)) & (ang < f32(157.5))] = 3
    return d


_NMS_NB = {0: ((0, 1), (0, -1)), 1: ((-1, 1), (1, -1)),
           2: ((-1, 0), (1, 0)), 3: ((-1, -1), (1, 1))}


def canny_cv2compat(gray, hysteresis_iters=8, return_internals=False):
    """morphology.py:458-509 -> edge map (B, H, W) uint8 {0,1}."""
    b01 = conv2d(gray, K["gauss5_canny"])
    thr255 = (otsu_threshold(b01) * f32(255.0)).astype(f32)
    b255 = (b01 * f32(255.0)).astype(f32)
    gx, gy = sobel(b255)
    mag = (np.abs(gx) + np.abs(gy)).astype(f32)
    d = nms_direction(gx, gy)
    nms = np.zeros_like(mag)
    for k, ((dy1, dx1), (dy2, dx2)) in _NMS_NB.items():
        keep = (mag >= _shift_rep(mag, dy1, dx1)) & (mag >= _shift_rep(mag, dy2, dx2))
        nms = np.where((d == k) & keep, mag, nms)
    t = thr255[:, None, None]
    strong = nms > t
    weak = nms > (f32(0.5) * t).astype(f32)
    edge = strong.astype(np.uint8)
    for _ in range(max(1, hysteresis_iters)):
        grown = _max3x3(edge, 0)
        edge = np.where(weak & (grown > 0), np.uint8(1), edge).astype(np.uint8)
    if return_internals:
        return edge, dict(blur=b01, thr=thr255 / f32(255.0), mag=mag, dir=d)
    return edge


def _nms(mag, gx, gy):
    d = nms_direction(gx, gy)
    out = np.zeros_like(mag)
    for k, ((dy1, dx1), (dy2, dx2)) in _NMS_NB.items():
        keep = (mag >= _shift_rep(mag, dy1, dx1)) & (mag >= _shift_rep(mag, dy2, dx2))
        out = np.where((d == k) & keep, mag, out)
    return out


def _hysteresis(strong, weak, iters):
    edge = strong.astype(np.uint8)
    for _ in range(max(1, iters)):
        grown = _max3x3(edge, 0)
        edge = np.where(weak & (grown > 0), np.uint8(1), edge).astype(np.uint8)
    return edge


def canny_legacy(gray):
    """morphology.py:512-540 (canny_impl='legacy'): blur, Sobel of the blur,
    L2 magnitude sqrt(gx^2 + gy^2 + 1e-12), NMS, per-image min-max
    normalisation of the NMS map, Otsu of that map, 2 hysteresis rounds."""
    blur = conv2d(gray, K["gauss5_canny"])
    gx, gy = sobel(blur)
    s = ((gx * gx).astype(f32) + (gy * gy).astype(f32)).astype(f32)
    mag = cr32(np.sqrt, (s + f32(1e-12)).astype(f32))
    n = normalize01(_nms(mag, gx, gy))
    t = otsu_threshold(n)[:, None, None]
    return _hysteresis(n > t, n > (f32(0.5) * t).astype(f32), 2)


def otsu_binarize(gray):
    """binarize_impl='otsu' (morphology.py:420-424, 546-547)."""
    return (gray > otsu_threshold(gray)[:, None, None]).astype(np.uint8)


def adaptive_binarize(gray, C=2.0):
    """morphology.py:551-573: g255 > G11(g255, replicate) - C."""
    g255 = (gray * f32(255.0)).astype(f32)
    mean = conv2d(g255, K["gauss11_adaptive"], pad="replicate")
    return (g255 > (mean - f32(C)).astype(f32)).astype(np.uint8)


def _tiles(a, tile):
    """(B, Hc, Wc) -> (B, ht, wt, tile*tile) row-major window order."""
    B, H, W = a.shape
    ht, wt = H // tile, W // tile
    t = a[:, :ht * tile, :wt * tile].reshape(B, ht, tile, wt, tile)
    return t.transpose(0, 1, 3, 2, 4).reshape(B, ht, wt, tile * tile)


def tile_mean_seq(a, tile):
    """avg_pool2d(tile): sequential row-major window sum / tile^2 (A.3)."""
    t = _tiles(a.astype(f32), tile)
    s = seq_sum(np.moveaxis(t, -1, 0))
    return (s / f32(tile * tile)).astype(f32)


def fractal_tiles(edge, tile, batch_offset=0, batch_total=None):
    """morphology.py:576-621 -> Df (B, ht, wt) in [1, 2].

    y-sums over the S scales reduce a (S, B*ht*wt) tensor: the ATen tail order
    depends on the tile's column in the WHOLE batch (batch_offset/total)."""
    B, H, W = edge.shape
    ht, wt = H // tile, W // tile
    scales = []
    s = 2
    while s <= tile:
        scales.append(s)
        s *= 2
    S = len(scales)
    if S < 2:
        return np.ones((B, ht, wt), f32)
    counts = []
    for s in scales:
        occ = edge[:, :ht * tile, :wt * tile].reshape(B, ht * tile // s, s, wt * tile // s, s).max(axis=(2, 4))
        k = tile // s
        n = occ.reshape(B, ht, k, wt, k).sum(axis=(2, 4)).astype(f32)
        counts.append(n)
    n = np.stack(counts)                                   # (S, B, ht, wt)
    x = cr32(np.log, np.array(scales, f32))                # (S,)
    y = cr32(np.log, (n + f32(1.0)).astype(f32))
    w = cr32(np.exp, (f32(-0.1) * np.arange(S, dtype=f32)).astype(f32))
    w_sum = aten_sum(w[:, None])[0]
    x_mean = (aten_sum((w * x).astype(f32)[:, None])[0] / w_sum).astype(f32)
    if batch_total is None:
        batch_total = B
    M = batch_total * ht * wt
    off = batch_offset * ht * wt
    wy = (w[:, None, None, None] * y).astype(f32).reshape(S, -1)
    y_mean = (aten_sum(wy, off, M) / w_sum).astype(f32).reshape(B, ht, wt)
    t1 = (w * (x - x_mean).astype(f32)).astype(f32)
    cov_terms = (t1[:, None, None, None] * (y - y_mean[None]).astype(f32)).astype(f32).reshape(S, -1)
    cov = aten_sum(cov_terms, off, M).reshape(B, ht, wt)
    dx = (x - x_mean).astype(f32)
    var = aten_sum((w * (dx * dx).astype(f32)).astype(f32)[:, None])[0]
    df = -(cov / (var + f32(1e-12))).astype(f32)
    return np.clip(df, f32(1.0), f32(2.0)).astype(f32)


LBP_SUM_ORDER = (8, 9, 0, 1, 2, 3, 4, 5, 6, 7)

# Arguments k/T^2 + 1e-10 (T <= 128) whose CPU torch.log2 is not the correctly
# rounded value: fp32 bit pattern of the argument -> bit pattern of the result.
LOG2_OVERRIDES = {
    0x3F4ABC00: 0xBEAC50B0,
    0x3F553400: 0xBE871FE6,
    0x3F5F7400: 0xBE48E134,
    0x3F6C9400: 0xBDE91E32,
    0x3F78CC00: 0xBD28A796,
    0x3F7A7C00: 0xBD00B59C,
    0x3F7B8000: 0xBCD1987E,
    0x3F7BE800: 0xBCBE853E,
    0x3F7CA400: 0xBC9C1DC6,
    0x3F7FFC00: 0xB8B8ABAC,   # 0x3F7B8000 = 0.982421875 is the only one for T <= 64
}


def log2_torch(a):
    """fp32 log2 as the reference's CPU run computes it for the LBP terms:
    correctly rounded, except the LOG2_OVERRIDES arguments."""
    a = np.asarray(a, f32)
    r = cr32(np.log2, a)
    ab = a.view(np.uint32)
    for k, v in LOG2_OVERRIDES.items():
        r = np.where(ab == np.uint32(k), np.array(v, np.uint32).view(f32), r)
    return r.astype(f32)
_LBP_OFFS = [(-1, -1), (-1, 0), (-1, 1), (0, 1), (1, 1), (1, 0), (1, -1), (0, -1)]


def lbp_labels(gray):
    """Uniform LBP label 0..9 per pixel (morphology.py:630-646)."""
    bits = [(_shift_rep(gray, dy, dx) >= gray) for dy, dx in _LBP_OFFS]
    bits = np.stack(bits).astype(np.int8)
    n1 = bits.sum(0)
    trans = np.abs(bits - np.roll(bits, 1, axis=0)).sum(0)
    return np.where(trans <= 2, n1, 9).astype(np.int8)


def lbp_entropy_tiles(gray, tile):
    """morphology.py:624-652: per-tile entropy of the 10-bin LBP histogram /
    log2(10).  one_hot(...).permute(0,3,1,2) makes the pooled histogram
    channels-last, so ATen sums the 10 bins of each tile as a contiguous inner
    row (vectorized_inner_sum, 8-wide vectors): the scalar tail (bins 8, 9) is
    summed from 0 first, then the 8 vector lanes (bins 0..7) are added in
    order."""
    B = gray.shape[0]
    lab = _tiles(lbp_labels(gray), tile)                   # (B, ht, wt, T2)
    ht, wt = lab.shape[1:3]
    T2 = tile * tile
    cnt = np.stack([(lab == i).sum(-1) for i in range(10)], axis=1).astype(f32)
    p = (cnt / f32(T2)).astype(f32)                        # (B, 10, ht, wt)
    lg = log2_torch(p + f32(1e-10))
    terms = (p * lg).astype(f32)
    acc = np.zeros((B, ht, wt), f32)
    for k in LBP_SUM_ORDER:
        acc = (acc + terms[:, k]).astype(f32)
    ent = -acc
    return (ent / f32(math.log2(10.0))).astype(f32)


def gradvar_tiles(gx, gy, tile):
    """morphology.py:655-670: v = Var(gx)+Var(gy) per tile; v/(v+1)."""
    def tvar(t):
        m = tile_mean_seq(t, tile)
        m2 = tile_mean_seq((t * t).astype(f32), tile)
        return np.maximum((m2 - (m * m).astype(f32)).astype(f32), f32(0.0))
    v = (tvar(gx) + tvar(gy)).astype(f32)
    return (v / (v + f32(1.0))).astype(f32)


_Q1 = {1, 2, 4, 8}
_Q3 = {7, 11, 13, 14}
_QD = {6, 9}


def euler_components_tiles(m, tile):
    """morphology.py:673-707: K = round(sum of per-window Euler quads) >= 1.
    Window (i, j) covers m[i-1..i, j-1..j] of the zero-padded map and is
    attributed to tile (i // tile, j // tile)."""
    B, H, W = m.shape
    mp = np.zeros((B, H + 2, W + 2), np.int32)
    mp[:, 1:-1, 1:-1] = m
    idx = (mp[:, :-1, :-1] + 2 * mp[:, :-1, 1:] + 4 * mp[:, 1:, :-1] + 8 * mp[:, 1:, 1:])
    e = np.zeros(idx.shape, f32)
    e[np.isin(idx, list(_Q1))] = f32(0.25)
    e[np.isin(idx, list(_Q3))] = f32(-0.25)
    e[np.isin(idx, list(_QD))] = f32(-0.5)
    ht, wt = H // tile, W // tile
    s = tile_mean_seq(e[:, :ht * tile, :wt * tile], tile)
    Kr = (s * f32(tile * tile)).astype(f32)
    return np.maximum(rint32(Kr), f32(1.0)).astype(f32)


def contour_tiles(binmask, tile, contour_components=True):
    """morphology.py:709-739 -> phi5 (B, ht, wt)."""
    m = binmask.astype(np.uint8)
    eroded = -_max3x3(-m.astype(np.int16), -32768)
    boundary = np.maximum(m.astype(np.int16) - eroded, 0).astype(f32)
    area = (tile_mean_seq(m.astype(f32), tile) * f32(tile * tile)).astype(f32)
    perim = (tile_mean_seq(boundary, tile) * f32(tile * tile)).astype(f32)
    den = ((f32(4.0 * math.pi) * area).astype(f32) + f32(1e-6)).astype(f32)
    ic = ((perim * perim).astype(f32) / den).astype(f32)
    if contour_components:
        ic = (ic / euler_components_tiles(m, tile)).astype(f32)
    phi5 = (f32(1.0) - (f32(1.0) / np.maximum(ic, f32(1.0))).astype(f32)).astype(f32)
    return np.where(area > 0, phi5, f32(0.0)).astype(f32)


def score_image(x, grid_size=8, feature_weights=None):
    """score_image (morphology.py:923-937): per-image mean over tiles of
    sum(alpha * phi[..., :5]), alpha = |w| / max(sum|w|, 1e-8), clamp [0, 1]."""
    phi = phi_tiles(x, grid_size)
    w = np.full(5, 0.2, np.float32) if feature_weights is None else np.asarray(feature_weights, np.float32)
    a = np.abs(w)
    a = (a / max(np.float32(a.sum()), np.float32(1e-8))).astype(np.float32)
    c = (phi[..., :5].astype(np.float64) * a.astype(np.float64)).sum(-1)
    return np.clip(c.mean(axis=(1, 2)), 0.0, 1.0).astype(np.float32)


def phi_tiles(x, grid_size=8, batch_offset=0, batch_total=None, internals=False, canny_impl="cv2compat",
              binarize_impl="adaptive", contour_components=True):
    """_phi_tiles_gpu (morphology.py:826-873) -> phi (B, ht, wt, 8); the
    analyzer switches of morphology.py:29-37 select the legacy variants."""
    B, C, H, W = x.shape
    tile = tile_size(H, grid_size)
    ht, wt = H // tile, W // tile
    Hc, Wc = ht * tile, wt * tile
    graw = channel_mean(x, Hc, Wc)
    gray = normalize01(graw)
    gx, gy = sobel(gray)
    edge, ci = canny_cv2compat(gray, return_internals=True)
    if canny_impl == "legacy":
        edge = canny_legacy(gray)
    binm = otsu_binarize(gray) if binarize_impl == "otsu" else adaptive_binarize(gray)
    p1 = (fractal_tiles(edge, tile, batch_offset, batch_total) / f32(2.0)).astype(f32)
    p2 = lbp_entropy_tiles(gray, tile)
    p3 = gradvar_tiles(gx, gy, tile)
    p4 = tile_mean_seq(edge.astype(f32), tile)
    p5 = contour_tiles(binm, tile, contour_components)
    p8 = cr32(np.sqrt, ((p4 * p5).astype(f32) + f32(1e-12)).astype(f32))
    phi = np.stack([p1, p2, p3, p4, p5, (p1 * p2).astype(f32), (p3 * p3).astype(f32), p8], axis=-1)
    if internals:
        return phi, dict(gray_raw=graw, gray=gray, gx=gx, gy=gy, edge=edge, binmask=binm,
                         blur=ci["blur"], otsu_thr=ci["thr"], tile=tile)
    return phi


# ---------------------------------------------------------------------------
# MLPs (fixed documented order; see module docstring)
# ---------------------------------------------------------------------------


def linear(x, Wt, b):
    """y_j = (sum_k fma over k from 0 in order) + b_j."""
    acc = np.zeros(x.shape[:-1] + (Wt.shape[0],), f32)
    for k in range(Wt.shape[1]):
        acc = fma32(x[..., k:k + 1], Wt[:, k][None, :], acc)
    return (acc + b[None, :]).astype(f32)


def tree_sum(x):
    """Pairwise tree over the last axis (N a power of two): adjacent pairs are
    added level by level.  This is the reduction order the HIP kernels use for
    LayerNorm statistics (a 64-lane xor butterfly produces exactly this tree)."""
    a = np.asarray(x, f32)
    while a.shape[-1] > 1:
        a = (a[..., 0::2] + a[..., 1::2]).astype(f32)
    return a[..., 0]


def layernorm(x, g, b, eps=1e-5):
    """LayerNorm over the last axis with a fixed order (module docstring):
    mean = tree_sum(x)/N; d = x - mean; var = tree_sum(d*d)/N;
    rstd = 1/sqrt(var + eps); y = ((d * rstd) * g) + b   (fp32, no FMA)."""
    N = x.shape[-1]
    mean = (tree_sum(x) / f32(N)).astype(f32)
    d = (x - mean[..., None]).astype(f32)
    var = (tree_sum((d * d).astype(f32)) / f32(N)).astype(f32)
    rstd = (f32(1.0) / cr32(np.sqrt, (var + f32(eps)).astype(f32))).astype(f32)
    return (((d * rstd[..., None]).astype(f32) * g[None, :]).astype(f32) + b[None, :]).astype(f32)


def sigmoid(z):
    e = cr32(np.exp, -z)
    return (f32(1.0) / (f32(1.0) + e).astype(f32)).astype(f32)


def complexity_mlp(phi, P):
    """morphology.py:81-97 on (N, 8) features."""
    h = linear(phi, P["complexity_analyzer.complexity_mlp.0.weight"], P["complexity_analyzer.complexity_mlp.0.bias"])
    h = np.maximum(layernorm(h, P["complexity_analyzer.complexity_mlp.1.weight"],
                             P["complexity_analyzer.complexity_mlp.1.bias"]), f32(0))
    h = linear(h, P["complexity_analyzer.complexity_mlp.3.weight"], P["complexity_analyzer.complexity_mlp.3.bias"])
    h = np.maximum(layernorm(h, P["complexity_analyzer.complexity_mlp.4.weight"],
                             P["complexity_analyzer.complexity_mlp.4.bias"]), f32(0))
    z = linear(h, P["complexity_analyzer.complexity_mlp.6.weight"], P["complexity_analyzer.complexity_mlp.6.bias"])
    return sigmoid(z)[..., 0]


def bilateral(c, sigma_r=0.1):
    """morphology.py:309-354 on the tile grid (B, ht, wt), 5x5, replicate."""
    B, H, W = c.shape
    sp = K["bilateral_spatial"].reshape(-1)
    pat = np.stack([_shift_rep(c, i - 2, j - 2) for i in range(5) for j in range(5)])  # (25,B,H,W)
    d = (pat - c[None]).astype(f32)
    rw = cr32(np.exp, (-(d * d).astype(f32) / f32(2 * sigma_r ** 2)).astype(f32))
    w = (sp[:, None, None, None] * rw).astype(f32)
    wp = (w * pat).astype(f32)
    out = np.empty((B, H, W), f32)
    for b in range(B):
        num = aten_sum(wp[:, b].reshape(25, -1))
        den = aten_sum(w[:, b].reshape(25, -1))
        out[b] = (num / (den + f32(1e-8))).reshape(H, W)
    return out


def analyzer_forward(x, P, grid_size=8, batch_offset=0, batch_total=None, **opts):
    """MorphologicalComplexityAnalyzer.forward (morphology.py:939-973)."""
    phi = phi_tiles(x, grid_size, batch_offset, batch_total, **opts)
    B, ht, wt, _ = phi.shape
    c = complexity_mlp(phi.reshape(-1, 8), P).reshape(B, ht, wt)
    return np.clip(bilateral(c), f32(0.0), f32(1.0)).astype(f32), phi, c


def batchnorm_eval(x, g, b, rm, rv, eps=1e-5):
    """alpha = g/sqrt(rv+eps) (as inv*g), beta = b - (rm*inv)*g; y = x*alpha + beta."""
    inv = (f32(1.0) / cr32(np.sqrt, (rv + f32(eps)).astype(f32))).astype(f32)
    alpha = (inv * g).astype(f32)
    beta = (b - ((rm * inv).astype(f32) * g).astype(f32)).astype(f32)
    return ((x * alpha[None, :]).astype(f32) + beta[None, :]).astype(f32)


def _finish_bits(bm, temperature, continuous, min_bits=2.0, max_bits=8.0):
    """Temperature multiply, STE clamp and STE round forward values
    (bit_allocation.py:264-278 / :72-79): v = b + (clamp(b) - b); r = v + (rint(v) - v)."""
    if temperature is not None:
        bm = (bm * f32(max(float(temperature), 0.1))).astype(f32)
    cl = np.clip(bm, f32(min_bits), f32(max_bits)).astype(f32)
    v = (bm + (cl - bm).astype(f32)).astype(f32)
    if not continuous:
        v = (v + (rint32(v) - v).astype(f32)).astype(f32)
    return v


def mlp_mapper(C, P, temperature=1.0, continuous=False, min_bits=2.0, max_bits=8.0, prefix="bit_mapper."):
    """ComplexityToBitMappingNetwork.forward (bit_allocation.py:218-280)."""
    c = np.clip(C, f32(0.0), f32(1.0)).astype(f32)
    z = np.stack([c, (c * c).astype(f32), cr32(np.log1p, c)], axis=-1).reshape(-1, 3)
    h = z
    for li, bi in ((0, 1), (3, 4), (6, 7)):
        h = linear(h, P[prefix + "mapping_network.%d.weight" % li], P[prefix + "mapping_network.%d.bias" % li])
        h = batchnorm_eval(h, P[prefix + "mapping_network.%d.weight" % bi], P[prefix + "mapping_network.%d.bias" % bi],
                           P[prefix + "mapping_network.%d.running_mean" % bi],
                           P[prefix + "mapping_network.%d.running_var" % bi])
        h = np.maximum(h, f32(0))
    zf = linear(h, P[prefix + "mapping_network.9.weight"], P[prefix + "mapping_network.9.bias"])
    hs = sigmoid(zf)[:, 0].reshape(C.shape)
    bm = (f32(min_bits) + (f32(max_bits - min_bits) * hs).astype(f32)).astype(f32)
    return _finish_bits(bm, temperature, continuous, min_bits, max_bits)


def quantile_rows(flat, q):
    """torch.quantile(flat, q, dim=1) linear interpolation."""
    s = np.sort(flat, axis=1)
    n = s.shape[1]
    rank = (f32(q) * f32(n - 1)).astype(f32)
    lo = int(rank)
    hi = int(math.ceil(float(rank)))
    w = (rank - f32(lo)).astype(f32)
    a = s[:, lo]
    b = s[:, hi]
    diff = (b - a).astype(f32)
    if abs(w) < 0.5:
        return fma32(w, diff, a)
    return fma32(-diff, (f32(1.0) - w).astype(f32), b)


def linear_mapper(C, temperature=1.0, continuous=False, min_bits=2.0, max_bits=8.0, eps_spread=1e-3):
    """LinearBitMapper.forward (bit_allocation.py:42-80)."""
    B = C.shape[0]
    flat = C.reshape(B, -1).astype(f32)
    lo = quantile_rows(flat, 0.02)[:, None, None]
    hi = quantile_rows(flat, 0.98)[:, None, None]
    spread = (hi - lo).astype(f32)
    rel = np.clip(((C - lo).astype(f32) / (spread + f32(1e-8)).astype(f32)).astype(f32), f32(0), f32(1))
    cn = np.where(spread > f32(eps_spread), rel, np.clip(C, f32(0), f32(1))).astype(f32)
    bm = (f32(min_bits) + (f32(max_bits - min_bits) * cn).astype(f32)).astype(f32)
    return _finish_bits(bm, temperature, continuous, min_bits, max_bits)


def normalize_complexity(C):
    """Optional per-image percentile normalisation (models/mcaq_yolo.py:427-432)."""
    B = C.shape[0]
    flat = C.reshape(B, -1).astype(f32)
    lo = quantile_rows(flat, 0.02)[:, None, None]
    hi = quantile_rows(flat, 0.98)[:, None, None]
    den = ((hi - lo).astype(f32) + f32(1e-8)).astype(f32)
    return np.clip(((C - lo).astype(f32) / den).astype(f32), f32(0), f32(1)).astype(f32)


# ---------------------------------------------------------------------------
# soft mask + quantizer
# ---------------------------------------------------------------------------


def nearest_index(out_size, in_size):
    """PyTorch 'nearest' source index for each output index (upsample_nearest)."""
    o = np.arange(out_size)
    if out_size == in_size:
        return o
    if out_size == 2 * in_size:
        return o >> 1
    scale = f32(in_size) / f32(out_size)
    return np.minimum(np.floor((o.astype(f32) * scale).astype(f32)).astype(np.int64), in_size - 1)


def adaptive_avg_pool(a, oh, ow):
    """adaptive_avg_pool2d on (B, H, W): window [floor(i*H/oh), ceil((i+1)*H/oh)),
    sequential row-major sum, then / kh / kw."""
    B, H, W = a.shape
    out = np.empty((B, oh, ow), f32)
    for i in range(oh):
        h0, h1 = (i * H) // oh, ((i + 1) * H + oh - 1) // oh
        for j in range(ow):
            w0, w1 = (j * W) // ow, ((j + 1) * W + ow - 1) // ow
            win = a[:, h0:h1, w0:w1].reshape(B, -1)
            s = seq_sum(win.T)
            out[:, i, j] = ((s / f32(h1 - h0)).astype(f32) / f32(w1 - w0)).astype(f32)
    return out


def soft_mask(bits, x, P, prefix="soft_mask.", absmean=None, threads=None):
    """LearnedSoftMask.forward (quantization.py:213-239) -> m (B, H, W).
    threads: torch thread count of the reference run (default REF_THREADS):
    ATen's softmax takes SLEEF's exp on vectorized lanes, glibc's on tails."""
    B, C, H, W = x.shape
    Ht, Wt = bits.shape[1:]
    if absmean is None:
        absmean = abs_channel_mean(x)
    act = adaptive_avg_pool(absmean, Ht, Wt)
    amax = act.max(axis=(1, 2), keepdims=True)
    act = (act / (amax + f32(1e-8)).astype(f32)).astype(f32)
    bn = np.clip(((bits.astype(f32) - f32(2.0)).astype(f32) / f32(6.0)).astype(f32), f32(0), f32(1))
    feats = np.stack([bn, act], axis=1)                   # (B, 2, Ht, Wt)
    w1 = P[prefix + "net.0.weight"]
    b1 = P[prefix + "net.0.bias"]
    w2 = P[prefix + "net.2.weight"]
    b2 = P[prefix + "net.2.bias"]
    # conv 3x3 (2->8), zero pad: (kh, kw) outer, ic inner, FMA from 0, + bias
    h1 = np.zeros((B, 8, Ht, Wt), f32)
    hh, ww = np.arange(Ht), np.arange(Wt)
    for oc in range(8):
        acc = np.zeros((B, Ht, Wt), f32)
        for i in range(3):
            for j in range(3):
                sh, sw = hh + i - 1, ww + j - 1
                vm = ((sh >= 0) & (sh < Ht))[:, None] & ((sw >= 0) & (sw < Wt))[None, :]
                for ic in range(2):
                    src = feats[:, ic][:, np.clip(sh, 0, Ht - 1)][:, :, np.clip(sw, 0, Wt - 1)]
                    acc = np.where(vm[None], fma32(w1[oc, ic, i, j], src, acc), acc).astype(f32)
        h1[:, oc] = np.maximum((acc + b1[oc]).astype(f32), f32(0))
    # conv 1x1 (8->2): accumulator starts at the bias, FMA over ic
    logit = np.zeros((B, 2, Ht, Wt), f32)
    for oc in range(2):
        acc = np.full((B, Ht, Wt), b2[oc], f32)
        for ic in range(8):
            acc = fma32(w2[oc, ic, 0, 0], h1[:, ic], acc)
        logit[:, oc] = acc
    mx = np.maximum(logit[:, 0], logit[:, 1])
    vl = aten_softmax_vec_lanes(B, Ht * Wt, REF_THREADS if threads is None else threads).reshape(B, Ht, Wt)
    a0 = (logit[:, 0] - mx).astype(f32)
    a1 = (logit[:, 1] - mx).astype(f32)
    e0 = np.where(vl, sleef_expf32(a0), cr32(np.exp, a0))
    e1 = np.where(vl, sleef_expf32(a1), cr32(np.exp, a1))
    mt = (e0 / (e0 + e1).astype(f32)).astype(f32)          # (B, Ht, Wt)
    up = mt[:, nearest_index(H, Ht)][:, :, nearest_index(W, Wt)]
    return conv2d(up, K["smooth5_softmask"], pad="replicate")


def qparams(xmin, xmax, b):
    """QuantizationParameters (quantization.py:26-66) for integer bit width b."""
    qmin, qmax = -(2 ** (b - 1)), 2 ** (b - 1) - 1
    rng = np.maximum((xmax - xmin).astype(f32), f32(1e-8))
    scale = (rng / f32(qmax - qmin)).astype(f32)
    zp = (f32(qmin) - (xmin / scale).astype(f32)).astype(f32)
    zp = np.clip(zp, f32(qmin), f32(qmax)).astype(f32)
    return scale, zp, f32(qmin), f32(qmax)


def quantize(x, bits, m=None, xmin=None, xmax=None):
    """SpatialAdaptiveQuantization inference (quantization.py:729-746) as the
    equivalent single pass: y = ((clamp(rint(x/s+zp)) - zp) * s) * m."""
    B, C, H, W = x.shape
    Ht, Wt = bits.shape[1:]
    if xmin is None:
        xmin = x.min(axis=(0, 2, 3))
        xmax = x.max(axis=(0, 2, 3))
    bpix = bits[:, nearest_index(H, Ht)][:, :, nearest_index(W, Wt)]   # (B, H, W)
    y = np.zeros_like(x)
    for bv in np.unique(bits):
        bi = int(round(float(bv)))
        s, zp, qmin, qmax = qparams(xmin, xmax, bi)
        s = s[None, :, None, None]
        zp = zp[None, :, None, None]
        t = ((x / s).astype(f32) + zp).astype(f32)
        q = np.clip(rint32(t), qmin, qmax)
        deq = ((q - zp).astype(f32) * s).astype(f32)
        sel = (bpix == bv)[:, None]
        y = np.where(sel, deq, y)
    if m is not None:
        y = (y * m[:, None]).astype(f32)
    return y.astype(f32)


def spatial_quantize_compat(x, bit_map, min_vals, max_vals, tile_h, tile_w, mask=None):
    """mcaq_cuda_ops.spatial_quantize contract (ops/src/mcaq_ops.cpp:22-68,
    mcaq_kernel.cu:12-99) with round-half-even: tile = min(h//tile_h, Ht-1),
    bits = clamp(rint(bit), 2, 8)."""
    B, C, H, W = x.shape
    Ht, Wt = bit_map.shape[1:]
    th = np.minimum(np.arange(H) // tile_h, Ht - 1)
    tw = np.minimum(np.arange(W) // tile_w, Wt - 1)
    bpix = np.clip(rint32(bit_map), 2, 8)[:, th][:, :, tw]
    xmin = np.asarray(min_vals, f32).reshape(-1)
    xmax = np.asarray(max_vals, f32).reshape(-1)
    y = np.zeros_like(x)
    for bi in range(2, 9):
        s, zp, qmin, qmax = qparams(xmin, xmax, bi)
        s = s[None, :, None, None]
        zp = zp[None, :, None, None]
        q = np.clip(rint32(((x / s).astype(f32) + zp).astype(f32)), qmin, qmax)
        deq = ((q - zp).astype(f32) * s).astype(f32)
        y = np.where((bpix == bi)[:, None], deq, y)
    if mask is not None:
        y = (y * np.asarray(mask, f32).reshape(B, 1, H, W)).astype(f32)
    return y


# ---------------------------------------------------------------------------
# the hook (models/mcaq_yolo.py:409-455), inference
# ---------------------------------------------------------------------------


def hook_forward(x, P, grid_size=8, mapper="mlp", temperature=1.0, smooth=True,
                 normalize=False, softmask_prefix="soft_mask.", xmin=None, xmax=None, **opts):
    """analyzer -> (normalize) -> mapper -> quantizer.  Returns dict.  opts:
    the analyzer switches (canny_impl, binarize_impl, contour_components)."""
    C, phi, c_mlp = analyzer_forward(x, P, grid_size, **opts)
    Cn = normalize_complexity(C) if normalize else C
    if mapper == "mlp":
        bits = mlp_mapper(Cn, P, temperature, continuous=False)
    else:
        bits = linear_mapper(Cn, temperature, continuous=False)
    m = soft_mask(bits, x, P, softmask_prefix) if smooth else None
    if xmin is None:
        xmin = x.min(axis=(0, 2, 3))
        xmax = x.max(axis=(0, 2, 3))
    y = quantize(x, bits, m, xmin, xmax)
    return dict(y=y, complexity=C, bits=bits, m=m, phi=phi, c_mlp=c_mlp, xmin=xmin, xmax=xmax)


def load_weights(path):
    d = np.load(path)
    return {k: d[k].astype(f32) if d[k].dtype.kind == "f" else d[k] for k in d.files}


# ---------------------------------------------------------------------------
# QAT quantizer: the training branch (BASELINE config 5)
# ---------------------------------------------------------------------------
def ema_running_stats(x, rmin=None, rmax=None, momentum=0.99):
    """update_running_stats (quantization.py:319-353), per channel: the first
    batch takes the batch min/max, later ones r <- momentum*r + (1-momentum)*new
    (Python scalars rounded to fp32, then fp32 ops: SURVEY App. A.9)."""
    xmin = x.min(axis=(0, 2, 3)).astype(f32)
    xmax = x.max(axis=(0, 2, 3)).astype(f32)
    if rmin is None:
        return xmin, xmax
    a, c = f32(momentum), f32(1.0 - momentum)
    return (((a * rmin).astype(f32) + (c * xmin).astype(f32)).astype(f32),
            ((a * rmax).astype(f32) + (c * xmax).astype(f32)).astype(f32))


def _qdq(x, xmin, xmax, b):
    """StraightThroughEstimator.forward (quantization.py:74-92) for integer bits b,
    per-channel parameters: (clamp(rint(x/s + zp)) - zp) * s."""
    s, zp, qmin, qmax = qparams(xmin, xmax, b)
    s = s[None, :, None, None]
    zp = zp[None, :, None, None]
    t = ((x / s).astype(f32) + zp).astype(f32)
    q = np.clip(rint32(t), qmin, qmax)
    return ((q - zp).astype(f32) * s).astype(f32)


def qat_forward(x, bits, xmin, xmax, m=None, max_bits=8):
    """_forward_pytorch training branch (quantization.py:699-727, 733-737):
    per pixel, with b the nearest-upsampled continuous tile bits,
    xq = (1 - f) * Q_floor(b)(x) + f * Q_floor(b)+1(x), f = b - floor(b)
    (Q_floor(b)+1 := Q_floor(b) past max_bits), y = xq * m.  Returns (y, parts)."""
    B, C, H, W = x.shape
    Ht, Wt = bits.shape[1:]
    bits = bits.astype(f32)
    bfl = np.floor(bits).astype(f32)
    fr = (bits - bfl).astype(f32)
    ri, ci = nearest_index(H, Ht), nearest_index(W, Wt)
    bfu = bfl[:, ri][:, :, ci]
    fu = fr[:, ri][:, :, ci][:, None]                       # (B, 1, H, W)
    q_lo = np.zeros_like(x)
    q_hi = np.zeros_like(x)
    for bv in np.unique(bfu):
        lo = int(bv)
        ql = _qdq(x, xmin, xmax, lo)
        qh = _qdq(x, xmin, xmax, lo + 1) if lo + 1 <= max_bits else ql
        sel = (bfu == bv)[:, None]
        q_lo = np.where(sel, ql, q_lo)
        q_hi = np.where(sel, qh, q_hi)
    one_m_f = (f32(1.0) - fu).astype(f32)
    xq = ((one_m_f * q_lo).astype(f32) + (fu * q_hi).astype(f32)).astype(f32)
    y = (xq * m[:, None]).astype(f32) if m is not None else xq
    return y, {"xq": xq, "q_lo": q_lo, "q_hi": q_hi, "fu": fu, "one_m_f": one_m_f, "ri": ri, "ci": ci}


def qat_backward(g, x, bits, xmin, xmax, m=None, max_bits=8):
    """Gradients of qat_forward through the reference's autograd graph, with the
    STE identity dQ/dx = 1 (quantization.py:94-118):
      grad_x    = gm*(1-f) + gm*f,  gm = g*m               (elementwise, exact order)
      grad_m    = sum_c g*xq                               (B, H, W)
      grad_bits = sum over each tile's pixels of sum_c gm*(q_hi - q_lo)   (B, Ht, Wt)
    The two sums are accumulated in float64 (ATen's reduction order is not
    pinned; the kernels are compared within tolerance there)."""
    B, C, H, W = x.shape
    Ht, Wt = bits.shape[1:]
    _, I = qat_forward(x, bits, xmin, xmax, m, max_bits)
    gm = (g * m[:, None]).astype(f32) if m is not None else g.astype(f32)
    gx = ((gm * I["one_m_f"]).astype(f32) + (gm * I["fu"]).astype(f32)).astype(f32)
    gmask = (g.astype(f64) * I["xq"].astype(f64)).sum(axis=1) if m is not None else None
    gfu = (gm.astype(f64) * (I["q_hi"].astype(f64) - I["q_lo"].astype(f64))).sum(axis=1)   # (B, H, W)
    gb = np.zeros((B, Ht, Wt), f64)
    np.add.at(gb, (np.arange(B)[:, None, None], I["ri"][None, :, None], I["ci"][None, None, :]), gfu)
    return gx, gb, gmask
