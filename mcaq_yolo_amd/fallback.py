"""Pure-PyTorch path of the MCAQ hook (CPU tensors; BASELINE config 1).

The reference keeps a torch-only path beside its CUDA extension
(core/quantization.py:14-23 import fallback, :631-634 dispatch, :681-746
`_forward_pytorch`; the tensor metric backend morphology.py:826-873).  This
module is this package's own torch implementation of the same hook, used by
`core.py` whenever a tensor lives on the CPU.  It never touches the HIP
library and never imports `oracle/` (the oracle is test infrastructure).

Design (SURVEY.md Appendix A is the arithmetic contract):

* integer / binary work is restated in whatever form is cheapest, because it
  is exact in any order: Otsu histograms by one batched `bincount`, Canny
  non-maximum suppression by gathering the two neighbours of each direction
  sector, hysteresis and erosion as boolean 3x3 dilations, uniform-LBP labels
  through a 256-entry lookup of the 8-neighbour code, Euler quad patterns
  through a 16-entry lookup, box/area/perimeter counts as integer tile sums;
* floating-point stages whose CPU value depends on ATen's reduction order or
  on its vector/scalar loop split (channel mean: A.1; oneDNN convolutions:
  A.2; tile `avg_pool2d` sums: A.3; SLEEF transcendentals: A.6 - the scalar
  tail of a vectorised loop uses libm, so the result of `log`/`log2`/`atan2`
  can depend on the element's position in memory) are evaluated with the
  ATen op on a tensor of the same shape and memory layout the reference's
  run hands it, so the values agree bit for bit;
* the quantizer is one elementwise pass: per-(width, channel) scale and
  zero-point tables gathered per pixel, `y = ((clamp(rint(x/s + zp)) - zp)
  * s) * m` (SURVEY 8(a) "verified single-pass equivalence"), instead of one
  full-tensor pass per distinct bit width;
* the training (QAT) quantizer is a custom autograd function with the
  reference's straight-through gradients (quantization.py:69-118, 699-727).
"""
import math

import torch
import torch.nn.functional as F

# ---------------------------------------------------------------------------
# geometry and constant kernels
# ---------------------------------------------------------------------------


def tile_size(H, grid_size):
    """morphology.py:359-376: largest power of two <= max(4, H // grid)."""
    raw = max(4, H // grid_size)
    return 1 << (raw.bit_length() - 1)


def _gauss2d(k, denom):
    """Normalised separable Gaussian exp(-t^2 / denom) / sum, as an outer
    product (1, 1, k, k).  Built with the torch ops and shapes the reference
    uses for its constants (morphology.py:485-488, 566-570; quantization.py:
    204-209), so the fp32 taps are identical."""
    t = torch.arange(k, dtype=torch.float32) - k // 2
    g = torch.exp(-(t * t) / denom)
    g = g / g.sum()
    return (g.unsqueeze(0) * g.unsqueeze(1)).view(1, 1, k, k)


_K_CANNY = _gauss2d(5, 2.0)                                   # sigma 1
_SIG11 = 0.3 * ((11 - 1) * 0.5 - 1) + 0.8                     # cv2 default sigma for k = 11
_K_ADAPT = _gauss2d(11, 2 * _SIG11 ** 2)
_K_SOBEL_X = torch.tensor([[-1., 0., 1.], [-2., 0., 2.], [-1., 0., 1.]]).view(1, 1, 3, 3)
_K_SOBEL_Y = torch.tensor([[-1., -2., -1.], [0., 0., 0.], [1., 2., 1.]]).view(1, 1, 3, 3)


def _on(t, ref):
    return t if t.device == ref.device else t.to(ref.device)


def _lbp_label_table():
    """Uniform LBP (P=8, R=1) label for every 8-bit neighbour code: the number
    of set bits when the circular code has <= 2 transitions, else 9
    (morphology.py:624-652)."""
    lut = []
    for code in range(256):
        b = [(code >> i) & 1 for i in range(8)]
        trans = sum(b[i] != b[i - 1] for i in range(8))
        lut.append(sum(b) if trans <= 2 else 9)
    return torch.tensor(lut, dtype=torch.long)


_LBP_LUT = _lbp_label_table()
# neighbour order of the circular code (bit i), as (dy, dx)
_LBP_RING = ((-1, -1), (-1, 0), (-1, 1), (0, 1), (1, 1), (1, 0), (1, -1), (0, -1))


def _euler_quad_table():
    """4 x Euler contribution of a 2x2 window with pattern code
    tl + 2 tr + 4 bl + 8 br (Gray's quads, 8-connectivity): one set pixel +1,
    three set pixels -1, the two diagonal pairs -2 (morphology.py:673-707)."""
    lut = [0] * 16
    for c in (1, 2, 4, 8):
        lut[c] = 1
    for c in (7, 11, 13, 14):
        lut[c] = -1
    for c in (6, 9):
        lut[c] = -2
    return torch.tensor(lut, dtype=torch.int32)


_EULER_LUT = _euler_quad_table()

# ---------------------------------------------------------------------------
# per-pixel planes
# ---------------------------------------------------------------------------


def gray_plane(x, Hc, Wc):
    """Channel mean of the tile-aligned crop, (B, 1, Hc, Wc) (morphology.py:837;
    ATen's cascade sum order, SURVEY A.1, is only reproduced by ATen's mean)."""
    return x[:, :, :Hc, :Wc].mean(dim=1, keepdim=True).float()


def unit_range(g):
    """Per-image (g - min) / (max - min + 1e-8) (morphology.py:379-383)."""
    lo = g.amin(dim=(1, 2, 3), keepdim=True)
    hi = g.amax(dim=(1, 2, 3), keepdim=True)
    return (g - lo) / (hi - lo + 1e-8)


def sobel(g):
    """3x3 Sobel, zero padding (morphology.py:386-395; oneDNN / mm order A.2)."""
    return (F.conv2d(g, _on(_K_SOBEL_X, g), padding=1),
            F.conv2d(g, _on(_K_SOBEL_Y, g), padding=1))


def otsu_thresholds(v, bins=256):
    """Per-image Otsu threshold of v (B, 1, H, W) in [0, 1] -> (B, 1, 1, 1)
    (morphology.py:398-418), all images at once.

    histc: bin = int(v * 256), v == 1 -> last bin, values outside [0, 1] are
    ignored.  The cumulative sums are taken in float64 and rounded once per
    prefix: CPU `cumsum` accumulates fp32 in double (A.4) and every prefix of
    these fp32 terms is exact in double, so the order does not matter."""
    B = v.shape[0]
    flat = v.reshape(B, -1)
    inside = (flat >= 0) & (flat <= 1)
    idx = (flat * bins).long().clamp(max=bins - 1)
    idx = idx + bins * torch.arange(B, device=v.device).view(B, 1)
    idx = torch.where(inside, idx, torch.full_like(idx, B * bins))
    hist = torch.bincount(idx.reshape(-1), minlength=B * bins + 1)[:B * bins].view(B, bins).float()
    p = hist / hist.sum(dim=1, keepdim=True).clamp(min=1.0)
    centers = (torch.arange(bins, dtype=torch.float32, device=v.device) + 0.5) / bins
    omega = p.double().cumsum(dim=1).float()
    mu = (p * centers).double().cumsum(dim=1).float()
    mu_t = mu[:, -1:]
    between = (mu_t * omega - mu) ** 2 / (omega * (1.0 - omega) + 1e-12)
    return centers[between.argmax(dim=1)].view(B, 1, 1, 1)


def _dilate3(b):
    """3x3 binary dilation of a bool plane (B, 1, H, W), outside = False."""
    p = F.pad(b.to(torch.uint8), (1, 1, 1, 1))
    H, W = b.shape[-2:]
    rows = p[..., :, 0:W] | p[..., :, 1:W + 1] | p[..., :, 2:W + 2]
    return (rows[..., 0:H, :] | rows[..., 1:H + 1, :] | rows[..., 2:H + 2, :]).bool()


def _erode3(b):
    """3x3 binary erosion over the in-image neighbours (a -inf padded min)."""
    p = F.pad(b.to(torch.uint8), (1, 1, 1, 1), value=1)
    H, W = b.shape[-2:]
    rows = p[..., :, 0:W] & p[..., :, 1:W + 1] & p[..., :, 2:W + 2]
    return (rows[..., 0:H, :] & rows[..., 1:H + 1, :] & rows[..., 2:H + 2, :]).bool()


def _grow(strong, weak, iters):
    """Hysteresis: `iters` rounds of weak pixels joining an 8-neighbour edge."""
    edge = strong
    for _ in range(max(1, iters)):
        edge = edge | (weak & _dilate3(edge))
    return edge


# direction sector -> the two compared neighbours (dy, dx), replicate border
_NMS_PAIRS = (((0, 1), (0, -1)), ((-1, 1), (1, -1)), ((-1, 0), (1, 0)), ((-1, -1), (1, 1)))


def suppress_non_maxima(mag, gx, gy):
    """Canny NMS over 4 direction sectors of atan2(gy, gx) in degrees folded to
    [0, 180) (morphology.py:427-449).  atan2 runs on the (B, 1, H, W) planes
    the reference hands it (SLEEF vector body / libm tail, A.6)."""
    ang = torch.atan2(gy, gx) * (180.0 / math.pi)
    ang = torch.where(ang < 0, ang + 180.0, ang)
    sector = ((ang >= 22.5) & (ang < 67.5)).long() + 2 * ((ang >= 67.5) & (ang < 112.5)).long() + \
        3 * ((ang >= 112.5) & (ang < 157.5)).long()
    H, W = mag.shape[-2:]
    pad = F.pad(mag, (1, 1, 1, 1), mode="replicate")

    def nb(dy, dx):
        return pad[..., 1 + dy:1 + dy + H, 1 + dx:1 + dx + W]

    first = torch.stack([nb(*p[0]) for p in _NMS_PAIRS])
    second = torch.stack([nb(*p[1]) for p in _NMS_PAIRS])
    s = sector.unsqueeze(0)
    keep = (mag >= first.gather(0, s)[0]) & (mag >= second.gather(0, s)[0])
    return torch.where(keep, mag, torch.zeros_like(mag))


def canny_cv2compat(gray, hysteresis_iters=8):
    """morphology.py:458-509: 5x5 Gaussian blur, Otsu threshold t of the
    blurred intensity, Sobel of 255*blur, L1 magnitude, NMS, strong > t,
    weak > t/2, hysteresis.  -> bool (B, 1, H, W)."""
    blur = F.conv2d(gray, _on(_K_CANNY, gray), padding=2)
    t = otsu_thresholds(blur) * 255.0
    gx, gy = sobel(blur * 255.0)
    nms = suppress_non_maxima(gx.abs() + gy.abs(), gx, gy)
    return _grow(nms > t, nms > 0.5 * t, hysteresis_iters)


def canny_legacy(gray):
    """morphology.py:512-540 (canny_impl='legacy'): blur, Sobel, L2 magnitude,
    NMS, Otsu of the min-max normalised NMS map, 2 hysteresis rounds."""
    blur = F.conv2d(gray, _on(_K_CANNY, gray), padding=2)
    gx, gy = sobel(blur)
    mag = torch.sqrt(gx ** 2 + gy ** 2 + 1e-12)
    n = unit_range(suppress_non_maxima(mag, gx, gy))
    t = otsu_thresholds(n)
    return _grow(n > t, n > 0.5 * t, 2)


def adaptive_mask(gray, block=11, C=2.0):
    """cv2.adaptiveThreshold(GAUSSIAN_C, 11, 2) restated (morphology.py:551-573):
    g255 > G11(g255, replicate border) - C."""
    g255 = gray * 255.0
    p = block // 2
    local = F.conv2d(F.pad(g255, (p, p, p, p), mode="replicate"), _on(_K_ADAPT, gray))
    return g255 > local - C


def otsu_mask(gray):
    """binarize_impl='otsu' (morphology.py:420-424): gray > per-image Otsu."""
    return gray > otsu_thresholds(gray)


# ---------------------------------------------------------------------------
# tile descriptors phi1..phi5
# ---------------------------------------------------------------------------


def _tile_counts(b, tile):
    """Number of set pixels per tile of a bool/0-1 plane (B, 1, H, W) -> float
    (B, ht, wt); exact integers."""
    B, _, H, W = b.shape
    ht, wt = H // tile, W // tile
    v = b[:, 0, :ht * tile, :wt * tile].to(torch.int32)
    return v.reshape(B, ht, tile, wt, tile).sum(dim=(2, 4)).float()


def _weighted_slope(xs, ys, w):
    """Weighted least-squares slope of ys (S, ...) on xs (S, 1, 1, 1) with
    weights w (S, 1, 1, 1); the sums over S are ATen outer reductions of the
    (S, B*ht*wt) tensors (A.1), as in morphology.py:614-620."""
    w_sum = w.sum(dim=0)
    x_bar = (w * xs).sum(dim=0) / w_sum
    y_bar = (w * ys).sum(dim=0) / w_sum
    cov = (w * (xs - x_bar) * (ys - y_bar)).sum(dim=0)
    var = (w * (xs - x_bar) ** 2).sum(dim=0)
    return cov / (var + 1e-12)


def box_count_dimension(edge, tile):
    """phi1 before /2: box-counting fractal dimension per tile (Algorithm 2,
    morphology.py:576-621): occupied s-boxes for s = 2, 4, ..., tile, slope
    of log(n + 1) on log s with weights exp(-0.1 i), clamped to [1, 2]."""
    B, _, H, W = edge.shape
    ht, wt = H // tile, W // tile
    scales = [1 << k for k in range(1, tile.bit_length()) if (1 << k) <= tile]
    if len(scales) < 2:
        return torch.ones(B, ht, wt, device=edge.device)
    e = edge[:, 0, :ht * tile, :wt * tile]
    n = []
    for s in scales:
        occ = e.reshape(B, ht * tile // s, s, wt * tile // s, s).amax(dim=(2, 4))
        k = tile // s
        n.append(occ.reshape(B, ht, k, wt, k).to(torch.int32).sum(dim=(2, 4)).float())
    n = torch.stack(n, dim=0)                                   # (S, B, ht, wt)
    S = len(scales)
    xs = torch.log(torch.tensor(scales, dtype=torch.float32, device=edge.device)).view(S, 1, 1, 1)
    ys = torch.log(n + 1.0)
    w = torch.exp(-0.1 * torch.arange(S, dtype=torch.float32, device=edge.device)).view(S, 1, 1, 1)
    return (-_weighted_slope(xs, ys, w)).clamp(1.0, 2.0)


def lbp_entropy(gray, tile):
    """phi2: entropy of the 10-bin uniform-LBP histogram per tile / log2(10)
    (morphology.py:624-652).  Labels come from the code lookup; the
    probabilities k / tile^2 are laid out (B, ht, wt, 10) - the memory order
    of the reference's channels-last pooled one-hot - so log2 and the 10-bin
    sum see the same vector/scalar split and inner-sum order (A.6)."""
    B, _, H, W = gray.shape
    ht, wt = H // tile, W // tile
    pad = F.pad(gray, (1, 1, 1, 1), mode="replicate")
    code = torch.zeros(gray.shape, dtype=torch.long, device=gray.device)
    for i, (dy, dx) in enumerate(_LBP_RING):
        code |= (pad[..., 1 + dy:1 + dy + H, 1 + dx:1 + dx + W] >= gray).long() << i
    label = _on(_LBP_LUT, gray)[code][:, 0, :ht * tile, :wt * tile]
    tid = (torch.arange(B, device=gray.device).view(B, 1, 1) * ht +
           (torch.arange(ht * tile, device=gray.device) // tile).view(1, -1, 1)) * wt + \
        (torch.arange(wt * tile, device=gray.device) // tile).view(1, 1, -1)
    cnt = torch.bincount((tid * 10 + label).reshape(-1), minlength=B * ht * wt * 10)
    p = cnt.view(B, ht, wt, 10).float() / float(tile * tile)
    ent = -(p * torch.log2(p + 1e-10)).sum(dim=-1)
    return ent / math.log2(10.0)


def gradient_variance(gx, gy, tile):
    """phi3 = v / (v + 1), v = Var(gx) + Var(gy) per tile (morphology.py:
    655-670); E[t], E[t^2] are avg_pool2d window sums (A.3)."""
    def var(t):
        m1 = F.avg_pool2d(t, kernel_size=tile, stride=tile)
        m2 = F.avg_pool2d(t * t, kernel_size=tile, stride=tile)
        return (m2 - m1 * m1).clamp(min=0.0)
    v = (var(gx) + var(gy))[:, 0]
    return v / (v + 1.0)


def euler_components(mask, tile):
    """K >= 1 per tile: round-half-even of the summed Euler quad contributions
    of the zero-padded mask, each 2x2 window attributed to the tile of its
    top-left pixel (morphology.py:673-707)."""
    B, _, H, W = mask.shape
    ht, wt = H // tile, W // tile
    m = F.pad(mask[:, 0].to(torch.int32), (1, 1, 1, 1))
    code = m[:, :-1, :-1] + 2 * m[:, :-1, 1:] + 4 * m[:, 1:, :-1] + 8 * m[:, 1:, 1:]
    e4 = _on(_EULER_LUT, mask)[code.long()][:, :ht * tile, :wt * tile]
    s = e4.reshape(B, ht, tile, wt, tile).sum(dim=(2, 4)).float()
    return torch.round(s / 4.0).clamp(min=1.0)


def contour_complexity(mask, tile, components=True):
    """phi5 (morphology.py:709-739): inverse circularity perim^2 / (4 pi area)
    of the foreground per tile (divided by the Euler component count K),
    mapped to 1 - 1/max(ic, 1); 0 for tiles without foreground."""
    boundary = mask & ~_erode3(mask)
    area = _tile_counts(mask, tile)
    perim = _tile_counts(boundary, tile)
    ic = (perim * perim) / (4.0 * math.pi * area + 1e-6)
    if components:
        ic = ic / euler_components(mask, tile)
    phi5 = 1.0 - 1.0 / ic.clamp(min=1.0)
    return torch.where(area > 0, phi5, torch.zeros_like(phi5))


def phi_tiles(features, grid_size, canny_impl="cv2compat", binarize_impl="adaptive",
              contour_components=True, internals=False):
    """_phi_tiles_gpu (morphology.py:826-873) on the CPU: (B, ht, wt, 8)
    [phi1..phi5, phi1 phi2, phi3^2, sqrt(phi4 phi5 + 1e-12)]."""
    x = features.detach().float()
    B, C, H, W = x.shape
    tile = tile_size(H, grid_size)
    ht, wt = H // tile, W // tile
    if ht < 1 or wt < 1:
        raise ValueError("feature map %dx%d smaller than one %d-pixel tile" % (H, W, tile))
    with torch.no_grad():
        gray = unit_range(gray_plane(x, ht * tile, wt * tile))
        gx, gy = sobel(gray)
        edge = canny_legacy(gray) if canny_impl == "legacy" else canny_cv2compat(gray)
        mask = otsu_mask(gray) if binarize_impl == "otsu" else adaptive_mask(gray)
        p1 = box_count_dimension(edge.float(), tile) / 2.0
        p2 = lbp_entropy(gray, tile)
        p3 = gradient_variance(gx, gy, tile)
        p4 = _tile_counts(edge, tile) / float(tile * tile)
        p5 = contour_complexity(mask, tile, contour_components)
        phi = torch.stack([p1, p2, p3, p4, p5, p1 * p2, p3 * p3, torch.sqrt(p4 * p5 + 1e-12)], dim=-1)
    if internals:
        return phi, {"gray": gray, "gx": gx, "gy": gy, "edge": edge, "binmask": mask, "tile": tile}
    return phi


# ---------------------------------------------------------------------------
# quantizer (inference): one pass
# ---------------------------------------------------------------------------


def width_tables(xmin, xmax, lo=2, hi=8):
    """QuantizationParameters (quantization.py:26-66) for every width lo..hi at
    once: scale (nb, C), zero point (nb, C), qmin / qmax (nb, 1).  fp32 ops in
    the reference's order: scale = max(range, 1e-8) / (qmax - qmin),
    zp = clamp(qmin - min / scale, qmin, qmax)."""
    widths = torch.arange(lo, hi + 1, dtype=torch.float64, device=xmin.device)
    qmin = (-(2.0 ** (widths - 1))).float().view(-1, 1)
    qmax = (2.0 ** (widths - 1) - 1).float().view(-1, 1)
    xmin = xmin.reshape(1, -1).float()
    xmax = xmax.reshape(1, -1).float()
    scale = (xmax - xmin).clamp(min=1e-8) / (qmax - qmin)
    zp = torch.maximum(torch.minimum(qmin - xmin / scale, qmax), qmin)
    return scale, zp, qmin, qmax


def pixel_bits(bits, H, W):
    """Nearest upsampling of the tile bit map (B, Ht, Wt) -> (B, 1, H, W)
    (the reference's F.interpolate(..., mode='nearest') tile masks)."""
    return F.interpolate(bits.unsqueeze(1).float(), size=(H, W), mode="nearest")


def quantize(x, bits, xmin, xmax, m=None, lo=2, hi=8):
    """Inference quantizer (quantization.py:729-746) as the single pass
    y = ((clamp(rint(x / s_b + zp_b), qmin_b, qmax_b) - zp_b) * s_b) * m."""
    B, C, H, W = x.shape
    scale, zp, qmin, qmax = width_tables(xmin.expand(C) if xmin.numel() == 1 else xmin,
                                         xmax.expand(C) if xmax.numel() == 1 else xmax, lo, hi)
    w = (torch.round(pixel_bits(bits, H, W)).long() - lo).clamp(0, hi - lo)[:, 0]     # (B, H, W)
    s = scale.t()[:, w].transpose(0, 1)                  # (B, C, H, W) views of the gathered tables
    z = zp.t()[:, w].transpose(0, 1)
    qlo = qmin[w].view(B, 1, H, W)
    qhi = qmax[w].view(B, 1, H, W)
    q = torch.round(x / s + z)
    y = (torch.maximum(torch.minimum(q, qhi), qlo) - z) * s
    return y if m is None else y * m


def spatial_quantize(x, bit_map, min_vals, max_vals, tile_h, tile_w, mask=None):
    """mcaq_cuda_ops.spatial_quantize semantics on CPU tensors: bits
    clamp(rint(b), 2, 8) of tile min(h // tile_h, Ht - 1) (mcaq_kernel.cu:
    36-60, with round-half-even as the PyTorch path)."""
    B, C, H, W = x.shape
    Ht, Wt = bit_map.shape[-2:]
    th = torch.clamp(torch.arange(H) // tile_h, max=Ht - 1)
    tw = torch.clamp(torch.arange(W) // tile_w, max=Wt - 1)
    b = torch.round(bit_map.float()).clamp(2, 8)[:, th][:, :, tw]          # (B, H, W)
    scale, zp, qmin, qmax = width_tables(min_vals.reshape(-1), max_vals.reshape(-1))
    w = b.long() - 2
    s = scale.t()[:, w].transpose(0, 1)
    z = zp.t()[:, w].transpose(0, 1)
    q = torch.round(x / s + z)
    y = (torch.maximum(torch.minimum(q, qmax[w].view(B, 1, H, W)), qmin[w].view(B, 1, H, W)) - z) * s
    return y if mask is None else y * mask.reshape(B, 1, H, W)


# ---------------------------------------------------------------------------
# quantizer (training): fractional bits + straight-through estimator
# ---------------------------------------------------------------------------


class FractionalQuant(torch.autograd.Function):
    """x_q = (1 - f) Q_floor(b)(x) + f Q_floor(b)+1(x), f = b - floor(b), per
    pixel from the nearest-upsampled continuous tile bits (quantization.py:
    699-727; Q_floor(b)+1 := Q_floor(b) past max_bits).  Straight-through
    backward (quantization.py:94-118): dQ/dx = 1, so
        grad_x    = g (1 - f) + g f
        grad_bits = tile sums of  sum_c g (Q_hi - Q_lo)
    xmin / xmax carry no gradient (EMA buffers)."""

    @staticmethod
    def _parts(x, bits, xmin, xmax, hi_bits):
        B, C, H, W = x.shape
        bfl = torch.floor(bits)
        f = pixel_bits(bits - bfl, H, W)                              # (B, 1, H, W)
        lo_w = pixel_bits(bfl, H, W).long()
        lo_b = int(lo_w.min()) if lo_w.numel() else 2
        scale, zp, qmin, qmax = width_tables(xmin, xmax, min(lo_b, hi_bits), hi_bits)
        base = min(lo_b, hi_bits)

        def q(width):
            wi = (width - base).clamp(0, hi_bits - base)[:, 0]
            s = scale.t()[:, wi].transpose(0, 1)
            z = zp.t()[:, wi].transpose(0, 1)
            r = torch.round(x / s + z)
            r = torch.maximum(torch.minimum(r, qmax[wi].view(B, 1, H, W)), qmin[wi].view(B, 1, H, W))
            return (r - z) * s

        q_lo = q(lo_w)
        q_hi = torch.where(lo_w + 1 <= hi_bits, q(torch.clamp(lo_w + 1, max=hi_bits)), q_lo)
        return f, q_lo, q_hi

    @staticmethod
    def forward(ctx, x, bits, xmin, xmax, hi_bits=8):
        xd = x.detach().float()
        f, q_lo, q_hi = FractionalQuant._parts(xd, bits.detach().float(), xmin, xmax, hi_bits)
        ctx.save_for_backward(xd, bits.detach().float(), xmin, xmax)
        ctx.hi_bits = hi_bits
        return (1.0 - f) * q_lo + f * q_hi

    @staticmethod
    def backward(ctx, g):
        xd, bits, xmin, xmax = ctx.saved_tensors
        f, q_lo, q_hi = FractionalQuant._parts(xd, bits, xmin, xmax, ctx.hi_bits)
        gx = g * (1.0 - f) + g * f if ctx.needs_input_grad[0] else None
        gb = None
        if ctx.needs_input_grad[1]:
            B, C, H, W = xd.shape
            Ht, Wt = bits.shape[-2:]
            per_pix = (g * (q_hi - q_lo)).sum(dim=1)                  # (B, H, W)
            rows = F.interpolate(torch.arange(Ht, dtype=torch.float32).view(1, 1, Ht, 1), size=(H, 1),
                                 mode="nearest").long().view(H)
            cols = F.interpolate(torch.arange(Wt, dtype=torch.float32).view(1, 1, 1, Wt), size=(1, W),
                                 mode="nearest").long().view(W)
            tid = (rows.view(H, 1) * Wt + cols.view(1, W)).to(xd.device)
            gb = torch.zeros(B, Ht * Wt, dtype=torch.float64, device=xd.device)
            gb.index_add_(1, tid.reshape(-1), per_pix.reshape(B, -1).double())
            gb = gb.view(B, Ht, Wt).to(g.dtype)
        return gx, gb, None, None, None


def ema_update(running_min, running_max, xmin, xmax, momentum):
    """update_running_stats (quantization.py:340-347): first batch takes the
    batch statistics, later ones r <- momentum r + (1 - momentum) new."""
    if running_min is None:
        return xmin.clone(), xmax.clone()
    return (momentum * running_min + (1 - momentum) * xmin,
            momentum * running_max + (1 - momentum) * xmax)
