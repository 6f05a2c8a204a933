"""Drop-in mirror of the reference's hot-path modules, running on the gfx950 kernels.

Same class names, constructor arguments, forward signatures, parameter /
buffer names (state_dict keys) and error behaviour as the reference:

    MorphologicalComplexityAnalyzer   mcaq_yolo/core/morphology.py:17-973
    ComplexityToBitMappingNetwork     mcaq_yolo/core/bit_allocation.py:83-303
    LinearBitMapper                   mcaq_yolo/core/bit_allocation.py:12-80
    LearnedSoftMask                   mcaq_yolo/core/quantization.py:168-239
    SpatialAdaptiveQuantization       mcaq_yolo/core/quantization.py:242-754

so a reference checkpoint loads unchanged (`load_state_dict`).

Dispatch (the reference's quantization.py:14-23, 631-634): CUDA (HIP) tensors
run through libmcaq_hip.so (include/mcaq_hip.h) - a missing library raises,
there is no silent torch fallback on the GPU; CPU tensors run this package's
own pure-PyTorch path (`fallback.py`, BASELINE config 1).  The numeric
contract is the reference's pure-PyTorch path (bit-exact decisions,
tests/test_core_gpu.py, tests/test_fallback_cpu.py).  When autograd needs a
gradient of a kernel-computed value (eval mode with grad enabled), the value
comes from the kernel and the backward recomputes the tile-sized torch graph
(`_kernel_value`), so gradients reach the reference's parameters.

Training (QAT, BASELINE config 5): the quantizer's per-element work - EMA
running statistics, the fractional-bit forward and the straight-through
backward - runs in the HIP kernels (mcaq_qat_forward / mcaq_qat_backward,
mcaq_ema_stats) behind a torch.autograd.Function; the soft mask's forward is
the HIP kernel and its (tile-sized) backward is recomputed with torch ops.
The complexity MLP + bilateral and the bit mapper in train mode are tile-level
(N_tiles x <=64) networks with batch-statistics BatchNorm: they run as torch
autograd ops on the GPU, restating morphology.py:309-354, 939-973 and
bit_allocation.py:199-280 (phi itself is no-grad side information computed by
the morph kernel, as in the reference).
"""
import ctypes
import functools
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import abi, fallback
from . import engine as _engine
from .engine import tile_size

_CM_SIZE, _MM_SIZE, _SM_SIZE = 2881, 4865, 170


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _need_cuda(t, what):
    if not torch.is_tensor(t):
        raise TypeError("%s must be a torch.Tensor, got %s" % (what, type(t)))
    if not t.is_cuda:
        raise RuntimeError("mcaq_yolo_amd runs on MI355X (HIP) only: %s is on %s" % (what, t.device))


def _f32c(t):
    return t.detach().float().contiguous()


def _wants_grad(inputs, params=()):
    return torch.is_grad_enabled() and (any(t.requires_grad for t in inputs) or
                                        any(p.requires_grad for p in params))


class _KernelValue(torch.autograd.Function):
    """Value from a HIP kernel, gradient from the torch restatement of the same
    tile-sized function (recomputed in backward).  args = n_in inputs followed
    by the module parameters torch_fn reads."""

    @staticmethod
    def forward(ctx, kernel_fn, torch_fn, n_in, *args):
        ctx.torch_fn, ctx.n_in = torch_fn, n_in
        ctx.save_for_backward(*args)
        with torch.no_grad():
            return kernel_fn(*[a.detach() for a in args[:n_in]])

    @staticmethod
    def backward(ctx, g):
        args = ctx.saved_tensors
        n_in = ctx.n_in
        need = ctx.needs_input_grad[3:]
        with torch.enable_grad():
            ins = [a.detach().requires_grad_(bool(r)) for a, r in zip(args[:n_in], need[:n_in])]
            out = ctx.torch_fn(*ins)
            targets = [t for t, r in zip(ins, need[:n_in]) if r] + [p for p, r in zip(args[n_in:], need[n_in:]) if r]
            grads = iter(torch.autograd.grad(out, targets, g, allow_unused=True) if targets else [])
        return (None, None, None) + tuple(next(grads) if r else None for r in need)


def _kernel_value(kernel_fn, torch_fn, inputs, params):
    params = [p for p in params if p.requires_grad]
    return _KernelValue.apply(kernel_fn, torch_fn, len(inputs), *inputs, *params)


_MFMA_IDX = {}


def _mfma_a_operands(w):
    """Device version of params.mfma_a_operands: (N_out, K) weight -> A operands
    of v_mfma_f32_16x16x4_f32 ([block][step][lane], lane l holds
    W[16*block + (l & 15)][4*step + (l >> 4)], K zero-padded to a multiple of 4)."""
    n, k = w.shape
    kp = (k + 3) // 4 * 4
    nb = (n + 15) // 16
    key = (n, k, w.device)
    idx = _MFMA_IDX.get(key)
    if idx is None:
        b = torch.arange(nb).view(nb, 1, 1)
        s = torch.arange(kp // 4).view(1, kp // 4, 1)
        lane = torch.arange(64).view(1, 1, 64)
        idx = ((16 * b + (lane & 15)) * kp + 4 * s + (lane >> 4)).reshape(-1).to(w.device)
        _MFMA_IDX[key] = idx
    wp = torch.zeros(nb * 16, kp, device=w.device, dtype=torch.float32)
    wp[:n, :k] = w
    return wp.reshape(-1)[idx]


class _BlobCache:
    """Packs module parameters into the flat blob a kernel reads, on the device,
    and re-packs only when a parameter changed (tensor version counters)."""

    def __init__(self):
        self.key = None
        self.blob = None
        self.pinned = None
        self.primed = False

    def prime(self, blob, key):
        """A blob packed by someone else's launch (train_step._prepack) for
        the next get(): taken as is, also under capture."""
        self.blob, self.key, self.primed = blob, key, True

    def get(self, tensors, pack):
        if self.pinned is not None:
            return self.pinned
        key = tuple((t.data_ptr(), t._version, t.device) for t in tensors)
        if self.primed:
            self.primed = False
            if self.key is None or self.key == key:     # packed under capture, or from these values
                return self.blob
        # under HIP-graph capture the pack is always recorded, so every replay
        # rebuilds the blob from the live parameters (an optimizer step inside
        # the captured step changes them in place); the captured blob holds
        # data only after a replay, so the next eager call packs afresh
        capturing = any(t.is_cuda for t in tensors) and torch.cuda.is_current_stream_capturing()
        if capturing or key != self.key:
            with torch.no_grad():
                self.blob = pack().contiguous()
            self.key = None if capturing else key
        return self.blob


def _pad4(t):
    """Blobs are read as 16-byte vectors: pad to a multiple of 4 floats."""
    n = (-t.numel()) % 4
    return torch.cat([t, t.new_zeros(n)]) if n else t


def _pack_segs(parts, mfma, base=0):
    """mcaq_pack segments (src, n, k, mode, dst) of one blob at `base`:
    `parts` copied back to back, then the MFMA A operands of the `mfma`
    weights; and the end offset."""
    segs, o = [], base
    for t in parts:
        segs.append((t.detach(), t.numel(), 1, 0, o))
        o += t.numel()
    for w in mfma:
        n, k = w.shape
        segs.append((w.detach(), n, k, 1, o))
        o += (n + 15) // 16 * ((k + 3) // 4) * 64
    return segs, o


def _pack_array(segs):
    arr = (abi.PackSeg * len(segs))()
    for a, (t, n, k, mode, dst) in zip(arr, segs):
        a.src, a.n, a.k, a.mode, a.dst = _p(t), n, k, mode, dst
    return arr


def _launch_pack(segs, out):
    abi.check(abi.lib().mcaq_pack(_pack_array(segs), len(segs), _p(out), out.numel(), _stream()), "mcaq_pack")


def _device_pack(parts, mfma, total):
    """The blob layout of _pack_* built by ONE kernel (mcaq_pack) from the live
    parameter tensors: `parts` copied back to back, then the MFMA A operands
    of the `mfma` weights, zero padded to `total` floats.  None when a tensor
    is not a contiguous fp32 CUDA tensor (the torch packing then runs)."""
    ts = list(parts) + list(mfma)
    if not all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in ts) or \
            len(ts) > abi.MCAQ_PACK_MAXSEG:
        return None
    segs, o = _pack_segs(parts, mfma)
    if o > total:
        raise ValueError("blob overflow")
    out = torch.empty(total, device=ts[0].device)
    _launch_pack(segs, out)
    return out


_CM_BLOB = (_CM_SIZE + 512 + 2048 + 3) // 4 * 4   # floats of the complexity-MLP blob


def _cmlp_pack_parts(seq):
    """(copied parts, MFMA weights) of the complexity-MLP blob."""
    l0, ln1, l3, ln4, l6 = seq[0], seq[1], seq[3], seq[4], seq[6]
    return [l0.weight, l0.bias, ln1.weight, ln1.bias, l3.weight, l3.bias, ln4.weight, ln4.bias, l6.weight,
            l6.bias], [l0.weight, l3.weight]


def _pack_cmlp(seq):
    l0, ln1, l3, ln4, l6 = seq[0], seq[1], seq[3], seq[4], seq[6]
    parts = [l0.weight, l0.bias, ln1.weight, ln1.bias, l3.weight, l3.bias, ln4.weight, ln4.bias,
             l6.weight, l6.bias]
    if sum(t.numel() for t in parts) == _CM_SIZE:
        blob = _device_pack(parts, [l0.weight, l3.weight], _CM_BLOB)
        if blob is not None:
            return blob
    flat = torch.cat([p.detach().float().reshape(-1) for p in parts])
    if flat.numel() != _CM_SIZE:
        raise ValueError("complexity MLP must be the reference Linear(8,64)-LN-ReLU-Linear(64,32)-LN-ReLU-"
                         "Linear(32,1) stack")
    return _pad4(torch.cat([flat, _mfma_a_operands(l0.weight.detach().float()),
                            _mfma_a_operands(l3.weight.detach().float())]))


def _pack_mapper(seq):
    parts = []
    for li, bi in ((0, 1), (3, 4), (6, 7)):
        lin, bn = seq[li], seq[bi]
        parts += [lin.weight, lin.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var]
    parts += [seq[9].weight, seq[9].bias]
    if sum(t.numel() for t in parts) == _MM_SIZE and len(parts) + 3 <= abi.MCAQ_PACK_MAXSEG:
        total = _MM_SIZE + sum((w.shape[0] + 15) // 16 * ((w.shape[1] + 3) // 4) * 64
                               for w in (seq[0].weight, seq[3].weight, seq[6].weight))
        blob = _device_pack(parts, [seq[i].weight for i in (0, 3, 6)], (total + 3) // 4 * 4)
        if blob is not None:
            return blob
    flat = torch.cat([p.detach().float().reshape(-1) for p in parts])
    if flat.numel() != _MM_SIZE:
        raise ValueError("bit mapper must use hidden_dims [32, 64, 32]")
    return _pad4(torch.cat([flat] + [_mfma_a_operands(seq[i].weight.detach().float()) for i in (0, 3, 6)]))


def _pack_softmask(seq):
    parts = [seq[0].weight, seq[0].bias, seq[2].weight, seq[2].bias]
    if sum(t.numel() for t in parts) == _SM_SIZE:
        blob = _device_pack(parts, [], (_SM_SIZE + 3) // 4 * 4)
        if blob is not None:
            return blob
    flat = torch.cat([p.detach().float().reshape(-1) for p in parts])
    if flat.numel() != _SM_SIZE:
        raise ValueError("soft mask must be the reference Conv2d(2,8,3)/Conv2d(8,2,1) net")
    return _pad4(flat)


def _morph_struct(B, H, W, tile, ht, wt, flags, **ptrs):
    s = abi.MorphScale()
    for k, v in ptrs.items():
        setattr(s, k, _p(v))
    s.B, s.H, s.W = B, H, W
    s.Hc, s.Wc, s.tile, s.ht, s.wt = ht * tile, wt * tile, tile, ht, wt
    s.batch_offset, s.batch_total = 0, B
    s.flags = flags
    s.hyst_iters = 8
    s.temperature, s.min_bits, s.max_bits = 1.0, 2.0, 8.0
    s.softmax_threads = torch.get_num_threads()   # the CPU reference's softmax partition
    return s


def _run_stats(x, gray=None, absmean=None, pmin=None, pmax=None, Hc=None, Wc=None):
    B, C, H, W = x.shape
    s = abi.StatsScale()
    s.x, s.gray, s.absmean, s.pmin, s.pmax = _p(x), _p(gray), _p(absmean), _p(pmin), _p(pmax)
    s.B, s.C, s.H, s.W = B, C, H, W
    s.Hc, s.Wc = (H if Hc is None else Hc), (W if Wc is None else Wc)
    abi.check(abi.lib().mcaq_stats(ctypes.byref(s), 1, _stream()), "mcaq_stats")


# Pass-1 sharing inside one hook call (train mode): the analyzer's pass 1
# (gray) also writes |x| channel means and the channel min/max partials of the
# same read, and the quantizer that follows on the same feature tensor
# (unchanged: data pointer, version, shape) takes them instead of reading x
# again.  One slot; False: every module runs its own pass 1.
PASS1_SHARE = True
_PASS1 = {"armed": False, "slot": None}


class pass1_sharing:
    """Scope of one hook call (MCAQHooks._run_scale_modules): inside it the
    analyzer leaves its pass-1 by-products for the quantizer; outside it
    nothing is cached (a recycled tensor address can never hit)."""

    def __enter__(self):
        _PASS1["armed"], _PASS1["slot"] = PASS1_SHARE, None
        return self

    def __exit__(self, *exc):
        _PASS1["armed"], _PASS1["slot"] = False, None
        return False


def _pass1_key(x):
    return (x.data_ptr(), x._version, tuple(x.shape), x.device, torch.cuda.current_stream(x.device).cuda_stream)


def _pass1_lookup(x):
    e = _PASS1["slot"]
    return e if (_PASS1["armed"] and e is not None and e["key"] == _pass1_key(x)) else None


def _channel_minmax(x, absmean=None, partials=None):
    """Per-channel min/max over (batch, H, W) (quantization.py:650-654) by pass 1
    + the finalize reduction; optionally the |x| channel mean in the same read
    (or both from the analyzer's pass 1 over the same tensor, _pass1_lookup,
    or `partials` = that pass's (pmin, pmax))."""
    B, C, H, W = x.shape
    L = abi.lib()
    units = L.mcaq_stats_units(B, C, H, W)
    hit = _pass1_lookup(x) if partials is None else {"pmin": partials[0], "pmax": partials[1], "absmean": absmean}
    if hit is not None and (absmean is None or absmean is hit["absmean"]):
        pmin, pmax = hit["pmin"], hit["pmax"]
    else:
        pmin = torch.empty(units, C, device=x.device)
        pmax = torch.empty(units, C, device=x.device)
        _run_stats(x, absmean=absmean, pmin=pmin, pmax=pmax)
    xmin = torch.empty(C, device=x.device)
    xmax = torch.empty(C, device=x.device)
    f = abi.FinalizeScale()
    f.pmin, f.pmax, f.min_out, f.max_out = _p(pmin), _p(pmax), _p(xmin), _p(xmax)
    f.C, f.nunits, f.min_stride = C, units, 1
    abi.check(L.mcaq_finalize(ctypes.byref(f), 1, _stream()), "mcaq_finalize")
    return xmin, xmax


# ---------------------------------------------------------------------------
# morphology.py
# ---------------------------------------------------------------------------
class MorphologicalComplexityAnalyzer(nn.Module):
    """morphology.py:17-973, tensor ("gpu") metric backend.

    forward(features) -> complexity map (B, ht, wt) in [0, 1]:
    channel mean -> phi1..phi5 per tile -> complexity MLP -> bilateral -> clamp
    (morphology.py:939-973), computed by mcaq_stats + mcaq_morph."""

    def __init__(self, grid_size: int = 8, device: str = "cuda", metric_backend: str = "gpu",
                 canny_impl: str = "cv2compat", binarize_impl: str = "adaptive",
                 contour_components: bool = True):
        super().__init__()
        if metric_backend != "gpu":
            raise NotImplementedError("metric_backend=%r: only the tensor ('gpu') backend is on the MI355X path "
                                      "(the cv2 backend is offline CPU scoring, out of scope)" % metric_backend)
        # as the reference: 'legacy' / 'otsu' select the legacy variants, any
        # other value the cv2-compatible defaults (morphology.py:451-455, 542-548)
        self.grid_size = grid_size
        self.device = device
        self.metric_backend = metric_backend
        self.canny_impl = canny_impl
        self.binarize_impl = binarize_impl
        self.contour_components = contour_components
        self.complexity_mlp = nn.Sequential(
            nn.Linear(8, 64), nn.LayerNorm(64), nn.ReLU(inplace=True),
            nn.Linear(64, 32), nn.LayerNorm(32), nn.ReLU(inplace=True),
            nn.Linear(32, 1), nn.Sigmoid(),
        )
        nn.init.xavier_uniform_(self.complexity_mlp[-2].weight, gain=3.0)
        nn.init.zeros_(self.complexity_mlp[-2].bias)
        self.register_buffer("feature_weights", torch.ones(5) / 5)
        self._blob = _BlobCache()
        self._gsink = _GradSink()
        if str(device).startswith("cuda") and torch.cuda.is_available():
            self.to(device)

    def _tile_size(self, H: int) -> int:
        """morphology.py:359-376: largest power of two <= max(4, H // grid_size)."""
        return tile_size(H, self.grid_size)

    def _flags(self):
        f = 0
        if self.binarize_impl == "otsu":
            f |= abi.F_BIN_OTSU
        if not self.contour_components:
            f |= abi.F_NO_EULER
        if self.canny_impl == "legacy":
            f |= abi.F_CANNY_LEGACY
        return f

    def cmlp_blob(self):
        ps = [p for p in self.complexity_mlp.parameters()]
        return self._blob.get(ps, lambda: _pack_cmlp(self.complexity_mlp))

    def _run(self, features, want_c, want_craw=False, image_batch=False):
        _need_cuda(features, "features")
        if features.dim() != 4:
            raise ValueError("features must be (B, C, H, W)")
        x = features.float().contiguous()
        B, C, H, W = x.shape
        T = tile_size(H, self.grid_size)
        ht, wt = H // T, W // T
        if ht < 1 or wt < 1 or T > 128:
            raise ValueError("feature map %dx%d: tile %d unsupported" % (H, W, T))
        dev = x.device
        gray = torch.empty(B, ht * T, wt * T, device=dev)
        if _PASS1["armed"] and self.training:
            # the quantizer of this hook reads the same x next: |x| means and
            # min/max partials in the same pass (_pass1_lookup)
            units = abi.lib().mcaq_stats_units(B, C, H, W)
            e = {"key": _pass1_key(x), "absmean": torch.empty(B, H, W, device=dev),
                 "pmin": torch.empty(units, C, device=dev), "pmax": torch.empty(units, C, device=dev)}
            _run_stats(x, gray=gray, absmean=e["absmean"], pmin=e["pmin"], pmax=e["pmax"], Hc=ht * T, Wc=wt * T)
            _PASS1["slot"] = e
        else:
            _run_stats(x, gray=gray, Hc=ht * T, Wc=wt * T)
        phi = torch.empty(B, ht, wt, 8, device=dev)
        flags = abi.F_PHI | self._flags() | (abi.F_IMAGE_BATCH if image_batch else 0)
        ptrs = dict(gray=gray, phi_out=phi, tile_tmp=torch.empty(B, ht * wt, 32, device=dev))
        L = abi.lib()
        if want_c:
            flags |= abi.F_CMLP
            ptrs["cmlp"] = self.cmlp_blob()
            ptrs["c_out"] = torch.empty(B, ht, wt, device=dev)
            if want_craw:
                ptrs["cmlp_out"] = torch.empty(B, ht, wt, device=dev)
        scratch = L.mcaq_morph_scratch_bytes(B, ht * T, wt * T, ht, wt)
        if scratch:
            ptrs["gscratch"] = torch.empty(scratch, device=dev, dtype=torch.uint8)
        wb = L.mcaq_morph_work_bytes(B, ht * T, wt * T, T) if _engine.BAND_PASS else 0
        if wb:
            ptrs["pwork"] = torch.empty(wb // 4, device=dev)   # pass A as band + edge workgroups
        s = _morph_struct(B, H, W, T, ht, wt, flags, **ptrs)
        abi.check(L.mcaq_morph(ctypes.byref(s), 1, _stream()), "mcaq_morph")
        if want_craw:
            return phi, ptrs.get("c_out"), ptrs.get("cmlp_out")
        return phi, ptrs.get("c_out")

    @staticmethod
    def _detailed(phi):
        return {"fractal": phi[..., 0], "texture": phi[..., 1], "gradient": phi[..., 2],
                "edge": phi[..., 3], "contour": phi[..., 4]}

    def compute_phi_tiles(self, features: torch.Tensor, image_batch: bool = False):
        """morphology.py:798-824: (phi (B,ht,wt,8), detailed dict of phi1..phi5).
        image_batch=True: every image as the reference's batch-1 call would
        see it (a few ATen reductions follow the tile's position in the whole
        batch) - one launch for the batch on the GPU."""
        if not features.is_cuda:
            if image_batch and features.shape[0] > 1:
                phi = torch.cat([fallback.phi_tiles(features[i:i + 1], self.grid_size, self.canny_impl,
                                                    self.binarize_impl, self.contour_components)
                                 for i in range(features.shape[0])])
            else:
                phi = fallback.phi_tiles(features, self.grid_size, self.canny_impl, self.binarize_impl,
                                         self.contour_components)
        else:
            phi, _ = self._run(features, want_c=False, image_batch=image_batch)
        return phi, self._detailed(phi)

    def score_image(self, features: torch.Tensor, image_batch: bool = False) -> torch.Tensor:
        """morphology.py:923-937: per-image Eq.(8) score for curriculum sorting,
        mean over tiles of sum_i alpha_i * phi_i (alpha = |feature_weights|
        normalised to sum 1), clamped to [0, 1].  phi comes from the morph
        kernel; the 5-term dot product is a (B, ht, wt) device reduction.
        image_batch: score every image as its own batch-1 call
        (compute_phi_tiles)."""
        phi, _ = self.compute_phi_tiles(features, image_batch=image_batch)
        with torch.no_grad():
            alpha = self.feature_weights.detach().abs().to(phi.device)
            alpha = alpha / alpha.sum().clamp(min=1e-8)
            c = (phi[..., :5] * alpha.view(1, 1, 1, 5)).sum(dim=-1)
            return c.mean(dim=(1, 2)).clamp(0.0, 1.0)

    def fit_feature_weights(self, batches, max_batches: int = 64):
        """morphology.py:876-921: NNLS fit of alpha so Eq.(8) tracks the trained
        complexity MLP (pre-bilateral), projected onto the simplex.  Offline
        curriculum utility: phi and the MLP target are computed on the GPU, the
        5-unknown NNLS solve runs on the host (scipy), as in the reference."""
        import numpy as np
        from scipy.optimize import nnls
        Ps, Cs = [], []
        dev = next(self.complexity_mlp.parameters()).device
        for i, x in enumerate(batches):
            if isinstance(x, dict):
                x = x.get("img")
            x = x.float()
            if x.dim() == 3:
                x = x.unsqueeze(0)
            if x.max() > 1.5:
                x = x / 255.0
            x = x.to(dev)
            phi, _ = self.compute_phi_tiles(x)
            with torch.no_grad():
                c = self.complexity_mlp(phi.reshape(-1, 8))
            Ps.append(phi[..., :5].reshape(-1, 5).cpu())
            Cs.append(c.reshape(-1, 1).cpu())
            if i + 1 >= max_batches:
                break
        P = torch.cat(Ps).double().numpy()
        C = torch.cat(Cs).double().numpy().ravel()
        alpha, _ = nnls(P, C)
        s = float(alpha.sum())
        alpha = alpha / s if s > 1e-12 else np.ones(5) / 5.0
        self.feature_weights.copy_(torch.as_tensor(alpha, dtype=self.feature_weights.dtype,
                                                   device=self.feature_weights.device))
        return alpha

    @staticmethod
    def bilateral_filter(complexity_map, sigma_spatial: float = 2.0, sigma_range: float = 0.1,
                         kernel_size: int = 5):
        """morphology.py:309-354, differentiable torch restatement (training path;
        inference runs it inside the morph kernel)."""
        B, H, W = complexity_map.shape
        pad = kernel_size // 2
        patches = F.unfold(F.pad(complexity_map.unsqueeze(1), (pad, pad, pad, pad), mode="replicate"),
                           kernel_size)
        center = complexity_map.reshape(B, 1, H * W)
        coords = torch.arange(kernel_size, dtype=torch.float32, device=complexity_map.device) - pad
        yy, xx = torch.meshgrid(coords, coords, indexing="ij")
        spatial_w = torch.exp(-(yy ** 2 + xx ** 2) / (2 * sigma_spatial ** 2)).reshape(1, -1, 1)
        range_w = torch.exp(-((patches - center) ** 2) / (2 * sigma_range ** 2))
        weights = spatial_w * range_w
        filtered = (weights * patches).sum(dim=1) / (weights.sum(dim=1) + 1e-8)
        return filtered.reshape(B, H, W)

    def _head(self, phi):
        """complexity MLP -> bilateral -> clamp on the tile features (morphology.py:959-968)."""
        B, ht, wt, _ = phi.shape
        c = self.complexity_mlp(phi.reshape(-1, 8)).reshape(B, ht, wt)
        return self.bilateral_filter(c).clamp(0.0, 1.0)

    def forward(self, features: torch.Tensor, return_detailed: bool = False):
        if not features.is_cuda:
            # pure-PyTorch path (morphology.py:939-973 on CPU tensors)
            phi, _ = self.compute_phi_tiles(features)
            c = self._head(phi)
        elif _wants_grad((), self.complexity_mlp.parameters()):
            # phi is no-grad side information (morph kernel); C is the kernel's
            # value and its gradient reaches complexity_mlp through the fused
            # head backward (mcaq_head_train_backward) or, FUSED_TRAIN off, the
            # torch restatement of the MLP + bilateral
            ht, wt = _tile_grid(features.shape[-2], features.shape[-1], self.grid_size)
            if FUSED_TRAIN and _head_bwd_fits(ht, wt):
                out = _HeadTrainFn.apply(self, features, *self.complexity_mlp.parameters())
                phi, c = self._last_phi, out
                self._last_phi = None
            else:
                phi, ck = self._run(features, want_c=True)
                c = _kernel_value(lambda p: ck, self._head, [phi], list(self.complexity_mlp.parameters()))
        else:
            phi, c = self._run(features, want_c=True)
        if return_detailed:
            return c, self._detailed(phi)
        return c


# ---------------------------------------------------------------------------
# bit_allocation.py
# ---------------------------------------------------------------------------
def _normalize_complexity_shape(complexity):
    """bit_allocation.py:145-172."""
    if not isinstance(complexity, torch.Tensor):
        raise TypeError(f"complexity must be torch.Tensor, got {type(complexity)}")
    if complexity.dim() == 2:
        complexity = complexity.unsqueeze(0)
    elif complexity.dim() == 3:
        pass
    elif complexity.dim() == 4:
        complexity = complexity.mean(dim=1)
    else:
        raise ValueError(f"Unsupported complexity dim={complexity.dim()}, expected 2, 3, or 4.")
    return complexity


def _run_mapper(c, flags, min_bits, max_bits, temperature, return_continuous, mapper_blob=None):
    _need_cuda(c, "complexity")
    c = _f32c(c)
    B, ht, wt = c.shape
    f = flags | abi.F_MAPPER
    if temperature is not None:
        f |= abi.F_HAS_T
    if return_continuous:
        f |= abi.F_CONT
    bits = torch.empty(B, ht, wt, device=c.device)
    s = _morph_struct(B, 4 * ht, 4 * wt, 4, ht, wt, f, c_in=c, bits_out=bits, mapper=mapper_blob)
    s.temperature = max(float(temperature if temperature is not None else 1.0), 0.1)
    s.min_bits, s.max_bits = float(min_bits), float(max_bits)
    abi.check(abi.lib().mcaq_morph(ctypes.byref(s), 1, _stream()), "mcaq_morph(mapper)")
    return bits


def _finish_bits(bit_map, min_bits, max_bits, temperature, return_continuous):
    """x max(T, 0.1), straight-through clamp to [min, max], straight-through
    round-half-even (bit_allocation.py:72-79 / 264-278)."""
    if temperature is not None:
        bit_map = bit_map * max(float(temperature), 0.1)
    clamped = torch.clamp(bit_map, min_bits, max_bits)
    bit_map = bit_map + (clamped - bit_map).detach()
    if not return_continuous:
        bit_map = bit_map + (torch.round(bit_map) - bit_map).detach()
    return bit_map


class LinearBitMapper(nn.Module):
    """bit_allocation.py:12-80: per-image 2-98 % percentile normalisation ->
    b = b_min + (b_max - b_min) * C_n, x temperature, clamp, round."""

    def __init__(self, min_bits: int = 2, max_bits: int = 8, eps_spread: float = 1e-3):
        super().__init__()
        self.min_bits = float(min_bits)
        self.max_bits = float(max_bits)
        if float(eps_spread) != 1e-3:
            raise NotImplementedError("eps_spread other than the reference default 1e-3")
        self.eps_spread = float(eps_spread)

    def constrained_weights(self):
        return []

    def enforce_weight_constraints(self):
        """No-op (parameter-free), as in the reference."""

    def _forward_torch(self, c, temperature, return_continuous):
        """bit_allocation.py:54-80 as torch ops (CPU path; the backward of the
        GPU path): quantile lerp, spread gate, affine, temperature, straight-
        through clamp and round."""
        B = c.shape[0]
        flat = c.reshape(B, -1).float()
        lo = torch.quantile(flat, 0.02, dim=1, keepdim=True).unsqueeze(-1)
        hi = torch.quantile(flat, 0.98, dim=1, keepdim=True).unsqueeze(-1)
        spread = hi - lo
        cn = torch.where(spread > self.eps_spread, ((c - lo) / (spread + 1e-8)).clamp(0.0, 1.0),
                         c.clamp(0.0, 1.0))
        return _finish_bits(self.min_bits + (self.max_bits - self.min_bits) * cn, self.min_bits,
                            self.max_bits, temperature, return_continuous)

    def forward(self, complexity: torch.Tensor, temperature: Optional[float] = None,
                return_continuous: bool = False) -> torch.Tensor:
        c = _normalize_complexity_shape(complexity)
        if not c.is_cuda:
            return self._forward_torch(c, temperature, return_continuous)

        def kernel(cc):
            return _run_mapper(cc, abi.F_MAP_LINEAR, self.min_bits, self.max_bits, temperature,
                               return_continuous)
        if _wants_grad((c,)):
            return _kernel_value(kernel, lambda cc: self._forward_torch(cc, temperature, return_continuous),
                                 [c], [])
        return kernel(c)


class ComplexityToBitMappingNetwork(nn.Module):
    """bit_allocation.py:83-303: z=[C, C^2, log1p C] -> 3 x (Linear, BN, ReLU)
    -> Linear -> sigmoid -> [b_min, b_max] -> x temperature -> STE clamp / round.
    Eval mode (BatchNorm running statistics)."""

    def __init__(self, min_bits: int = 2, max_bits: int = 8, hidden_dims: list = [32, 64, 32],
                 enforce_monotonicity: bool = True):
        super().__init__()
        if list(hidden_dims) != [32, 64, 32]:
            raise NotImplementedError("hidden_dims other than the reference [32, 64, 32]")
        self.min_bits = float(min_bits)
        self.max_bits = float(max_bits)
        self.enforce_monotonicity = enforce_monotonicity
        layers = []
        d = 3
        for h in hidden_dims:
            layers += [nn.Linear(d, h), nn.BatchNorm1d(h), nn.ReLU(inplace=True)]
            d = h
        layers += [nn.Linear(d, 1), nn.Sigmoid()]
        self.mapping_network = nn.Sequential(*layers)
        self.apply(self._init_weights)
        self._blob = _BlobCache()
        self._gsink = _GradSink()

    _normalize_complexity_shape = staticmethod(_normalize_complexity_shape)

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            nn.init.xavier_uniform_(m.weight, gain=0.5)
            if self.enforce_monotonicity:
                m.weight.data = torch.abs(m.weight.data)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0.1)

    def constrained_weights(self):
        """The parameters enforce_weight_constraints projects onto |W| (Linear
        weights and BatchNorm gammas; none without enforce_monotonicity) -
        for optim.ClipAdamW(project_abs=...), which folds the projection into
        the optimizer launch."""
        if not self.enforce_monotonicity:
            return []
        return [m.weight for m in self.mapping_network.modules() if isinstance(m, (nn.Linear, nn.BatchNorm1d))]

    def enforce_weight_constraints(self):
        """Eq.18: |W| for Linear layers and BatchNorm gammas (bit_allocation.py:186-197)."""
        if self.enforce_monotonicity:
            ws = [m.weight.data for m in self.mapping_network.modules() if isinstance(m, (nn.Linear, nn.BatchNorm1d))]
            # in place (parameter storage stays put for graph capture); one
            # multi-tensor launch on the GPU instead of one per layer
            if ws and all(w.is_cuda for w in ws):
                torch._foreach_abs_(ws)
            else:
                for w in ws:
                    w.abs_()

    def create_augmented_features(self, complexity: torch.Tensor) -> torch.Tensor:
        """bit_allocation.py:199-216: z0 = [C, C^2, log1p C]."""
        return torch.cat([complexity, complexity ** 2, torch.log1p(complexity)], dim=-1)

    def _forward_torch(self, complexity, temperature, return_continuous):
        """bit_allocation.py:247-280 as torch autograd ops: the CPU path, train
        mode (BatchNorm over the batch's tiles) and the backward of the GPU
        eval path."""
        c = _normalize_complexity_shape(complexity).clamp(0.0, 1.0)
        B, H, W = c.shape
        h = self.mapping_network(self.create_augmented_features(c.reshape(-1, 1)))
        bit_map = (self.min_bits + (self.max_bits - self.min_bits) * h).reshape(B, H, W)
        return _finish_bits(bit_map, self.min_bits, self.max_bits, temperature, return_continuous)

    def _fusable(self):
        """The fused train-mode kernels take the reference stack with plain
        BatchNorm1d layers, or with dist.GroupBatchNorm1d layers of one
        process group (statistics over every rank's tiles: the kernels run one
        stage per launch with the collectives between them)."""
        from .dist import GroupBatchNorm1d
        net = self.mapping_network
        bns = [net[i] for i in (1, 4, 7)]
        if not all(type(b) in (nn.BatchNorm1d, GroupBatchNorm1d) and b.track_running_stats and
                   b.momentum is not None and b.affine for b in bns):
            return False
        return len({getattr(b, "process_group", None) for b in bns}) == 1

    def mapper_blob(self):
        net = self.mapping_network
        ts = list(net.parameters()) + [net[i].running_mean for i in (1, 4, 7)] + \
            [net[i].running_var for i in (1, 4, 7)]
        return self._blob.get(ts, lambda: _pack_mapper(net))

    def forward(self, complexity: torch.Tensor, temperature: Optional[float] = None,
                return_continuous: bool = False) -> torch.Tensor:
        c = _normalize_complexity_shape(complexity)
        if self.training and c.is_cuda and FUSED_TRAIN and self._fusable():
            return _MapperTrainFn.apply(self, c, temperature, return_continuous, *self.mapping_network.parameters())
        if self.training or not c.is_cuda:
            return self._forward_torch(c, temperature, return_continuous)

        def kernel(cc):
            return _run_mapper(cc, 0, self.min_bits, self.max_bits, temperature, return_continuous,
                               mapper_blob=self.mapper_blob())
        if _wants_grad((c,), self.mapping_network.parameters()):
            return _kernel_value(kernel, lambda cc: self._forward_torch(cc, temperature, return_continuous),
                                 [c], list(self.mapping_network.parameters()))
        return kernel(c)


# ---------------------------------------------------------------------------
# quantization.py
# ---------------------------------------------------------------------------
class LearnedSoftMask(nn.Module):
    """quantization.py:168-239: per-tile [bits_norm, |x| activation] -> conv3x3
    -> ReLU -> conv1x1 -> softmax[0] -> nearest upsample -> 5x5 Gaussian
    (replicate pad).  Returns m (B, 1, H, W)."""

    def __init__(self, hidden: int = 8, kernel_size: int = 5):
        super().__init__()
        if hidden != 8 or kernel_size != 5:
            raise NotImplementedError("soft mask hidden=8, kernel_size=5 only (reference defaults)")
        self.net = nn.Sequential(nn.Conv2d(2, hidden, 3, padding=1), nn.ReLU(inplace=True),
                                 nn.Conv2d(hidden, 2, 1))
        nn.init.normal_(self.net[-1].weight, std=1e-3)
        with torch.no_grad():
            self.net[-1].bias.copy_(torch.tensor([4.0, 0.0]))
        k = kernel_size
        sigma = k / 3.0
        xs = torch.arange(k, dtype=torch.float32) - k // 2
        g1 = torch.exp(-xs ** 2 / (2 * sigma ** 2))
        g1 = g1 / g1.sum()
        self.register_buffer("smooth_kernel", (g1.unsqueeze(0) * g1.unsqueeze(1)).unsqueeze(0).unsqueeze(0))
        self.kernel_size = k
        self._blob = _BlobCache()
        self._gsink = _GradSink()

    def blob(self):
        return self._blob.get(list(self.net.parameters()), lambda: _pack_softmask(self.net))

    def _run(self, bit_map, x, absmean, plane):
        _need_cuda(bit_map, "bit_map")
        _need_cuda(x, "x")
        B, C, H, W = x.shape
        bits = _f32c(bit_map)
        _, ht, wt = bits.shape
        if absmean is None:
            absmean = torch.empty(B, H, W, device=x.device)
            _run_stats(_f32c(x), absmean=absmean)
        if 4 * ht > H or 4 * wt > W:
            # the launcher's geometry check wants >= 4 pixels per tile (every
            # hook tile grid has them: tile = pow2floor(max(4, H // grid)))
            raise NotImplementedError("soft mask on a tile grid finer than 4 pixels per tile")
        out = torch.empty(B, 1, H, W, device=x.device) if plane else torch.empty(B, ht, wt, device=x.device)
        # tile / crop fields only satisfy the launcher: the soft-mask stage
        # pools and upsamples over (H, W) like adaptive_avg_pool2d / nearest
        ptrs = dict(absmean=absmean, bits_in=bits, smask=self.blob())
        ptrs["m_out" if plane else "mt_out"] = out
        s = _morph_struct(B, H, W, 4, ht, wt, abi.F_SOFTMASK, **ptrs)
        abi.check(abi.lib().mcaq_morph(ctypes.byref(s), 1, _stream()), "mcaq_morph(soft mask)")
        return out

    def forward(self, bit_map: torch.Tensor, x: torch.Tensor, absmean: Optional[torch.Tensor] = None):
        if not x.is_cuda:
            # pure-PyTorch path: per-pixel channel mean of |x| (no grad to x)
            if absmean is None:
                absmean = x.detach().float().abs().mean(1)
            return self._torch_forward(bit_map, absmean)
        if torch.is_grad_enabled() and (bit_map.requires_grad or any(p.requires_grad for p in self.net.parameters())):
            _need_cuda(x, "x")
            if absmean is None:
                B, C, H, W = x.shape
                absmean = torch.empty(B, H, W, device=x.device)
                _run_stats(_f32c(x), absmean=absmean)
            return _SoftMaskFn.apply(bit_map, absmean, self, *self.net.parameters())
        return self._run(bit_map, x, absmean, plane=True)

    def _torch_forward(self, bit_map, absmean):
        """quantization.py:213-239 as torch ops (the backward recomputation);
        absmean = x.abs().mean(1) from pass 1 (bit-identical to ATen's)."""
        B, H, W = absmean.shape
        Ht, Wt = bit_map.shape[-2:]
        with torch.no_grad():
            act = F.adaptive_avg_pool2d(absmean.unsqueeze(1), (Ht, Wt))
            act = act / (act.amax(dim=(2, 3), keepdim=True) + 1e-8)
        bits_norm = ((bit_map.unsqueeze(1).float() - 2.0) / 6.0).clamp(0.0, 1.0)
        logits = self.net(torch.cat([bits_norm, act.float()], dim=1))
        m = torch.softmax(logits, dim=1)[:, :1]
        m = _nearest_up(m, H, W)
        p = self.kernel_size // 2
        return F.conv2d(F.pad(m, (p, p, p, p), mode="replicate"), self.smooth_kernel)

    def tile_values(self, bit_map, x, absmean=None):
        """m per tile before upsampling/smoothing (B, Ht, Wt); the quant pass
        turns it into m(p) on the fly."""
        return self._run(bit_map, x, absmean, plane=False)


@functools.lru_cache(maxsize=None)
def _block_nearest(n_in, n_out):
    """True when ATen's nearest index floor(o * fp32(n_in / n_out)) is the block
    index o // (n_out / n_in) for every output o (UpSampleKernel nearest_idx)."""
    if n_out % n_in:
        return False
    s = n_out // n_in
    sc = torch.tensor(n_in / n_out, dtype=torch.float32)
    o = torch.arange(n_out, dtype=torch.float32)
    return bool(torch.equal(torch.floor(o * sc).long(), torch.arange(n_out) // s))


def _nearest_up(m, H, W):
    """F.interpolate(m, (H, W), 'nearest') with the same values; on the GPU,
    when the index map is a block map, as an expand whose backward is a
    per-tile sum (ATen's upsample_nearest2d_backward kernel takes ~67 us per
    call at config 5).  CPU tensors keep the reference op (bit-exact grads)."""
    Ht, Wt = m.shape[-2:]
    if m.is_cuda and _block_nearest(Ht, H) and _block_nearest(Wt, W):
        B, C = m.shape[:2]
        return m[:, :, :, None, :, None].expand(B, C, Ht, H // Ht, Wt, W // Wt).reshape(B, C, H, W)
    return F.interpolate(m, size=(H, W), mode="nearest")


class _SoftMaskFn(torch.autograd.Function):
    """m(p) forward by the morph kernel (bit-exact with the reference); backward
    by recomputing the tile-sized soft-mask net with torch autograd."""

    @staticmethod
    def forward(ctx, bit_map, absmean, mod, *params):
        ctx.mod = mod
        ctx.save_for_backward(bit_map, absmean)
        B, H, W = absmean.shape
        m = mod._run(bit_map.detach(), torch.empty(B, 1, H, W, device=absmean.device), absmean, plane=True)
        return m

    @staticmethod
    def backward(ctx, gm):
        bit_map, absmean = ctx.saved_tensors
        mod = ctx.mod
        params = list(mod.net.parameters())
        if FUSED_TRAIN and _smask_bwd_fits(absmean.shape[-2], absmean.shape[-1], bit_map.shape[-2], bit_map.shape[-1]):
            return _smask_backward_fused(ctx, mod, bit_map, absmean, gm, params)
        with torch.enable_grad():
            b = bit_map.detach().requires_grad_(ctx.needs_input_grad[0])
            m = mod._torch_forward(b, absmean)
            ins = ([b] if ctx.needs_input_grad[0] else []) + [p for p in params if p.requires_grad]
            grads = torch.autograd.grad(m, ins, gm, allow_unused=True) if ins else []
        it = iter(grads)
        gb = next(it) if ctx.needs_input_grad[0] else None
        gp = [next(it) if p.requires_grad else None for p in params]
        return (gb, None, None) + tuple(gp)


# ---------------------------------------------------------------------------
# train-mode tile networks on the fused kernels (csrc/mcaq_train.h)
# ---------------------------------------------------------------------------
# False: the torch autograd restatement of the analyzer head, the train-mode
# mapper and the soft-mask backward (the r02 path; A/B and cross-check)
FUSED_TRAIN = True


# LDS the fused train-mode backwards stage per workgroup (csrc/mcaq_train.h
# launchers; the kernels take at most 159 KiB): when an image does not fit,
# the call takes the torch restatement (the FUSED_TRAIN = False branch)
_TRAIN_LDS_LIMIT = 160 * 1024 - 1024


def _head_bwd_fits(ht, wt):
    """mcaq_head_train_backward: 53 floats per tile of one image."""
    return 53 * ht * wt * 4 <= _TRAIN_LDS_LIMIT


def _smask_bwd_fits(H, W, ht, wt):
    """mcaq_smask_train_backward: one image's m(p) gradient plus tile and
    row tables."""
    return (22 * ht * wt + 64 + 1024 + 176 + H * wt + H * W) * 4 + 2 * (ht + wt) * 4 <= _TRAIN_LDS_LIMIT


def _tile_grid(H, W, grid_size):
    tile = tile_size(H, grid_size)
    return H // tile, W // tile


def _split_flat(flat, params):
    out, o = [], 0
    for p in params:
        n = p.numel()
        out.append(flat[o:o + n].view_as(p))
        o += n
    return out


# The fused backwards of the modules shared by the three hook scales (the
# complexity MLP and the bit mapper) accumulate their parameter gradients
# directly into one persistent flat buffer whose views are the parameters'
# .grad (as fused optimizers do), instead of returning them to autograd,
# which would add the three scales' gradients with one ATen kernel per
# parameter tensor (54 launches per QAT step).  Consequence: those gradients
# reach .grad through backward() / loss.backward(), not through
# torch.autograd.grad(..., inputs=params).  False: returned to autograd.
DIRECT_GRAD_ACCUM = True


def _grads_observed(params):
    """True when something outside backward() must see these parameters'
    gradients as autograd results: torch DDP's reducer (it hooks every
    parameter's AccumulateGrad and would never see a gradient written straight
    into .grad) or any parameter hook.  Direct accumulation is then off and the
    gradients go back to autograd.  A torch.distributed process group alone
    counts as observed (a DDP wrapper may hold the parameters) - unless every
    parameter is marked as synchronised by this package's own data-parallel
    step (dist.shard_hooks: dist.allreduce_gradients reads the sinks, no
    reducer is involved)."""
    for p in params:
        if getattr(p, "_backward_hooks", None) or getattr(p, "_post_accumulate_grad_hooks", None):
            return True
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return not all(getattr(p, "_mcaq_dp_manual", False) for p in params)
    return False


class _GradArena:
    """The gradient sinks of several nets as consecutive slices of ONE flat
    device buffer (dist.shard_hooks), so the data-parallel step's gradient
    bucket is that buffer, all-reduced in place (dist.allreduce_gradients)."""

    def __init__(self, pairs, device):
        n = sum(p.numel() for _, ps in pairs for p in ps)
        self.flat = torch.zeros(n, device=device)
        o = 0
        for sk, ps in pairs:
            k = sum(p.numel() for p in ps)
            old = sk.views
            sk.flat = self.flat[o:o + k]
            sk.views = _split_flat(sk.flat, ps)
            for i, (p, v) in enumerate(zip(ps, sk.views)):
                # a .grad that was the old sink's view moves into the arena
                if old is not None and i < len(old) and p.grad is not None and \
                        p.grad.data_ptr() == old[i].data_ptr() and p.grad.shape == v.shape:
                    v.copy_(p.grad)
                    p.grad = v
            o += k


class _GradSink:
    """Flat gradient storage for a module's parameters; `target(params)`
    returns (flat buffer, accumulate flag) for the next backward, or None when
    some parameter's .grad is neither None nor this sink's view (gradients
    from elsewhere: return them to autograd)."""

    def __init__(self):
        self.flat = None
        self.views = None

    def _plan(self, params):
        """1 (accumulate into the sink), 0 (fresh: .grad to become the
        sink's views) or None (autograd); no .grad is touched."""
        if not DIRECT_GRAD_ACCUM or not all(p.requires_grad for p in params):
            return None
        if _grads_observed(params):
            return None
        n = sum(p.numel() for p in params)
        dev = params[0].device
        if self.flat is None or self.flat.numel() != n or self.flat.device != dev:
            if dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
                return None          # first use must happen outside capture (warm-up step)
            self.flat = torch.zeros(n, device=dev)
            self.views = _split_flat(self.flat, params)
        mine = [p.grad is not None and p.grad.data_ptr() == v.data_ptr() and p.grad.shape == v.shape
                for p, v in zip(params, self.views)]
        if all(mine):
            return 1
        if any(p.grad is not None for p in params):
            return None
        return 0

    def _take(self, params, acc):
        if acc == 0:
            for p, v in zip(params, self.views):
                p.grad = v
        return self.flat, acc

    def target(self, params):
        acc = self._plan(params)
        return None if acc is None else self._take(params, acc)

    @staticmethod
    def target_all(pairs):
        """[(sink, params), ...] -> every sink's (flat, accumulate), or None
        (and no .grad touched) when any of them must go through autograd."""
        plans = [sk._plan(ps) for sk, ps in pairs]
        if any(a is None for a in plans):
            return None
        return [sk._take(ps, a) for (sk, ps), a in zip(pairs, plans)]


class _HeadTrainFn(torch.autograd.Function):
    """Analyzer in train mode: phi, C (= clamp(bilateral(MLP(phi)))) and the
    MLP output from the morph kernel (bit-exact forward); the backward is the
    fused bilateral adjoint + complexity MLP backward."""

    @staticmethod
    def forward(ctx, mod, features, *params):
        phi, c, craw = mod._run(features, want_c=True, want_craw=True)
        mod._last_phi = phi
        ctx.mod = mod
        ctx.conc = concurrent_scales.active
        ctx.save_for_backward(phi, craw, *params)
        return c

    @staticmethod
    def backward(ctx, gc):
        phi, craw = ctx.saved_tensors[:2]
        params = ctx.saved_tensors[2:]
        B, ht, wt = craw.shape
        n = B * ht * wt
        L = abi.lib()
        q = abi.CmlpParams(*[_p(p.detach()) for p in params])
        gcraw = torch.empty(n, device=craw.device)
        mod_params = list(ctx.mod.complexity_mlp.parameters())
        sink = ctx.mod._gsink.target(mod_params) if len(mod_params) == len(params) else None
        gflat, acc = sink if sink is not None else (torch.empty(_CM_SIZE, device=craw.device), 0)
        gpart = torch.empty(L.mcaq_head_gpart_floats(n), device=craw.device)
        if ctx.conc is not None:
            ctx.conc.join_after_backward()
        conc = ctx.conc if sink is not None else None    # shared flat buffer, scales on several streams
        abi.check(L.mcaq_head_train_backward(ctypes.byref(q), _p(phi), _p(craw), _p(_f32c(gc)), B, ht, wt, _p(gcraw),
                                             None if conc else _p(gflat), _p(gpart), acc, _stream()),
                  "mcaq_head_train_backward")
        if conc is not None:
            conc.ordered(ctx.mod._gsink, lambda: abi.check(
                L.mcaq_head_train_grad_reduce(n, _p(gpart), _p(gflat), acc, _stream()), "mcaq_head_train_grad_reduce"))
        if sink is not None:
            return (None, None) + (None,) * len(params)
        return (None, None) + tuple(_split_flat(gflat, params))


# ---------------------------------------------------------------------------
# hook scales on concurrent streams (train mode, MCAQHooks.forward_features)
# ---------------------------------------------------------------------------
class concurrent_scales:
    """Scope of one train-mode hook step whose scales run on their own HIP
    streams (each scale's forward, and so its backward, on its stream).  The
    modules the scales share get ordered here instead of by one stream:
      * the complexity-MLP blob is packed once, before the fork (pinned);
      * the train-mode mapper's BatchNorm running statistics: each scale's
        forward leaves its batch mean / unbiased variance in its work buffer
        (update_stats 2) and `finish` applies the updates in scale order on
        the joining stream (mcaq_mapper_running_update: the values the scales
        would have left one after another);
      * gradients accumulated in-kernel into the shared flat buffers
        (_GradSink): each backward's reduction launch waits for the previous
        one (events, in autograd's launch order) - a fixed order of fp32 sums.
    Entered by the caller on its own stream; `finish(stream)` after the join."""

    active = None

    def __init__(self, analyzer=None, main=None, streams=()):
        self.analyzer = analyzer
        self.mapper = {}          # id(module) -> [q, works, ns, momentum, keepalive]
        self.events = {}          # grad sink -> event of its last reduction launch
        self.main, self.streams = main, list(streams)
        self._join_queued = False

    def __enter__(self):
        if concurrent_scales.active is not None:
            raise RuntimeError("concurrent_scales scopes do not nest")
        if self.analyzer is not None:
            an = self.analyzer
            an._blob.pinned = an.cmlp_blob()
        concurrent_scales.active = self
        return self

    def __exit__(self, *exc):
        concurrent_scales.active = None
        if self.analyzer is not None:
            self.analyzer._blob.pinned = None
        return False

    def defer_mapper(self, mod, q, work, n, momentum):
        e = self.mapper.setdefault(id(mod), [q, [], [], momentum, mod])
        e[1].append(work)
        e[2].append(n)

    def finish(self):
        """On the joining stream, after every scale's stream: the deferred
        mapper running-statistics updates, in scale order."""
        L = abi.lib()
        for q, works, ns, momentum, _mod in self.mapper.values():
            for k in range(0, len(works), 8):
                w, n = works[k:k + 8], ns[k:k + 8]
                wa = (abi.P * len(w))(*[_p(t) for t in w])
                na = (abi.I * len(n))(*n)
                abi.check(L.mcaq_mapper_running_update(ctypes.byref(q), wa, na, len(w), float(momentum), _stream()),
                          "mcaq_mapper_running_update")
        self.mapper = {}

    def join_after_backward(self):
        """Called from the backward of a scale's node: once per backward pass,
        queue an engine callback that makes the stream the forward joined on
        wait for every scale stream (the in-kernel gradient accumulations on
        those streams are not autograd results, so the engine's own leaf-stream
        sync need not cover them)."""
        if self._join_queued or self.main is None:
            return
        self._join_queued = True

        def join():
            self._join_queued = False
            for st in self.streams:
                self.main.wait_stream(st)
        torch.autograd.Variable._execution_engine.queue_callback(join)

    def ordered(self, key, launch):
        """Run `launch()` (a reduction into a buffer the scales share) on the
        current stream after the previous one of the same key."""
        st = torch.cuda.current_stream()
        ev = self.events.get(key)
        if ev is not None:
            st.wait_event(ev)
        launch()
        ev = torch.cuda.Event()
        ev.record(st)
        self.events[key] = ev


# one-launch train-mode mapper (grid barriers between its batch-statistics
# stages) instead of one launch per stage: measured slower at config 5 (the
# agent-scope release / acquire around each barrier costs more than a kernel
# boundary: forward 46.7 vs 37.6 us, backward 68.7 vs ~55 us per scale,
# profiles/r03_qat/one_launch_mapper_ab.txt), so off by default
MAPPER_ONE_LAUNCH = False
_GRID_SYNC = {}


def _grid_sync_counter(device):
    """Zeroed uint32 pair for the mapper's grid barriers: one persistent buffer
    per (device, stream) - launches on one stream run one after another and
    each leaves it zeroed; launches on different streams get different
    buffers.  Created inside a graph capture, the buffer's zero fill is
    captured too (every replay re-zeroes it).  None when MAPPER_ONE_LAUNCH is
    off (multi-launch path)."""
    if not MAPPER_ONE_LAUNCH:
        return None
    key = (torch.device(device), torch.cuda.current_stream(device).cuda_stream)
    buf = _GRID_SYNC.get(key)
    if buf is None:
        buf = torch.zeros(2, dtype=torch.int32, device=device)
        _GRID_SYNC[key] = buf
    return buf


class _MapperTrainFn(torch.autograd.Function):
    """ComplexityToBitMappingNetwork in train mode (batch-statistics
    BatchNorm, running stats updated, straight-through clamp / round) on the
    fused kernels: 4 forward launches, 5 backward launches."""

    @staticmethod
    def forward(ctx, mod, c, temperature, return_continuous, *params):
        net = mod.mapping_network
        cf = _f32c(c).reshape(-1)
        n = cf.numel()
        L = abi.lib()
        bns = [net[i] for i in (1, 4, 7)]
        q = abi.MapperParams()
        for k, t in zip(("w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4"),
                        (net[0].weight, net[0].bias, net[3].weight, net[3].bias, net[6].weight, net[6].bias,
                         net[9].weight, net[9].bias)):
            setattr(q, k, _p(t.detach()))
        for i, bn in enumerate(bns, 1):
            for k, t in (("g", bn.weight), ("be", bn.bias), ("rm", bn.running_mean), ("rv", bn.running_var),
                         ("nbt", bn.num_batches_tracked)):
                setattr(q, "%s%d" % (k, i), _p(t.detach()) if t is not None else None)
        T = max(float(temperature), 0.1) if temperature is not None else 0.0
        work = torch.empty(L.mcaq_mapper_work_floats(n), device=c.device)
        bits = torch.empty(n, device=c.device)
        pg = _mapper_group(net)
        ctx.pg, ctx.gath1 = pg, None
        conc = concurrent_scales.active if pg is None else None
        ctx.conc = conc
        if pg is None:
            # scales on concurrent streams: the shared running statistics are
            # updated later, in scale order (concurrent_scales.finish)
            abi.check(L.mcaq_mapper_train_forward(ctypes.byref(q), _p(cf), n, mod.min_bits, mod.max_bits, T,
                                                  float(bns[0].momentum), 0 if return_continuous else 1,
                                                  2 if conc is not None else 1, _p(bits),
                                                  _p(work), _p(_grid_sync_counter(c.device)), _stream()),
                      "mcaq_mapper_train_forward")
            if conc is not None:
                conc.defer_mapper(mod, q, work, n, float(bns[0].momentum))
        else:
            # batch sharded over the group (GroupBatchNorm1d): the BatchNorm
            # statistics of every layer span the ranks' tiles - each rank's
            # (mean, M2, n) all-gathered between the stage launches
            import torch.distributed as dist
            world = dist.get_world_size(pg)
            gath = [None] * 4
            for st in (1, 2, 3, 4):
                abi.check(L.mcaq_mapper_train_forward_stage(
                    ctypes.byref(q), _p(cf), n, mod.min_bits, mod.max_bits, T, float(bns[0].momentum),
                    0 if return_continuous else 1, 1, _p(bits), _p(work), st, _p(gath[st - 1]), world, _stream()),
                    "mcaq_mapper_train_forward_stage")
                if st <= 3:
                    rk = torch.empty(_RANK_ENT, device=c.device)
                    abi.check(L.mcaq_mapper_train_reduce(_p(work), n, 0, st, _p(rk), _stream()),
                              "mcaq_mapper_train_reduce")
                    gath[st] = _all_gather_flat(rk, pg, world)
            ctx.gath1, ctx.world = gath[1], world
        ctx.q, ctx.T, ctx.mod = q, T, mod
        ctx.save_for_backward(cf, work, *params)
        return bits.view(c.shape)

    @staticmethod
    def backward(ctx, gbits):
        cf, work = ctx.saved_tensors[:2]
        params = ctx.saved_tensors[2:]
        n = cf.numel()
        L = abi.lib()
        mod = ctx.mod
        gc = torch.empty(n, device=cf.device)
        sink = mod._gsink.target(list(mod.mapping_network.parameters()))
        gflat, acc = sink if sink is not None else (torch.empty(_MAPPER_G_SIZE, device=cf.device), 0)
        gpart = torch.empty(L.mcaq_mapper_gpart_floats(n), device=cf.device)
        gb = _f32c(gbits)
        if ctx.conc is not None:
            ctx.conc.join_after_backward()
        conc = ctx.conc if sink is not None else None
        if ctx.pg is None and conc is not None:
            # the scales' reductions into the shared flat buffer, one after another
            abi.check(L.mcaq_mapper_train_backward(ctypes.byref(ctx.q), _p(cf), n, _p(gb), mod.min_bits,
                                                   mod.max_bits, ctx.T, _p(work), _p(gc), None, _p(gpart), acc,
                                                   None, _stream()), "mcaq_mapper_train_backward")
            conc.ordered(mod._gsink, lambda: abi.check(
                L.mcaq_mapper_train_grad_reduce(n, _p(gpart), _p(gflat), acc, _stream()),
                "mcaq_mapper_train_grad_reduce"))
        elif ctx.pg is None:
            abi.check(L.mcaq_mapper_train_backward(ctypes.byref(ctx.q), _p(cf), n, _p(gb), mod.min_bits,
                                                   mod.max_bits, ctx.T, _p(work), _p(gc), _p(gflat), _p(gpart), acc,
                                                   _p(_grid_sync_counter(cf.device)), _stream()),
                      "mcaq_mapper_train_backward")
        else:
            # BN backward sums (S1, S2) of each layer all-reduced over the
            # ranks before the stage that consumes them (the autograd of
            # GroupBatchNorm1d's all-reduce); parameter gradients stay this
            # rank's own, for the gradient all-reduce
            import torch.distributed as dist
            gs = [None] * 5
            for st in (4, 3, 2, 1):
                abi.check(L.mcaq_mapper_train_backward_stage(
                    ctypes.byref(ctx.q), _p(cf), n, _p(gb), mod.min_bits, mod.max_bits, ctx.T, _p(work), _p(gc),
                    _p(gpart), st, _p(gs[st]), _p(ctx.gath1), ctx.world, _stream()),
                    "mcaq_mapper_train_backward_stage")
                if st >= 2:
                    bs = torch.empty(128, device=cf.device)
                    abi.check(L.mcaq_mapper_train_reduce(_p(work), n, 1, st - 1, _p(bs), _stream()),
                              "mcaq_mapper_train_reduce")
                    dist.all_reduce(bs, group=ctx.pg)
                    gs[st - 1] = bs
            abi.check(L.mcaq_mapper_train_grad_reduce(n, _p(gpart), _p(gflat), acc, _stream()),
                      "mcaq_mapper_train_grad_reduce")
        if sink is not None:
            return (None, gc.view(gbits.shape), None, None) + (None,) * len(params)
        return (None, gc.view(gbits.shape), None, None) + tuple(_split_flat(gflat, params))


_MAPPER_G_SIZE = 4609
_RANK_ENT = 129          # (mean[64], M2[64], n) of one rank's tiles (csrc/mcaq_train.h RANK_ENT)


def _mapper_group(net):
    """The process group of a mapping network whose BatchNorm layers are
    dist.GroupBatchNorm1d over one group, else None."""
    pg = getattr(net[1], "process_group", None)
    if pg is None:
        return None
    import torch.distributed as dist
    return pg if dist.is_available() and dist.is_initialized() else None


def _all_gather_flat(t, pg, world):
    """All ranks' copies of the flat tensor t, concatenated in rank order."""
    import torch.distributed as dist
    if dist.get_backend(pg) == "nccl":
        out = torch.empty(world * t.numel(), device=t.device, dtype=t.dtype)
        dist.all_gather_into_tensor(out, t, group=pg)
        return out
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=pg)
    return torch.cat(parts)


def _smask_backward_fused(ctx, mod, bit_map, absmean, gm, params):
    """LearnedSoftMask backward on the fused kernel: grads of the bit map and
    of the net's parameters from the m(p) gradient."""
    B, H, W = absmean.shape
    _, ht, wt = bit_map.shape
    L = abi.lib()
    q = abi.SmaskParams(*[_p(p.detach()) for p in params])
    gb = torch.empty(B, ht, wt, device=absmean.device)
    gflat = torch.empty(_SM_SIZE, device=absmean.device)
    gpart = torch.empty(L.mcaq_smask_gpart_floats(B), device=absmean.device)
    abi.check(L.mcaq_smask_train_backward(ctypes.byref(q), _p(_f32c(bit_map)), _p(absmean), _p(_f32c(gm)), B, H, W,
                                          ht, wt, _p(gb), 0, _p(gflat), _p(gpart), _stream()),
              "mcaq_smask_train_backward")
    gp = _split_flat(gflat, params)
    return (gb if ctx.needs_input_grad[0] else None, None, None) + tuple(
        g if p.requires_grad else None for g, p in zip(gp, params))


def _qat_struct(x, bits, m, xmin, xmax):
    B, C, H, W = x.shape
    q = abi.QatScale()
    q.x, q.bits, q.m, q.xmin, q.xmax = _p(x), _p(bits), _p(m), _p(xmin), _p(xmax)
    q.B, q.C, q.H, q.W = B, C, H, W
    q.ht, q.wt = bits.shape[-2], bits.shape[-1]
    return q


def qat_quantize(x, bits, m, xmin, xmax):
    """Fractional-bit QAT forward (quantization.py:699-727, 733-737) on the HIP
    kernel: y = ((1-f) Q_floor(b) + f Q_floor(b)+1)(x) * m.  No autograd."""
    y = torch.empty_like(x)
    q = _qat_struct(x, bits, m, xmin, xmax)
    q.y = _p(y)
    abi.check(abi.lib().mcaq_qat_forward(ctypes.byref(q), 1, _stream()), "mcaq_qat_forward")
    return y


# The backward's in-launch fold (arrival counters, last unit of each tile-row
# band folds it) measured slower than backward kernel + fold kernel at config
# 5 (46.4 vs 32.1 + 8.5 us: every unit drains its stores before counting in),
# so the two-kernel form is the default; the in-launch form stays selectable.
FOLD_IN_LAUNCH = False
_ARRIVE = {}


def _arrive_counters(B, device):
    """Zeroed per-image arrival counters for the in-launch fold of
    mcaq_qat_backward (the kernel leaves them zeroed): one persistent int32
    buffer per (device, stream), created outside graph capture.  Launches on
    one stream run one after another, and each leaves the counters zeroed, so
    the scales of a step may share a buffer; launches on different streams
    (batches in flight) get different buffers.  While a HIP graph is being
    captured and none exists yet, a fresh zeroed buffer is captured (its fill
    node re-zeroes it on each replay)."""
    key = (torch.device(device), torch.cuda.current_stream(device).cuda_stream)
    buf = _ARRIVE.get(key)
    if buf is not None and buf.numel() >= B:
        return buf
    if torch.cuda.is_current_stream_capturing():
        return torch.zeros(B, dtype=torch.int32, device=device)
    buf = torch.zeros(max(B, 1024), dtype=torch.int32, device=device)
    _ARRIVE[key] = buf
    return buf


def qat_quantize_backward(g, x, bits, m, xmin, xmax, want_gm=True, want_gb=True):
    """Straight-through backward (quantization.py:94-118 + the autograd graph of
    :699-737): (grad_x, grad_bits (B,ht,wt) or None, grad_m (B,H,W) or None)."""
    B, C, H, W = x.shape
    L = abi.lib()
    gx = torch.empty_like(x)
    gm = torch.empty(B, H, W, device=x.device) if (want_gm and m is not None) else None
    gb = torch.empty(bits.shape, device=x.device) if want_gb else None
    work = torch.empty(L.mcaq_qat_work_floats(B, C, H, W), device=x.device)
    q = _qat_struct(x, bits, m, xmin, xmax)
    q.g, q.gx, q.gm, q.gb, q.work = _p(g), _p(gx), _p(gm), _p(gb), _p(work)
    if FOLD_IN_LAUNCH and (gm is not None or gb is not None) and 16 <= W <= 512:
        q.arrive = _p(_arrive_counters(B * bits.shape[-2], x.device))   # fold inside the backward launch
    abi.check(L.mcaq_qat_backward(ctypes.byref(q), 1, _stream()), "mcaq_qat_backward")
    return gx, gb, gm


class _QATQuantFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bit_map, m, xmin, xmax):
        xf, bits = _f32c(x), _f32c(bit_map)
        mf = None if m is None else _f32c(m)
        ctx.save_for_backward(xf, bits, mf, xmin, xmax)
        return qat_quantize(xf, bits, mf, xmin, xmax)

    @staticmethod
    def backward(ctx, g):
        xf, bits, mf, xmin, xmax = ctx.saved_tensors
        gx, gb, gm = qat_quantize_backward(_f32c(g), xf, bits, mf, xmin, xmax,
                                           want_gm=ctx.needs_input_grad[2], want_gb=ctx.needs_input_grad[1])
        if gm is not None:
            gm = gm.view(mf.shape)
        return gx, gb, gm, None, None


class SpatialAdaptiveQuantization(nn.Module):
    """quantization.py:242-754, inference: per-channel (batch, H, W) min/max (or
    frozen calibration stats) -> per-tile 2..8-bit quant/dequant x m(p).
    One read of x for min/max + |x| mean, one read + one write for y."""

    def __init__(self, calibration_mode: str = "minmax", smooth_transitions: bool = True,
                 per_channel: bool = True, learned_rounding: bool = False, momentum: float = 0.99):
        super().__init__()
        if calibration_mode != "minmax":
            raise NotImplementedError("calibration_mode=%r: the hooks use 'minmax' "
                                      "(models/mcaq_yolo.py:466-470)" % calibration_mode)
        if learned_rounding:
            raise NotImplementedError("learned_rounding is never enabled by the reference hooks")
        self.calibration_mode = calibration_mode
        self.smooth_transitions = smooth_transitions
        self.per_channel = per_channel
        self.momentum = momentum
        self.register_buffer("running_min", None)
        self.register_buffer("running_max", None)
        self.register_buffer("num_batches_tracked", torch.tensor(0))
        self.register_buffer("stats_frozen", torch.tensor(False))
        self.learned_rounding = None
        self.soft_mask = LearnedSoftMask() if smooth_transitions else None
        self.register_buffer("calibration_histogram", None)
        self.histogram_bins = 2048
        self._frozen_cached = False
        # data-parallel training: set to a torch.distributed group to make the
        # EMA statistics global; None = this process's batch only
        self.process_group = None

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        """quantization.py:297-312: materialise the lazy running_min/max buffers."""
        for name in ("running_min", "running_max"):
            key = prefix + name
            if key in state_dict and getattr(self, name) is None:
                setattr(self, name, torch.zeros_like(state_dict[key]))
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)

    def freeze_calibration(self):
        self.stats_frozen = torch.tensor(True, device=self.stats_frozen.device)

    def _frozen(self):
        """bool(stats_frozen) without a device sync while a HIP graph is being
        captured (the flag cannot change inside a captured step)."""
        if self.stats_frozen.is_cuda and torch.cuda.is_current_stream_capturing():
            return self._frozen_cached
        self._frozen_cached = bool(self.stats_frozen)
        return self._frozen_cached

    def batch_minmax(self, x, absmean=None):
        """Per-channel (or per-tensor) min/max of the batch, expanded to C entries."""
        xmin, xmax = _channel_minmax(x, absmean)
        if not self.per_channel:
            xmin = xmin.amin().expand(x.shape[1]).contiguous()
            xmax = xmax.amax().expand(x.shape[1]).contiguous()
        return xmin, xmax

    def _global_minmax(self, xmin, xmax):
        """Batch-sharded data parallelism: min/max over the global batch with one
        all-reduce (MAX over [-min, max]) when a process group is set."""
        if self.process_group is None:
            return xmin, xmax
        import torch.distributed as dist
        shape = xmin.shape
        vec = torch.cat([-xmin.reshape(-1), xmax.reshape(-1)])
        dist.all_reduce(vec, op=dist.ReduceOp.MAX, group=self.process_group)
        n = xmin.numel()
        return (-vec[:n]).reshape(shape).contiguous(), vec[n:].reshape(shape).contiguous()

    def _batch_stats_torch(self, x):
        """Per-channel (keepdim (1, C, 1, 1)) or per-tensor min/max of the batch
        (quantization.py:330-338, 423-429)."""
        if self.per_channel:
            dims = [0] + list(range(2, x.dim()))
            return x.amin(dim=dims, keepdim=True), x.amax(dim=dims, keepdim=True)
        return x.min(), x.max()

    @torch.no_grad()
    def _update_running_stats_torch(self, x):
        xmin, xmax = self._global_minmax(*self._batch_stats_torch(x.detach().float()))
        self.running_min, self.running_max = fallback.ema_update(self.running_min, self.running_max, xmin,
                                                                 xmax, self.momentum)
        self.num_batches_tracked += 1

    @torch.no_grad()
    def update_running_stats(self, x: torch.Tensor, absmean: Optional[torch.Tensor] = None, want_copies=False,
                             partials=None):
        """quantization.py:319-353: EMA(momentum) of the batch min/max (pass 1 +
        finalize + mcaq_ema_stats; absmean, if given, is filled by the same read).
        want_copies (per-channel, GPU): also return copies (xmin, xmax) of the
        updated statistics, written by the EMA launch itself (the values this
        step's quantizer reads; the running buffers change in place later)."""
        if self._frozen():
            return None
        if not x.is_cuda:
            return self._update_running_stats_torch(x)
        _need_cuda(x, "x")
        xf = _f32c(x)
        xmin, xmax = _channel_minmax(xf, absmean, partials)
        if self.process_group is not None:
            # data-parallel QAT: the EMA sees the global batch's min/max (one
            # all-reduce, MAX over [-min, max]), as a single process would
            import torch.distributed as dist
            vec = torch.cat([-xmin, xmax])
            dist.all_reduce(vec, op=dist.ReduceOp.MAX, group=self.process_group)
            C0 = xmin.numel()
            xmin, xmax = -vec[:C0], vec[C0:].contiguous()
            xmin = xmin.contiguous()
        C = x.shape[1]
        if self.per_channel:
            shape = (1, C) + (1,) * (x.dim() - 2)
            nmin, nmax = xmin.view(shape), xmax.view(shape)
        else:
            nmin, nmax = xmin.amin(), xmax.amax()
        first = self.running_min is None
        if not first and self.running_min.numel() != nmin.numel():
            raise RuntimeError("running stats have %d entries, batch has %d"
                               % (self.running_min.numel(), nmin.numel()))
        inplace = not first and all(t.dtype == torch.float32 and t.is_contiguous() and t.device == nmin.device
                                    for t in (self.running_min, self.running_max))
        if inplace:
            # updated in place (persistent buffers: a captured HIP graph replays
            # the EMA); consumers of the statistics take copies
            rmin, rmax = self.running_min, self.running_max
        else:
            rmin, rmax = nmin.clone(), nmax.clone()
            if not first:
                rmin.copy_(self.running_min.reshape(nmin.shape))
                rmax.copy_(self.running_max.reshape(nmax.shape))
        nbt = self.num_batches_tracked
        kernel_nbt = (nbt.device == nmin.device and nbt.dtype == torch.int64 and nbt.numel() == 1
                      and nbt.is_contiguous())
        cmin = cmax = None
        if want_copies and self.per_channel:
            cmin = torch.empty(nmin.numel(), device=nmin.device)
            cmax = torch.empty(nmin.numel(), device=nmin.device)
        # EMA, this step's copies and num_batches_tracked += 1 in one launch
        abi.check(abi.lib().mcaq_ema_stats_ex(_p(nmin), _p(nmax), _p(rmin), _p(rmax), nmin.numel(),
                                              float(self.momentum), 1 if first else 0, _p(cmin), _p(cmax),
                                              _p(nbt) if kernel_nbt else None, _stream()), "mcaq_ema_stats_ex")
        self.running_min, self.running_max = rmin, rmax
        if not kernel_nbt:
            self.num_batches_tracked += 1
        return (cmin, cmax) if cmin is not None else None

    def _stats_c(self, t, C):
        t = t.reshape(-1).float()
        return (t.expand(C) if t.numel() == 1 else t).contiguous()

    def _forward_train(self, x, bit_map):
        """quantization.py:604-613 + 699-727, 733-737: EMA update, then the
        fractional-bit straight-through quantizer x m(p)."""
        _need_cuda(x, "x")
        _need_cuda(bit_map, "bit_map")
        B, C, H, W = x.shape
        if bit_map.dim() != 3 or bit_map.shape[0] != B:
            raise AssertionError(f"Batch size mismatch: {B} vs {bit_map.shape[0]}")
        want_m = self.smooth_transitions and self.soft_mask is not None
        xf = _f32c(x)
        hit = _pass1_lookup(xf)
        absmean = (hit["absmean"] if hit is not None else torch.empty(B, H, W, device=x.device)) if want_m else None
        frozen = self._frozen()
        copies = None
        if frozen:
            if want_m and hit is None:
                _run_stats(xf, absmean=absmean)
        else:
            copies = self.update_running_stats(xf, absmean, want_copies=self.training)
        # _calibrate_minmax (quantization.py:409-434): running stats in train
        # mode or when frozen, else this batch's min/max (copies: the running
        # buffers are updated in place by later steps)
        if copies is not None:
            xmin, xmax = copies
        elif self.running_min is not None and (self.training or frozen):
            xmin = self._stats_c(self.running_min, C).clone()
            xmax = self._stats_c(self.running_max, C).clone()
        else:
            xmin, xmax = self.batch_minmax(xf)
        m = self.soft_mask(bit_map, x, absmean=absmean) if want_m else None
        return _QATQuantFn.apply(x, bit_map, m, xmin, xmax)

    def _minmax_for_quant(self, x):
        """_calibrate_minmax (quantization.py:409-434): running statistics in
        train mode or when frozen, else this batch's (all-reduced over the
        process group, if any)."""
        if self.running_min is not None and (self.training or self._frozen()):
            return self.running_min.detach(), self.running_max.detach()
        return self._global_minmax(*self._batch_stats_torch(x.detach().float()))

    def _forward_torch(self, x, bit_map, training):
        """The pure-PyTorch quantizer (quantization.py:604-634, 681-746) for CPU
        tensors: one elementwise pass (fallback.quantize) at inference, the
        fractional-bit straight-through quantizer in training."""
        B, C, H, W = x.shape
        if bit_map.dim() != 3 or bit_map.shape[0] != B:
            raise AssertionError(f"Batch size mismatch: {B} vs {bit_map.shape[0]}")
        if training:
            self.update_running_stats(x)
        xmin, xmax = self._minmax_for_quant(x)
        xmin = xmin.reshape(-1).float().expand(C) if xmin.numel() == 1 else xmin.reshape(-1).float()
        xmax = xmax.reshape(-1).float().expand(C) if xmax.numel() == 1 else xmax.reshape(-1).float()
        if training:
            xq = fallback.FractionalQuant.apply(x.float(), bit_map, xmin.contiguous(), xmax.contiguous())
        else:
            with torch.no_grad():
                xq = fallback.quantize(x.detach().float(), bit_map.detach(), xmin, xmax).contiguous()
        if self.smooth_transitions and self.soft_mask is not None:
            xq = xq * self.soft_mask(bit_map, x)
        return xq

    def forward(self, x: torch.Tensor, bit_map: torch.Tensor, training: Optional[bool] = None) -> torch.Tensor:
        if training is None:
            training = self.training
        if not x.is_cuda:
            return self._forward_torch(x, bit_map, training)
        if training:
            return self._forward_train(x, bit_map)
        _need_cuda(x, "x")
        _need_cuda(bit_map, "bit_map")
        xf = _f32c(x)
        B, C, H, W = xf.shape
        if bit_map.dim() != 3 or bit_map.shape[0] != B:
            raise AssertionError(f"Batch size mismatch: {B} vs {bit_map.shape[0]}")
        bits = _f32c(bit_map)
        _, ht, wt = bits.shape
        want_m = self.smooth_transitions and self.soft_mask is not None
        absmean = torch.empty(B, H, W, device=xf.device) if want_m else None
        frozen = bool(self.stats_frozen) and self.running_min is not None
        if frozen:
            xmin = self.running_min.reshape(-1).float().expand(C).contiguous() \
                if self.running_min.numel() == 1 else self.running_min.reshape(-1).float().contiguous()
            xmax = self.running_max.reshape(-1).float().expand(C).contiguous() \
                if self.running_max.numel() == 1 else self.running_max.reshape(-1).float().contiguous()
            if want_m:
                _run_stats(xf, absmean=absmean)
        else:
            xmin, xmax = self.batch_minmax(xf, absmean)
        mt = self.soft_mask.tile_values(bits, xf, absmean=absmean) if want_m else None
        y = torch.empty_like(xf)
        q = abi.QuantScale()
        q.x, q.y, q.bits, q.mt, q.xmin, q.xmax = _p(xf), _p(y), _p(bits), _p(mt), _p(xmin), _p(xmax)
        q.B, q.C, q.H, q.W, q.ht, q.wt = B, C, H, W, ht, wt
        q.bits_lo, q.nbits = 2, 7
        q.stats_cover_x = 0 if frozen else 1
        abi.check(abi.lib().mcaq_quant(ctypes.byref(q), 1, _stream()), "mcaq_quant")
        return y

    def extra_repr(self) -> str:
        return (f"calibration_mode={self.calibration_mode}, smooth_transitions={self.smooth_transitions}, "
                f"per_channel={self.per_channel}")
