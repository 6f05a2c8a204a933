"""Drop-in for the reference's Torch extension `mcaq_cuda_ops`
(mcaq_yolo/ops/src/mcaq_ops.cpp:22-77, kernel mcaq_kernel.cu:12-123).

    spatial_quantize(input, bit_map, min_vals, max_vals, tile_h, tile_w, mask=None) -> Tensor

Same signature, argument meaning, output ownership (a new tensor, inputs
read-only) and errors (RuntimeError when min/max do not hold one entry per
channel or the mask is not N*H*W); additionally the dtype / device /
contiguity checks the reference lacks.  Runs
mcaq_launch_spatial_quantization (include/mcaq_hip.h) on the current stream,
asynchronously.  One deliberate difference: q is rounded half-to-even
(torch.round, the reference's PyTorch path) instead of the CUDA kernel's
roundf, so this op and SpatialAdaptiveQuantization._forward_pytorch agree
bit-for-bit.

To let the unmodified reference pick it up (`import mcaq_cuda_ops` at
core/quantization.py:14-23) call `install()` before importing it.  The
launch itself is the torch.library operator `torch.ops.mcaq.spatial_quantize`
(with a fake implementation), so graphs that call it can be traced by
torch.compile / torch.export.
"""
import ctypes
import sys
from typing import Optional

import torch

from . import abi


_HALF = (torch.float16, torch.bfloat16)


def _check(t, what, half_ok=False):
    if not torch.is_tensor(t):
        raise TypeError("%s must be a Tensor" % what)
    if not t.is_cuda:
        raise RuntimeError("%s must be a CUDA (HIP) tensor, got %s" % (what, t.device))
    if t.dtype != torch.float32 and not (half_ok and t.dtype in _HALF):
        raise RuntimeError("%s must be float32%s, got %s" % (what, " (or float16 / bfloat16)" if half_ok else "",
                                                             t.dtype))
    if not t.is_contiguous():
        raise RuntimeError("%s must be contiguous" % what)


def spatial_quantize(input, bit_map, min_vals, max_vals, tile_h, tile_w, mask=None):
    """input may also be fp16 / bf16 (an autocast region; the reference op
    raises there, data_ptr<float>): quantized in fp32 arithmetic on
    input.float() (exact); the result takes torch's type promotion of
    input x mask (fp32 with an fp32 mask, as the reference's _forward_pytorch
    returns x_quantized * m, quantization.py:742-744; else the input's dtype,
    rounded to nearest even)."""
    _check(input, "input", half_ok=True)
    if input.dtype in _HALF:
        out_dt = input.dtype if mask is None else torch.promote_types(input.dtype, mask.dtype)
        return spatial_quantize(input.float(), bit_map, min_vals, max_vals, tile_h, tile_w,
                                None if mask is None else mask.float().contiguous()).to(out_dt)
    for t, n in ((bit_map, "bit_map"), (min_vals, "min_vals"), (max_vals, "max_vals")):
        _check(t, n)
    if input.dim() != 4:
        raise RuntimeError("input must be (N, C, H, W)")
    if bit_map.dim() != 3:
        raise RuntimeError("bit_map must be (N, Ht, Wt)")
    N, C, H, W = input.shape
    if min_vals.numel() != C or max_vals.numel() != C:
        raise RuntimeError("min_vals/max_vals must have one entry per channel (C=%d), got %d - expand "
                           "per-tensor stats before calling (see SpatialAdaptiveQuantization._forward_cuda)"
                           % (C, min_vals.numel()))
    if mask is not None:
        _check(mask, "mask")
        if mask.numel() != N * H * W:
            raise RuntimeError("mask must be (N, 1, H, W)")
    if bit_map.shape[0] != N:
        raise RuntimeError("bit_map batch %d != input batch %d" % (bit_map.shape[0], N))
    return torch.ops.mcaq.spatial_quantize(input, bit_map, min_vals, max_vals, int(tile_h), int(tile_w), mask)


# The launch as a torch.library operator (mcaq::spatial_quantize), so the
# call is an opaque node that torch.compile / torch.export / FakeTensor
# tracing can carry (its fake implementation gives the output's shape, dtype
# and device); the checks above run in Python before it, on real or fake
# tensors alike.
@torch.library.custom_op("mcaq::spatial_quantize", mutates_args=())
def _spatial_quantize_op(input: torch.Tensor, bit_map: torch.Tensor, min_vals: torch.Tensor,
                         max_vals: torch.Tensor, tile_h: int, tile_w: int,
                         mask: Optional[torch.Tensor]) -> torch.Tensor:
    out = torch.empty_like(input)
    if out.numel() == 0:
        return out
    N, C, H, W = input.shape
    n_th, n_tw = int(bit_map.shape[1]), int(bit_map.shape[2])
    mptr = ctypes.c_void_p(mask.data_ptr()) if mask is not None else None
    err = abi.lib().mcaq_launch_spatial_quantization(
        ctypes.c_void_p(input.data_ptr()), ctypes.c_void_p(bit_map.data_ptr()),
        ctypes.c_void_p(min_vals.data_ptr()), ctypes.c_void_p(max_vals.data_ptr()), mptr,
        ctypes.c_void_p(out.data_ptr()), N, C, H, W, int(tile_h), int(tile_w), n_th, n_tw,
        ctypes.c_void_p(torch.cuda.current_stream(input.device).cuda_stream))
    abi.check(err, "mcaq_launch_spatial_quantization")
    return out


@_spatial_quantize_op.register_fake
def _spatial_quantize_fake(input, bit_map, min_vals, max_vals, tile_h, tile_w, mask):
    return torch.empty_like(input)


def install():
    """Register this module as the top-level `mcaq_cuda_ops` extension."""
    sys.modules["mcaq_cuda_ops"] = sys.modules[__name__]
