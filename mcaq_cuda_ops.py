"""Top-level `mcaq_cuda_ops`: the module name the reference imports
(mcaq_yolo/core/quantization.py:14-16, `import mcaq_cuda_ops`; built there by
mcaq_yolo/ops/setup.py from ops/src/mcaq_ops.cpp:22-77 + mcaq_kernel.cu).

With this repository on the Python path (PYTHONPATH, or the working
directory) `import mcaq_cuda_ops` resolves here with no install() call and no
edit to the reference: the reference's HAS_CUDA becomes True and its
`_forward_cuda` (quantization.py:636-679) calls

    mcaq_cuda_ops.spatial_quantize(x, bit_map, x_min, x_max, tile_h, tile_w, m)

which runs `mcaq_launch_spatial_quantization` of libmcaq_hip.so (the HIP
kernel for gfx950) on the current stream.  Same argument names and defaults
as the reference's pybind11 binding (mcaq_ops.cpp:73-77), same errors; see
mcaq_yolo_amd/mcaq_cuda_ops.py for the checks and the torch.library operator.
"""
from mcaq_yolo_amd.mcaq_cuda_ops import spatial_quantize  # noqa: F401

__all__ = ["spatial_quantize"]
