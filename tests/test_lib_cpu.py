"""The C-ABI library: builds for gfx950, loads without a GPU, exports every
symbol include/mcaq_hip.h declares, and its ctypes mirror matches the header."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from mcaq_yolo_amd import abi

HDR = os.path.join(ROOT, "include", "mcaq_hip.h")


def declared_functions():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^(?:int|size_t|void\*|long long)\s+(mcaq_\w+)\s*\(", src, re.M)))


def test_library_built_and_exports_header_symbols():
    if not os.path.exists(abi.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(abi.LIB_PATH)
    names = declared_functions()
    assert set(names) == set(abi.EXPORTS)
    for n in names:
        assert hasattr(lib, n), n
    assert lib.mcaq_abi_version() == abi.ABI_VERSION


def test_struct_layouts_match_header():
    """Field order / count of the ctypes mirrors equal the C structs."""
    src = open(HDR).read()
    for cname, py in (("mcaq_stats_scale", abi.StatsScale), ("mcaq_finalize_scale", abi.FinalizeScale),
                      ("mcaq_morph_scale", abi.MorphScale), ("mcaq_quant_scale", abi.QuantScale),
                      ("mcaq_qat_scale", abi.QatScale), ("mcaq_mapper_seg", abi.MapperSeg),
                      ("mcaq_head_seg", abi.HeadSeg), ("mcaq_smask_seg", abi.SmaskSeg),
                      ("mcaq_reduce_seg", abi.ReduceSeg), ("mcaq_ema_seg", abi.EmaSeg)):
        body = re.search(r"typedef struct \{([^{}]*)\} %s;" % cname, src).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            names = decl.split(None, 1)[1] if not decl.startswith("const") else decl.split(None, 2)[2]
            for n in names.split(","):
                fields.append(n.strip().lstrip("*").strip())
        assert fields == [f[0] for f in py._fields_], cname


def test_invalid_args_rejected_without_gpu():
    """Size validation happens before any launch (no GPU needed)."""
    if not os.path.exists(abi.LIB_PATH):
        pytest.skip("library not built")
    lib = abi._declare(ctypes.CDLL(abi.LIB_PATH))
    err = lib.mcaq_launch_spatial_quantization(None, None, None, None, None, None, 0, 1, 1, 1, 1, 1, 1, 1, None)
    assert err != 0
    s = abi.MorphScale()
    s.tile = 3
    assert lib.mcaq_morph(ctypes.byref(s), 1, None) != 0
    assert lib.mcaq_stats(ctypes.byref(abi.StatsScale()), 0, None) != 0


def test_reference_cpp_linkage_symbol_exported():
    """launch_spatial_quantization with the reference's C++ declaration
    (MCAQPlugin.cpp:15-23, hipStream_t for cudaStream_t) is exported under its
    Itanium-mangled name, so a caller compiled against that declaration links."""
    if not os.path.exists(abi.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(abi.LIB_PATH)
    mangled = "_Z27launch_spatial_quantizationPKfS0_S0_S0_S0_PfiiiiiiiiP12ihipStream_t"
    assert hasattr(lib, mangled)


def test_top_level_mcaq_cuda_ops_importable_fresh_process(tmp_path):
    """`import mcaq_cuda_ops` - the reference's module name
    (quantization.py:14-16) - resolves in a fresh process with only the
    repository on the Python path (no install() call), and spatial_quantize
    has the argument names / default of the reference's pybind11 binding
    (ops/src/mcaq_ops.cpp:73-77).  No GPU needed: nothing is launched."""
    import subprocess
    import sys
    code = ("import inspect, mcaq_cuda_ops; s = inspect.signature(mcaq_cuda_ops.spatial_quantize); "
            "print(list(s.parameters)); print(s.parameters['mask'].default)")
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert lines[-2] == str(["input", "bit_map", "min_vals", "max_vals", "tile_h", "tile_w", "mask"])
    assert lines[-1] == "None"


def test_in_launch_exchange_sizes_and_refusals_without_gpu():
    """The round-6 one-launch entries: their sync-buffer sizes (header words,
    then 8-byte granules) and the refusals that happen before any launch -
    no buffer, a short buffer, more workgroups / chunks than the chip holds
    at once, the one-launch optimizer without clipping."""
    if not os.path.exists(abi.LIB_PATH):
        pytest.skip("library not built")
    lib = abi._declare(ctypes.CDLL(abi.LIB_PATH))
    mx = lib.mcaq_mapper_fused_max_wg()
    assert mx == 256
    assert lib.mcaq_mapper_sync_bytes(0) == 0
    assert lib.mcaq_mapper_sync_bytes(57) == 64 * 4 + 3 * 129 * 8 * 57
    assert lib.mcaq_head_sync_bytes(57) == 64 * 4 + 57 * 2881 * 8
    assert lib.mcaq_clip_adamw_sync_bytes(9000, 40) == 64 * 4 + 9 * 40 * 8
    fake = ctypes.c_void_p(0x1000)      # never dereferenced: every call below is refused first
    q = abi.MapperParams()
    segs = (abi.MapperSeg * 1)()
    segs[0].c = segs[0].bits = segs[0].work = segs[0].gbits = segs[0].gc = segs[0].gpart = 0x1000
    segs[0].n = 64 * (mx + 1)
    nb = lib.mcaq_mapper_sync_bytes(mx + 1)
    assert lib.mcaq_mapper_train_forward_fused(ctypes.byref(q), segs, 1, 2.0, 8.0, 1.0, 0.1, 0, 0, fake, nb, None) != 0
    assert lib.mcaq_mapper_train_backward_fused(ctypes.byref(q), segs, 1, 2.0, 8.0, 1.0, None, 0, fake, nb, None) != 0
    segs[0].n = 64
    assert lib.mcaq_mapper_train_forward_fused(ctypes.byref(q), segs, 1, 2.0, 8.0, 1.0, 0.1, 0, 0, None, 0, None) != 0
    assert lib.mcaq_mapper_train_forward_fused(ctypes.byref(q), segs, 1, 2.0, 8.0, 1.0, 0.1, 0, 0, fake, 100, None) != 0
    a = (abi.AdamwSeg * 1)()
    a[0].param = a[0].grad = a[0].exp_avg = a[0].exp_avg_sq = 0x1000
    a[0].n = 1024 * 257
    big = lib.mcaq_clip_adamw_sync_bytes(a[0].n, 1)
    assert lib.mcaq_clip_adamw_fused(a, 1, fake, 1, fake, 1.0, None, fake, big, None) != 0   # 257 chunks
    a[0].n = 100
    assert lib.mcaq_clip_adamw_fused(a, 1, fake, 1, fake, 0.0, None, fake, big, None) != 0   # no clipping
    assert lib.mcaq_clip_adamw_fused(a, 1, fake, 1, fake, 1.0, None, fake, 8, None) != 0     # short buffer


def test_sync_buffers_one_per_module_and_layout():
    """train_step._sync_buffer: one zeroed buffer per module, size function and
    segment layout (a layout seen before gets its buffer back), none above
    the resident-workgroup limit."""
    if not os.path.exists(abi.LIB_PATH):
        pytest.skip("library not built")
    import torch
    from mcaq_yolo_amd import train_step
    lib = abi.lib()

    class M:
        pass
    m = M()
    b1 = train_step._sync_buffer(m, torch.device("cpu"), [1600, 1600, 400], lib.mcaq_mapper_sync_bytes)
    assert b1.dtype == torch.int64 and b1.numel() * 8 >= lib.mcaq_mapper_sync_bytes(57) and not bool(b1.any())
    b2 = train_step._sync_buffer(m, torch.device("cpu"), [800, 800, 200], lib.mcaq_mapper_sync_bytes)
    assert b2 is not b1
    assert train_step._sync_buffer(m, torch.device("cpu"), [1600, 1600, 400], lib.mcaq_mapper_sync_bytes) is b1
    h = train_step._sync_buffer(m, torch.device("cpu"), [1600, 1600, 400], lib.mcaq_head_sync_bytes)
    assert h is not b1 and h.numel() * 8 >= lib.mcaq_head_sync_bytes(57)
    assert train_step._sync_buffer(m, torch.device("cpu"), [64 * 257], lib.mcaq_mapper_sync_bytes) is None
    assert len(m._mapx) == 3
