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
