"""Load the reference's tensor-backend modules by FILE PATH (fixture generation only).

Runs only in the build container, where /root/reference exists. Nothing on the
GPU box imports this file (tests read the committed .npz fixtures instead).

`mcaq_yolo/core/morphology.py` imports `cv2` and `skimage.feature` at module
top (morphology.py:8, 13) but the tensor ("gpu") backend that is on the hot path
never touches them (they serve only the cv2 backend, morphology.py:110-307,
741-796).  OpenCV / scikit-image are absent here, so we pre-seed `sys.modules`
with modules whose every attribute use RAISES: if any stubbed symbol were ever
called while generating fixtures, generation would fail instead of silently
producing non-reference values.  `bit_allocation.py` and `quantization.py`
import only torch/numpy and load unmodified.

Loading by file path avoids `mcaq_yolo/__init__.py:16-19`, which eagerly
imports ultralytics-dependent modules.
"""
import importlib.util
import sys
import types

REF_ROOT = "/root/reference/mcaq_yolo/core"


class _Forbidden(types.ModuleType):
    def __getattr__(self, name):  # pragma: no cover - must never fire
        if name.startswith("__"):
            raise AttributeError(name)
        raise RuntimeError(f"stub module {self.__name__!r}: attribute {name!r} "
                           "was used - the tensor backend must not need it")


def _install_stubs():
    if "cv2" not in sys.modules:
        sys.modules["cv2"] = _Forbidden("cv2")
    if "skimage" not in sys.modules:
        sk = _Forbidden("skimage")
        feat = types.ModuleType("skimage.feature")

        def local_binary_pattern(*a, **k):  # pragma: no cover
            raise RuntimeError("skimage stub called (cv2 backend only)")

        feat.local_binary_pattern = local_binary_pattern
        sk.feature = feat
        sys.modules["skimage"] = sk
        sys.modules["skimage.feature"] = feat


def _load(name, fname):
    spec = importlib.util.spec_from_file_location(name, f"{REF_ROOT}/{fname}")
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    """Returns (morphology, bit_allocation, quantization) reference modules."""
    import warnings
    _install_stubs()
    morph = _load("ref_morphology", "morphology.py")
    bits = _load("ref_bit_allocation", "bit_allocation.py")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # 'mcaq_cuda_ops not found' warning
        quant = _load("ref_quantization", "quantization.py")
    assert not quant.HAS_CUDA
    return morph, bits, quant
