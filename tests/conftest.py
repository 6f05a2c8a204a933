import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) GPU and the built libmcaq_hip.so")
    # the golden fixtures were generated with 8 torch threads, and the soft
    # mask's softmax exp per tile follows ATen's thread partition
    # (oracle.mcaq_oracle.REF_THREADS): the CPU path and the HIP path
    # (softmax_threads default = torch.get_num_threads()) reproduce that run
    import torch
    from oracle.mcaq_oracle import REF_THREADS
    torch.set_num_threads(REF_THREADS)


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        have_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        have_gpu = False
    if have_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def case_names():
    return sorted(f[5:-4] for f in os.listdir(GOLDEN) if f.startswith("case_") and f.endswith(".npz"))


def load_case(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, "case_%s.npz" % name))


def load_weights():
    from oracle.mcaq_oracle import load_weights as lw
    return lw(os.path.join(GOLDEN, "weights.npz"))
