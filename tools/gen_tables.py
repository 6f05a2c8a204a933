"""Write mcaq_yolo_amd/csrc/mcaq_tables.h from the oracle's constant kernels.

The values are the CPU values of the reference's run-time constant tensors
(Gaussian kernels, bilateral spatial weights); tests/test_oracle_cpu.py pins
oracle.K against tests/golden/constants.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.mcaq_oracle import K  # noqa: E402

HDR = os.path.join(ROOT, "mcaq_yolo_amd", "csrc", "mcaq_tables.h")


def table(name, arr):
    a = np.asarray(arr, np.float32).reshape(-1)
    words = ", ".join("0x%08Xu" % int(v) for v in a.view(np.uint32))
    return "MCAQ_TABLE uint32_t %s_bits[%d] = {%s};\n" % (name, a.size, words)


def main():
    body = "".join(table(n, K[k]) for n, k in (
        ("k_gauss5", "gauss5_canny"), ("k_gauss11", "gauss11_adaptive"),
        ("k_smooth5", "smooth5_softmask"), ("k_bilat_sp", "bilateral_spatial")))
    src = open(HDR).read()
    a = src.index("// @@TABLES@@")
    b = src.index("}  // namespace mcaq")
    src = src[:a] + "// @@TABLES@@\n" + body + src[b:]
    open(HDR, "w").write(src)
    print("wrote", HDR)


if __name__ == "__main__":
    main()
