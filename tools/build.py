"""Build the in-tree native library mcaq_yolo_amd/lib/libmcaq_hip.so for gfx950.

    python tools/build.py [--force]

One hipcc invocation; the library links libamdhip64 by SONAME, so inside a
Python process that imported torch first it binds to torch's HIP runtime (one
runtime per process; checked by tests/test_lib_cpu.py on the GPU box)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mcaq_yolo_amd", "csrc")
OUT = os.path.join(ROOT, "mcaq_yolo_amd", "lib", "libmcaq_hip.so")
SRCS = [os.path.join(CSRC, "mcaq_kernels.hip")]
DEPS = SRCS + [os.path.join(CSRC, f) for f in ("mcaq_math.h", "mcaq_morph.h", "mcaq_band.h", "mcaq_tiles_batch.h", "mcaq_tables.h", "mcaq_mlp_mfma.h", "mcaq_qat.h", "mcaq_nms.h", "mcaq_train.h", "mcaq_optim.h", "mcaq_dp.h")] + \
    [os.path.join(ROOT, "include", "mcaq_hip.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-result"]


def build(force=False, verbose=True, stamps=False, defines=(), out=None):
    """defines / out: A/B variant builds (tools/gpu_ab.sh), e.g.
    python tools/build.py --variant tools/probe/ab/x.so -DMCAQ_TILES_EXCL"""
    out = out or (OUT.replace(".so", "_stamps.so") if stamps else OUT)
    if not force and not defines and os.path.exists(out) and \
            all(os.path.getmtime(out) >= os.path.getmtime(d) for d in DEPS):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = [HIPCC] + FLAGS + (["-DMCAQ_STAMPS"] if stamps else []) + list(defines) + ["-o", tmp] + SRCS
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    a = sys.argv[1:]
    out = a[a.index("--variant") + 1] if "--variant" in a else None
    print(build(force="--force" in a, stamps="--stamps" in a, out=out,
                defines=[x for x in a if x.startswith("-D")]))
