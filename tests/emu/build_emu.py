"""Build tests/emu/libmcaq_emu.so (host emulation of the morph kernel)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libmcaq_emu.so")
SRC = os.path.join(HERE, "morph_emu.cpp")
DEPS = [SRC] + [os.path.join(HERE, "..", "..", "mcaq_yolo_amd", "csrc", f)
                for f in ("mcaq_morph.h", "mcaq_band.h", "mcaq_tiles_batch.h", "mcaq_math.h", "mcaq_tables.h")] + \
       [os.path.join(HERE, "..", "..", "include", "mcaq_hip.h")]


def build(force=False):
    if not force and os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(d) for d in DEPS):
        return LIB
    # private output, then an atomic rename: parallel test workers that find
    # the library stale each build their own copy and never load a partial file
    tmp = "%s.%d.tmp" % (LIB, os.getpid())
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
           "-o", tmp, SRC, "-lm"]
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True))
