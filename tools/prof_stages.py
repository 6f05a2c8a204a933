"""Time kernel variants (stage flags) on the bench workload: where does time go?"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd import abi  # noqa: E402
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom  # noqa: E402


def timeit(fn, reps=20):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize()
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda:0")
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    name, B, chans, grid, mapper = bench.CONFIGS[cfg]
    feats = [bench.synth_features(B, c, h, w, 1000 * cfg + i, dev) for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))]
    cm, mm, sm = bench.load_blobs(dev)
    plan = HookPlan([ScaleGeom(B, c, h, w, grid) for c, (h, w) in zip(chans, bench.SIZES)], dev)
    plan.prepare(feats, cm, mm, [sm] * 3)
    L = plan.lib
    sh = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    n = plan._n
    res = {}
    res["stats(all)"] = timeit(lambda: L.mcaq_stats(plan._st, n, sh()))
    saved = [(s.absmean, s.pmin, s.pmax) for s in plan._st]
    for s in plan._st:
        s.absmean = s.pmin = s.pmax = None
    res["stats(gray only)"] = timeit(lambda: L.mcaq_stats(plan._st, n, sh()))
    for s, (a, b, c) in zip(plan._st, saved):
        s.absmean, s.pmin, s.pmax = a, b, c
    res["finalize"] = timeit(lambda: L.mcaq_finalize(plan._fz, n, sh()))
    full = [s.flags for s in plan._mo]
    for label, mask in (("morph PHI", abi.F_PHI), ("morph PHI+CMLP", abi.F_PHI | abi.F_CMLP),
                        ("morph PHI+CMLP+MAP", abi.F_PHI | abi.F_CMLP | abi.F_MAPPER | abi.F_HAS_T),
                        ("morph all", None), ("morph pass B only", ~abi.F_PHI)):
        for s, f in zip(plan._mo, full):
            s.flags = f if mask is None else (f & mask)
        res[label] = timeit(lambda: L.mcaq_morph(plan._mo, n, sh()))
    for s, f in zip(plan._mo, full):
        s.flags = f
    for i in range(n):   # per scale
        res["morph all scale%d" % i] = timeit(lambda: L.mcaq_morph(ctypes.byref(plan._mo[i]), 1, sh()))
    res["morph_finalize all"] = timeit(lambda: L.mcaq_morph_finalize(plan._mo, n, plan._fz, n, sh()))
    res["quant"] = timeit(lambda: L.mcaq_quant(plan._qs, n, sh()))
    for k, v in res.items():
        print("%-24s %9.1f us" % (k, v))


if __name__ == "__main__":
    main()
