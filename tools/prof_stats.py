"""Diagnostic: stats/quant kernel time per scale and against a plain HBM read."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom  # noqa: E402
from prof_stages import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    name, B, chans, grid, mapper = bench.CONFIGS[cfg]
    feats = [bench.synth_features(B, c, h, w, 1000 * cfg + i, dev) for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))]
    cm, mm, sm = bench.load_blobs(dev)
    plan = HookPlan([ScaleGeom(B, c, h, w, grid) for c, (h, w) in zip(chans, bench.SIZES)], dev)
    plan.prepare(feats, cm, mm, [sm] * 3)
    plan.launch()
    L = plan.lib
    sh = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for i in range(plan._n):
        nb = feats[i].numel() * 4
        t = timeit(lambda: L.mcaq_stats(ctypes.byref(plan._st[i]), 1, sh()))
        print("stats scale%d  %8.1f us  %7.1f GB/s" % (i, t, nb / t / 1e3))
        t = timeit(lambda: L.mcaq_quant(ctypes.byref(plan._qs[i]), 1, sh()))
        print("quant scale%d  %8.1f us  %7.1f GB/s" % (i, t, 2 * nb / t / 1e3))
    st = plan._st[0]
    saved = (st.gray, st.absmean, st.pmin, st.pmax)
    nb = feats[0].numel() * 4
    for label, keep in (("no minmax", (1, 1, 0)), ("gray only", (1, 0, 0)), ("minmax only", (0, 0, 1)),
                        ("nothing", (0, 0, 0))):
        st.gray = saved[0] if keep[0] else None
        st.absmean = saved[1] if keep[1] else None
        st.pmin, st.pmax = (saved[2], saved[3]) if keep[2] else (None, None)
        t = timeit(lambda: L.mcaq_stats(ctypes.byref(st), 1, sh()))
        print("stats scale0 %-12s %8.1f us  %7.1f GB/s" % (label, t, nb / t / 1e3))
    st.gray, st.absmean, st.pmin, st.pmax = saved
    tot = sum(f.numel() * 4 for f in feats)
    t = timeit(lambda: L.mcaq_stats(plan._st, plan._n, sh()))
    print("stats all     %8.1f us  %7.1f GB/s" % (t, tot / t / 1e3))
    t = timeit(lambda: L.mcaq_quant(plan._qs, plan._n, sh()))
    print("quant all     %8.1f us  %7.1f GB/s" % (t, 2 * tot / t / 1e3))
    # torch reference points for the same bytes
    t = timeit(lambda: [f.sum() for f in feats])
    print("torch sum     %8.1f us  %7.1f GB/s" % (t, tot / t / 1e3))
    outs = [torch.empty_like(f) for f in feats]
    t = timeit(lambda: [o.copy_(f) for o, f in zip(outs, feats)])
    print("torch copy    %8.1f us  %7.1f GB/s" % (t, 2 * tot / t / 1e3))
    big = torch.empty(256 * 2**20, device=dev)
    big2 = torch.empty_like(big)
    t = timeit(lambda: big2.copy_(big))
    print("copy 1GiB     %8.1f us  %7.1f GB/s" % (t, 2 * big.numel() * 4 / t / 1e3))


if __name__ == "__main__":
    main()
