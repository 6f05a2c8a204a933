"""Per-dispatch device time of the two HBM passes alone, x cold.

    python tools/stream_bench.py [--config 2] [--reps 40] [--lib path/to/variant.so]

Config-2 shapes, 4 input batches cycled (367 MB of x: no dispatch finds its
x in the 256 MiB Infinity Cache): pass 1 (mcaq_stats) of batch r % 4, then,
in a second loop, pass 2 (mcaq_quant) of batch r % 4 with the morphology
outputs prepared once.  Each dispatch is timed by its own hipExtLaunchKernel
start/stop events.  Prints one JSON line: medians, GB/s of the algorithmic
bytes (pass 1: 4 B, pass 2: 8 B per element) and the plain-kernel ceilings
of profiles/r03_probes (read 15.4 us, copy 31.4 us at these sizes)."""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    from mcaq_yolo_amd import abi
    if args.lib:
        abi.LIB_PATH = os.path.abspath(args.lib)
    import bench
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    dev = torch.device("cuda:0")
    name, B, chans, grid, mapper = bench.CONFIGS[args.config]
    cm, mm, sm = bench.load_blobs(dev)
    geoms = [ScaleGeom(B, c, h, w, grid) for c, (h, w) in zip(chans, bench.SIZES)]
    plans = []
    for p in range(4):
        feats = [bench.synth_features(B, c, h, w, 1000 * args.config + i + 104729 * p, dev)
                 for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))]
        plan = HookPlan(geoms, dev)
        plan.prepare(feats, cm, mm, [sm] * 3, temperature=1.0, mapper_kind=mapper)
        plan.feats = feats
        plan.launch(torch.cuda.current_stream())
        plans.append(plan)
    torch.cuda.synchronize()
    L = plans[0].lib
    st = torch.cuda.current_stream()
    elems = sum(B * c * h * w for c, (h, w) in zip(chans, bench.SIZES))
    out = {"tag": args.tag, "lib": os.path.basename(abi.LIB_PATH)}
    for name_, fn, nbytes in (("stats", lambda p: p.launch_stats(st), 4 * elems),
                              ("quant", lambda p: p.launch_quant(st), 8 * elems)):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record(st)
            b.record(st)
        for r in range(8):
            fn(plans[r % 4])
        torch.cuda.synchronize()
        for r, (a, b) in enumerate(ev):
            L.mcaq_time_next_launch(ctypes.c_void_p(a.cuda_event), ctypes.c_void_p(b.cuda_event))
            fn(plans[r % 4])
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
        med = t[len(t) // 2]
        out[name_] = {"us": round(med, 2), "min": round(t[0], 2), "GB/s": round(nbytes / med / 1e3, 1),
                      "frac": round(nbytes / med / 1e3 / 8000.0, 4)}
    # back to back (the streaming stream of the staged schedule): pass 1 (i) + pass 2 (i-3)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = args.reps
    e0.record(st)
    for r in range(n):
        plans[r % 4].launch_stats(st)
        plans[(r + 1) % 4].launch_quant(st)
    e1.record(st)
    torch.cuda.synchronize()
    step = e0.elapsed_time(e1) * 1e3 / n
    out["stats+quant back to back"] = {"us_per_step": round(step, 2), "path_frac_if_hidden":
                                       round(12 * elems / step / 1e3 / 8000.0, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
