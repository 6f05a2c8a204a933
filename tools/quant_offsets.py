"""Pass 2 (mcaq_quant) per-dispatch time, x cold, with y placed at several
byte offsets from a 2 MiB-aligned base, beside a flat torch copy of the same
bytes (the box's copy ceiling).  Box-to-box pass-2 times varied 36-43 us in
r03 while pass 1 did not: is it the placement of y relative to x?

    python tools/quant_offsets.py [--reps 40]
"""
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
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--offsets", default="0,256,1024,4096,65536,1048576")
    args = ap.parse_args()
    import bench
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    dev = torch.device("cuda:0")
    name, B, chans, grid, mapper = bench.CONFIGS[2]
    cm, mm, sm = bench.load_blobs(dev)
    geoms = [ScaleGeom(B, c, h, w, grid) for c, (h, w) in zip(chans, bench.SIZES)]
    sizes = [B * c * h * w for c, (h, w) in zip(chans, bench.SIZES)]
    plans = []
    for p in range(4):
        feats = [bench.synth_features(B, c, h, w, 2000 + i + 104729 * p, dev)
                 for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))]
        plan = HookPlan(geoms, dev)
        plan.prepare(feats, cm, mm, [sm] * 3, temperature=1.0, mapper_kind=mapper)
        plan.feats = feats
        plan.launch(torch.cuda.current_stream())
        plans.append(plan)
    torch.cuda.synchronize()
    L = plans[0].lib
    st = torch.cuda.current_stream()
    elems = sum(sizes)
    out = {}

    def timed(fn):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record(st)
            b.record(st)
        for r in range(8):
            fn(r % 4, None)
        torch.cuda.synchronize()
        for r, (a, b) in enumerate(ev):
            fn(r % 4, (a, b))
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
        return t[len(t) // 2]

    # flat copy reference: x of plan k (3 scale tensors) into a y buffer
    ybuf = [torch.empty(elems, device=dev) for _ in range(4)]

    def copy(k, evs):
        if evs:
            evs[0].record(st)
        o = 0
        for f in plans[k].feats:
            n = f.numel()
            ybuf[k][o:o + n].view_as(f).copy_(f)
            o += n
        if evs:
            evs[1].record(st)
    out["torch copy (3 launches, events around)"] = round(timed(copy), 2)

    def quant(k, evs):
        if evs:
            L.mcaq_time_next_launch(ctypes.c_void_p(evs[0].cuda_event), ctypes.c_void_p(evs[1].cuda_event))
        plans[k].launch_quant(st)
    out["quant (plan y)"] = round(timed(quant), 2)
    for off in [int(x) for x in args.offsets.split(",")]:
        bufs = []
        for k, plan in enumerate(plans):
            raw = torch.empty(elems * 4 + off + (4 << 20), dtype=torch.uint8, device=dev)
            base = (raw.data_ptr() + (2 << 20) - 1) // (2 << 20) * (2 << 20) + off
            bufs.append(raw)
            o = base
            for i in range(len(plan.geoms)):
                plan._qs[i].y = ctypes.c_void_p(o)
                o += 4 * sizes[i]
        out["quant y at 2MiB+%d" % off] = round(timed(quant), 2)
        del bufs
    for k, v in list(out.items()):
        nb = (8 if "quant" in k or "copy" in k else 4) * elems
        out[k] = {"us": v, "GB/s": round(nb / v / 1e3, 1)}
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
