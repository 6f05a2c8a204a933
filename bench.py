"""Benchmark of the MCAQ spatial-adaptive-quantization hook path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--pipeline D]
                    [--no-cpu] [--no-e2e] [--e2e [--amp]] [--eager]

The headline (`metric`, `value`) is the HOOK PATH: a step = the three
backbone hooks (C3/C4/C5) of one batch - channel statistics, morphological
complexity (phi1..5, MLP, bilateral), bit mapper, soft mask and the tile-wise
2..8-bit quant/dequant, every output the reference hook produces - computed
by the HIP kernels on inputs already resident in HBM.  The end-to-end image
rate (YOLOv8 network on MIOpen + hooks + HIP NMS, `run_e2e`) is measured in
the same run and reported beside it under "e2e" (or alone with --e2e).

Throughput: `--pipeline D` (default 3) independent batches are in flight on D
HIP streams, so one batch's latency-bound per-image morphology overlaps the
HBM passes of the others; `value` = images of all K timed steps / wall time.
`path_roofline` is the north-star figure (12 B per feature element over the
step time); `roofline` is the dominant kernel, pass 2, timed with HIP events
around each of its launches in single-batch steps run in sequence (the
context `rocprofv3 ... bench.py --pipeline 1` profiles).  `cpu_baseline` is this
package's pure-PyTorch path (fallback.py) at the same config on the host.

N > 1: one process per GPU (torch.distributed.run), each rank takes its own
batch shard (weak scaling); the per-channel batch min/max is made global with
one RCCL all-reduce per step, so every rank quantizes exactly like the
reference run on the whole global batch.  --config 5: the QAT training step.

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from mcaq_yolo_amd import params  # noqa: E402
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom  # noqa: E402

# BASELINE.json configs that fit this harness: name -> (per-GPU batch, channels, grid, mapper)
CONFIGS = {
    2: ("yolov8n", 32, (64, 128, 256), 8, "mlp"),
    3: ("yolov8s", 64, (128, 256, 512), 16, "mlp"),
    4: ("yolov8m", 32, (192, 384, 576), 8, "mlp"),   # bs256 = 32 per GPU x 8
}
SIZES = ((80, 80), (40, 40), (20, 20))  # C3/C4/C5 at 640x640 (strides 8/16/32)
HBM_PEAK_GBS = 8000.0                   # MI355X_MICROARCH.md chip table (spec)


def synth_features(B, C, H, W, seed, device):
    """silu(1.5*randn + 2*bilinear_up(randn(B,C,H/8,W/8)))."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    lo = torch.randn(B, C, max(1, H // 8), max(1, W // 8), generator=g)
    hi = torch.randn(B, C, H, W, generator=g)
    up = F.interpolate(lo, size=(H, W), mode="bilinear", align_corners=False)
    return F.silu(1.5 * hi + 2.0 * up).contiguous().to(device)


def load_blobs(device):
    import numpy as np
    w = np.load(os.path.join(ROOT, "tests", "golden", "weights.npz"))
    sd = {k: w[k] for k in w.files}
    cm = torch.from_numpy(params.pack_complexity_mlp(params.sub(sd, "complexity_analyzer."))).to(device)
    mm = torch.from_numpy(params.pack_mapper_mlp(params.sub(sd, "bit_mapper."))).to(device)
    sm = torch.from_numpy(params.pack_soft_mask(params.sub(sd, "soft_mask."))).to(device)
    return cm, mm, sm


# BASELINE config 5: yolov8n QAT step, bs128 = 16 per GPU x 8 (weak scaling)
QAT_CONFIG = ("yolov8n", 16, (64, 128, 256), 8, "mlp")


def hook_state_dict(device):
    """The seeded reference-layout weights (tests/golden/weights.npz) as an
    MCAQHooks state_dict: one analyzer, one mapper, a soft mask per scale."""
    import numpy as np
    w = np.load(os.path.join(ROOT, "tests", "golden", "weights.npz"))
    sd = {}
    for k in w.files:
        t = torch.from_numpy(np.array(w[k])).to(device)
        if k.startswith("soft_mask."):
            for idx in (4, 6, 9):
                sd["quantizers.%d.%s" % (idx, k)] = t
        else:
            sd[k] = t
    return sd


def cpu_baseline_qat(budget_s=12.0):
    """The same QAT step on the host: this package's pure-PyTorch CPU path
    (core / fallback.py modules in train mode - the reference's own
    _forward_pytorch training branch, EMA statistics, train-mode mapper,
    soft mask, fractional-bit STE quantizer), the bit-budget loss, backward,
    and optim.ClipAdamW's torch-op step, at config 5's per-GPU batch, on the
    process's torch threads; whole steps repeated for ~budget_s seconds."""
    from mcaq_yolo_amd.hooks import MCAQHooks
    from mcaq_yolo_amd.optim import ClipAdamW
    name, B, chans, grid, mapper = QAT_CONFIG
    cpu = torch.device("cpu")
    torch.manual_seed(0)
    h = MCAQHooks(grid_size=grid, bit_mapping=mapper, device=cpu)
    h.load_state_dict(hook_state_dict(cpu), strict=False)
    h.train()
    feats = [synth_features(B, c, hh, ww, 5000 + i, "cpu").requires_grad_(True)
             for i, (c, (hh, ww)) in enumerate(zip(chans, SIZES))]
    gen = torch.Generator(device="cpu").manual_seed(77)
    G = [1e-3 * torch.randn(f.shape, generator=gen) for f in feats]
    ps = [p for p in h.parameters() if p.requires_grad]
    opt = ClipAdamW(ps, lr=1e-3, weight_decay=0.05, betas=(0.9, 0.999), max_norm=1.0,
                    project_abs=h.bit_mapper.constrained_weights())
    w_bit = torch.full((), 0.1)

    def step():
        opt.zero_grad(set_to_none=True)
        for f in feats:
            f.grad = None
        outs, aux = h.forward_features(feats, temperature=1.0)
        torch.autograd.backward(list(outs) + [h.bit_budget_loss(aux, 4.0)], list(G) + [w_bit])
        opt.step()
    step()              # warm-up (lazy state)
    t0 = time.perf_counter()
    n = 0
    while True:
        step()
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n * B / dt, 3), "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": "%d whole QAT steps of %s bs%d (3 hook scales, train mode, bit-budget loss, backward, "
                      "clip + AdamW + |W|) on this package's pure-PyTorch CPU path (the reference's "
                      "_forward_pytorch training branch), %d torch threads, %.1f s"
                      % (n, name, B, torch.get_num_threads(), dt)}


def main_qat(args, world, rank, dev, pg):
    """BASELINE config 5 at the hook level: one QAT training step of the three
    MCAQ hooks (train mode) per batch - EMA statistics, analyzer (phi kernel +
    complexity MLP with autograd), continuous bits (train-mode mapper), soft
    mask, fractional-bit quantizer forward; backward from the upstream feature
    gradients the YOLOv8 neck would return (synthetic, fixed), straight-through
    into the backbone features and into the hook parameters; gradient
    all-reduce (N > 1), clip 1.0, AdamW step, |W| projection (train.py:615-641)."""
    from mcaq_yolo_amd import abi, core
    from mcaq_yolo_amd.hooks import MCAQHooks
    name, B, chans, grid, mapper = QAT_CONFIG
    torch.manual_seed(0)
    h = MCAQHooks(grid_size=grid, bit_mapping=mapper, device=dev)
    h.load_state_dict(hook_state_dict(dev), strict=False)
    h.train()
    if pg is not None:
        # global-batch EMA statistics and mapper BatchNorm
        from mcaq_yolo_amd.dist import shard_hooks
        shard_hooks(h, pg, rank, world, B)
    feats = [synth_features(B, c, hh, ww, 5000 + i + 7919 * rank, dev).requires_grad_(True)
             for i, (c, (hh, ww)) in enumerate(zip(chans, SIZES))]
    gen = torch.Generator(device="cpu").manual_seed(77 + rank)
    G = [(1e-3 * torch.randn(f.shape, generator=gen)).to(dev) for f in feats]
    params_ = [p for p in h.parameters() if p.requires_grad]
    # the reference's optimizer end of the step (train.py:140-150, 626-641:
    # clip_grad_norm_ 1.0, AdamW lr 1e-3 weight decay 0.05 betas 0.9 / 0.999,
    # the mapper's |W| projection): by default optim.ClipAdamW, all three in
    # one launch; --torch-optim: torch's clip + fused capturable AdamW + the
    # projection as separate kernels (~14 per step)
    fused_opt = not args.torch_optim
    if fused_opt:
        from mcaq_yolo_amd.optim import ClipAdamW
        opt = ClipAdamW(params_, lr=1e-3, weight_decay=0.05, betas=(0.9, 0.999), max_norm=1.0,
                        project_abs=h.bit_mapper.constrained_weights())
        from mcaq_yolo_amd import optim as _optim
        opt_kind = "optim.ClipAdamW (clip_grad_norm 1.0 + AdamW + |W| projection, %s)" % (
            "one launch" if _optim.ONE_LAUNCH else "two launches")
    else:
        try:
            opt = torch.optim.AdamW(params_, lr=1e-3, weight_decay=0.05, betas=(0.9, 0.999), fused=True,
                                    capturable=True)
            opt_kind = "AdamW (fused, capturable) + clip_grad_norm_ 1.0 + enforce_weight_constraints"
        except (RuntimeError, TypeError, ValueError):
            opt = torch.optim.AdamW(params_, lr=1e-3, weight_decay=0.05, betas=(0.9, 0.999), foreach=True,
                                    capturable=True)
            opt_kind = "AdamW (foreach, capturable) + clip_grad_norm_ 1.0 + enforce_weight_constraints"
    target_bits = 4.0
    h.target_bits = target_bits
    w_bit = torch.full((), 0.1, device=dev)          # the bit-budget loss weight (loss_weights['bit_budget'])

    # how the train-mode mapper ran (fused kernels, or the torch autograd path)
    from mcaq_yolo_amd import train_step
    fused = {"calls": 0}
    orig_apply, orig_multi = core._MapperTrainFn.apply, train_step._MapperMulti.apply

    def counted(*a, **k):
        fused["calls"] += 1
        return orig_apply(*a, **k)

    def counted_multi(*a, **k):          # one call for every hook scale
        fused["calls"] += a[3]
        return orig_multi(*a, **k)
    core._MapperTrainFn.apply = counted
    train_step._MapperMulti.apply = counted_multi

    def step():
        opt.zero_grad(set_to_none=True)
        for f in feats:
            f.grad = None
        outs, aux = h.forward_features(feats, temperature=1.0)   # curriculum stage 3: temperature 1
        # MCAQLoss.compute_bit_budget_loss (models/mcaq_yolo.py:110-118) with weight 0.1
        lbit = h.bit_budget_loss(aux, target_bits)
        torch.autograd.backward(list(outs) + [lbit], list(G) + [w_bit])
        if pg is not None:
            from mcaq_yolo_amd.dist import allreduce_gradients
            allreduce_gradients(params_, pg, static_pattern=True)   # the sink arena, in place over RCCL
        if fused_opt:
            opt.step()
        else:
            torch.nn.utils.clip_grad_norm_(params_, max_norm=1.0)
            opt.step()
            h.bit_mapper.enforce_weight_constraints()

    # warm up on a side stream (lazy state: running stats, momentum buffers),
    # then (N = 1) capture the whole step - forward, backward, clip, AdamW,
    # projection - as one HIP graph: ~300 small launches replayed at once
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(max(args.warmup, 3)):
            step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    # N > 1 on the nccl (RCCL) backend: the step's collectives (EMA min/max,
    # the mapper's BatchNorm statistics, the gradient bucket) are captured in
    # the graph too; gloo (the CPU-collective rehearsal) runs eagerly
    use_graph = (pg is None or _backend(pg) == "nccl") and not args.eager
    run = step
    if use_graph:
        graph = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        # thread_local: the process group's watchdog thread polls its work
        # events while this thread captures (global mode would fail its calls)
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            step()
        run = graph.replay
        for _ in range(2):
            run()
    torch.cuda.synchronize()

    # HBM-side bytes per launch of the QAT kernels (rocprofv3 PMC passes,
    # tools/gpu/pmc_r04.sh -> profiles/pmc_traffic_config5.json)
    qat_traffic = {}
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic_config5.json")
    if os.path.exists(tpath):
        qat_traffic = {k: v["total"] for k, v in json.load(open(tpath)).get("kernels", {}).items()}
    # per-kernel device time of the QAT quantizer over the three scales in one launch
    L = abi.lib()
    stream = torch.cuda.current_stream()
    sh = abi.ctypes.c_void_p(stream.cuda_stream)
    xs = [f.detach() for f in feats]
    bits = [torch.rand(B, hh // grid, ww // grid, device=dev) * 6 + 2 for (hh, ww) in SIZES]
    ms = [torch.rand(B, hh, ww, device=dev) * 0.1 + 0.9 for (hh, ww) in SIZES]
    mm = [core._channel_minmax(x) for x in xs]
    ys = [torch.empty_like(x) for x in xs]
    gxs = [torch.empty_like(x) for x in xs]
    gms = [torch.empty(B, hh, ww, device=dev) for (hh, ww) in SIZES]
    gbs = [torch.empty_like(b) for b in bits]
    works = [torch.empty(L.mcaq_qat_work_floats(*x.shape), device=dev) for x in xs]
    arrive = torch.zeros(3, B * max(hh // grid for (hh, _) in SIZES), dtype=torch.int32, device=dev)
    arr, arr_u = (abi.QatScale * 3)(), (abi.QatScale * 3)()
    for i in range(3):
        q = core._qat_struct(xs[i], bits[i], ms[i], mm[i][0], mm[i][1])
        q.g, q.y, q.gx, q.gm, q.gb, q.work = core._p(G[i]), core._p(ys[i]), core._p(gxs[i]), core._p(gms[i]), \
            core._p(gbs[i]), core._p(works[i])
        arr_u[i] = q
        q.arrive = core._p(arrive[i])
        arr[i] = q
    # each dispatch timed by its own start/stop events (hipExtLaunchKernel,
    # mcaq_time_launch: skip 0 = the quantizer kernel, skip 1 = the fold the
    # backward launcher issues after it), 20 launches in sequence.  The
    # product backward folds inside its launch (arrival counters); the
    # two-kernel form (no counters) is timed beside it for comparison.
    kt = {}
    reps = 20
    for k, fn, skip in (("qat_forward", lambda: L.mcaq_qat_forward(arr_u, 3, sh), 0),
                        ("qat_backward_kernel", lambda: L.mcaq_qat_backward(arr_u, 3, sh), 0),
                        ("qat_fold", lambda: L.mcaq_qat_backward(arr_u, 3, sh), 1),
                        ("qat_backward_fold_in_launch", lambda: L.mcaq_qat_backward(arr, 3, sh), 0)):
        abi.check(fn(), k)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a_, b_ in ev:
            a_.record(stream)
            b_.record(stream)
        torch.cuda.synchronize()
        for a_, b_ in ev:
            L.mcaq_time_launch(skip, abi.ctypes.c_void_p(a_.cuda_event), abi.ctypes.c_void_p(b_.cuda_event))
            fn()
        torch.cuda.synchronize()
        kt[k] = sum(a_.elapsed_time(b_) for a_, b_ in ev) * 1e3 / reps
    kt["qat_backward"] = kt["qat_backward_kernel"] + kt["qat_fold"]    # the product's two-kernel form

    if pg is not None:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    step_s = (time.perf_counter() - t0) / args.steps
    core._MapperTrainFn.apply = orig_apply
    train_step._MapperMulti.apply = orig_multi
    # one step alone (device idle before it): its latency, and how long the
    # host takes to issue it
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    run()
    t_one_enq = time.perf_counter() - t1
    torch.cuda.synchronize()
    t_one = time.perf_counter() - t1
    fused_per_step = fused["calls"] / max(1, args.steps + max(args.warmup, 3)) if not use_graph else None
    if pg is not None:
        import torch.distributed as dist
        t = torch.tensor([step_s], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier()
        step_s = float(t.item())
    elems = sum(B * c * hh * ww for c, (hh, ww) in zip(chans, SIZES))
    if rank == 0:
        kern = {}
        # fold: reads the 2 x ceil(C/32) partial planes (the work buffer), writes grad_m + grad_bits
        pix = sum(B * hh * ww for (hh, ww) in SIZES)
        fold_b = sum(4 * 2 * ((c + 31) // 32) * B * hh * ww for c, (hh, ww) in zip(chans, SIZES)) + 4 * pix
        for k, nb in (("qat_forward", 8 * elems + 4 * pix), ("qat_backward_kernel", 12 * elems + 4 * pix),
                      ("qat_fold", fold_b), ("qat_backward", 12 * elems + 4 * pix),
                      ("qat_backward_fold_in_launch", 12 * elems + 4 * pix)):
            gbs_ = nb / (kt[k] * 1e-6) / 1e9
            kern[k] = {"us": round(kt[k], 2), "alg_bytes": nb, "GB/s": round(gbs_, 1),
                       "frac": round(gbs_ / HBM_PEAK_GBS, 4)}
        achieved = 24 * elems / step_s / 1e9
        out = {
            "metric": "images/sec QAT hook step (BASELINE config 5), 1/2/4/8 MI355X; % HBM roofline",
            "value": round(world * B / step_s, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic silu features + fixed synthetic upstream gradients, seeded weights",
            "config": {"workload": "%s QAT bs%d/GPU 640x640 MCAQ hooks C3/C4/C5 train step (grid %d, %s mapper, "
                                   "continuous bits, STE, stage-3 temperature 1); YOLOv8 network excluded"
                                   % (name, B, grid, mapper),
                       "global_batch": world * B, "parallelism": "dp%d" % world, "hip_graph": use_graph,
                       "rccl_in_graph": use_graph and pg is not None,
                       "scales": _qat_scales_mode(h, feats),
                       "optimizer": opt_kind + " (train.py:626-641)",
                       "host_enqueue_us_per_step": round(t_enq / args.steps * 1e6, 1),
                       "single_step_latency_us": round(t_one * 1e6, 1),
                       "single_step_enqueue_us": round(t_one_enq * 1e6, 1)},
            "roofline": {"bound": "hbm", "achieved": kern["qat_backward_kernel"]["GB/s"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": kern["qat_backward_kernel"]["frac"],
                         "traffic": qat_traffic.get("mcaq_qat_kernel<bwd>"),
                         "kernel": "mcaq_qat_kernel<bwd> (read g, x + write grad_x: 12 B per element, + 4 B per "
                                   "pixel of mask); its fold kernel is kernels.qat_fold",
                         "alg_bytes_per_launch": kern["qat_backward_kernel"]["alg_bytes"],
                         "us_per_launch": kern["qat_backward_kernel"]["us"]},
            "step_roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                              "kernel": "whole QAT step, 24 B per feature element (fwd 12 + bwd 12)",
                              "alg_bytes_per_step": 24 * elems},
            "kernels": kern,
            "cpu_baseline": None,
            "mapper": {"fused_kernels": fused["calls"] > 0,
                       "batchnorm": type(h.bit_mapper.mapping_network[1]).__name__,
                       "fused_calls_per_eager_step": fused_per_step},
        }
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline_qat()
        print(json.dumps(out), flush=True)
    if pg is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


# independent batches per launch set (engine.HookPlan batches): measured
# DESIGN.md s.3 "Round 5"
LAUNCH_BATCHES = 2
# per config, measured (profiles/r06_configs/): config 3's batch
# is 1.1 GB of x, two of them per launch lose to one (283.7 vs 271.9 k img/s);
# configs 2 and 4 gain from two (540 k; 199.3 vs 188.9 k)
LAUNCH_BATCHES_BY_CONFIG = {2: 2, 3: 1, 4: 2}

HOOK_METRIC = ("images/sec @640x640 MCAQ hook path (C3/C4/C5 complexity + bit mapper + 2-8 bit quant), "
               "1/2/4/8 MI355X; % HBM roofline")
E2E_METRIC = "images/sec @640x640 end-to-end MCAQ infer (YOLOv8 + hooks + NMS), 1/2/4/8 MI355X"
E2E_CONF, E2E_IOU, E2E_MAX_DET = 0.25, 0.45, 1000    # Predictor defaults (inference.py:45-48)
E2E_TARGET_CANDIDATES = 64       # anchors per image above conf after the class-bias shift (NMS does work)


def _shift_class_bias(m, imgs, target=E2E_TARGET_CANDIDATES):
    """Seeded random weights put every class score far below conf 0.25
    (Detect.bias_init), so NMS would see no candidates.  Shift all class
    biases by one constant so that about `target` anchors per image clear
    the threshold: a detector-like workload, fixed by the seed."""
    det = m.model.model[-1]
    with torch.no_grad():
        (y, _), _ = m(imgs, temperature=1.0, return_aux=True)
        s = y[:, 4:].amax(dim=1).clamp(1e-7, 1 - 1e-7)             # (B, N) best class score
        logit = torch.log(s) - torch.log1p(-s)
        kth = logit.topk(min(target, logit.shape[1]), dim=1).values[:, -1]
        thr = math.log(E2E_CONF / (1 - E2E_CONF))
        delta = float(thr - kth.median()) + 1e-3
        for seq in det.cv3:
            seq[-1].bias.add_(delta)
    return delta


def run_e2e(cfg, steps, warmup, world, rank, dev, pg, amp=False, eager=False, fuse=True, channels_last=False,
            inflight=2):
    """End-to-end MCAQ inference: YOLOv8 (MIOpen
    convolutions, seeded weights) with the MCAQ hooks at C3/C4/C5 on the HIP
    kernels, Detect decode, batched HIP NMS; N > 1: each rank its batch shard,
    hook min/max all-reduced, detections all-gathered over RCCL.  N = 1: the
    whole step is one HIP graph, and `inflight` batches (own input, own hook
    buffers - MCAQHooks.plan_slot - own graph) are in flight on as many HIP
    streams, so one batch's latency-bound hook chain runs beside another
    batch's convolutions (inference.py:383-455 predicts batch after batch).
    Returns the measurement dict (rank 0)."""
    from mcaq_yolo_amd.postprocess import gather_detections, nms_padded
    from mcaq_yolo_amd.yolo import MCAQYOLO
    name, B, chans, grid, mapper = CONFIGS[cfg]
    torch.manual_seed(0)
    m = MCAQYOLO(name, grid_size=grid, bit_mapping=mapper, device=dev)
    m.load_state_dict(hook_state_dict(dev), strict=False)
    m.eval()
    if fuse:
        m.fuse()        # Conv + BN folded, as the reference's ultralytics predictor does
    if pg is not None:
        m.process_group, m.batch_offset, m.batch_total = pg, rank * B, world * B
    g = torch.Generator(device="cpu").manual_seed(1000 * cfg + rank)
    imgs = torch.rand(B, 3, 640, 640, generator=g).to(dev)
    if channels_last:
        m.model.to(memory_format=torch.channels_last)
        imgs = imgs.contiguous(memory_format=torch.channels_last)
    delta = _shift_class_bias(m, imgs)

    def step(hooks=True):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            if hooks:
                (y, _), aux = m(imgs, temperature=1.0, return_aux=True)
            else:
                y, _ = m.model(imgs)
        out, cnt = nms_padded(y.float(), E2E_CONF, E2E_IOU, E2E_MAX_DET)
        if pg is not None:
            out, cnt = gather_detections(out, cnt, pg)
        return out, cnt

    def timed(fn, n, sync=lambda: None):
        if pg is not None:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        sync()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        if pg is not None:
            import torch.distributed as dist
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    # N > 1 on RCCL: the hook all-reduce and the detections' all-gather are
    # captured in the step's graph; one batch in flight (one stream), so the
    # replays issue the communicator's collectives in order on every rank
    use_graph = not eager and (pg is None or _backend(pg) == "nccl")
    nin = max(1, inflight) if (pg is None and use_graph) else 1
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    inputs = [imgs] + [torch.rand(imgs.shape, generator=g).to(dev).contiguous(memory_format=fmt) for _ in range(nin - 1)]

    def step_on(k, hooks=True):
        nonlocal imgs
        imgs = inputs[k]
        m.plan_slot = k
        return step(hooks)

    runs = {}
    with torch.no_grad():
        for hooks in (True, False):
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(max(warmup, 2)):
                    for k in range(nin):
                        step_on(k, hooks)
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            if use_graph:
                streams = [torch.cuda.Stream() for _ in range(nin)]
                graphs = []
                for k in range(nin):
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph, stream=streams[k], capture_error_mode="thread_local"):
                        r = step_on(k, hooks)
                    graphs.append(graph)
                    if k == 0:
                        res = r
                ctr = [0]

                def fn(graphs=graphs, streams=streams):
                    k = ctr[0] % len(graphs)
                    ctr[0] += 1
                    with torch.cuda.stream(streams[k]):
                        graphs[k].replay()
                for k in range(nin):
                    streams[k].wait_stream(torch.cuda.current_stream())
                for _ in range(nin):
                    fn()

                def sync(streams=streams):
                    for st_ in streams:
                        torch.cuda.current_stream().wait_stream(st_)
            else:
                res = step_on(0, hooks)
                fn = lambda h=hooks: step_on(0, h)
                sync = lambda: None
            torch.cuda.synchronize()
            runs[hooks] = (timed(fn, steps, sync), res)
    m.plan_slot = 0
    step_s, (out, cnt) = runs[True]
    net_s = runs[False][0]
    return {
        "metric": E2E_METRIC, "value": round(world * B / step_s, 2), "unit": "images/s", "n_gpus": world,
        "steps": steps, "warmup": warmup, "ms_per_step": round(step_s * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16-net/bf16-maps-f32-math-hooks" if amp else "f32",
        "data": "synthetic torch.rand images 640x640, seeded YOLOv8 + MCAQ weights, class biases shifted "
                "by %.3f so ~%d anchors/image clear conf %.2f" % (delta, E2E_TARGET_CANDIDATES, E2E_CONF),
        "config": {"workload": "%s bs%d/GPU 640x640 end-to-end: YOLOv8 (MIOpen) + MCAQ hooks C3/C4/C5 (HIP) + "
                               "Detect decode + HIP NMS (conf %.2f, IoU %.2f, max_det %d)%s"
                               % (name, B, E2E_CONF, E2E_IOU, E2E_MAX_DET,
                                  " + RCCL detection all-gather" if pg is not None else ""),
                   "global_batch": world * B, "grid_size": grid, "mapper": mapper,
                   "parallelism": "dp%d" % world, "hip_graph": use_graph,
                   "rccl_in_graph": use_graph and pg is not None,
                   "conv_bn_fused": fuse, "channels_last": channels_last, "batches_in_flight": nin,
                   "network_only_ms_per_step": round(net_s * 1e3, 4),
                   # both legs run NMS: the difference is the hooks' cost per step
                   "mcaq_hooks_ms_per_step": round((step_s - net_s) * 1e3, 4),
                   "hook_share_of_step": round((step_s - net_s) / step_s, 4),
                   "detections_per_image": round(float(cnt.float().mean()), 2)},
    }


def main_score(args, world, rank, dev, pg):
    """Curriculum scoring of a dataset (SURVEY 8(f) rank 4,
    utils/dataset.py:276-401 tensor path): 640x640 RGB images (0..255
    values, as a dataset yields them) scored `--score-batch` at a time by
    mcaq_yolo_amd.dataset.score_batch - per-image /255, phi kernel with every
    image as its own batch of one, Eq.(8) dot and tile mean - with the images
    already resident in HBM.  cpu_baseline: the same per-image scores through
    the pure-PyTorch path (the reference's algorithm, one image per call as
    the reference loops) on the host's threads."""
    from mcaq_yolo_amd import core
    from mcaq_yolo_amd.dataset import score_batch
    import numpy as np
    bs = max(1, args.score_batch)
    torch.manual_seed(0)
    w = np.load(os.path.join(ROOT, "tests", "golden", "weights.npz"))
    sd = {k[len("complexity_analyzer."):]: torch.from_numpy(np.array(w[k])) for k in w.files
          if k.startswith("complexity_analyzer.")}
    a = core.MorphologicalComplexityAnalyzer(device=dev, grid_size=8)
    a.load_state_dict(sd)
    a = a.to(dev).eval()
    g = torch.Generator(device="cpu").manual_seed(31 + rank)
    nb = 3
    xs = [(torch.rand(bs, 3, 640, 640, generator=g) * 255).round().to(dev) for _ in range(nb)]
    out = torch.empty(args.steps + args.warmup, bs, device=dev)
    for i in range(max(args.warmup, 1)):
        out[i % out.shape[0]] = score_batch(a, xs[i % nb])
    torch.cuda.synchronize()
    if pg is not None:
        import torch.distributed as dist
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        out[i] = score_batch(a, xs[i % nb])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    if pg is not None:
        import torch.distributed as dist
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    res = {"metric": "images/sec curriculum scoring @640x640 (compute_dataset_complexity tensor path), MI355X",
           "value": round(world * bs / dt, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f32", "data": "synthetic 0..255 RGB 640x640 images, seeded analyzer",
           "config": {"workload": "score_batch of %d images 640x640x3 (grid 8: tile 64, 10x10 tiles; planes in "
                                  "global scratch), scores kept on the device" % bs,
                      "global_batch": world * bs, "parallelism": "dp%d" % world},
           "cpu_baseline": None}
    if rank == 0 and not args.no_cpu and world == 1:
        threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
        torch.set_num_threads(threads)
        ac = core.MorphologicalComplexityAnalyzer(device="cpu", grid_size=8)
        ac.load_state_dict(sd)
        ac.eval()
        xc = xs[0][:4].cpu()
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 10.0:
            score_batch(ac, xc[n % 4:n % 4 + 1])
            n += 1
        dtc = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(n / dtc, 3), "unit": "images/s", "cores": torch.get_num_threads(),
                               "kind": "port", "sample": "%d images 640x640, one per call (as the reference's loop), "
                               "pure-PyTorch path (fallback.py), %.1f s" % (n, dtc)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if pg is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


def main_e2e(args, world, rank, dev, pg):
    if args.find:
        torch.backends.cudnn.benchmark = True
    out = run_e2e(args.config, args.steps, args.warmup, world, rank, dev, pg, args.amp, args.eager,
                  not args.no_fuse, args.channels_last, args.e2e_inflight)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


def cpu_baseline(cfg_id, budget_s=10.0):
    """This package's pure-PyTorch path (fallback.py through MCAQHooks on CPU
    tensors - the reference's own algorithm and op order, bit-exact against
    its fixtures) at the config's full batch and shapes, on the host's
    threads: whole batches of the three hooks until ~budget_s -> images/s."""
    from mcaq_yolo_amd.hooks import MCAQHooks
    name, B, chans, grid, mapper = CONFIGS[cfg_id]
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    torch.set_num_threads(threads)
    h = MCAQHooks(grid_size=grid, bit_mapping=mapper, device="cpu")
    h.load_state_dict(hook_state_dict("cpu"), strict=False)
    h.eval()
    xs = [synth_features(B, c, hh, ww, 1000 * cfg_id + i, "cpu") for i, (c, (hh, ww)) in
          enumerate(zip(chans, SIZES))]
    with torch.no_grad():
        h.forward_features(xs)                # first-call allocations out of the timing
        t0 = time.perf_counter()
        n = 0
        while True:
            h.forward_features(xs)
            n += 1
            if time.perf_counter() - t0 > budget_s:
                break
    dt = time.perf_counter() - t0
    return {"value": round(n * B / dt, 3), "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": "%d batches x %d images x 3 hook scales (%s %s, grid %d, %s mapper) through the package's "
                      "pure-PyTorch path (mcaq_yolo_amd/fallback.py), fp32, %d threads, %.1f s"
                      % (n, B, name, "x".join(map(str, chans)), grid, mapper, torch.get_num_threads(), dt)}


def _qat_scales_mode(h, feats):
    """How MCAQHooks.forward_features runs this train step (the order it tries)."""
    from mcaq_yolo_amd import train_step
    hk = _hooks_mod()
    if hk.MULTI_SCALE_TRAIN and train_step.multi_ok(h, feats):
        return "multi-segment launches (one per stage for all scales, one stream)"
    if hk.CONCURRENT_TRAIN_SCALES and h._concurrent_ok(feats):
        return "per-scale modules on concurrent streams"
    return "per-scale modules, one stream"


def _hooks_mod():
    from mcaq_yolo_amd import hooks
    return hooks


def _engine_mod():
    from mcaq_yolo_amd import engine
    return engine


class _RunMixin:
    def run(self, steps):
        for _ in range(steps):
            self.step()

    def prepare(self, steps):
        pass


class Runner(_RunMixin):
    """Issues hook-path launch sets.  Independent HookPlans (own inputs and
    buffers; each a launch set of `batches` batches) cycled over `depth` HIP
    streams: launch i runs plan i % len(plans) on stream i % depth, so the
    per-image morphology of one launch set (latency-bound) overlaps the HBM
    passes of the others.  A launch is one HIP-graph replay - with N > 1 on
    the nccl (RCCL) backend the min/max all-reduce is captured inside it; on
    gloo (CPU collectives, the functional rehearsal) it is two replays around
    the eager all-reduce."""

    def __init__(self, plans, pg, use_graph, depth):
        self.plans, self.pg = plans, pg
        self.streams = [torch.cuda.Stream() for _ in range(depth)]
        self.graphs = [None] * len(plans)
        self.i = 0
        self.batches = plans[0].batches
        # RCCL inside the graphs only where the replays cannot run two
        # collectives of the communicator at once: one rank (no peers), or one
        # stream.  With peers and several streams in flight, graphs replayed
        # on different streams would put their all-reduce kernels on the GPU
        # concurrently, in an order that can differ between ranks; there the
        # all-reduce is issued eagerly between two replays - on the process
        # group's own stream, in the host's (rank-identical) order.
        capturable = pg is None or (_backend(pg) == "nccl" and (_world(pg) == 1 or depth == 1))
        if pg is not None and os.environ.get("MCAQ_BENCH_EAGER_COLLECTIVE") == "1":
            # rehearsal of the N > 1 schedule on one rank: split graphs around
            # the eager all-reduce even where capture would be allowed
            capturable = False
        self.captured_collective = use_graph and pg is not None and capturable
        if use_graph:
            torch.cuda.synchronize()
            for p, plan in enumerate(plans):
                st = self.streams[p % depth]
                with torch.cuda.stream(st):
                    for _ in range(2):          # warm the launchers outside capture
                        plan.launch(st, self.pg)
                st.synchronize()
                segs = [lambda pl=plan: pl.launch(torch.cuda.current_stream(), self.pg)] if capturable else \
                    [lambda pl=plan: pl.launch_pre(torch.cuda.current_stream()),
                     lambda pl=plan: pl.launch_quant(torch.cuda.current_stream())]
                gs = []
                for seg in segs:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st, capture_error_mode="thread_local"):
                        seg()
                    gs.append(g)
                self.graphs[p] = gs
            torch.cuda.synchronize()

    def run(self, steps):
        """`steps` batches = steps / batches launch sets (steps a multiple)."""
        for _ in range(steps // self.batches):
            self.step()

    def step(self):
        p = self.i % len(self.plans)
        plan, st, gs = self.plans[p], self.streams[self.i % len(self.streams)], self.graphs[p]
        self.i += 1
        with torch.cuda.stream(st):
            if gs is None:
                plan.launch(st, self.pg)
            elif len(gs) == 1:
                gs[0].replay()
            else:
                gs[0].replay()
                plan.allreduce_stats(self.pg, st)
                gs[1].replay()

    def sync(self):
        for st in self.streams:
            torch.cuda.current_stream().wait_stream(st)


def _backend(pg):
    import torch.distributed as dist
    return str(dist.get_backend(pg)).lower()


def _world(pg):
    import torch.distributed as dist
    return dist.get_world_size(pg)


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N rank processes of this
    same command (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set
    as torch.distributed.run sets them) and wait for them.  This process
    never touches the GPU; rank 0's one JSON line is passed through."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = procs[0].communicate()[0]
    rcs = [procs[0].returncode]
    for p_ in procs[1:]:
        try:
            rcs.append(p_.wait(timeout=600))
        except subprocess.TimeoutExpired:
            p_.kill()
            rcs.append(-9)
    if any(rcs):
        for p_ in procs:
            if p_.poll() is None:
                p_.kill()
        raise SystemExit("bench.py --gpus %d: rank exit codes %s" % (n, rcs))
    sys.stdout.write(out.decode())
    sys.stdout.flush()


def kernel_timing(plans, reps=40, evict=None):
    """Per-launch device time of each kernel of a step, in sequence: `reps`
    single-batch steps on one stream, cycling the plans (>= 4 input batches:
    367 MB of x at config 2, more than the 256 MiB Infinity Cache).  Pass 1
    and pass 2 are launched through hipExtLaunchKernel with start/stop events
    (mcaq_time_next_launch: the dispatch's own start and end, as a kernel
    trace reports them); the morphology launch (two kernels + finalize) by
    events around it.  evict: a tensor > 256 MiB read by a torch reduction
    right before each timed pass-1 and pass-2 dispatch, so neither finds x in
    the Infinity Cache (pass 2 otherwise re-reads the x that pass 1 of the
    same batch has just read); read-only, so the timed dispatch does not pay
    for the write-back of the sweep's own lines."""
    st = torch.cuda.current_stream()
    L = plans[0].lib
    names = ("stats", "morph_finalize", "quant")
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(reps)]
    for e in ev:            # create the HIP events (lazily created on first record)
        for x in e:
            x.record(st)
    torch.cuda.synchronize()
    for r, e in enumerate(ev):
        plan = plans[r % len(plans)]
        if evict is not None:
            torch.sum(evict)
        L.mcaq_time_next_launch(ctypes.c_void_p(e[0].cuda_event), ctypes.c_void_p(e[1].cuda_event))
        plan.launch_stats(st)
        e[2].record(st)
        plan.launch_morph(st)
        e[3].record(st)
        if evict is not None:
            torch.sum(evict)
        L.mcaq_time_next_launch(ctypes.c_void_p(e[4].cuda_event), ctypes.c_void_p(e[5].cuda_event))
        plan.launch_quant(st)
    torch.cuda.synchronize()
    pairs = ((0, 1), (2, 3), (4, 5))
    # median over the launches (a kernel trace's per-dispatch durations have a
    # long upper tail: profiles/r02_v6 p1 trace, quant mean 36.5 / median 36.1 us)
    return {k: sorted(e[a].elapsed_time(e[b]) for e in ev)[reps // 2] * 1e3 for k, (a, b) in zip(names, pairs)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400, help="timed steps (400 x ~65 us: the pipeline fill / drain is < 0.5 %% of the window)")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS) + [5],
                    help="2/3/4: inference hook path; 5: QAT hook training step")
    ap.add_argument("--pipeline", type=int, default=3, help="launch sets in flight (HIP streams)")
    ap.add_argument("--launch-batches", type=int, default=None,
                    help="independent batches per launch set (each kernel launch carries that many batches, "
                         "each with its own statistics and outputs; ms_per_step still counts one batch)")
    ap.add_argument("--inputs", type=int, default=0,
                    help="distinct input batches cycled through (default max(3, pipeline): >= 276 MB of x at "
                         "config 2, more than the 256 MiB Infinity Cache, so no step finds its input cached)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (YOLOv8 + hooks + NMS) leg")
    ap.add_argument("--e2e", action="store_true", help="only the end-to-end line (run_e2e)")
    ap.add_argument("--torch-optim", action="store_true",
                    help="--config 5: torch clip_grad_norm_ + fused AdamW + projection instead of optim.ClipAdamW")
    ap.add_argument("--score", action="store_true",
                    help="only the curriculum-scoring line (compute_dataset_complexity tensor path, 640x640 images)")
    ap.add_argument("--score-batch", type=int, default=32, help="--score: images per launch")
    ap.add_argument("--e2e-inflight", type=int, default=2,
                    help="end-to-end leg: batches in flight on as many HIP streams (one graph each)")
    ap.add_argument("--amp", action="store_true",
                    help="--e2e: network under bf16 autocast (the hooks read the bf16 maps natively, fp32 arithmetic)")
    ap.add_argument("--no-fuse", action="store_true", help="--e2e: keep Conv and BatchNorm separate")
    ap.add_argument("--channels-last", action="store_true", help="--e2e: NHWC network (experiment)")
    ap.add_argument("--find", action="store_true", help="--e2e: MIOpen Find (torch.backends.cudnn.benchmark)")
    ap.add_argument("--eager", action="store_true", help="no HIP graphs")
    ap.add_argument("--schedule", choices=("streams",), default="streams",
                    help="streams: --pipeline batches in flight on as many HIP streams, one graph each (the staged, "
                         "split and prefetch schedules of rounds 2-4 measured slower and were removed, DESIGN.md)")
    ap.add_argument("--m-plane", action="store_true",
                    help="pass B writes the m(p) plane and pass 2 reads it (instead of regenerating m per slice)")
    ap.add_argument("--qat-scales", choices=("multi", "concurrent", "sequential"), default=None,
                    help="--config 5: every stage once for all hook scales (multi-segment launches), the per-scale "
                         "modules on concurrent streams, or one after another (default: hooks')")
    ap.add_argument("--pass-b", choices=("image", "batch"), default=None,
                    help="morphology pass B: per-image workgroups or batch-wide tile kernels (default: engine's)")
    ap.add_argument("--pass-a", choices=("image", "band"), default=None,
                    help="morphology pass A: per-image workgroups or 16-row band workgroups (default: engine's)")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher rehearsal without a GPU: the ranks rendezvous over gloo, all-reduce their ranks "
                         "and rank 0 prints one JSON line (tests/test_bench_cpu.py)")
    args = ap.parse_args()
    if args.qat_scales is not None:
        from mcaq_yolo_amd import hooks as _hooks
        _hooks.MULTI_SCALE_TRAIN = args.qat_scales == "multi"
        _hooks.CONCURRENT_TRAIN_SCALES = args.qat_scales == "concurrent"
    if args.pass_b is not None:
        from mcaq_yolo_amd import engine as _engine
        _engine.TILES_BATCH = args.pass_b == "batch"
    if args.pass_a is not None:
        from mcaq_yolo_amd import engine as _engine
        _engine.BAND_PASS = args.pass_a == "band"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)          # self-launched: one process per GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.launch_check:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"metric": "launch check", "n_gpus": world, "rank_sum": float(t[0]),
                              "pid_differs": os.getpid() != os.getppid()}), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return
    # MCAQ_BENCH_BACKEND=gloo + more ranks than GPUs: functional rehearsal of
    # the N > 1 path on a one-GPU box (never a measurement)
    backend = os.environ.get("MCAQ_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1) if backend != "nccl" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    # MCAQ_BENCH_SHARDED=1 at N = 1: run the batch-sharded code path anyway
    # (a world_size 1 process group: the RCCL collectives captured in the
    # step's graph), to measure what N > 1 adds per step on one GPU
    if world > 1 or os.environ.get("MCAQ_BENCH_SHARDED") == "1":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        pg = dist.group.WORLD

    if args.config == 5:
        return main_qat(args, world, rank, dev, pg)
    if args.e2e:
        return main_e2e(args, world, rank, dev, pg)
    if args.score:
        return main_score(args, world, rank, dev, pg)
    name, B, chans, grid, mapper = CONFIGS[args.config]
    depth = max(1, args.pipeline)
    if args.launch_batches is None:
        args.launch_batches = LAUNCH_BATCHES_BY_CONFIG.get(args.config, LAUNCH_BATCHES)
    nbat = max(1, args.launch_batches)
    # whole launch sets: K (and the warmup) rounded up to a multiple of the batches per launch
    args.steps = -(-args.steps // nbat) * nbat
    args.warmup = -(-max(args.warmup, 1) // nbat) * nbat
    cm, mm, sm = load_blobs(dev)
    geoms = [ScaleGeom(B, c, h, w, grid) for c, (h, w) in zip(chans, SIZES)]
    plans = []
    nin = max(args.inputs or max(3, depth), depth)
    for p in range(nin):
        # each batch in flight has its own synthetic input (seeded per rank and slot)
        feats = [[synth_features(B, c, h, w, 1000 * args.config + i + 7919 * rank + 104729 * (p * nbat + k), dev)
                  for i, (c, (h, w)) in enumerate(zip(chans, SIZES))] for k in range(nbat)]
        plan = HookPlan(geoms, dev, batches=nbat)
        plan.prepare(feats if nbat > 1 else feats[0], cm, mm, [sm, sm, sm], temperature=1.0, mapper_kind=mapper,
                     batch_offset=rank * B, batch_total=world * B, m_plane=args.m_plane,
                     shared_stats=pg is not None)
        plan.feats = feats
        plans.append(plan)
    torch.cuda.synchronize()

    use_graph = not args.eager
    runner = Runner(plans, pg, use_graph, depth)
    runner.run(args.warmup)
    runner.sync()
    torch.cuda.synchronize()

    # per-kernel device times: in sequence (pass 2 right behind its own pass 1
    # and morphology) and with x evicted from the Infinity Cache before each
    # timed HBM pass (the roofline figure)
    kt_seq = kernel_timing(plans)
    sweep = torch.ones(96 << 20, device=dev)         # 384 MiB
    kt = kernel_timing(plans, evict=sweep)
    del sweep
    # single-batch latency: one batch through its chain with nothing in flight
    # beside it (the plan's own launch sequence on one stream)
    lat = []
    for _ in range(10):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        plans[0].launch(torch.cuda.current_stream())
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t1)
    latency_ms = sorted(lat)[len(lat) // 2] * 1e3
    runner.run(4 * nbat)  # plans[0] was re-run alone: a few more steps to be safe, then settle
    runner.sync()

    # ---- timed region: K steps, `depth` batches in flight.  Every window
    # starts and ends synchronised, so it carries one pipeline fill and one
    # drain (~ one batch's chain latency).  Two windows, K and 2K steps: their
    # difference is K steady-state steps (the fill and drain cancel), which
    # is what ms_per_step reports; the raw K-step window is kept beside it.
    def window(k):
        runner.sync()
        if pg is not None:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        runner.run(k)
        t_enq = time.perf_counter() - t0
        runner.sync()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if pg is not None:
            import torch.distributed as dist
            t = torch.tensor([wall], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.barrier()
            wall = float(t.item())
        return wall, t_enq

    # the K / 2K pair is repeated (5 pairs up to K = 100, else 3) and the
    # median slope reported: one host hiccup in a short window otherwise moves
    # the slope by several %; the first K-step window stays the raw figure
    npairs = 5 if args.steps <= 100 else 3
    slopes = []
    for i in range(npairs):
        wk, te = window(args.steps)
        w2k, _ = window(2 * args.steps)
        if i == 0:
            wall_k, t_enq, wall_2k = wk, te, w2k
        slopes.append((w2k - wk) / args.steps)
    step_s = sorted(slopes)[npairs // 2]
    if step_s <= 0.0:          # clock noise: fall back to the raw window
        step_s = wall_k / args.steps
    quant_us = kt["quant"]

    elems = sum(B * c * h * w for c, (h, w) in zip(chans, SIZES))    # per batch (= per step)
    lelems = nbat * elems                                            # per kernel launch
    alg_bytes = 12 * elems                       # 2 reads of x + 1 write of y, fp32
    # HBM-side bytes per launch from the rocprofv3 PMC passes of tools/pmc_traffic.sh
    # (FETCH_SIZE and WRITE_SIZE in separate runs, FETCH doubled per the gfx950
    # calibration), committed per config under profiles/
    traffic, traffic_k = None, {}
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic_config%d.json" % args.config)
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        traffic = tj.get("step_total")
        traffic_k = {k: v["total"] for k, v in tj.get("kernels", {}).items()}
    achieved = alg_bytes / step_s / 1e9
    value = world * B / step_s
    out = None
    if rank == 0:
        q_gbs = 8 * lelems / (quant_us * 1e-6) / 1e9
        seq = "hipExtLaunchKernel start/stop events of each launch, median of 40 single-launch steps in sequence " \
              "on one stream over %d input launch sets (%d batch(es) each), x evicted from the Infinity Cache " \
              "(384 MiB sweep) before each timed pass" % (len(plans), nbat)
        kern = {"quant": {"us": round(quant_us, 2), "alg_bytes": 8 * lelems, "GB/s": round(q_gbs, 1),
                          "frac": round(q_gbs / HBM_PEAK_GBS, 4), "timing": seq,
                          "us_in_sequence": round(kt_seq["quant"], 2)}}
        gbs = 4 * lelems / (kt["stats"] * 1e-6) / 1e9
        kern["stats"] = {"us": round(kt["stats"], 2), "alg_bytes": 4 * lelems, "GB/s": round(gbs, 1),
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "timing": seq,
                         "us_in_sequence": round(kt_seq["stats"], 2)}
        kern["morph_finalize"] = {"us": round(kt_seq["morph_finalize"], 2), "bound": "latency (per-image chain)",
                                  "timing": "events around the launch, in sequence"}
        out = {
            "metric": HOOK_METRIC,
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic silu(1.5*randn+2*up(randn)) C3/C4/C5 features, seeded weights",
            "config": {"workload": "%s bs%d/GPU 640x640 MCAQ hook path C3/C4/C5 (grid %d, %s mapper): channel "
                                   "stats, phi1..5, complexity MLP, bilateral, bit mapper, soft mask, 2-8 bit "
                                   "quant/dequant; YOLOv8 network excluded (see e2e)" % (name, B, grid, mapper),
                       "global_batch": world * B, "grid_size": grid, "mapper": mapper,
                       "parallelism": "dp%d" % world,
                       "pass_a": "16-row band workgroups" if _engine_mod().BAND_PASS else "per-image workgroups",
                       "pass_b": "batch-wide tile kernels" if _engine_mod().TILES_BATCH else "per-image workgroups",
                       "hip_graph": use_graph,
                       "rccl_in_graph": runner.captured_collective,
                       "sharded_code_path": pg is not None,
                       "batches_per_launch": nbat,
                       "launch_sets_in_flight": depth,
                       "batches_in_flight": depth * nbat,
                       "schedule": "streams: %d launch-set chains (%d independent batch(es) per launch, each with "
                                   "its own statistics) on %d streams, one HIP graph each" % (depth, nbat, depth),
                       "input_batches": len(plans) * nbat,
                       "latency_ms_single_launch": round(latency_ms, 4),
                       "host_enqueue_us_per_step": round(t_enq / args.steps * 1e6, 1),
                       "timing": "steady state: median over %d pairs of (wall(2K steps) - wall(K steps)) / K, "
                                 "each window synchronised on both sides (the pipeline fill and drain cancel)" % npairs,
                       "slopes_ms_per_step": [round(x * 1e3, 5) for x in slopes],
                       "raw_window_ms_per_step": round(wall_k / args.steps * 1e3, 5),
                       "raw_window_2k_ms_per_step": round(wall_2k / (2 * args.steps) * 1e3, 5)},
            # north star: the whole fused complexity + quant path,
            # 12 B per feature element over the wall time of a step
            "path_roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(achieved / HBM_PEAK_GBS, 4), "target_frac": 0.70, "traffic": traffic,
                              "kernel": "whole step: mcaq_stats + mcaq_morph_kernel + mcaq_tiles_kernel + "
                                        "mcaq_quant, 12 B per feature element per step",
                              "alg_bytes_per_step": alg_bytes},
            # the dominant kernel (pass 2): algorithmic bytes per launch over its
            # launch time (HIP events on its stream, single-batch steps in sequence)
            "roofline": {"bound": "hbm", "achieved": kern["quant"]["GB/s"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": kern["quant"]["frac"],
                         "traffic": traffic_k.get("mcaq_quant_tile_kernel", traffic_k.get("mcaq_quant_kernel")),
                         "kernel": "%s (pass 2: read x + write y, 8 B per feature element)"
                                   % ("mcaq_quant_tile_kernel" if "mcaq_quant_tile_kernel" in traffic_k
                                      else "mcaq_quant_kernel"),
                         "alg_bytes_per_launch": 8 * lelems, "us_per_launch": kern["quant"]["us"]},
            "kernels": kern,
            "cpu_baseline": None,
        }
    if not args.no_e2e:
        for p_ in plans:
            p_.feats = None
        del runner
        try:
            e2e = run_e2e(args.config, 20, 3, world, rank, dev, pg, inflight=args.e2e_inflight)
            e2e.pop("metric", None)
            if out is not None:
                out["e2e"] = e2e
        except Exception as exc:          # the hook-path line must still print
            if out is not None:
                out["e2e"] = {"error": repr(exc)[:300]}
    if rank == 0:
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.config)
        print(json.dumps(out), flush=True)
    if pg is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
