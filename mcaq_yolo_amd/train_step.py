"""The three hook scales of one QAT training step as multi-scale launches.

The per-scale train path (hooks.MCAQHooks._run_scale_modules: analyzer,
mapper, quantizer module by module, models/mcaq_yolo.py:409-455 in train
mode) issues every kernel once per scale: ~85 launches per step at config 5,
each a few microseconds of kernel and a kernel boundary.  Here every stage
runs once for all scales (the kernels take per-scale segments: mcaq_stats /
mcaq_morph / mcaq_qat_* with nscales = 3, the mcaq_*_multi train launchers of
csrc/mcaq_train.h), so a single-stream HIP graph of the step carries about a
third of the nodes and each node costs about its slowest scale instead of the
sum.  The values are those of the per-scale path, bit for bit
(tests/test_train_multi_gpu.py): the same per-scale kernels' bodies run on
the same data; the mapper's BatchNorm running statistics are updated in scale
order after the forward (as the per-scale calls leave them); the shared
modules' parameter gradients are reduced in the order autograd runs the
per-scale backwards (the last scale first).

Autograd: one Function per stage spans the scales (_HeadMulti, _MapperMulti,
_SoftMaskMulti, _QATMulti); LinearBitMapper, normalize_complexity and frozen /
per-tensor quantizers keep their per-scale pieces in between.
"""
import ctypes
import os

import torch

from . import abi, core
from .core import _f32c, _p, _stream


def _cmlp_params(an):
    return list(an.complexity_mlp.parameters())


_SM_BLOBS = {"key": None, "blobs": None, "primed": False}
_PREPACK = {"pending": None}


def _flush_prepack():
    """The pending blob pack on its own (when no pass-1 launch took it)."""
    p = _PREPACK["pending"]
    _PREPACK["pending"] = None
    if p is not None:
        arr, n, out, _ = p
        abi.check(abi.lib().mcaq_pack(arr, n, _p(out), out.numel(), _stream()), "mcaq_pack")


def _prepack(an, mods):
    """The step's two blob re-packs - the analyzer's complexity-MLP blob
    (core._pack_cmlp's layout, MFMA operands included) and every scale's
    soft-mask blob (_softmask_blobs') - as ONE mcaq_pack launch into one
    buffer, primed into both caches; when both would pack now (after an
    optimizer step, and always under HIP-graph capture).  Otherwise each
    cache packs for itself."""
    seq = an.complexity_mlp
    cps = list(seq.parameters())
    sps = [p for m in mods for p in m.net.parameters()]
    parts, mfma = core._cmlp_pack_parts(seq)
    ts = cps + sps
    if an._blob.pinned is not None or an._blob.primed or _SM_BLOBS["primed"] or \
            not all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in ts) or \
            len(parts) + len(mfma) + len(sps) > abi.MCAQ_PACK_MAXSEG or \
            sum(t.numel() for t in parts) != core._CM_SIZE or \
            any(sum(p.numel() for p in m.net.parameters()) != core._SM_SIZE for m in mods):
        return
    capturing = torch.cuda.is_current_stream_capturing()
    ckey = tuple((t.data_ptr(), t._version, t.device) for t in cps)
    skey = tuple((p.data_ptr(), p._version) for p in sps)
    if not capturing and (ckey == an._blob.key or skey == _SM_BLOBS["key"]):
        return
    segs, o = core._pack_segs(parts, mfma)
    if o > core._CM_BLOB:
        raise ValueError("blob overflow")
    stride = (core._SM_SIZE + 3) // 4 * 4
    for i, m in enumerate(mods):
        o = core._CM_BLOB + i * stride
        for p in m.net.parameters():
            segs.append((p.detach(), p.numel(), 1, 0, o))
            o += p.numel()
    out = torch.empty(core._CM_BLOB + len(mods) * stride, device=cps[0].device)
    # launched by the analyzer's pass-1 launch as extra workgroups (mcaq_stats_pack)
    _PREPACK["pending"] = (core._pack_array(segs), len(segs), out, segs)
    an._blob.prime(out[:core._CM_BLOB], None if capturing else ckey)
    _SM_BLOBS["blobs"] = [out[core._CM_BLOB + i * stride:core._CM_BLOB + (i + 1) * stride] for i in range(len(mods))]
    _SM_BLOBS["key"] = None if capturing else skey
    _SM_BLOBS["primed"] = True


def _softmask_blobs(mods):
    """The soft-mask blobs of every scale's quantizer (core._pack_softmask
    layout, each padded to a 16-byte multiple) packed by ONE mcaq_pack launch
    into one buffer; re-packed when a parameter changed (version counters)
    and always under HIP-graph capture, as core._BlobCache."""
    ps = [p for m in mods for p in m.net.parameters()]
    if _SM_BLOBS["primed"]:
        _SM_BLOBS["primed"] = False
        if _SM_BLOBS["key"] is None or _SM_BLOBS["key"] == tuple((p.data_ptr(), p._version) for p in ps):
            return _SM_BLOBS["blobs"]
    if not all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() for p in ps) or \
            len(ps) > abi.MCAQ_PACK_MAXSEG or any(sum(p.numel() for p in m.net.parameters()) != core._SM_SIZE
                                                  for m in mods):
        return [m.blob() for m in mods]
    key = tuple((p.data_ptr(), p._version) for p in ps)
    capturing = torch.cuda.is_current_stream_capturing()
    if capturing or key != _SM_BLOBS["key"]:
        stride = (core._SM_SIZE + 3) // 4 * 4
        segs = (abi.PackSeg * len(ps))()
        k = 0
        for i, m in enumerate(mods):
            o = i * stride
            for p in m.net.parameters():
                segs[k].src, segs[k].n, segs[k].k, segs[k].mode, segs[k].dst = _p(p.detach()), p.numel(), 1, 0, o
                o += p.numel()
                k += 1
        out = torch.empty(len(mods) * stride, device=ps[0].device)
        abi.check(abi.lib().mcaq_pack(segs, len(ps), _p(out), out.numel(), _stream()), "mcaq_pack")
        _SM_BLOBS["blobs"] = [out[i * stride:(i + 1) * stride] for i in range(len(mods))]
        _SM_BLOBS["key"] = None if capturing else key
    return _SM_BLOBS["blobs"]


def _ema_multi_ok(qs, xs):
    """Every quantizer in the state the one-launch EMA covers: per-channel
    running statistics that exist (fp32, contiguous, on the device, C
    entries), not frozen, unsharded, num_batches_tracked an int64 scalar on
    the device; otherwise each quantizer runs update_running_stats."""
    if len({id(q.process_group) for q in qs}) != 1:
        return False
    for q, x in zip(qs, xs):
        if not q.per_channel or q._frozen() or q.running_min is None:
            return False
        C = x.shape[1]
        for t in (q.running_min, q.running_max):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != x.device or t.numel() != C:
                return False
        nbt = q.num_batches_tracked
        if nbt.device != x.device or nbt.dtype != torch.int64 or nbt.numel() != 1:
            return False
    return True


# The quantizers' EMA launch (with the mapper's running-statistics update),
# deferred by _quantize_multi to ride on the soft-mask launch of
# _MaskQuantMulti (mcaq_morph_ema); flushed on its own if nothing took it.
_PENDING_EMA = {"args": None}


def _flush_ema():
    p = _PENDING_EMA["args"]
    _PENDING_EMA["args"] = None
    if p is not None:
        _launch_ema(*p)


def _launch_ema(segs, n, running, keep):
    L = abi.lib()
    if running is not None:
        rq, wa, na, cnt, mom = running
        abi.check(L.mcaq_ema_stats_multi_running(segs, n, ctypes.byref(rq), wa, na, cnt, mom, _stream()),
                  "mcaq_ema_stats_multi_running")
    else:
        abi.check(L.mcaq_ema_stats_multi(segs, n, _stream()), "mcaq_ema_stats_multi")


def _ema_multi(qs, xs, box, running=None, defer=False):
    """quantization.py:319-353 for every scale's quantizer: the batch min /
    max from the analyzer's pass-1 partials (one finalize launch for all
    scales), then the EMA, this step's copies and num_batches_tracked (one
    launch): the values of q.update_running_stats(x, want_copies=True)."""
    L = abi.lib()
    n = len(qs)
    fz = (abi.FinalizeScale * n)()
    segs = (abi.EmaSeg * n)()
    mins, maxs, keep = [], [], []
    fold = all("bmin" in b for b in box[:n])      # reduced by the analyzer's morph launch
    for i, (q, x) in enumerate(zip(qs, xs)):
        C = x.shape[1]
        if fold:
            bmin, bmax = box[i]["bmin"], box[i]["bmax"]
        else:
            bmin, bmax = torch.empty(C, device=x.device), torch.empty(C, device=x.device)
        cmin, cmax = torch.empty(C, device=x.device), torch.empty(C, device=x.device)
        keep += [bmin, bmax]
        f = fz[i]
        f.pmin, f.pmax, f.min_out, f.max_out = _p(box[i]["pmin"]), _p(box[i]["pmax"]), _p(bmin), _p(bmax)
        f.C, f.nunits, f.min_stride = C, box[i]["pmin"].shape[0], 1
        e = segs[i]
        e.batch_min, e.batch_max = _p(bmin), _p(bmax)
        e.running_min, e.running_max = _p(q.running_min), _p(q.running_max)
        e.copy_min, e.copy_max, e.num_batches = _p(cmin), _p(cmax), _p(q.num_batches_tracked)
        e.C, e.first, e.momentum = C, 0, float(q.momentum)
        mins.append(cmin); maxs.append(cmax)
    if not fold:
        abi.check(L.mcaq_finalize(fz, n, _stream()), "mcaq_finalize")
    pg = qs[0].process_group
    if pg is not None and not (fold and all(b.get("bglobal") for b in box[:n])):
        # data-parallel QAT: every scale's batch min / max over the global
        # batch in ONE all-reduce (MAX over [-min, max]; per quantizer the
        # values of update_running_stats' own all-reduce)
        import torch.distributed as dist
        vec = torch.cat([t for i in range(n) for t in (-keep[2 * i], keep[2 * i + 1])])
        dist.all_reduce(vec, op=dist.ReduceOp.MAX, group=pg)
        o = 0
        for i, x in enumerate(xs):
            C = x.shape[1]
            keep[2 * i].copy_(-vec[o:o + C])
            keep[2 * i + 1].copy_(vec[o + C:o + 2 * C])
            o += 2 * C
    if defer:
        _PENDING_EMA["args"] = (segs, n, running, keep)
    else:
        _launch_ema(segs, n, running, keep)
    return mins, maxs


def _flush_running(pending):
    """The mapper's deferred BatchNorm running-statistics update on its own."""
    q, wa, na, n, mom = pending
    abi.check(abi.lib().mcaq_mapper_running_update(ctypes.byref(q), wa, na, n, mom, _stream()),
              "mcaq_mapper_running_update")


def _run_analyzer_multi(an, xs):
    """Pass 1 (gray, |x| means, channel min/max partials) and the morphology
    (phi, complexity MLP, bilateral -> C) of every scale: 2 launches of
    mcaq_stats / mcaq_morph instead of 2 per scale."""
    L = abi.lib()
    n = len(xs)
    stats = (abi.StatsScale * n)()
    morphs = (abi.MorphScale * n)()
    outs, keep = [], []
    blob = an.cmlp_blob()
    flags = abi.F_PHI | abi.F_CMLP | an._flags()
    for i, x in enumerate(xs):
        B, C, H, W = x.shape
        T = core.tile_size(H, an.grid_size)
        ht, wt = H // T, W // T
        if ht < 1 or wt < 1 or T > 128:
            raise ValueError("feature map %dx%d: tile %d unsupported" % (H, W, T))
        dev = x.device
        units = L.mcaq_stats_units(B, C, H, W)
        o = {"gray": torch.empty(B, ht * T, wt * T, device=dev), "absmean": torch.empty(B, H, W, device=dev),
             "pmin": torch.empty(units, C, device=dev), "pmax": torch.empty(units, C, device=dev),
             "phi": torch.empty(B, ht, wt, 8, device=dev), "c": torch.empty(B, ht, wt, device=dev),
             "craw": torch.empty(B, ht, wt, device=dev), "tile_tmp": torch.empty(B, ht * wt, 32, device=dev)}
        s = stats[i]
        s.x, s.gray, s.absmean, s.pmin, s.pmax = _p(x), _p(o["gray"]), _p(o["absmean"]), _p(o["pmin"]), _p(o["pmax"])
        s.B, s.C, s.H, s.W, s.Hc, s.Wc = B, C, H, W, ht * T, wt * T
        ptrs = dict(gray=o["gray"], phi_out=o["phi"], tile_tmp=o["tile_tmp"], cmlp=blob, c_out=o["c"],
                    cmlp_out=o["craw"])
        scratch = L.mcaq_morph_scratch_bytes(B, ht * T, wt * T, ht, wt)
        if scratch:
            ptrs["gscratch"] = torch.empty(scratch, device=dev, dtype=torch.uint8)
            keep.append(ptrs["gscratch"])
        wb = L.mcaq_morph_work_bytes(B, ht * T, wt * T, T) if core._engine.BAND_PASS else 0
        if wb:
            ptrs["pwork"] = torch.empty(wb // 4, device=dev)   # pass A as band + edge workgroups, as core.py
            keep.append(ptrs["pwork"])
        morphs[i] = core._morph_struct(B, H, W, T, ht, wt, flags, **ptrs)
        outs.append(o)
    # the quantizers' batch min / max ride along with the morph launch as its
    # channel-reduction workgroups (as in inference): the EMA then needs no
    # finalize launch of its own (_ema_multi)
    fz = (abi.FinalizeScale * n)()
    for i, (x, o) in enumerate(zip(xs, outs)):
        C = x.shape[1]
        o["bmin"], o["bmax"] = torch.empty(C, device=x.device), torch.empty(C, device=x.device)
        f = fz[i]
        f.pmin, f.pmax, f.min_out, f.max_out = _p(o["pmin"]), _p(o["pmax"]), _p(o["bmin"]), _p(o["bmax"])
        f.C, f.nunits, f.min_stride = C, o["pmin"].shape[0], 1
    pend = _PREPACK["pending"]
    _PREPACK["pending"] = None
    if pend is not None:      # the step's blob pack rides on pass 1
        arr, npk, out, _ = pend
        abi.check(L.mcaq_stats_pack(stats, n, arr, npk, _p(out), out.numel(), _stream()), "mcaq_stats_pack")
    else:
        abi.check(L.mcaq_stats(stats, n, _stream()), "mcaq_stats")
    abi.check(L.mcaq_morph_finalize(morphs, n, fz, n, _stream()), "mcaq_morph_finalize")
    return outs


class _HeadMulti(torch.autograd.Function):
    """Analyzer of every scale in train mode: C per scale (values of the morph
    kernel); backward = bilateral adjoint + complexity MLP backward of every
    scale in 2 launches, parameter gradients reduced in one."""

    @staticmethod
    def forward(ctx, an, n, box, *args):
        xs, params = args[:n], args[n:]
        outs = _run_analyzer_multi(an, [x.detach() for x in xs])
        box.extend(outs)                    # pass-1 by-products for the quantizers
        an._last_phi = outs[-1]["phi"]
        ctx.an, ctx.n = an, n
        ctx.save_for_backward(*[o["phi"] for o in outs], *[o["craw"] for o in outs], *params)
        return tuple(o["c"] for o in outs)

    @staticmethod
    def backward(ctx, *gcs):
        n = ctx.n
        phis, craws = ctx.saved_tensors[:n], ctx.saved_tensors[n:2 * n]
        params = ctx.saved_tensors[2 * n:]
        L = abi.lib()
        dev = craws[0].device
        q = abi.CmlpParams(*[_p(p.detach()) for p in params])
        segs = (abi.HeadSeg * n)()
        gparts, keep = [], []
        for i in range(n):
            B, ht, wt = craws[i].shape
            m = B * ht * wt
            g = _f32c(gcs[i]) if gcs[i] is not None else torch.zeros(B, ht, wt, device=dev)
            gcraw = torch.empty(m, device=dev)
            gp = torch.empty(L.mcaq_head_gpart_floats(m), device=dev)
            keep += [g, gcraw]
            gparts.append((gp, gp.numel() // core._CM_SIZE))      # one partial per backward workgroup
            sg = segs[i]
            sg.phi, sg.craw, sg.gC, sg.gcraw, sg.gpart = _p(phis[i]), _p(craws[i]), _p(g), _p(gcraw), _p(gp)
            sg.B, sg.ht, sg.wt = B, ht, wt
        ride = _PENDING_REDUCE["segs"]
        _PENDING_REDUCE["segs"] = None
        mod_params = _cmlp_params(ctx.an)
        sink = ctx.an._gsink.target(mod_params) if len(mod_params) == len(params) else None
        gflat, acc = sink if sink is not None else (torch.empty(core._CM_SIZE, device=dev), 0)
        sync = _sync_buffer(ctx.an, dev, [c.numel() for c in craws], L.mcaq_head_sync_bytes) if HEAD_FUSED else None
        if sync is not None:
            # the MLP's parameter reduction inside its own launch; the mapper's
            # (if pending) riding on the bilateral launch
            abi.check(L.mcaq_head_train_backward_fused(ctypes.byref(q), segs, n, ride[0] if ride else None,
                                                       ride[1] if ride else 0, _p(gflat), acc, 0.0, _p(sync),
                                                       sync.numel() * 8, _stream()),
                      "mcaq_head_train_backward_fused")
        else:
            if ride is not None:     # the mapper's gradient reduction as extra workgroups of the bilateral launch
                abi.check(L.mcaq_head_train_backward_multi_ride(ctypes.byref(q), segs, n, ride[0], ride[1],
                                                                _stream()), "mcaq_head_train_backward_multi_ride")
            else:
                abi.check(L.mcaq_head_train_backward_multi(ctypes.byref(q), segs, n, _stream()),
                          "mcaq_head_train_backward_multi")
            _reduce_chain(gparts, gflat, acc, core._CM_SIZE)
        grads = (None,) * len(params) if sink is not None else tuple(core._split_flat(gflat, params))
        return (None, None, None) + (None,) * n + grads


def _chain_segs(gparts, out, acc, count, scale=0.0):
    """ReduceSeg chain: every scale's per-workgroup partials into `out`, in
    the order the per-scale backwards accumulate them (autograd runs the last
    scale's first); scale (0: none) multiplies the launch's sum."""
    n = len(gparts)
    segs = (abi.ReduceSeg * n)()
    for k, (gp, nparts) in enumerate(reversed(gparts)):
        s = segs[k]
        s.part, s.out, s.nparts, s.stride, s.count, s.accumulate = _p(gp), _p(out), nparts, count, count, acc
        s.scale = scale
    return segs


def _reduce_chain(gparts, out, acc, count, scale=0.0):
    abi.check(abi.lib().mcaq_train_reduce_multi(_chain_segs(gparts, out, acc, count, scale), len(gparts), 1,
                                                _stream()), "mcaq_train_reduce_multi")


# The bit mapper's parameter-gradient reduction, deferred from its backward
# to ride on the analyzer head's backward launch (the next node autograd runs
# on this path; the mapper's .grad are views of its _GradSink buffer, which
# nothing reads before the optimizer).  An engine callback at the end of
# backward launches it on its own if no head backward took it.
_PENDING_REDUCE = {"segs": None}


def _flush_pending_reduce():
    p = _PENDING_REDUCE["segs"]
    _PENDING_REDUCE["segs"] = None
    if p is not None:
        segs, n, keep = p
        abi.check(abi.lib().mcaq_train_reduce_multi(segs, n, 1, _stream()), "mcaq_train_reduce_multi")


# The soft masks' parameter-gradient reductions (one per scale, into each
# net's _GradSink), deferred from _MaskQuantMulti.backward to ride on the
# bit mapper's first backward launch (the next node on this path) the same
# way; an engine callback launches them on their own otherwise.
_PENDING_SM_REDUCE = {"segs": None}


def _flush_pending_sm_reduce():
    p = _PENDING_SM_REDUCE["segs"]
    _PENDING_SM_REDUCE["segs"] = None
    if p is not None:
        segs, n, keep = p
        abi.check(abi.lib().mcaq_train_reduce_multi(segs, n, 0, _stream()), "mcaq_train_reduce_multi")


# ---------------------------------------------------------------------------
# batch-sharded step (dist.shard_hooks): the bit mapper on the global batch
# ---------------------------------------------------------------------------
# The mapper's train-mode BatchNorm statistics span the global batch
# (bit_allocation.py:126 on the single process).  Instead of one collective
# per batch-statistics stage in each direction (3 + 3), every rank
# all-gathers the mapper's inputs once - with the quantizers' batch channel
# min / max riding along - runs the mapper on the GLOBAL batch of tiles (a
# few thousand tiles: the stage launches' cost is their latency, not the
# tile count) and keeps its own slice; the backward all-gathers the bits'
# gradients once and runs the mapper's backward on the global batch: every
# rank then holds the WHOLE mapper gradient and contributes 1 / world of it
# to the gradient all-reduce (whose sum is that gradient again).  Bits,
# BatchNorm batch and running statistics, EMA min / max and the mapper's
# input gradients are the single-process values bit for bit; 2 collectives
# instead of 7.  False: the staged per-layer collectives.
DP_GLOBAL_MAPPER = True

# The train-mode mapper as ONE launch per direction (mcaq_mapper_train_*_fused):
# the workgroups exchange the batch statistics between the layers inside the
# launch (write-through granules, no grid barrier, no fence) instead of
# ending a launch at each of the 3 + 3 statistics barriers; bit-identical to
# the staged launches (False), which also serve more workgroups than the
# chip holds at once.  MCAQ_MAPPER_FUSED=0 selects the staged launches (A/B).
MAPPER_FUSED = os.environ.get("MCAQ_MAPPER_FUSED", "1") != "0"


def _sync_buffer(mod, dev, ns, nbytes):
    """An in-launch exchange's sync buffer for segments of ns tiles (64 per
    workgroup): one per module and segment layout, zeroed when made (epochs
    and granules start over); None above the resident-workgroup limit."""
    L = abi.lib()
    wgs = tuple((int(n) + 63) // 64 for n in ns)
    total = sum(wgs)
    if total > L.mcaq_mapper_fused_max_wg():
        return None
    cache = mod.__dict__.setdefault("_mapx", {})
    key = (str(dev), nbytes.__name__, wgs)
    buf = cache.get(key)
    if buf is None:
        buf = torch.zeros((nbytes(total) + 7) // 8, dtype=torch.int64, device=dev)
        cache[key] = buf
    return buf


def _mapx_buffer(mod, dev, ns):
    """The fused mapper launches' sync buffer (forward and backward share it)."""
    return _sync_buffer(mod, dev, ns, abi.lib().mcaq_mapper_sync_bytes) if MAPPER_FUSED else None


def mapper_sync_status(mod):
    """Nonzero when an in-launch exchange of a fused launch of `mod` (the
    mapper's, or the analyzer head's backward) timed out (its results are
    then invalid); 0 otherwise.  Synchronises."""
    st = 0
    for key, buf in getattr(mod, "_mapx", {}).items():
        w = abi.MAPPER_SYNC_STATUS_WORD if key[1] == "mcaq_mapper_sync_bytes" else abi.ADAMW_SYNC_STATUS_WORD
        st |= int(buf.view(torch.int32)[w].item())
    return st


# The complexity MLP's backward with its parameter reduction inside the
# launch (mcaq_head_train_backward_fused: partials exchanged as granules,
# bit-identical to the separate chain reduction).  Off by default: measured
# no faster than the separate launch (19.8 vs 13.9 + 5.7 us, step within
# noise: profiles/r06_fuse/r06_fuse3) - the 2,881 partials per workgroup
# cost as much written and swept write-through as the launch boundary they
# replace.  MCAQ_HEAD_FUSED=1 selects it.
HEAD_FUSED = os.environ.get("MCAQ_HEAD_FUSED", "0") == "1"


def _consecutive(ts):
    """The flat concatenation of ts when they already lie back to back in one
    buffer (no copy), else None."""
    if not all(t.is_contiguous() and t.dtype == torch.float32 for t in ts):
        return None
    st = ts[0].untyped_storage()
    o = ts[0].storage_offset()
    for t in ts:
        if t.untyped_storage().data_ptr() != st.data_ptr() or t.storage_offset() != o:
            return None
        o += t.numel()
    out = torch.empty(0, dtype=torch.float32, device=ts[0].device)
    out.set_(st, ts[0].storage_offset(), (o - ts[0].storage_offset(),))
    return out


def _dp_exchange(parts, specs, pg):
    """all-gather the concatenation of `parts` (this rank's flat fp32 pieces)
    over pg in ONE collective and unpack it in ONE launch: specs are
    (out, offset in the send buffer, n, mode) - mode 0 writes the pieces of
    every rank back to back (world * n), mode 1 / 2 the min / max over ranks."""
    import torch.distributed as dist
    world = dist.get_world_size(pg)
    send = _consecutive(parts)
    if send is None:
        send = torch.cat(parts)
    g = core._all_gather_flat(send, pg, world)
    arr = (abi.DpSeg * len(specs))()
    for a, (out, off, n, mode) in zip(arr, specs):
        a.out, a.off, a.n, a.mode = _p(out), off, n, mode
    abi.check(abi.lib().mcaq_dp_unpack(_p(g), world, send.numel(), arr, len(specs), _stream()), "mcaq_dp_unpack")
    return g


def _dp_mapper_inputs(mapper, ncs, box, with_minmax):
    """The global-batch mapper inputs of every scale (and, riding along, the
    quantizers' global batch min / max written into box) - or None when the
    sharded step keeps the staged collectives."""
    if not DP_GLOBAL_MAPPER or not isinstance(mapper, core.ComplexityToBitMappingNetwork):
        return None
    pg = core._mapper_group(mapper.mapping_network)
    if pg is None:
        return None
    if len(ncs) * 3 > abi.MCAQ_DP_MAXSEG:
        return None
    import torch.distributed as dist
    world, rank = dist.get_world_size(pg), dist.get_rank(pg)
    cf = [_f32c(c).reshape(-1) for c in ncs]
    parts, specs, cg, o = list(cf), [], [], 0
    for c in cf:
        g = torch.empty(world * c.numel(), device=c.device)
        cg.append(g)
        specs.append((g, o, c.numel(), 0))
        o += c.numel()
    if with_minmax:
        for b in box[:len(ncs)]:
            for key, mode in (("bmin", 1), ("bmax", 2)):
                t = b[key]
                parts.append(t)
                specs.append((t, o, t.numel(), mode))      # written in place: the global batch's
                o += t.numel()
            b["bglobal"] = True
    _dp_exchange(parts, specs, pg)
    return {"cg": cg, "rank": rank, "world": world, "pg": pg}


class _MapperMulti(torch.autograd.Function):
    """Train-mode bit mapper of every scale: one forward launch (MAPPER_FUSED:
    the batch statistics exchanged inside it; else 4 launches, one per
    batch-statistics barrier) + the running-statistics update in scale order;
    one backward launch (else 4) + one parameter reduction."""

    @staticmethod
    def forward(ctx, mod, temperature, return_continuous, n, *args):
        cs, params = args[:n], args[n:]
        net = mod.mapping_network
        L = abi.lib()
        dev = cs[0].device
        bns = [net[i] for i in (1, 4, 7)]
        q = abi.MapperParams()
        for k, t in zip(("w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4"),
                        (net[0].weight, net[0].bias, net[3].weight, net[3].bias, net[6].weight, net[6].bias,
                         net[9].weight, net[9].bias)):
            setattr(q, k, _p(t.detach()))
        for i, bn in enumerate(bns, 1):
            for k, t in (("g", bn.weight), ("be", bn.bias), ("rm", bn.running_mean), ("rv", bn.running_var),
                         ("nbt", bn.num_batches_tracked)):
                setattr(q, "%s%d" % (k, i), _p(t.detach()) if t is not None else None)
        T = max(float(temperature), 0.1) if temperature is not None else 0.0
        segs = (abi.MapperSeg * n)()
        cfs, works, bits = [], [], []
        dp = getattr(mod, "_dp", None)       # batch sharded: the global batch (_dp_mapper_inputs)
        for i, c in enumerate(cs):
            cf = _f32c(c).reshape(-1) if dp is None else dp["cg"][i]
            m = cf.numel()
            w = torch.empty(L.mcaq_mapper_work_floats(m), device=dev)
            b = torch.empty(m, device=dev)
            cfs.append(cf); works.append(w); bits.append(b)
            segs[i].c, segs[i].bits, segs[i].work, segs[i].n = _p(cf), _p(b), _p(w), m
        mom = float(bns[0].momentum)
        pg = core._mapper_group(net) if dp is None else None
        ctx.pg, ctx.gath1, ctx.world, ctx.dp = pg, None, 1, dp
        sync = _mapx_buffer(mod, dev, [c.numel() for c in cfs]) if pg is None else None
        ctx.sync = sync
        if sync is not None:
            abi.check(L.mcaq_mapper_train_forward_fused(ctypes.byref(q), segs, n, mod.min_bits, mod.max_bits, T, mom,
                                                        0 if return_continuous else 1, 2, _p(sync),
                                                        sync.numel() * 8, _stream()),
                      "mcaq_mapper_train_forward_fused")
        elif pg is None:
            abi.check(L.mcaq_mapper_train_forward_multi(ctypes.byref(q), segs, n, mod.min_bits, mod.max_bits, T,
                                                        mom, 0 if return_continuous else 1, 2, _stream()),
                      "mcaq_mapper_train_forward_multi")
        else:
            # batch sharded (GroupBatchNorm1d): between the stage launches every
            # scale's (mean, M2, n) of this rank, all-gathered in ONE collective
            import torch.distributed as dist
            world = dist.get_world_size(pg)
            gath = [None] * 4
            for st in (1, 2, 3, 4):
                gp = (abi.P * n)(*[_p(t) for t in gath[st - 1]]) if st >= 2 else None
                abi.check(L.mcaq_mapper_train_forward_stage_multi(
                    ctypes.byref(q), segs, n, mod.min_bits, mod.max_bits, T, mom, 0 if return_continuous else 1, 2,
                    st, gp, world, _stream()), "mcaq_mapper_train_forward_stage_multi")
                if st <= 3:
                    rk = torch.empty(n, core._RANK_ENT, device=dev)
                    for i in range(n):
                        abi.check(L.mcaq_mapper_train_reduce(_p(works[i]), cfs[i].numel(), 0, st, _p(rk[i]), _stream()),
                                  "mcaq_mapper_train_reduce")
                    g_all = core._all_gather_flat(rk.reshape(-1), pg, world)
                    gath[st] = list(g_all.view(world, n, core._RANK_ENT).transpose(0, 1).contiguous())
            ctx.gath1, ctx.world = gath[1], world
        wa = (abi.P * n)(*[_p(w) for w in works])
        na = (abi.I * n)(*[c.numel() for c in cfs])
        if pg is None and getattr(mod, "_defer_running", False):    # (sharded on the global batch too)
            # the quantizers' EMA launch that follows applies it (forward_features)
            mod._pending_running = (q, wa, na, n, mom)
        else:
            _flush_running((q, wa, na, n, mom))
        ctx.q, ctx.T, ctx.mod, ctx.n = q, T, mod, n
        ctx.shapes = [c.shape for c in cs]
        ctx.save_for_backward(*cfs, *works, *params)
        if dp is not None:       # this rank's tiles of the global batch
            r = dp["rank"]
            return tuple(b[r * c.numel():(r + 1) * c.numel()].view(c.shape) for b, c in zip(bits, cs))
        return tuple(b.view(c.shape) for b, c in zip(bits, cs))

    @staticmethod
    def backward(ctx, *gbits):
        n, mod = ctx.n, ctx.mod
        cfs, works = ctx.saved_tensors[:n], ctx.saved_tensors[n:2 * n]
        params = ctx.saved_tensors[2 * n:]
        L = abi.lib()
        dev = cfs[0].device
        segs = (abi.MapperSeg * n)()
        gcs, gparts, keep = [], [], []
        dp = ctx.dp
        gls = [(_f32c(gbits[i]).reshape(-1) if gbits[i] is not None else
                torch.zeros(ctx.shapes[i].numel(), device=dev)) for i in range(n)]
        if dp is not None:
            # every rank's bit gradients of every scale: ONE all-gather
            r, world = dp["rank"], dp["world"]
            ggs, specs, o = [], [], 0
            for g in gls:
                gg = torch.empty(world * g.numel(), device=dev)
                ggs.append(gg)
                specs.append((gg, o, g.numel(), 0))
                o += g.numel()
            keep.append(_dp_exchange(gls, specs, dp["pg"]))
            gls = ggs
        for i in range(n):
            m = cfs[i].numel()
            g = gls[i]
            gc = torch.empty(m, device=dev)
            gp = torch.empty(L.mcaq_mapper_gpart_floats(m), device=dev)
            keep.append(g)
            npart = gp.numel() // core._MAPPER_G_SIZE             # one partial per backward workgroup
            if dp is not None:
                ml = ctx.shapes[i].numel()
                gcs.append(gc[r * ml:(r + 1) * ml])               # this rank's tiles
            else:
                gcs.append(gc)
            gparts.append((gp, npart))
            s = segs[i]
            s.c, s.work, s.gbits, s.gc, s.gpart, s.n = _p(cfs[i]), _p(works[i]), _p(g), _p(gc), _p(gp), m
        ride = _PENDING_SM_REDUCE["segs"] if ctx.pg is None else None
        if ctx.pg is None and ctx.sync is not None:
            # one launch, the soft masks' reductions (if pending) riding along
            _PENDING_SM_REDUCE["segs"] = None
            abi.check(L.mcaq_mapper_train_backward_fused(ctypes.byref(ctx.q), segs, n, mod.min_bits, mod.max_bits,
                                                         ctx.T, ride[0] if ride is not None else None,
                                                         ride[1] if ride is not None else 0, _p(ctx.sync),
                                                         ctx.sync.numel() * 8, _stream()),
                      "mcaq_mapper_train_backward_fused")
        elif ride is not None:
            # the soft masks' gradient reductions as extra workgroups of the first stage launch
            _PENDING_SM_REDUCE["segs"] = None
            abi.check(L.mcaq_mapper_train_backward_multi_ride(ctypes.byref(ctx.q), segs, n, mod.min_bits, mod.max_bits,
                                                              ctx.T, ride[0], ride[1], _stream()),
                      "mcaq_mapper_train_backward_multi_ride")
        elif ctx.pg is None:
            abi.check(L.mcaq_mapper_train_backward_multi(ctypes.byref(ctx.q), segs, n, mod.min_bits, mod.max_bits,
                                                         ctx.T, _stream()), "mcaq_mapper_train_backward_multi")
        else:
            # BN backward sums (S1, S2) of every scale all-reduced in ONE
            # collective before the stage that consumes them; parameter
            # gradients stay this rank's own (for the gradient all-reduce)
            import torch.distributed as dist
            gs = [None] * 5
            g1p = (abi.P * n)(*[_p(t) for t in ctx.gath1])
            for st in (4, 3, 2, 1):
                gsp = (abi.P * n)(*[_p(t) for t in gs[st]]) if st <= 3 else None
                abi.check(L.mcaq_mapper_train_backward_stage_multi(
                    ctypes.byref(ctx.q), segs, n, mod.min_bits, mod.max_bits, ctx.T, st, gsp,
                    g1p if st <= 3 else None, ctx.world, _stream()), "mcaq_mapper_train_backward_stage_multi")
                if st >= 2:
                    bs = torch.empty(n, 128, device=dev)
                    for i in range(n):
                        abi.check(L.mcaq_mapper_train_reduce(_p(works[i]), cfs[i].numel(), 1, st - 1, _p(bs[i]),
                                                             _stream()), "mcaq_mapper_train_reduce")
                    dist.all_reduce(bs, group=ctx.pg)
                    gs[st - 1] = list(bs)
        sink = mod._gsink.target(list(mod.mapping_network.parameters()))
        gflat, acc = sink if sink is not None else (torch.empty(core._MAPPER_G_SIZE, device=dev), 0)
        # batch sharded on the global batch: every rank computed the WHOLE
        # mapper gradient (all ranks' tiles); it contributes 1 / world of it
        # to the gradient all-reduce, whose sum is then that gradient
        sc = 1.0 / dp["world"] if dp is not None else 0.0
        if sink is not None and ctx.pg is None and _PENDING_REDUCE["segs"] is None:
            _PENDING_REDUCE["segs"] = (_chain_segs(gparts, gflat, acc, core._MAPPER_G_SIZE, sc), n, (gparts, keep))
            torch.autograd.Variable._execution_engine.queue_callback(_flush_pending_reduce)
        else:
            _reduce_chain(gparts, gflat, acc, core._MAPPER_G_SIZE, sc)
        grads = (None,) * len(params) if sink is not None else tuple(core._split_flat(gflat, params))
        return (None, None, None, None) + tuple(g.view(s) for g, s in zip(gcs, ctx.shapes)) + grads


class _SoftMaskMulti(torch.autograd.Function):
    """LearnedSoftMask of every scale (each quantizer its own net): m(p)
    planes by one morph launch; backward by one launch + one reduction."""

    @staticmethod
    def forward(ctx, mods, n, *args):
        bits, absmeans = args[:n], args[n:2 * n]
        L = abi.lib()
        morphs = (abi.MorphScale * n)()
        ms = []
        blobs = _softmask_blobs(mods)
        for i in range(n):
            b = _f32c(bits[i]).detach()
            B, H, W = absmeans[i].shape
            _, ht, wt = b.shape
            if 4 * ht > H or 4 * wt > W:
                raise NotImplementedError("soft mask on a tile grid finer than 4 pixels per tile")
            m = torch.empty(B, 1, H, W, device=b.device)
            ms.append(m)
            morphs[i] = core._morph_struct(B, H, W, 4, ht, wt, abi.F_SOFTMASK, absmean=absmeans[i], bits_in=b,
                                           smask=blobs[i], m_out=m)
        abi.check(L.mcaq_morph(morphs, n, _stream()), "mcaq_morph(soft mask)")
        ctx.mods, ctx.n = mods, n
        ctx.save_for_backward(*bits, *absmeans)
        return tuple(ms)

    @staticmethod
    def backward(ctx, *gms):
        n = ctx.n
        bits, absmeans = ctx.saved_tensors[:n], ctx.saved_tensors[n:2 * n]
        L = abi.lib()
        segs = (abi.SmaskSeg * n)()
        rsegs = (abi.ReduceSeg * n)()
        gbs, gflats, keep = [], [], []
        for i in range(n):
            b = _f32c(bits[i])
            B, H, W = absmeans[i].shape
            _, ht, wt = b.shape
            gm = _f32c(gms[i]) if gms[i] is not None else torch.zeros(B, H, W, device=b.device)
            gb = torch.empty(B, ht, wt, device=b.device)
            gp = torch.empty(L.mcaq_smask_gpart_floats(B), device=b.device)
            gf = torch.empty(core._SM_SIZE, device=b.device)
            keep += [b, gm, gp]
            gbs.append(gb); gflats.append(gf)
            s = segs[i]
            s.P = abi.SmaskParams(*[_p(p.detach()) for p in ctx.mods[i].net.parameters()])
            s.bits, s.absmean, s.gm, s.gbits, s.gpart = _p(b), _p(absmeans[i]), _p(gm), _p(gb), _p(gp)
            s.B, s.H, s.W, s.ht, s.wt, s.accumulate = B, H, W, ht, wt, 0
            r = rsegs[i]
            r.part, r.out, r.nparts, r.stride, r.count, r.accumulate = _p(gp), _p(gf), B, core._SM_SIZE, \
                core._SM_SIZE, 0
        abi.check(L.mcaq_smask_train_backward_multi(segs, n, _stream()), "mcaq_smask_train_backward_multi")
        abi.check(L.mcaq_train_reduce_multi(rsegs, n, 0, _stream()), "mcaq_train_reduce_multi")
        pgrads = []
        for i in range(n):
            params = list(ctx.mods[i].net.parameters())
            pgrads += [g if p.requires_grad else None for g, p in zip(core._split_flat(gflats[i], params), params)]
        return (None, None) + tuple(gbs[i] if ctx.needs_input_grad[2 + i] else None for i in range(n)) + \
            (None,) * n + tuple(pgrads)


# The soft masks, the quantizers and the bit budget of every scale as ONE
# autograd node (_MaskQuantMulti): the quantizer backward's fold, the soft-mask
# backward and the bit-budget gradient then meet in one launch, so the bit
# maps receive ONE gradient (no ATen adds between the quantizer's, the soft
# mask's and the avg_bits term's contributions) and avg_bits / its loss cost
# one small launch instead of ~20 ATen kernels.  False: the separate
# _SoftMaskMulti / _QATMulti nodes and avg_bits as torch ops.
FUSED_MASK_QAT = True


class _MaskQuantMulti(torch.autograd.Function):
    """LearnedSoftMask + fractional-bit STE quantizer of every scale, plus the
    bit budget avg_bits = mean_k mean(bits_k) and (avg_bits - target)^2
    (models/mcaq_yolo.py:572-577, 110-118).  Forward: the soft-mask planes
    (one morph launch), the quantizer (one launch), the bit budget (one
    launch).  Backward: the quantizer (one launch, partials only), then fold +
    soft-mask backward + bit-budget gradient (one launch), the soft-mask
    parameter reduction (one launch).  Per tile the bit-map gradient is
    (c + grad_bits(quantizer)) + grad_bits(soft mask), the order autograd
    sums them in the per-scale step."""

    @staticmethod
    def forward(ctx, mods, n, target, *args):
        ctx.set_materialize_grads(False)
        bits, absmeans, xs, mins, maxs = (args[k * n:(k + 1) * n] for k in range(5))
        L = abi.lib()
        st = _stream()
        blobs = _softmask_blobs(mods)
        morphs = (abi.MorphScale * n)()
        ms, bf = [], []
        for i in range(n):
            b = _f32c(bits[i]).detach()
            bf.append(b)
            B, H, W = absmeans[i].shape
            _, ht, wt = b.shape
            if 4 * ht > H or 4 * wt > W:
                raise NotImplementedError("soft mask on a tile grid finer than 4 pixels per tile")
            m = torch.empty(B, 1, H, W, device=b.device)
            ms.append(m)
            morphs[i] = core._morph_struct(B, H, W, 4, ht, wt, abi.F_SOFTMASK, absmean=absmeans[i], bits_in=b,
                                           smask=blobs[i], m_out=m)
        ema = _PENDING_EMA["args"]
        _PENDING_EMA["args"] = None
        if ema is not None:
            # the quantizers' EMA (+ the mapper's running update) rides on this launch
            segs_e, ne, running, _ = ema
            if running is not None:
                rq, wa, na, cnt, mom = running
                abi.check(L.mcaq_morph_ema(morphs, n, segs_e, ne, ctypes.byref(rq), wa, na, cnt, mom, st),
                          "mcaq_morph_ema")
            else:
                abi.check(L.mcaq_morph_ema(morphs, n, segs_e, ne, None, None, None, 0, 0.0, st), "mcaq_morph_ema")
        else:
            abi.check(L.mcaq_morph(morphs, n, st), "mcaq_morph(soft mask)")
        xs = [_f32c(x) for x in xs]
        arr = (abi.QatScale * n)()
        ys = []
        for i in range(n):
            y = torch.empty_like(xs[i])
            ys.append(y)
            q = core._qat_struct(xs[i], bf[i], ms[i], mins[i], maxs[i])
            q.y = _p(y)
            arr[i] = q
        dev = xs[0].device
        avg = torch.empty((), device=dev)
        loss = torch.empty((), device=dev)
        bp = (abi.P * n)(*[_p(b) for b in bf])
        bn = (abi.I * n)(*[b.numel() for b in bf])
        # the quantizer and the bit budget (one extra workgroup) in one launch
        abi.check(L.mcaq_qat_forward_budget(arr, n, bp, bn, n, float(target), _p(avg), _p(loss), st),
                  "mcaq_qat_forward_budget")
        ctx.mods, ctx.n, ctx.target = mods, n, float(target)
        ctx.save_for_backward(*xs, *bf, *ms, *absmeans, *mins, *maxs, avg)
        return tuple(ys) + (avg, loss)

    @staticmethod
    def backward(ctx, *grads):
        n = ctx.n
        sv = ctx.saved_tensors
        xs, bits, ms, absmeans, mins, maxs = (sv[k * n:(k + 1) * n] for k in range(6))
        avg = sv[6 * n]
        gys, g_avg, g_loss = grads[:n], grads[n], grads[n + 1]
        L = abi.lib()
        st = _stream()
        arr = (abi.QatScale * n)()
        segs = (abi.QatSmaskSeg * n)()
        rsegs = (abi.ReduceSeg * n)()
        gxs, gbs, gflats, keep = [], [], [], []
        # the scales' bit-map gradients back to back in one buffer (a sharded
        # step all-gathers them as they are, _MapperMulti.backward)
        gb_all = torch.empty(sum(b.numel() for b in bits), device=xs[0].device)
        gbo = 0
        for i in range(n):
            x = xs[i]
            B, C, H, W = x.shape
            g = _f32c(gys[i]) if gys[i] is not None else torch.zeros_like(x)
            gx = torch.empty_like(x)
            work = torch.empty(L.mcaq_qat_work_floats(B, C, H, W), device=x.device)
            keep += [g, work]
            q = core._qat_struct(x, bits[i], ms[i], mins[i], maxs[i])
            q.g, q.gx, q.work = _p(g), _p(gx), _p(work)     # gm = gb = NULL: partials only, folded below
            arr[i] = q
            gxs.append(gx)
            _, ht, wt = bits[i].shape
            gb = gb_all[gbo:gbo + B * ht * wt].view(B, ht, wt)
            gbo += B * ht * wt
            gp = torch.empty(L.mcaq_smask_gpart_floats(B), device=x.device)
            gf = torch.empty(core._SM_SIZE, device=x.device)
            keep.append(gp)
            gbs.append(gb)
            gflats.append(gf)
            sg = segs[i]
            sg.P = abi.SmaskParams(*[_p(p.detach()) for p in ctx.mods[i].net.parameters()])
            sg.bits, sg.absmean, sg.qat_work, sg.gbits, sg.gpart = _p(bits[i]), _p(absmeans[i]), _p(work), _p(gb), \
                _p(gp)
            sg.B, sg.C, sg.H, sg.W, sg.ht, sg.wt = B, C, H, W, ht, wt
            r = rsegs[i]
            r.part, r.out, r.nparts, r.stride, r.count, r.accumulate = _p(gp), _p(gf), B, core._SM_SIZE, \
                core._SM_SIZE, 0
        abi.check(L.mcaq_qat_backward(arr, n, st), "mcaq_qat_backward")
        ga = _f32c(g_avg) if g_avg is not None else None
        gl = _f32c(g_loss) if g_loss is not None else None
        bb = abi.BitBudget(_p(avg), _p(ga), _p(gl), ctx.target, n)
        abi.check(L.mcaq_qat_smask_backward_multi(segs, n, ctypes.byref(bb), st), "mcaq_qat_smask_backward_multi")
        # every net's gradients straight into its _GradSink (their .grad), the
        # reduction deferred to the mapper's backward launch; otherwise
        # reduced here and handed to autograd
        sinks = None
        if _PENDING_SM_REDUCE["segs"] is None:
            sinks = core._GradSink.target_all([(ctx.mods[i]._gsink, list(ctx.mods[i].net.parameters()))
                                               for i in range(n)])
        if sinks is not None:
            for i, (gf, acc) in enumerate(sinks):
                rsegs[i].out, rsegs[i].accumulate = _p(gf), acc
            _PENDING_SM_REDUCE["segs"] = (rsegs, n, keep)
            torch.autograd.Variable._execution_engine.queue_callback(_flush_pending_sm_reduce)
            nig = ctx.needs_input_grad
            return (None, None, None) + tuple(gbs[i] if nig[3 + i] else None for i in range(n)) + (None,) * n + \
                tuple(gxs[i] if nig[3 + 2 * n + i] else None for i in range(n)) + (None,) * (2 * n) + \
                (None,) * sum(len(list(m.net.parameters())) for m in ctx.mods)
        abi.check(L.mcaq_train_reduce_multi(rsegs, n, 0, st), "mcaq_train_reduce_multi")
        pgrads = []
        for i in range(n):
            params = list(ctx.mods[i].net.parameters())
            pgrads += [gg if p.requires_grad else None for gg, p in zip(core._split_flat(gflats[i], params), params)]
        nig = ctx.needs_input_grad
        return (None, None, None) + tuple(gbs[i] if nig[3 + i] else None for i in range(n)) + (None,) * n + \
            tuple(gxs[i] if nig[3 + 2 * n + i] else None for i in range(n)) + (None,) * (2 * n) + tuple(pgrads)


class _QATMulti(torch.autograd.Function):
    """Fractional-bit straight-through quantizer x m(p) of every scale: one
    forward launch, one backward launch (+ its fold)."""

    @staticmethod
    def forward(ctx, n, *args):
        xs, bits, ms, mins, maxs = (args[k * n:(k + 1) * n] for k in range(5))
        xs = [_f32c(x) for x in xs]
        bits = [_f32c(b) for b in bits]
        ms = [None if m is None else _f32c(m) for m in ms]
        arr = (abi.QatScale * n)()
        ys = []
        for i in range(n):
            y = torch.empty_like(xs[i])
            ys.append(y)
            q = core._qat_struct(xs[i], bits[i], ms[i], mins[i], maxs[i])
            q.y = _p(y)
            arr[i] = q
        abi.check(abi.lib().mcaq_qat_forward(arr, n, _stream()), "mcaq_qat_forward")
        ctx.n = n
        ctx.has_m = [m is not None for m in ms]
        ctx.save_for_backward(*xs, *bits, *[m for m in ms if m is not None], *mins, *maxs)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *gys):
        n = ctx.n
        sv = ctx.saved_tensors
        xs, bits = sv[:n], sv[n:2 * n]
        nm = sum(ctx.has_m)
        mit = iter(sv[2 * n:2 * n + nm])
        ms = [next(mit) if h else None for h in ctx.has_m]
        mins, maxs = sv[2 * n + nm:3 * n + nm], sv[3 * n + nm:]
        L = abi.lib()
        arr = (abi.QatScale * n)()
        gxs, gbs, gmsl, keep = [], [], [], []
        for i in range(n):
            x = xs[i]
            B, C, H, W = x.shape
            g = _f32c(gys[i]) if gys[i] is not None else torch.zeros_like(x)
            gx = torch.empty_like(x)
            gm = torch.empty(B, H, W, device=x.device) if (ms[i] is not None and ctx.needs_input_grad[1 + 2 * n + i]) \
                else None
            gb = torch.empty(bits[i].shape, device=x.device) if ctx.needs_input_grad[1 + n + i] else None
            work = torch.empty(L.mcaq_qat_work_floats(B, C, H, W), device=x.device)
            keep += [g, work]
            q = core._qat_struct(x, bits[i], ms[i], mins[i], maxs[i])
            q.g, q.gx, q.gm, q.gb, q.work = _p(g), _p(gx), _p(gm), _p(gb), _p(work)
            arr[i] = q
            gxs.append(gx); gbs.append(gb); gmsl.append(None if gm is None else gm.view(ms[i].shape))
        abi.check(L.mcaq_qat_backward(arr, n, _stream()), "mcaq_qat_backward")
        return (None,) + tuple(gxs) + tuple(gbs) + tuple(gmsl) + (None,) * (2 * n)


def multi_ok(hooks, feats):
    """The multi-scale step covers train mode with the fused kernels on one
    device, an unsharded batch and the reference modules (mlp or linear mapper,
    per-channel or per-tensor quantizers).  The mapper and every quantizer
    must be in train mode themselves, as the multi-scale launches assume
    (batch-statistics BatchNorm with running-stat updates, EMA statistics);
    a module frozen with .eval() inside a training hook set takes the
    per-scale modules, which follow each module's own flag."""
    if not (hooks.training and core.FUSED_TRAIN and len(feats) > 1):
        return False
    if not hooks.bit_mapper.training or not all(q.training for q in hooks.quantizers.values()):
        return False
    if not all(torch.is_tensor(f) and f.is_cuda and f.dim() == 4 for f in feats):
        return False
    if len({f.device for f in feats}) != 1 or len(feats) > abi.MCAQ_TRAIN_MAXSEG:
        return False
    # data parallel: every quantizer and the mapper's BatchNorm over ONE group
    pgs = {id(q.process_group) for q in hooks.quantizers.values()}
    if len(pgs) != 1:
        return False
    qpg = next(iter(hooks.quantizers.values())).process_group
    an = hooks.complexity_analyzer
    if any(not core._head_bwd_fits(*core._tile_grid(f.shape[2], f.shape[3], an.grid_size)) for f in feats):
        return False
    if isinstance(hooks.bit_mapper, core.ComplexityToBitMappingNetwork):
        if not hooks.bit_mapper._fusable():
            return False
        if getattr(hooks.bit_mapper.mapping_network[1], "process_group", None) is not qpg:
            return False
    elif qpg is not None:
        return False
    for idx, f in zip(hooks.backbone_out_indices, feats):
        q = hooks.quantizers[str(idx)]
        if q.smooth_transitions and q.soft_mask is not None:
            ht, wt = core._tile_grid(f.shape[2], f.shape[3], an.grid_size)
            if not core._smask_bwd_fits(f.shape[2], f.shape[3], ht, wt):
                return False
    return True


def forward_features(hooks, feats, state):
    """models/mcaq_yolo.py:409-455 in train mode for all scales at once;
    appends one aux entry per scale to state['aux'] and returns the quantized
    maps (or the inputs when state['quantize'] is False)."""
    n = len(feats)
    an, mapper = hooks.complexity_analyzer, hooks.bit_mapper
    idxs = list(hooks.backbone_out_indices)[:n]
    xs = [f.float().contiguous() for f in feats]
    box = []
    qs = [hooks.quantizers[str(i)] for i in idxs]
    smods = [q.soft_mask for q in qs]
    if FUSED_MASK_QAT and state.get("quantize", True) and \
            all(q.smooth_transitions and m is not None for q, m in zip(qs, smods)):
        _prepack(an, smods)          # the step's two blob packs in one launch
    try:
        cs = list(_HeadMulti.apply(an, n, box, *xs, *_cmlp_params(an)))
    finally:
        _flush_prepack()             # normally taken by the pass-1 launch
    if hooks.normalize_complexity:
        for i, c in enumerate(cs):
            B = c.shape[0]
            flat = c.reshape(B, -1)
            lo = torch.quantile(flat, 0.02, dim=1, keepdim=True).unsqueeze(-1)
            hi = torch.quantile(flat, 0.98, dim=1, keepdim=True).unsqueeze(-1)
            cs[i] = ((c - lo) / (hi - lo + 1e-8)).clamp(0.0, 1.0)
    T = state.get("temperature", 1.0)
    quantize = state.get("quantize", True)
    per_quantizer = not (quantize and _ema_multi_ok(qs, xs))
    try:
        if isinstance(mapper, core.ComplexityToBitMappingNetwork):
            ncs = [core._normalize_complexity_shape(c) for c in cs]
            # the mapper's running-statistics update rides on the EMA launch
            mapper._defer_running, mapper._pending_running = not per_quantizer, None
            # batch sharded: the mapper on the global batch, EMA min / max riding along
            mapper._dp = _dp_mapper_inputs(mapper, ncs, box, with_minmax=not per_quantizer)
            bits = list(_MapperMulti.apply(mapper, T, True, n, *ncs, *mapper.mapping_network.parameters()))
        else:
            bits = [mapper(c, T, return_continuous=True) for c in cs]
        return _quantize_multi(hooks, feats, state, n, idxs, xs, box, cs, bits, qs, per_quantizer)
    finally:
        pend = getattr(mapper, "_pending_running", None)
        mapper._defer_running, mapper._pending_running, mapper._dp = False, None, None
        if pend is not None:
            _flush_running(pend)


def _quantize_multi(hooks, feats, state, n, idxs, xs, box, cs, bits, qs, per_quantizer):
    """forward_features after the mapper: EMA statistics, soft masks, the
    quantizers (and the bit budget)."""
    mapper = hooks.bit_mapper
    quantize = state.get("quantize", True)
    if not quantize:
        for i in range(n):
            state.setdefault("aux", []).append({"layer": idxs[i], "complexity": cs[i], "bit_map": bits[i],
                                                "features_q": feats[i]})
        return list(feats)
    mins, maxs = [], []
    for i, x in enumerate(xs):
        if bits[i].dim() != 3 or bits[i].shape[0] != x.shape[0]:
            raise AssertionError(f"Batch size mismatch: {x.shape[0]} vs {bits[i].shape[0]}")
    want = [q.smooth_transitions and q.soft_mask is not None for q in qs]
    fused = FUSED_MASK_QAT and all(want) and n <= abi.MCAQ_TRAIN_MAXSEG
    if not per_quantizer:
        running = getattr(mapper, "_pending_running", None)
        mapper._pending_running = None
        # on the fused path the EMA launch rides on the soft-mask launch
        mins, maxs = _ema_multi(qs, xs, box, running, defer=fused)
    for i, (q, x) in enumerate(zip(qs, xs) if per_quantizer else ()):
        B, C, H, W = x.shape
        p1 = box[i]
        copies = None
        frozen = q._frozen()
        if not frozen:
            copies = q.update_running_stats(x, p1["absmean"], want_copies=q.training,
                                            partials=(p1["pmin"], p1["pmax"]))
        if copies is not None:
            xmin, xmax = copies
        elif q.running_min is not None and (q.training or frozen):
            xmin = q._stats_c(q.running_min, C).clone()
            xmax = q._stats_c(q.running_max, C).clone()
        else:
            xmin, xmax = q.batch_minmax(x, None)
        mins.append(xmin); maxs.append(xmax)
    if fused:
        target = float(getattr(hooks, "target_bits", 4.0))
        try:
            res = _MaskQuantMulti.apply([q.soft_mask for q in qs], n, target, *bits, *[b["absmean"] for b in box],
                                        *feats, *mins, *maxs, *[p for q in qs for p in q.soft_mask.net.parameters()])
        finally:
            _flush_ema()         # normally taken by the soft-mask launch
        ys, budget = list(res[:n]), {"avg_bits": res[n], "loss_bit": res[n + 1], "target": target, "bits": bits}
        for i in range(n):
            state.setdefault("aux", []).append({"layer": idxs[i], "complexity": cs[i], "bit_map": bits[i],
                                                "features_q": ys[i], "_bit_budget": budget})
        return ys
    ms = [None] * n
    if all(want):
        ms = list(_SoftMaskMulti.apply([q.soft_mask for q in qs], n, *bits, *[b["absmean"] for b in box],
                                       *[p for q in qs for p in q.soft_mask.net.parameters()]))
    elif any(want):
        ms = [q.soft_mask(b, x, absmean=p1["absmean"]) if w else None
              for q, b, x, p1, w in zip(qs, bits, xs, box, want)]
    ys = list(_QATMulti.apply(n, *feats, *bits, *ms, *mins, *maxs))
    for i in range(n):
        state.setdefault("aux", []).append({"layer": idxs[i], "complexity": cs[i], "bit_map": bits[i],
                                            "features_q": ys[i]})
    return ys
