"""Launch sequencing for the MCAQ hook path on MI355X.

A step over up to three hook scales (C3/C4/C5) is four kernel launches on one
HIP stream:

    mcaq_stats            HBM pass 1: x -> gray, |x| channel means, min/max partials
    mcaq_morph_finalize   one workgroup per image: phi, complexity, bits, soft
                          mask; plus workgroups reducing the per-channel batch
                          min/max                (+ optional RCCL all-reduce)
    mcaq_quant            HBM pass 2: y = dequant(quant_b(x)) * m

All buffers of a `HookPlan` are allocated once, so `HookPlan.run` only
enqueues launches and can be captured into a HIP graph (torch.cuda.CUDAGraph);
batched throughput comes from several plans' graphs replayed on as many
streams (bench.py Runner).

A launch takes up to abi.MAX_SEGMENTS segments, a segment being one hook scale
of one batch.  `HookPlan(geoms, dev, batches=k)` is a LAUNCH SET: k independent
batches (each with its own input, statistics, outputs and batch_offset /
batch_total, exactly as if run alone) in one launch of each kernel, so every
node of the chain carries k batches of streaming work while the per-image
morphology latency stays that of one image.

Batch-sharded runs (one process per GPU) keep every segment's channel
statistics as [-min | max] in ONE contiguous buffer (`HookPlan.mm`): the
finalize writes the negated min, pass 2 reads it back negated, and the only
operation between them is one in-place MAX all-reduce of that buffer - an RCCL
collective that can be captured inside the step's HIP graph.

This module is the HIP path only: non-CUDA tensors or a missing library
raise here.  CPU tensors take the pure-PyTorch path (fallback.py), which the
modules in core.py / hooks.py dispatch to, as the reference does.
"""
import ctypes

import torch

from . import abi


def tile_size(H, grid_size):
    """morphology.py:359-376: largest power of two <= max(4, H // grid)."""
    raw = max(4, H // grid_size)
    return 1 << (raw.bit_length() - 1)


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("mcaq_yolo_amd runs on MI355X (HIP) only; got a %s tensor" % t.device)


# feature-map element types the kernels read natively (include/mcaq_hip.h
# MCAQ_DTYPE_*): fp32, and the fp16 / bf16 maps an autocast region hands the
# hooks (train.py:582-585, 748-749).  fp16 / bf16 widen exactly in pass 1 and
# pass 2, all arithmetic is fp32 (the analyzer's gray / |x| sums are those of
# x.float(), morphology.py:834-837).  y takes the reference's result type: the
# input's dtype, or fp32 where the fp32 soft mask multiplies it
# (quantization.py:742-744 promotes fp16 * fp32 to fp32).
_DTYPES = {torch.float32: abi.DTYPE_F32, torch.float16: abi.DTYPE_F16, torch.bfloat16: abi.DTYPE_BF16}


def half_native_ok(geom, min_bits=2.0, max_bits=8.0):
    """True when pass 2 takes an fp16 / bf16 map of this geometry natively
    (the tile-aligned kernel: the map a power-of-two multiple of the tile
    grid, tiles >= 4 pixels wide, H*W % 4 == 0, <= 1024 tiles, <= 8 widths);
    otherwise callers quantize x.float()."""
    def pow2_mult(n, t):
        k = 0
        while (t << k) < n:
            k += 1
        return (t << k) == n, k
    okh, _ = pow2_mult(geom.H, geom.ht)
    okw, sw = pow2_mult(geom.W, geom.wt)
    return okh and okw and sw >= 2 and (geom.H * geom.W) % 4 == 0 and geom.ht * geom.wt <= 1024 and \
        int(max_bits) - int(min_bits) + 1 <= 8


def _stream_handle(stream):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


# Pass A of the morphology as band + edge workgroups (csrc/mcaq_band.h) for
# every scale that supports it.  Bit-identical to the per-image pass A, but
# measured slower in the pipelined step (r04: 66.4-67.2 vs 62.2-62.8 us per
# step at config 2, profiles/r04_morph/): its 16-row bands run ~30 us each
# on 1-4 waves per SIMD, so its CU-time is no lower.  Off by default.
BAND_PASS = False

# Pass B of the morphology as batch-wide tile kernels (csrc/mcaq_tiles_batch.h)
# wherever the flags allow it.  Bit-identical to the per-image pass B but
# measured slower in the pipelined step (r04, bench --pass-b, 3 interleaved
# rounds: 502-507 k vs 518-530 k img/s at config 2, profiles/r04_passb/):
# off by default; True for A/B and the cross-check tests.
TILES_BATCH = False


class ScaleGeom:
    """Shape bookkeeping for one hook scale."""

    def __init__(self, B, C, H, W, grid_size):
        self.B, self.C, self.H, self.W, self.grid = B, C, H, W, grid_size
        self.tile = tile_size(H, grid_size)
        self.ht, self.wt = H // self.tile, W // self.tile
        self.Hc, self.Wc = self.ht * self.tile, self.wt * self.tile
        if self.ht < 1 or self.wt < 1:
            raise ValueError("feature map %dx%d smaller than one %d-pixel tile" % (H, W, self.tile))
        if self.tile > 128:
            raise ValueError("tile %d > 128 not supported (H=%d, grid=%d)" % (self.tile, H, grid_size))

    @property
    def key(self):
        return (self.B, self.C, self.H, self.W, self.grid)


class HookPlan:
    """Buffers + launch descriptors for a fixed set of hook-scale shapes.

    want: subset of {"phi", "cmlp", "debug"} extra outputs.
    batches: independent batches of those shapes per launch (a launch set);
    segment j is scale j // batches of batch j % batches (scale-major, so the
    heaviest scale's segments start first in pass 1)."""

    def __init__(self, geoms, device, want=(), batches=1):
        nbat = int(batches)
        if nbat < 1 or not 1 <= len(geoms) or len(geoms) * nbat > abi.MAX_SEGMENTS:
            raise ValueError("1..%d segments (scales x batches) per launch, got %d x %d"
                             % (abi.MAX_SEGMENTS, len(geoms), nbat))
        self.scale_geoms = list(geoms)
        self.batches = nbat
        self.seg = [(si, k) for si in range(len(geoms)) for k in range(nbat)]
        self.geoms = [geoms[si] for si, _ in self.seg]
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("HookPlan needs a CUDA (HIP) device")
        self.lib = abi.lib()
        d = self.device
        self.bufs = []
        # planes in global memory for every scale when one scale's planes
        # exceed the LDS budget (the mode is common to a launch's scales)
        glob = any(self.lib.mcaq_morph_scratch_bytes(g.B, g.Hc, g.Wc, g.ht, g.wt) for g in self.geoms)
        # channel statistics of every segment in one buffer: [min | max] per
        # segment, or [-min | max] when the plan runs batch-sharded (one MAX
        # all-reduce of the whole buffer makes them global)
        self.mm = torch.empty(2 * sum(g.C for g in self.geoms), device=d)
        self._neg = False
        mo = 0
        for g in self.geoms:
            units = self.lib.mcaq_stats_units(g.B, g.C, g.H, g.W)
            nb = {}
            nb["units"] = units
            nb["gray"] = torch.empty(g.B, g.Hc, g.Wc, device=d)
            nb["absmean"] = torch.empty(g.B, g.H, g.W, device=d)
            nb["pmin"] = torch.empty(units, g.C, device=d)
            nb["pmax"] = torch.empty(units, g.C, device=d)
            nb["xmin"] = self.mm[mo:mo + g.C]           # holds -min in sharded runs
            nb["xmax"] = self.mm[mo + g.C:mo + 2 * g.C]
            mo += 2 * g.C
            nb["complexity"] = torch.empty(g.B, g.ht, g.wt, device=d)
            nb["bits"] = torch.empty(g.B, g.ht, g.wt, device=d)
            nb["mt"] = torch.empty(g.B, g.ht, g.wt, device=d)          # soft-mask tile values
            nb["m"] = torch.empty(g.B, 1, g.H, g.W, device=d) if "debug" in want else None
            nb["y"] = torch.empty(g.B, g.C, g.H, g.W, device=d)
            nb["phi"] = torch.empty(g.B, g.ht, g.wt, 8, device=d)
            nb["tile_tmp"] = torch.empty(g.B, g.ht * g.wt, 32, device=d)   # pass A -> pass B of mcaq_morph
            nb["cmlp"] = torch.empty(g.B, g.ht, g.wt, device=d) if "cmlp" in want else None
            if "debug" in want:
                nb["edge"] = torch.empty(g.B, g.Hc, g.Wc, device=d, dtype=torch.uint8)
                nb["binmask"] = torch.empty(g.B, g.Hc, g.Wc, device=d, dtype=torch.uint8)
            else:
                nb["edge"] = nb["binmask"] = None
            sb = self.lib.mcaq_morph_scratch_bytes_global(g.B, g.Hc, g.Wc) if glob else 0
            nb["gscratch"] = torch.empty(max(sb, 16), device=d, dtype=torch.uint8) if sb else None
            # pass A in band mode (NMS plane + per-band Otsu histograms); 0 bytes:
            # the scale keeps the per-image pass A
            wb = 0 if not BAND_PASS else self.lib.mcaq_morph_work_bytes(g.B, g.Hc, g.Wc, g.tile)
            nb["pwork"] = torch.empty(wb // 4, device=d) if wb else None
            self.bufs.append(nb)

    # ------------------------------------------------------------------
    def batch_bufs(self, k=0):
        """Buffer dicts of batch k, in scale order."""
        return [b for b, (_, kk) in zip(self.bufs, self.seg) if kk == k]

    def channel_minmax(self, j):
        """(min, max) of segment j as the quantizer used them."""
        b = self.bufs[j]
        return (-b["xmin"] if self._neg else b["xmin"]), b["xmax"]

    def run(self, feats, cmlp, mapper, smasks, stream=None, process_group=None, **kw):
        """Enqueue one step (prepare + launch).  feats: list of (B,C,H,W) fp32
        (or fp16 / bf16, see half_native_ok) CUDA tensors matching the plan
        (batches > 1: one such list per batch).
        cmlp/mapper: packed blobs (CUDA fp32); smasks: one packed soft-mask
        blob per scale or None (smooth_transitions=False).  Keyword options:
        see prepare().  Returns the buffer dicts (overwritten by the next run)."""
        kw.setdefault("shared_stats", process_group is not None)
        self.prepare(feats, cmlp, mapper, smasks, **kw)
        self.launch(stream, process_group)
        return self.bufs

    def prepare(self, feats, cmlp, mapper, smasks, temperature=1.0, mapper_kind="mlp", continuous=False,
                normalize=False, minmax=None, batch_offset=0, batch_total=None, binarize_otsu=False,
                contour_components=True, canny_legacy=False, min_bits=2.0, max_bits=8.0, quantize=True, hysteresis_iters=8,
                per_tensor=False, softmax_threads=None, m_plane=False, shared_stats=False):
        """Validate inputs and build the launch descriptors (pointers are baked
        in: the tensors must stay alive and in place until the last launch).
        A call with the same blobs, buffers and options as the previous one
        only rebinds x and the y / complexity / bits outputs.
        minmax: optional per-scale (xmin, xmax) frozen calibration stats.
        per_tensor: one batch min/max over all channels (per_channel=False,
        quantization.py:655-661), broadcast to the C entries the kernel reads.
        softmax_threads: thread count of the CPU reference whose soft-mask
        softmax is reproduced bit for bit (ATen picks SLEEF or glibc exp per
        tile by its thread partition); default torch.get_num_threads().
        m_plane: pass B writes the soft-mask plane m(p) and pass 2 reads it,
        instead of pass 2 regenerating m(p) from the tile values per channel
        slice (+4 B per pixel written, +4 B per pixel per slice read).
        shared_stats: the statistics of a batch-sharded run - the finalize
        writes [-min | max] into `mm` and pass 2 reads the min negated, so
        launch(process_group=...) combines them with ONE in-place all-reduce.
        With batches > 1, feats is one list per batch; smasks and minmax are
        per scale and shared by the batches."""
        ns = len(self.scale_geoms)
        if self.batches > 1:
            if len(feats) != self.batches or any(len(fb) != ns for fb in feats):
                raise ValueError("expected %d batches of %d feature maps" % (self.batches, ns))
            feats = [feats[k][si] for si, k in self.seg]
        if len(smasks) != ns:
            raise ValueError("expected %d soft-mask blobs" % ns)
        smasks = [smasks[si] for si, _ in self.seg]
        if minmax is not None:
            if len(minmax) != ns:
                raise ValueError("expected %d minmax entries" % ns)
            minmax = [minmax[si] for si, _ in self.seg]
        n = len(self.geoms)
        L = self.lib
        if m_plane:
            for g, b in zip(self.geoms, self.bufs):
                if b["m"] is None:
                    b["m"] = torch.empty(g.B, 1, g.H, g.W, device=self.device)
        if len(feats) != n:
            raise ValueError("expected %d feature maps" % n)
        for f, g in zip(feats, self.geoms):
            _require_cuda(f)
            if f.dtype not in _DTYPES or not f.is_contiguous() or tuple(f.shape) != (g.B, g.C, g.H, g.W):
                raise ValueError("feature map must be contiguous fp32 / fp16 / bf16 %s, got %s %s"
                                 % ((g.B, g.C, g.H, g.W), tuple(f.shape), f.dtype))
        dtype = feats[0].dtype
        if any(f.dtype != dtype for f in feats):
            raise ValueError("one feature-map dtype per launch, got %s" % sorted({str(f.dtype) for f in feats}))
        if dtype != torch.float32:
            if m_plane or not all(half_native_ok(g, min_bits, max_bits) for g in self.geoms):
                raise ValueError("%s feature maps need the tile-aligned quantizer (engine.half_native_ok)" % dtype)
        ydt = [torch.float32 if (sm is not None and quantize) else dtype for sm in smasks]
        for b, g, yd in zip(self.bufs, self.geoms, ydt):
            if b["y"].dtype != yd:          # y in the reference's result type
                b["y"] = torch.empty(g.B, g.C, g.H, g.W, device=self.device, dtype=yd)
        # descriptor reuse: an eager hook calls prepare once per forward with
        # new x / output tensors and otherwise the same blobs, buffers and
        # options; then only those pointers are patched into the structs
        sig = self._signature(cmlp, mapper, smasks, minmax, (
            float(temperature if temperature is not None else 1.0), mapper_kind, bool(continuous), bool(normalize),
            int(batch_offset), batch_total, bool(binarize_otsu), bool(contour_components), bool(canny_legacy),
            float(min_bits), float(max_bits), bool(quantize), int(hysteresis_iters), bool(per_tensor),
            int(softmax_threads) if softmax_threads else torch.get_num_threads(), bool(m_plane),
            bool(shared_stats), str(dtype)))
        if sig is not None and sig == getattr(self, "_sig", None):
            self._rebind(feats)
            self._keep = (list(feats), cmlp, mapper, list(smasks), minmax)
            return
        self._sig = None
        self._keep = (list(feats), cmlp, mapper, list(smasks), minmax)
        self._neg = bool(shared_stats) and quantize
        with_mask = [sm is not None for sm in smasks]
        # ---- pass 1
        st = (abi.StatsScale * n)()
        for i, (f, g, b) in enumerate(zip(feats, self.geoms, self.bufs)):
            s = st[i]
            s.x = _p(f)
            s.gray = _p(b["gray"])
            s.absmean = _p(b["absmean"]) if with_mask[i] else None
            need_mm = quantize and (minmax is None or minmax[i] is None)
            s.pmin = _p(b["pmin"]) if need_mm else None
            s.pmax = _p(b["pmax"]) if need_mm else None
            s.B, s.C, s.H, s.W, s.Hc, s.Wc = g.B, g.C, g.H, g.W, g.Hc, g.Wc
            s.dtype = _DTYPES[dtype]
        self._st = st
        self._fz = self._qs = None
        # ---- channel min/max
        if quantize:
            fz = (abi.FinalizeScale * n)()
            for i, (g, b) in enumerate(zip(self.geoms, self.bufs)):
                s = fz[i]
                s.C, s.nunits, s.min_stride = g.C, b["units"], 1
                s.per_tensor = 1 if per_tensor else 0
                s.neg_min = 1 if self._neg else 0
                s.min_out, s.max_out = _p(b["xmin"]), _p(b["xmax"])
                if minmax is not None and minmax[i] is not None:
                    lo, hi = minmax[i]
                    _require_cuda(lo, hi)
                    lo = lo.float().contiguous().reshape(-1)
                    hi = hi.float().contiguous().reshape(-1)
                    self._keep += (lo, hi)
                    s.min_in, s.max_in = _p(lo), _p(hi)
                    if lo.numel() == 1:
                        s.min_stride = 0
                else:
                    s.pmin, s.pmax = _p(b["pmin"]), _p(b["pmax"])
            self._fz = fz
        # ---- morph
        mo = (abi.MorphScale * n)()
        flags = abi.F_PHI | abi.F_CMLP | abi.F_MAPPER | abi.F_HAS_T
        if continuous:
            flags |= abi.F_CONT
        if normalize:
            flags |= abi.F_NORM_C
        if mapper_kind == "linear":
            flags |= abi.F_MAP_LINEAR
        if binarize_otsu:
            flags |= abi.F_BIN_OTSU
        if not contour_components:
            flags |= abi.F_NO_EULER
        if canny_legacy:
            flags |= abi.F_CANNY_LEGACY
        T = max(float(temperature if temperature is not None else 1.0), 0.1)
        for i, (g, b) in enumerate(zip(self.geoms, self.bufs)):
            s = mo[i]
            s.gray, s.absmean = _p(b["gray"]), _p(b["absmean"])
            s.cmlp, s.mapper = _p(cmlp), _p(mapper) if mapper is not None else None
            s.smask = _p(smasks[i]) if with_mask[i] else None
            s.phi_out, s.cmlp_out = _p(b["phi"]), _p(b["cmlp"])
            s.c_out, s.bits_out = _p(b["complexity"]), _p(b["bits"])
            s.m_out = _p(b["m"]) if (with_mask[i] and quantize) else None
            s.mt_out = _p(b["mt"]) if (with_mask[i] and quantize) else None
            s.edge_out, s.bin_out = _p(b["edge"]), _p(b["binmask"])
            s.gscratch = _p(b["gscratch"])
            s.pwork = _p(b["pwork"])
            s.tile_tmp = _p(b["tile_tmp"])
            s.B, s.H, s.W, s.Hc, s.Wc = g.B, g.H, g.W, g.Hc, g.Wc
            s.tile, s.ht, s.wt = g.tile, g.ht, g.wt
            s.batch_offset = batch_offset
            s.batch_total = batch_total if batch_total is not None else g.B
            s.flags = flags | (abi.F_SOFTMASK if (with_mask[i] and quantize) else 0) | \
                (0 if TILES_BATCH else abi.F_TILES_IMAGE)
            s.hyst_iters = hysteresis_iters
            s.softmax_threads = int(softmax_threads) if softmax_threads else torch.get_num_threads()
            s.temperature, s.min_bits, s.max_bits = T, float(min_bits), float(max_bits)
        self._mo = mo
        # ---- pass 2
        if quantize:
            qs = (abi.QuantScale * n)()
            lo_b = int(min_bits)
            nb = int(max_bits) - lo_b + 1
            for i, (f, g, b) in enumerate(zip(feats, self.geoms, self.bufs)):
                s = qs[i]
                s.x, s.y, s.bits = _p(f), _p(b["y"]), _p(b["bits"])
                if with_mask[i] and m_plane:
                    s.m = _p(b["m"])                              # m(p) plane written by pass B
                else:
                    s.mt = _p(b["mt"]) if with_mask[i] else None  # m(p) generated in the quant pass
                s.xmin, s.xmax = _p(b["xmin"]), _p(b["xmax"])
                s.B, s.C, s.H, s.W, s.ht, s.wt = g.B, g.C, g.H, g.W, g.ht, g.wt
                s.bits_lo, s.nbits = lo_b, nb
                # batch statistics of this x (pass 1 + finalize, all-reduced or not)
                s.stats_cover_x = 1 if (minmax is None or minmax[i] is None) else 0
                s.neg_min = 1 if self._neg else 0
                s.dtype = _DTYPES[dtype]
                s.ydtype = _DTYPES[b["y"].dtype]
            self._qs = qs
        self._n = n
        self._sig = sig

    # pointers rebound per call (the eager hook hands out fresh outputs)
    _REBOUND = ("y", "complexity", "bits")

    def _signature(self, cmlp, mapper, smasks, minmax, opts):
        """Everything the descriptors depend on except x and the rebound
        outputs; None (never reused) when a frozen min/max would be copied."""
        def ptr(t):
            return None if t is None else t.data_ptr()
        mm = None
        if minmax is not None:
            mm = []
            for e in minmax:
                if e is None:
                    mm.append(None)
                    continue
                lo, hi = e
                if not all(t.dtype == torch.float32 and t.is_contiguous() for t in (lo, hi)):
                    return None
                mm.append((lo.data_ptr(), hi.data_ptr(), lo.numel()))
            mm = tuple(mm)
        bufs = tuple(tuple(ptr(v) if torch.is_tensor(v) else v for k, v in sorted(b.items()) if k not in self._REBOUND)
                     for b in self.bufs)
        return (ptr(cmlp), ptr(mapper), tuple(ptr(s) for s in smasks), mm, opts, bufs)

    def _rebind(self, feats):
        for i, (f, b) in enumerate(zip(feats, self.bufs)):
            self._st[i].x = _p(f)
            self._mo[i].c_out, self._mo[i].bits_out = _p(b["complexity"]), _p(b["bits"])
            if self._qs is not None:
                q = self._qs[i]
                q.x, q.y, q.bits = _p(f), _p(b["y"]), _p(b["bits"])

    def launch_stats(self, stream=None):
        """Pass 1 only."""
        abi.check(self.lib.mcaq_stats(self._st, self._n, _stream_handle(stream)), "mcaq_stats")

    def launch_morph(self, stream=None):
        """Morphology passes A + B (+ the channel min/max reduction); needs pass 1."""
        nf = self._n if self._fz is not None else 0
        abi.check(self.lib.mcaq_morph_finalize(self._mo, self._n, self._fz, nf, _stream_handle(stream)),
                  "mcaq_morph_finalize")

    def launch_pre(self, stream=None):
        """Pass 1 + morphology (+ the channel min/max reduction)."""
        self.launch_stats(stream)
        self.launch_morph(stream)

    def launch_quant(self, stream=None):
        """Pass 2."""
        if self._qs is not None:
            abi.check(self.lib.mcaq_quant(self._qs, self._n, _stream_handle(stream)), "mcaq_quant")

    def launch(self, stream=None, process_group=None):
        """Enqueue the prepared step on `stream` (default: current stream).
        With a process group (batch sharded over ranks) the per-channel min/max
        of every segment is combined by ONE all-reduce so the quantizer sees
        the global-batch statistics of the reference: in place on `mm` when
        the plan was prepared with shared_stats (no other op, capturable in a
        HIP graph with the nccl / RCCL backend), else through
        sync_channel_minmax."""
        L = self.lib
        n = self._n
        sh = _stream_handle(stream)
        abi.check(L.mcaq_stats(self._st, n, sh), "mcaq_stats")
        # the channel min/max reduction rides along as extra workgroups of the
        # morph launch (the per-image workgroups leave most CUs idle)
        nf = n if self._fz is not None else 0
        abi.check(L.mcaq_morph_finalize(self._mo, n, self._fz, nf, sh), "mcaq_morph_finalize")
        if self._fz is not None and process_group is not None:
            self.allreduce_stats(process_group, stream)
        if self._qs is not None:
            abi.check(L.mcaq_quant(self._qs, n, sh), "mcaq_quant")
        return self.bufs

    def allreduce_stats(self, process_group, stream=None):
        """The collective between the finalize (which writes the statistics)
        and pass 2 (which reads them), on the launch stream."""
        with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream()):
            if self._neg:
                import torch.distributed as dist
                dist.all_reduce(self.mm, op=dist.ReduceOp.MAX, group=process_group)
            else:
                sync_channel_minmax(self.bufs, process_group)


def sync_channel_minmax(bufs, process_group):
    """Exact global-batch channel min/max across ranks with one all-reduce:
    pack [-min_s, max_s] for every scale, reduce with MAX, unpack."""
    import torch.distributed as dist
    vec = torch.cat([t for b in bufs for t in (-b["xmin"], b["xmax"])])
    dist.all_reduce(vec, op=dist.ReduceOp.MAX, group=process_group)
    o = 0
    for b in bufs:
        C = b["xmin"].numel()
        b["xmin"].copy_(-vec[o:o + C])
        b["xmax"].copy_(vec[o + C:o + 2 * C])
        o += 2 * C
