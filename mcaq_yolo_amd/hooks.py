"""The MCAQ forward hook (models/mcaq_yolo.py:402-473) on the fused HIP path.

`MCAQHooks` owns the hot-path modules under the reference's attribute names
(`complexity_analyzer`, `bit_mapper`, `quantizers[str(idx)]`), so a reference
MCAQYOLO state_dict restricted to those prefixes loads into it, and speaks
the reference's hook protocol: the shared `_mcaq_state` dict with keys
`active`, `temperature`, `quantize`, `calibrating`, `aux`; each hook appends
`{layer, complexity, bit_map, features_q}` to `aux` and returns the quantized
map (replacing the layer output) or None.

Inference calls go through one `HookPlan` per feature shape: 3 launches
(pass 1, morphology + channel min/max, pass 2) instead of the reference's
analyzer -> mapper -> soft mask -> quantizer chain.  Calibration
(`calibrating=True`) first folds the batch min/max into the quantizer's EMA
statistics (quantization.py:319-353), then quantizes like inference.
Train mode (QAT) and CPU tensors (the pure-PyTorch path) run the modules one
by one with autograd (`_run_scale_modules`), exactly as the reference hook.
"""
import torch
import torch.nn as nn

from .core import (ComplexityToBitMappingNetwork, LinearBitMapper, MorphologicalComplexityAnalyzer,
                   SpatialAdaptiveQuantization)
from . import core, engine, train_step
from .engine import HookPlan, ScaleGeom

DEFAULT_INDICES = (4, 6, 9)   # models/mcaq_yolo.py:361 fallback (C3/C4/C5 of YOLOv8)

# Train mode (QAT) through forward_features, fastest first:
#  * MULTI_SCALE_TRAIN: every stage once for all scales (train_step.py: one
#    launch per stage with per-scale segments, one stream) - values equal the
#    per-scale path's (tests/test_train_multi_gpu.py);
#  * CONCURRENT_TRAIN_SCALES: the per-scale modules, each scale's chain of
#    launches (and, through autograd's stream semantics, its backward) on its
#    own HIP stream; the state the scales share is ordered by
#    core.concurrent_scales (tests/test_concurrent_scales_gpu.py).  Captured
#    in a HIP graph this is a multi-stream graph, which ROCm issues node by
#    node (tools/probe/graph_replay_probe.py), so it is the second choice;
#  * else one stream, scale after scale.
MULTI_SCALE_TRAIN = True
CONCURRENT_TRAIN_SCALES = True


class MCAQHooks(nn.Module):
    def __init__(self, grid_size=8, min_bits=2, max_bits=8, bit_mapping="mlp", normalize_complexity=False,
                 device="cuda", indices=DEFAULT_INDICES):
        super().__init__()
        self.complexity_analyzer = MorphologicalComplexityAnalyzer(grid_size=grid_size, device=device)
        if bit_mapping == "mlp":
            self.bit_mapper = ComplexityToBitMappingNetwork(min_bits=min_bits, max_bits=max_bits)
        elif bit_mapping == "linear":
            self.bit_mapper = LinearBitMapper(min_bits=min_bits, max_bits=max_bits)
        else:
            raise ValueError("bit_mapping must be 'mlp' or 'linear'")
        self.bit_mapping = bit_mapping
        self.normalize_complexity = normalize_complexity
        self.quantizers = nn.ModuleDict()
        self.backbone_out_indices = list(indices)
        for idx in self.backbone_out_indices:
            self.quantizers[str(idx)] = SpatialAdaptiveQuantization(calibration_mode="minmax",
                                                                    smooth_transitions=True, per_channel=True)
        self._mcaq_state = {"active": False}
        # batch-sharded inference (one process per GPU): the per-channel batch
        # min/max is made global by one all-reduce per hook, and the fractal
        # regression's reduction order follows the image's global batch index
        self.process_group = None
        self.batch_offset, self.batch_total = 0, None
        # thread count of the CPU reference run whose soft-mask softmax the
        # kernels reproduce bit for bit (ATen's exp per tile follows its thread
        # partition); None = torch.get_num_threads() at each call,
        # an int pins it (results then independent of this process's threads)
        self.softmax_threads = None
        # bit budget target of the QAT loss (MCAQYOLO.target_bits, models/
        # mcaq_yolo.py:70-77, 333; the curriculum sets it per stage)
        self.target_bits = 4.0
        self._handles = []
        self._plans = {}
        # buffer set of the per-shape HookPlans: steps captured into HIP graphs
        # that run concurrently (batches in flight on several streams) each
        # take their own slot, so they never share the hook's device buffers
        self.plan_slot = 0
        if str(device).startswith("cuda") and torch.cuda.is_available():
            self.to(device)

    # -- registration (models/mcaq_yolo.py:459-473)
    def register(self, layers):
        """Attach one forward hook per backbone index to `layers` (a list /
        nn.Sequential of the detector's modules)."""
        layers = list(layers)
        for idx in self.backbone_out_indices:
            if 0 <= idx < len(layers):
                self._handles.append(layers[idx].register_forward_hook(self.make_hook(idx)))
        return self

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []

    def begin(self, temperature=1.0, quantize=True, calibrating=False):
        """Open a forward (models/mcaq_yolo.py:556-561); returns the aux list."""
        self._mcaq_state = {"active": True, "temperature": temperature, "quantize": quantize,
                            "calibrating": calibrating, "aux": []}
        return self._mcaq_state["aux"]

    def end(self):
        aux = self._mcaq_state.get("aux", [])
        self._mcaq_state = {"active": False}
        return aux

    @staticmethod
    def _budget(aux):
        """The bit budget the multi-scale train step computed with these bit
        maps (train_step._MaskQuantMulti), if aux is exactly that step's."""
        b = aux[0].get("_bit_budget") if aux else None
        if b is None or len(aux) != len(b["bits"]):
            return None
        if any(a.get("_bit_budget") is not b or a["bit_map"] is not m for a, m in zip(aux, b["bits"])):
            return None
        return b

    @staticmethod
    def avg_bits(aux):
        """models/mcaq_yolo.py:572-577: mean over scales of each bit map's mean.
        After a multi-scale train step the value its bit-budget launch
        computed (same definition, a fixed-order device reduction; its
        gradient is folded into that step's backward launch)."""
        if not aux:
            return None
        b = MCAQHooks._budget(aux)
        if b is not None:
            return b["avg_bits"]
        return torch.stack([a["bit_map"].float().mean() for a in aux]).mean()

    def bit_budget_loss(self, aux, target_bits=None):
        """MCAQLoss.compute_bit_budget_loss (models/mcaq_yolo.py:110-118):
        (avg_bits - target)^2, target default self.target_bits.  After a
        multi-scale train step run with that target: its fused value."""
        t = float(self.target_bits if target_bits is None else target_bits)
        b = MCAQHooks._budget(aux)
        if b is not None and b["target"] == t:
            return b["loss_bit"]
        return (MCAQHooks.avg_bits(aux) - t) ** 2

    # -- the hook body (models/mcaq_yolo.py:409-455)
    def make_hook(self, layer_idx):
        def hook(module, inputs, output):
            state = self._mcaq_state
            if not state.get("active", False):
                return None
            if not torch.is_tensor(output) or output.dim() != 4:
                return None
            return self.run_scale(layer_idx, output, state)
        return hook

    def _plan(self, feat):
        key = (tuple(feat.shape), feat.device, self.complexity_analyzer.grid_size, self.plan_slot)
        plan = self._plans.get(key)
        if plan is None:
            plan = HookPlan([ScaleGeom(*feat.shape, self.complexity_analyzer.grid_size)], feat.device)
            self._plans[key] = plan
        return plan

    def _run_scale_modules(self, layer_idx, feat, state):
        """models/mcaq_yolo.py:409-455 module by module: train mode (QAT,
        BASELINE config 5: analyzer with autograd into complexity_mlp,
        continuous bits from the train-mode mapper, fractional-bit STE
        quantizer on the HIP kernels) and every CPU tensor (the pure-PyTorch
        path, BASELINE config 1)."""
        B = feat.shape[0]
        bt = self.batch_total
        if not self.training and not feat.is_cuda and bt is not None and bt > B:
            return self._run_scale_shard_cpu(layer_idx, feat, state)
        if feat.is_cuda:
            with core.pass1_sharing():
                return self._run_scale_modules_body(layer_idx, feat, state)
        return self._run_scale_modules_body(layer_idx, feat, state)

    def _run_scale_modules_body(self, layer_idx, feat, state):
        complexity = self.complexity_analyzer(feat)
        if self.normalize_complexity:
            B = complexity.shape[0]
            flat = complexity.reshape(B, -1)
            lo = torch.quantile(flat, 0.02, dim=1, keepdim=True).unsqueeze(-1)
            hi = torch.quantile(flat, 0.98, dim=1, keepdim=True).unsqueeze(-1)
            complexity = ((complexity - lo) / (hi - lo + 1e-8)).clamp(0.0, 1.0)
        bit_map = self.bit_mapper(complexity, state.get("temperature", 1.0), return_continuous=self.training)
        quantize = state.get("quantize", True)
        quantizer = self.quantizers[str(layer_idx)]
        q_training = self.training or state.get("calibrating", False)
        feat_q = quantizer(feat, bit_map, training=q_training) if quantize else feat
        state.setdefault("aux", []).append({"layer": layer_idx, "complexity": complexity,
                                            "bit_map": bit_map, "features_q": feat_q})
        return feat_q if quantize else None

    def _run_scale_shard_cpu(self, layer_idx, feat, state):
        """A batch shard on the pure-PyTorch path (inference / calibration).
        Several CPU ATen results depend on a value's position in the WHOLE
        batch, not only on the image: the fractal regression's outer sums
        over the scales (a tile's global column picks the vectorised or the
        row_sum order, morphology.py:614-620), the vector-body / scalar-tail
        split of SLEEF log / log2 / exp and the softmax thread partition
        (SURVEY App. A.1, A.6), and oneDNN vs MKL for single-image 3x3
        convolutions (A.2).  So the shard runs on a tensor of the global batch
        shape: rows batch_offset .. batch_offset + B - 1 hold this shard's
        images and the other rows repeat them (which leaves the shard's
        channel min/max unchanged; the process group's all-reduce then makes
        it global).  The shard's rows of every output are exactly those of
        the single-process run on the global batch, at world_size x the CPU
        work of the shard."""
        B = feat.shape[0]
        off, bt = self.batch_offset, self.batch_total
        if not 0 <= off <= bt - B:
            raise ValueError("batch_offset %d + shard %d exceeds batch_total %d" % (off, B, bt))
        rows = (torch.arange(bt) - off) % B
        sub = {"temperature": state.get("temperature", 1.0), "quantize": state.get("quantize", True),
               "calibrating": state.get("calibrating", False), "aux": []}
        saved = self.batch_total
        self.batch_total = None
        try:
            out = self._run_scale_modules(layer_idx, feat.index_select(0, rows.to(feat.device)), sub)
        finally:
            self.batch_total = saved
        a = sub["aux"][0]
        sl = slice(off, off + B)
        feat_q = a["features_q"][sl] if state.get("quantize", True) else feat
        state.setdefault("aux", []).append({"layer": layer_idx, "complexity": a["complexity"][sl],
                                            "bit_map": a["bit_map"][sl], "features_q": feat_q})
        return feat_q if out is not None else None

    def run_scale(self, layer_idx, feat, state):
        if self.training or not feat.is_cuda:
            return self._run_scale_modules(layer_idx, feat, state)
        quantize = state.get("quantize", True)
        quantizer = self.quantizers[str(layer_idx)]
        # fp16 / bf16 maps (an autocast region) are read natively by pass 1 and
        # pass 2 (fp32 arithmetic, y in the input's dtype) where the quantizer's
        # tile-aligned kernel takes the shape; otherwise quantized as x.float()
        half = feat.dtype in (torch.float16, torch.bfloat16)
        x = feat.contiguous() if half else feat.float().contiguous()
        plan = self._plan(x)
        if half and not all(engine.half_native_ok(g, self.bit_mapper.min_bits, self.bit_mapper.max_bits)
                            for g in plan.geoms):
            x = x.float()
        if state.get("calibrating", False) and quantize:
            quantizer.update_running_stats(x.float())
        b = plan.bufs[0]
        for k in ("y", "complexity", "bits"):      # fresh outputs: the caller keeps them
            b[k] = torch.empty_like(b[k])
        minmax = None
        if quantizer._frozen() and quantizer.running_min is not None:
            minmax = [(quantizer.running_min.reshape(-1), quantizer.running_max.reshape(-1))]
        an = self.complexity_analyzer
        sm = quantizer.soft_mask.blob() if (quantizer.smooth_transitions and quantizer.soft_mask is not None) \
            else None
        mapper_blob = self.bit_mapper.mapper_blob() if self.bit_mapping == "mlp" else None
        plan.run([x], an.cmlp_blob(), mapper_blob, [sm], temperature=state.get("temperature", 1.0),
                 mapper_kind=self.bit_mapping, normalize=self.normalize_complexity, minmax=minmax,
                 binarize_otsu=an.binarize_impl == "otsu", contour_components=an.contour_components,
                 canny_legacy=an.canny_impl == "legacy", min_bits=self.bit_mapper.min_bits, max_bits=self.bit_mapper.max_bits, quantize=quantize,
                 per_tensor=not quantizer.per_channel, softmax_threads=self.softmax_threads, process_group=self.process_group if minmax is None else None,
                 batch_offset=self.batch_offset, batch_total=self.batch_total)
        feat_q = b["y"] if quantize else feat
        state.setdefault("aux", []).append({"layer": layer_idx, "complexity": b["complexity"],
                                            "bit_map": b["bits"], "features_q": feat_q})
        return feat_q if quantize else None

    def forward_features(self, feats, temperature=1.0, quantize=True):
        """Run the hook body directly on a list of (C3, C4, C5) feature maps
        (one per backbone index); returns (quantized maps, aux).  In train mode
        on the GPU the scales run on concurrent streams (CONCURRENT_TRAIN_SCALES)."""
        aux = self.begin(temperature=temperature, quantize=quantize)
        if MULTI_SCALE_TRAIN and train_step.multi_ok(self, feats):
            outs = train_step.forward_features(self, feats, self._mcaq_state)
        elif self._concurrent_ok(feats):
            outs = self._forward_features_concurrent(feats)
        else:
            outs = []
            for idx, f in zip(self.backbone_out_indices, feats):
                y = self.run_scale(idx, f, self._mcaq_state)
                outs.append(f if y is None else y)
        self.end()
        return outs, aux

    def _concurrent_ok(self, feats):
        if not (CONCURRENT_TRAIN_SCALES and self.training and core.FUSED_TRAIN and len(feats) > 1):
            return False
        if not all(torch.is_tensor(f) and f.is_cuda and f.dim() == 4 for f in feats):
            return False
        if len({f.device for f in feats}) != 1:
            return False
        # batch-sharded steps keep one stream: their collectives sit between
        # the stage launches (dist.shard_hooks)
        if self.process_group is not None or any(q.process_group is not None for q in self.quantizers.values()):
            return False
        if isinstance(self.bit_mapper, ComplexityToBitMappingNetwork) and \
                core._mapper_group(self.bit_mapper.mapping_network) is not None:
            return False
        return True

    def _scale_streams(self, device, n):
        key = (torch.device(device), n)
        cache = self.__dict__.setdefault("_streams", {})
        if key not in cache:
            cache[key] = [torch.cuda.Stream(device=device) for _ in range(n)]
        return cache[key]

    def _forward_features_concurrent(self, feats):
        dev = feats[0].device
        main = torch.cuda.current_stream(dev)
        streams = self._scale_streams(dev, len(feats))
        outs = []
        with core.concurrent_scales(self.complexity_analyzer, main, streams) as scope:
            for st in streams:
                st.wait_stream(main)
            for idx, f, st in zip(self.backbone_out_indices, feats, streams):
                with torch.cuda.stream(st):
                    y = self.run_scale(idx, f, self._mcaq_state)
                outs.append(f if y is None else y)
            for st in streams:
                main.wait_stream(st)
            # outputs allocated on the side streams are used on the main one:
            # the caching allocator must not hand their blocks back to the
            # side streams' pools before the main stream is done with them
            for f, y in zip(feats, outs):
                if y is not f:
                    y.record_stream(main)
            scope.finish()
        return outs
