"""YOLOv8 host network for the end-to-end MCAQ inference path (SURVEY 8(f)
rank 1) and the reference's `MCAQYOLO` wrapper (models/mcaq_yolo.py:222-589).

ultralytics (and its weights) is not available offline, so the detector is
defined here from the public YOLOv8 architecture: the `yolov8.yaml` layer
table (scales n/s/m = depth 0.33/0.33/0.67, width 0.25/0.50/0.75, max
channels 1024/1024/768), ultralytics module semantics (Conv = conv+BN(eps
1e-3)+SiLU, C2f, SPPF, nearest Upsample, Concat, Detect with DFL and
dist2bbox decode).  Module and parameter names follow ultralytics'
DetectionModel (`model.<i>.cv1.conv.weight`, `model.22.dfl.conv.weight`, ...)
so an ultralytics state_dict loads with `load_state_dict`, and every layer
carries ultralytics' `.i` / `.f` / `.type` attributes so the reference's
backbone discovery (`_find_backbone_out_indices`, models/mcaq_yolo.py:
351-400) runs unchanged on it.  Weights are seeded random (ultralytics init:
BN eps 1e-3 / momentum 0.03, Detect bias init).  Parity of the network
against ultralytics is unpinned (no ultralytics, no weights).

The network's convolutions run on MIOpen; the MCAQ hooks at the backbone
outputs (C3/C4/C5) and the NMS are the HIP kernels of this package.
"""
import math
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F

from .hooks import MCAQHooks

# scale: (depth_multiple, width_multiple, max_channels) - ultralytics yolov8.yaml
SCALES = {"n": (0.33, 0.25, 1024), "s": (0.33, 0.50, 1024), "m": (0.67, 0.75, 768),
          "l": (1.00, 1.00, 512), "x": (1.00, 1.25, 512)}

# (from, repeats, module, args) - ultralytics yolov8.yaml backbone + head
YOLOV8_LAYERS = [
    (-1, 1, "Conv", [64, 3, 2]),        # 0 P1/2
    (-1, 1, "Conv", [128, 3, 2]),       # 1 P2/4
    (-1, 3, "C2f", [128, True]),        # 2
    (-1, 1, "Conv", [256, 3, 2]),       # 3 P3/8
    (-1, 6, "C2f", [256, True]),        # 4   <- C3 hook
    (-1, 1, "Conv", [512, 3, 2]),       # 5 P4/16
    (-1, 6, "C2f", [512, True]),        # 6   <- C4 hook
    (-1, 1, "Conv", [1024, 3, 2]),      # 7 P5/32
    (-1, 3, "C2f", [1024, True]),       # 8
    (-1, 1, "SPPF", [1024, 5]),         # 9   <- C5 hook
    (-1, 1, "Upsample", [None, 2, "nearest"]),  # 10
    ([-1, 6], 1, "Concat", [1]),        # 11
    (-1, 3, "C2f", [512]),              # 12
    (-1, 1, "Upsample", [None, 2, "nearest"]),  # 13
    ([-1, 4], 1, "Concat", [1]),        # 14
    (-1, 3, "C2f", [256]),              # 15 (P3/8-small)
    (-1, 1, "Conv", [256, 3, 2]),       # 16
    ([-1, 12], 1, "Concat", [1]),       # 17
    (-1, 3, "C2f", [512]),              # 18 (P4/16-medium)
    (-1, 1, "Conv", [512, 3, 2]),       # 19
    ([-1, 9], 1, "Concat", [1]),        # 20
    (-1, 3, "C2f", [1024]),             # 21 (P5/32-large)
    ([15, 18, 21], 1, "Detect", ["nc"]),  # 22
]


def make_divisible(x, divisor=8):
    return int(math.ceil(x / divisor) * divisor)


class Conv(nn.Module):
    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, k // 2 if p is None else p, groups=g, bias=False)
        self.bn = nn.BatchNorm2d(c2, eps=1e-3, momentum=0.03)
        self.act = nn.SiLU() if act else nn.Identity()

    def forward(self, x):
        return self.act(self.bn(self.conv(x)))

    @torch.no_grad()
    def fuse(self):
        """Fold the (eval) BatchNorm into the convolution, as ultralytics'
        inference AutoBackend does by default (fuse_conv_and_bn): w' = w * g /
        sqrt(var + eps), b' = beta - mean * g / sqrt(var + eps)."""
        if isinstance(self.bn, nn.Identity):
            return self
        bn, conv = self.bn, self.conv
        scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        fused = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding,
                          groups=conv.groups, bias=True).to(conv.weight.device)
        fused.weight.copy_(conv.weight * scale.reshape(-1, 1, 1, 1))
        fused.bias.copy_(bn.bias - bn.running_mean * scale)
        self.conv, self.bn = fused, nn.Identity()
        return self


class Bottleneck(nn.Module):
    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, k[0], 1)
        self.cv2 = Conv(c_, c2, k[1], 1, g=g)
        self.add = shortcut and c1 == c2

    def forward(self, x):
        y = self.cv2(self.cv1(x))
        return x + y if self.add else y


class C2f(nn.Module):
    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        self.c = int(c2 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut, g, k=(3, 3), e=1.0) for _ in range(n))

    def forward(self, x):
        y = list(self.cv1(x).chunk(2, 1))
        for m in self.m:
            y.append(m(y[-1]))
        return self.cv2(torch.cat(y, 1))


class SPPF(nn.Module):
    def __init__(self, c1, c2, k=5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * 4, c2, 1, 1)
        self.m = nn.MaxPool2d(kernel_size=k, stride=1, padding=k // 2)

    def forward(self, x):
        y = [self.cv1(x)]
        for _ in range(3):
            y.append(self.m(y[-1]))
        return self.cv2(torch.cat(y, 1))


class Concat(nn.Module):
    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def forward(self, x):
        return torch.cat(x, self.d)


class DFL(nn.Module):
    """Distribution focal loss integral: softmax over reg_max bins . arange."""

    def __init__(self, c1=16):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        self.conv.weight.data[:] = torch.arange(c1, dtype=torch.float).view(1, c1, 1, 1)
        self.c1 = c1

    def forward(self, x):
        b, _, a = x.shape
        return self.conv(x.view(b, 4, self.c1, a).transpose(2, 1).softmax(1)).view(b, 4, a)


def make_anchors(feats, strides, offset=0.5):
    pts, strd = [], []
    for x, s in zip(feats, strides):
        _, _, h, w = x.shape
        sx = torch.arange(w, device=x.device, dtype=x.dtype) + offset
        sy = torch.arange(h, device=x.device, dtype=x.dtype) + offset
        sy, sx = torch.meshgrid(sy, sx, indexing="ij")
        pts.append(torch.stack((sx, sy), -1).view(-1, 2))
        strd.append(torch.full((h * w, 1), float(s), dtype=x.dtype, device=x.device))
    return torch.cat(pts), torch.cat(strd)


def dist2bbox(distance, anchor_points, xywh=True, dim=-1):
    lt, rb = distance.chunk(2, dim)
    x1y1 = anchor_points - lt
    x2y2 = anchor_points + rb
    if xywh:
        return torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), dim)
    return torch.cat((x1y1, x2y2), dim)


class Detect(nn.Module):
    def __init__(self, nc=80, ch=()):
        super().__init__()
        self.nc, self.nl, self.reg_max = nc, len(ch), 16
        self.no = nc + self.reg_max * 4
        self.stride = torch.zeros(self.nl)
        c2 = max((16, ch[0] // 4, self.reg_max * 4))
        c3 = max(ch[0], min(self.nc, 100))
        self.cv2 = nn.ModuleList(nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 4 * self.reg_max, 1))
                                 for x in ch)
        self.cv3 = nn.ModuleList(nn.Sequential(Conv(x, c3, 3), Conv(c3, c3, 3), nn.Conv2d(c3, self.nc, 1))
                                 for x in ch)
        self.dfl = DFL(self.reg_max)
        self._anchor_key = None

    def bias_init(self):
        for a, b, s in zip(self.cv2, self.cv3, self.stride):
            a[-1].bias.data[:] = 1.0
            b[-1].bias.data[: self.nc] = math.log(5 / self.nc / (640 / float(s)) ** 2)

    def forward(self, x):
        for i in range(self.nl):
            x[i] = torch.cat((self.cv2[i](x[i]), self.cv3[i](x[i])), 1)
        if self.training:
            return x
        shape = x[0].shape
        key = (tuple(shape), x[0].device, x[0].dtype)
        if self._anchor_key != key:       # anchors cached per input shape (graph-capture safe)
            a, s = make_anchors(x, self.stride, 0.5)
            self.anchors, self.strides = a.transpose(0, 1), s.transpose(0, 1)
            self._anchor_key = key
        x_cat = torch.cat([xi.view(shape[0], self.no, -1) for xi in x], 2)
        box, cls = x_cat.split((self.reg_max * 4, self.nc), 1)
        dbox = dist2bbox(self.dfl(box), self.anchors.unsqueeze(0), xywh=True, dim=1) * self.strides
        return torch.cat((dbox, cls.sigmoid()), 1), x


_MODULES = {"Conv": Conv, "C2f": C2f, "SPPF": SPPF, "Concat": Concat, "Detect": Detect}


class DetectionModel(nn.Module):
    """ultralytics DetectionModel equivalent for yolov8{n,s,m,l,x}."""

    def __init__(self, cfg="yolov8n", nc=80, ch=3):
        super().__init__()
        scale = cfg[-1] if cfg.startswith("yolov8") else cfg
        if scale not in SCALES:
            raise ValueError("unknown YOLOv8 scale %r" % cfg)
        depth, width, max_ch = SCALES[scale]
        self.yaml = {"cfg": cfg, "nc": nc, "scale": scale}
        chs, layers, save = [ch], [], []
        for i, (f, n, mname, args) in enumerate(YOLOV8_LAYERS):
            n_ = max(round(n * depth), 1) if n > 1 else n
            if mname in ("Conv", "C2f", "SPPF"):
                c1, c2 = chs[f], args[0]
                c2 = make_divisible(min(c2, max_ch) * width, 8)
                if mname == "C2f":
                    m = C2f(c1, c2, n_, *args[1:])
                elif mname == "SPPF":
                    m = SPPF(c1, c2, *args[1:])
                else:
                    m = Conv(c1, c2, *args[1:])
            elif mname == "Upsample":
                m, c2 = nn.Upsample(None, args[1], args[2]), chs[f]
            elif mname == "Concat":
                m, c2 = Concat(args[0]), sum(chs[x] for x in f)
            elif mname == "Detect":
                m, c2 = Detect(nc, [chs[x] for x in f]), None
            else:
                raise ValueError(mname)
            m.i, m.f, m.type = i, f, mname
            save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
            layers.append(m)
            if i == 0:
                chs = []
            chs.append(c2)
        self.model = nn.Sequential(*layers)
        self.save = sorted(set(save))
        self.names = {i: "class%d" % i for i in range(nc)}
        det = self.model[-1]
        det.stride = torch.tensor([8.0, 16.0, 32.0])
        self.stride = det.stride
        det.bias_init()

    def fuse(self):
        """Conv + BatchNorm folding for inference (ultralytics DetectionModel.fuse)."""
        for mod in self.modules():
            if isinstance(mod, Conv):
                mod.fuse()
        return self

    def forward(self, x):
        y = []
        for m in self.model:
            if m.f != -1:
                x = y[m.f] if isinstance(m.f, int) else [x if j == -1 else y[j] for j in m.f]
            x = m(x)
            y.append(x if m.i in self.save else None)
        return x


def find_backbone_out_indices(layers):
    """models/mcaq_yolo.py:351-400: the backbone ends at SPPF; every neck
    layer's from-index pointing strictly below SPPF is a skip (P3/P4); P5 is
    the SPPF output.  Fallback [4, 6, 9]."""
    fallback = [4, 6, 9]
    layers = list(layers)
    sppf = None
    for i, m in enumerate(layers):
        if m.__class__.__name__ == "SPPF":
            sppf = i
    if sppf is None:
        warnings.warn("[MCAQ] SPPF layer not found - falling back to backbone indices %s." % fallback)
        return [i for i in fallback if i < len(layers)]
    refs = set()
    for m in layers[sppf + 1:]:
        f = getattr(m, "f", None)
        if f is None:
            continue
        for j in (f if isinstance(f, (list, tuple)) else [f]):
            if isinstance(j, int) and j != -1 and 0 <= j < sppf:
                refs.add(j)
    idx = sorted(refs | {sppf})
    if len(idx) < 2:
        warnings.warn("[MCAQ] Could not derive backbone->neck connections - falling back to %s." % fallback)
        return [i for i in fallback if i < len(layers)]
    return idx


class MCAQYOLO(MCAQHooks):
    """models/mcaq_yolo.py:222-589 on this package: a YOLOv8 DetectionModel
    (`self.model`) with the MCAQ hooks registered on its C3/C4/C5 outputs.
    Attribute names (model, complexity_analyzer, bit_mapper, quantizers) and
    therefore state_dict keys are the reference's.  `pretrained=True` needs
    ultralytics weights, which are unavailable offline: pass `weights=` (a
    state_dict file readable by safetensors or torch.load(weights_only=True))
    instead.  The training loss (MCAQYOLOLoss) is out of scope."""

    def __init__(self, model_name="yolov8n", pretrained=False, min_bits=2, max_bits=8, target_bits=4.0,
                 device="cuda", num_classes=80, grid_size=8, bit_mapping="mlp", normalize_complexity=False,
                 weights=None):
        if pretrained and weights is None:
            raise RuntimeError("pretrained ultralytics weights are not available offline; pass weights=<file>")
        model = DetectionModel(model_name, nc=num_classes)
        indices = find_backbone_out_indices(model.model)
        super().__init__(grid_size=grid_size, min_bits=min_bits, max_bits=max_bits, bit_mapping=bit_mapping,
                         normalize_complexity=normalize_complexity, device=device, indices=indices)
        self.model = model
        self.num_classes = num_classes
        self.target_bits = target_bits
        self.min_bits, self.max_bits = min_bits, max_bits
        self.device = device
        if weights is not None:
            self.load_checkpoint(_load_weights(weights))
        if str(device).startswith("cuda") and torch.cuda.is_available():
            self.to(device)
        self.register(self.model.model)

    def fuse(self):
        """Fold every Conv's BatchNorm into its convolution for inference (what
        the reference's ultralytics Predictor does through AutoBackend(fuse=True));
        the hooks stay registered on the same layers."""
        self.model.fuse()
        return self

    def load_checkpoint(self, sd):
        """Load a reference MCAQYOLO state_dict ('model.model.<i>...', hook
        modules) or a bare ultralytics DetectionModel one ('model.<i>...',
        remapped).  Non-strict like the reference's fallback (inference.py:
        105-115), but a checkpoint that leaves detector weights unloaded
        raises instead of silently running on random weights."""
        if sd and not any(k.startswith("model.model.") for k in sd) and any(k.startswith("model.") for k in sd):
            sd = {("model." + k if k.startswith("model.") else k): v for k, v in sd.items()}
        res = self.load_state_dict(sd, strict=False)
        missing = [k for k in res.missing_keys if k.startswith("model.") and not k.endswith("num_batches_tracked")]
        if missing:
            raise RuntimeError("checkpoint leaves %d detector tensors unloaded (first: %s)" % (len(missing), missing[0]))
        if res.unexpected_keys:
            warnings.warn("[MCAQ] %d unexpected checkpoint keys ignored (first: %s)"
                          % (len(res.unexpected_keys), res.unexpected_keys[0]))
        return res

    def forward(self, x, temperature=1.0, return_aux=True, targets=None, quantize=True):
        """models/mcaq_yolo.py:527-589."""
        aux = self.begin(temperature=temperature, quantize=quantize)
        try:
            outputs = self.model(x)
        finally:
            self.end()
        if not return_aux:
            return outputs
        bit_maps = [r["bit_map"] for r in aux]
        avg_bits = self.avg_bits(aux) if bit_maps else torch.tensor(float(self.target_bits), device=x.device)
        return outputs, {"complexity_map": [r["complexity"] for r in aux], "bit_map": bit_maps,
                         "avg_bits": avg_bits, "quantized_features": [r["features_q"] for r in aux],
                         "feature_layers": [r["layer"] for r in aux], "detailed_metrics": {}}

    @torch.no_grad()
    def calibrate(self, dataloader, num_images=1000):
        """models/mcaq_yolo.py:475-508: EMA min/max over ~num_images, then freeze."""
        self.eval()
        seen = 0
        for batch in dataloader:
            imgs = batch["img"] if isinstance(batch, dict) else (batch[0] if isinstance(batch, (list, tuple))
                                                                  else batch)
            imgs = imgs.to(next(self.model.parameters()).device).float()
            if imgs.max() > 1.5:
                imgs = imgs / 255.0
            self.begin(temperature=1.0, quantize=True, calibrating=True)
            try:
                self.model(imgs)
            finally:
                self.end()
            seen += imgs.shape[0]
            if seen >= num_images:
                break
        for q in self.quantizers.values():
            q.freeze_calibration()
        return seen


def _load_weights(path):
    if str(path).endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    return sd.get("model", sd) if isinstance(sd, dict) else sd
