"""Probe: which ATen ops the QAT hook step (bench.py --config 5) issues
besides the fused kernels - one eager step under torch.profiler, ops grouped
by name and by the innermost package / bench source line that issued them."""
import collections
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mcaq_yolo_amd.hooks import MCAQHooks  # noqa: E402

dev = torch.device("cuda:0")
name, B, chans, grid, mapper = bench.QAT_CONFIG
torch.manual_seed(0)
h = MCAQHooks(grid_size=grid, bit_mapping=mapper, device=dev)
h.load_state_dict(bench.hook_state_dict(dev), strict=False)
h.train()
feats = [bench.synth_features(B, c, hh, ww, 5000 + i, dev).requires_grad_(True)
         for i, (c, (hh, ww)) in enumerate(zip(chans, bench.SIZES))]
G = [1e-3 * torch.randn(f.shape, device=dev) for f in feats]
params_ = [p for p in h.parameters() if p.requires_grad]
opt = torch.optim.SGD(params_, lr=1e-3, momentum=0.9)


def step():
    opt.zero_grad(set_to_none=True)
    for f in feats:
        f.grad = None
    outs, aux = h.forward_features(feats, temperature=1.0)
    lbit = (MCAQHooks.avg_bits(aux) - 4.0) ** 2
    torch.autograd.backward(list(outs) + [0.1 * lbit], list(G) + [torch.ones((), device=dev)])
    torch.nn.utils.clip_grad_norm_(params_, max_norm=1.0)
    opt.step()
    h.bit_mapper.enforce_weight_constraints()


for _ in range(3):
    step()
torch.cuda.synchronize()
# record the Python call site of every dispatched op that launches a kernel
sites = collections.Counter()
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402


class Where(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        st = traceback.extract_stack()
        loc = "?"
        for fr in reversed(st[:-1]):
            if ("mcaq_yolo_amd" in fr.filename or "bench.py" in fr.filename or "qat_ops" in fr.filename) \
                    and "_python_dispatch" not in fr.filename:
                loc = "%s:%d" % (os.path.basename(fr.filename), fr.lineno)
                break
        sites[(str(func), loc)] += 1
        return func(*args, **(kwargs or {}))


with Where():
    step()
torch.cuda.synchronize()
for (f, loc), n in sorted(sites.items(), key=lambda x: -x[1]):
    if any(k in f for k in ("view", "detach", "t.default", "as_strided", "_reshape_alias", "unsqueeze", "squeeze",
                            "expand", "permute", "select", "slice", "alias", "size", "stride")):
        continue
    print("%4d  %-45s %s" % (n, f[:45], loc))
