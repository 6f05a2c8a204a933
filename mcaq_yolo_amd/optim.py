"""The optimizer end of the reference's QAT step (train.py:626-641) as two
kernel launches on the GPU:

    torch.nn.utils.clip_grad_norm_(params, max_norm=1.0)   # ~9 ATen kernels
    optimizer.step()                                       # AdamW (train.py:140-150), 4 multi-tensor kernels
    model.bit_mapper.enforce_weight_constraints()          # |W|, 1 multi-tensor kernel

`ClipAdamW` is a torch.optim.Optimizer with AdamW's hyper-parameters, state
(`exp_avg`, `exp_avg_sq`, `step` per parameter; torch.optim.AdamW's
state_dict layout, so checkpoints move between the two) and update rule;
`max_norm` clips the gradients of every parameter it holds first (the
gradients are scaled in place, as clip_grad_norm_ does) and `project_abs`
names the parameters projected onto |W| after the update.  On CUDA (HIP)
parameters the whole step is `mcaq_clip_adamw` (csrc/mcaq_optim.h): no host
sync, capturable in a HIP graph.  CPU parameters run the same three steps as
torch ops.  Values agree with torch's clip + fused AdamW within fp32
rounding (the norms reduce in another order): tests/test_optim_gpu.py.
The two launches: per-chunk squared-norm partials, then the norm and the
update of every chunk (csrc/mcaq_optim.h).
"""
import ctypes

import torch

from . import abi


class ClipAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_norm=None,
                 project_abs=()):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self.max_norm = None if max_norm is None else float(max_norm)
        self._abs = {id(p) for p in project_abs}
        self.last_total_norm = None
        self._flat = None
        self._step_t = None
        self._segs = None
        self._seg_key = None

    def _params(self):
        return [(g, p) for g in self.param_groups for p in g["params"]]

    def _init_state(self):
        """exp_avg / exp_avg_sq of every parameter as views of two flat
        device buffers, and one shared device step counter (outside capture:
        the first step is a warm-up)."""
        ps = [p for _, p in self._params()]
        if self._flat is not None or not ps:
            return
        dev = ps[0].device
        n = sum(p.numel() for p in ps)
        self._flat = (torch.zeros(n, device=dev), torch.zeros(n, device=dev))
        self._step_t = torch.zeros((), device=dev)
        o = 0
        for p in ps:
            k = p.numel()
            st = self.state[p]
            st["exp_avg"] = self._flat[0][o:o + k].view_as(p)
            st["exp_avg_sq"] = self._flat[1][o:o + k].view_as(p)
            st["step"] = self._step_t
            o += k

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        # re-home the loaded state into the flat buffers the kernel updates
        loaded = {p: dict(self.state[p]) for _, p in self._params() if p in self.state}
        self._flat = None
        self._segs = None
        self._init_state()
        for p, st in loaded.items():
            if "exp_avg" in st:
                self.state[p]["exp_avg"].copy_(st["exp_avg"])
                self.state[p]["exp_avg_sq"].copy_(st["exp_avg_sq"])
            if "step" in st:
                self._step_t.fill_(float(st["step"]))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        items = [(g, p) for g, p in self._params() if p.grad is not None]
        if not items:
            return loss
        self._init_state()
        if items[0][1].is_cuda:
            self._step_cuda(items)
        else:
            self._step_torch(items)
        return loss

    def _step_cuda(self, items):
        if len(items) > abi.MCAQ_OPT_MAXSEG:
            raise ValueError("ClipAdamW: at most %d parameter tensors per launch" % abi.MCAQ_OPT_MAXSEG)
        for _, p in items:
            if p.dtype != torch.float32 or p.grad.dtype != torch.float32 or not p.is_contiguous() or \
                    not p.grad.is_contiguous():
                raise ValueError("ClipAdamW on the GPU takes contiguous fp32 parameters and gradients")
        # descriptors are rebuilt only when a gradient or parameter moved (a
        # captured step keeps them; a set_to_none zero_grad allocates anew)
        key = tuple((p.data_ptr(), p.grad.data_ptr(), g["lr"], g["weight_decay"], g["betas"], g["eps"])
                    for g, p in items)
        if key != self._seg_key:
            hps = []
            segs = (abi.AdamwSeg * len(items))()
            for s, (g, p) in zip(segs, items):
                st = self.state[p]
                hp = (float(g["lr"]), float(g["weight_decay"]), float(g["betas"][0]), float(g["betas"][1]),
                      float(g["eps"]))
                if hp not in hps:
                    hps.append(hp)
                s.param, s.grad = p.data_ptr(), p.grad.data_ptr()
                s.exp_avg, s.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                s.n, s.project_abs, s.group = p.numel(), 1 if id(p) in self._abs else 0, hps.index(hp)
            if len(hps) > abi.MCAQ_OPT_MAXGROUPS:
                raise ValueError("ClipAdamW: at most %d distinct hyper-parameter groups" % abi.MCAQ_OPT_MAXGROUPS)
            self._groups = (abi.AdamwGroup * len(hps))(*[abi.AdamwGroup(*hp) for hp in hps])
            self._segs, self._seg_key = segs, key
            self._norm_t = torch.empty(1, device=items[0][1].device)
            total = sum(p.numel() for _, p in items)
            self._work = torch.empty(abi.lib().mcaq_clip_adamw_work_floats(total), device=items[0][1].device)
        mn = self.max_norm if self.max_norm is not None else 0.0
        st = ctypes.c_void_p(torch.cuda.current_stream(items[0][1].device).cuda_stream)
        abi.check(abi.lib().mcaq_clip_adamw(self._segs, len(items), self._groups, len(self._groups),
                                            ctypes.c_void_p(self._step_t.data_ptr()), mn,
                                            ctypes.c_void_p(self._norm_t.data_ptr()),
                                            ctypes.c_void_p(self._work.data_ptr()), st), "mcaq_clip_adamw")
        self.last_total_norm = self._norm_t[0] if self.max_norm is not None else None
        # the kernel updated the tensors through raw pointers: bump their
        # version counters as an in-place torch op would, so caches keyed on
        # them (the packed weight blobs, core._BlobCache) see the new values
        for _, p in items:
            torch.autograd.graph.increment_version(p)
            if self.max_norm is not None:
                torch.autograd.graph.increment_version(p.grad)

    def _step_torch(self, items):
        """The same step as torch ops (CPU parameters)."""
        if self.max_norm is not None:
            self.last_total_norm = torch.nn.utils.clip_grad_norm_([p for _, p in items], self.max_norm)
        self._step_t += 1
        t = float(self._step_t)
        for g, p in items:
            st = self.state[p]
            b1, b2 = g["betas"]
            p.mul_(1 - g["lr"] * g["weight_decay"])
            st["exp_avg"].mul_(b1).add_(p.grad, alpha=1 - b1)
            st["exp_avg_sq"].mul_(b2).addcmul_(p.grad, p.grad, value=1 - b2)
            denom = (st["exp_avg_sq"].sqrt() / (1 - b2 ** t) ** 0.5).add_(g["eps"])
            p.addcdiv_(st["exp_avg"], denom, value=-g["lr"] / (1 - b1 ** t))
            if id(p) in self._abs:
                p.abs_()
