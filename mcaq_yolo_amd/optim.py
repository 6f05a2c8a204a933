"""The optimizer end of the reference's QAT step (train.py:626-641) as two
kernel launches on the GPU:

    torch.nn.utils.clip_grad_norm_(params, max_norm=1.0)   # ~9 ATen kernels
    optimizer.step()                                       # AdamW (train.py:140-150), 4 multi-tensor kernels
    model.bit_mapper.enforce_weight_constraints()          # |W|, 1 multi-tensor kernel

`ClipAdamW` is a torch.optim.Optimizer with AdamW's hyper-parameters, state
(`exp_avg`, `exp_avg_sq`, `step` per parameter - a parameter without a
gradient keeps its step, as in torch; torch.optim.AdamW's state_dict layout,
so checkpoints move between the two) and update rule;
`max_norm` clips the gradients of every parameter it holds first (the
gradients are scaled in place, as clip_grad_norm_ does) and `project_abs`
names the parameters projected onto |W| after the update.  On CUDA (HIP)
parameters the whole step is `mcaq_clip_adamw` (csrc/mcaq_optim.h): no host
sync, capturable in a HIP graph (the hyper-parameters are read from a device
table at run time: `sync_hyperparameters()` after an lr schedule changes them
between graph replays).  CPU parameters run the same three steps as
torch ops.  Values agree with torch's clip + fused AdamW within fp32
rounding (the norms reduce in another order): tests/test_optim_gpu.py.
The two launches: per-chunk squared-norm partials, then the norm and the
update of every chunk (csrc/mcaq_optim.h).  With clipping and up to 256
chunks of 1,024 elements (ONE_LAUNCH) both run in ONE launch, the partials
exchanged inside it (`mcaq_clip_adamw_fused`, bit-identical).
"""
import ctypes
import os

import torch

from . import abi


# one launch for the clipped step when its chunks fit the chip at once
# (MCAQ_ADAMW_ONE_LAUNCH=0: the two launches, A/B)
ONE_LAUNCH = os.environ.get("MCAQ_ADAMW_ONE_LAUNCH", "1") != "0"


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
        self._steps_t = None
        self._index = None
        self._hp_t = None
        self._hp_host = None
        self._segs = None
        self._seg_key = None
        self._sync = None
        self._sync_key = None
        self._retired = []

    def _params(self):
        return [(g, p) for g in self.param_groups for p in g["params"]]

    def _init_state(self):
        """exp_avg / exp_avg_sq of every parameter as views of two flat
        device buffers and one step counter per parameter (torch.optim.AdamW
        keeps a step per parameter and skips parameters without a gradient),
        views of one device array (outside capture: the first step is a
        warm-up)."""
        ps = [p for _, p in self._params()]
        if self._flat is not None or not ps:
            return
        dev = ps[0].device
        n = sum(p.numel() for p in ps)
        self._flat = (torch.zeros(n, device=dev), torch.zeros(n, device=dev))
        self._steps_t = torch.zeros(len(ps), device=dev)
        self._index = {id(p): i for i, p in enumerate(ps)}
        o = 0
        for i, p in enumerate(ps):
            k = p.numel()
            st = self.state[p]
            st["exp_avg"] = self._flat[0][o:o + k].view_as(p)
            st["exp_avg_sq"] = self._flat[1][o:o + k].view_as(p)
            st["step"] = self._steps_t[i]
            o += k

    def state_dict(self):
        """torch.optim.AdamW's layout.  Every parameter's step is its own CPU
        float tensor (a non-capturable AdamW's form; a capturable or fused one
        moves it to the device on load), never a view of this optimizer's
        device counters: an AdamW loading it then steps its own copies."""
        sd = super().state_dict()
        sd["state"] = {k: {kk: (vv.detach().to("cpu", torch.float32).clone() if kk == "step" and torch.is_tensor(vv)
                                else vv) for kk, vv in v.items()} for k, v in sd["state"].items()}
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        # re-home the loaded state into the flat buffers the kernel updates;
        # the launch descriptors point at the old buffers: rebuild them
        loaded = {p: dict(self.state[p]) for _, p in self._params() if p in self.state}
        self._flat = None
        self._retire()
        self._hp_host = None
        self._init_state()
        for p, st in loaded.items():
            if "exp_avg" in st:
                self.state[p]["exp_avg"].copy_(st["exp_avg"])
                self.state[p]["exp_avg_sq"].copy_(st["exp_avg_sq"])
            if "step" in st:
                self._steps_t[self._index[id(p)]].fill_(float(st["step"]))

    def _retire(self):
        """Forget the launch descriptors; their device buffers stay alive (a
        graph captured earlier may still write into them)."""
        if self._segs is not None:
            self._retired.append((self._work, self._norm_t, self._sync))
        self._segs = None
        self._seg_key = None

    def _hparams(self):
        return tuple((float(g["lr"]), float(g["weight_decay"]), float(g["betas"][0]), float(g["betas"][1]),
                      float(g["eps"])) for g in self.param_groups)

    def sync_hyperparameters(self):
        """Write every group's lr / weight decay / betas / eps into the device
        table the kernel reads.  Eager steps do it themselves when a value
        changed; a step captured in a HIP graph reads the table at replay, so
        after an lr scheduler step between replays call this (outside
        capture)."""
        hp = self._hparams()
        if len(hp) > abi.MCAQ_OPT_MAXGROUPS:
            raise ValueError("ClipAdamW: at most %d parameter groups" % abi.MCAQ_OPT_MAXGROUPS)
        if self._hp_t is None:
            dev = self.param_groups[0]["params"][0].device
            self._hp_t = torch.zeros(abi.MCAQ_OPT_MAXGROUPS * 5, dtype=torch.float64, device=dev)
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("ClipAdamW: hyper-parameters changed inside graph capture; call "
                               "sync_hyperparameters() before capturing")
        self._hp_t[:5 * len(hp)].copy_(torch.tensor([v for row in hp for v in row], dtype=torch.float64))
        self._hp_host = hp

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        items = [(gi, p) for gi, g in enumerate(self.param_groups) for p in g["params"] if p.grad is not None]
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
        if self._hparams() != self._hp_host:
            self.sync_hyperparameters()
        # descriptors are rebuilt only when a gradient or parameter moved (a
        # captured step keeps them; a set_to_none zero_grad allocates anew)
        key = tuple((p.data_ptr(), p.grad.data_ptr(), gi) for gi, p in items)
        if key != self._seg_key:
            self._retire()
            segs = (abi.AdamwSeg * len(items))()
            for s, (gi, p) in zip(segs, items):
                st = self.state[p]
                s.param, s.grad = p.data_ptr(), p.grad.data_ptr()
                s.exp_avg, s.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                s.n, s.project_abs, s.group = p.numel(), 1 if id(p) in self._abs else 0, gi
                s.step_idx = self._index[id(p)]
            self._segs, self._seg_key = segs, key
            self._norm_t = torch.empty(1, device=items[0][1].device)
            total = sum(p.numel() for _, p in items)
            self._work = torch.empty(abi.lib().mcaq_clip_adamw_work_floats(total), device=items[0][1].device)
            # the one-launch form's exchange buffer: one per (elements,
            # tensors) layout, zeroed when made - descriptors rebuilt for moved
            # gradients (set_to_none) keep it, its epoch carries on
            lay = (total, len(items), items[0][1].device)
            if self.max_norm is None or self.max_norm <= 0 or -(-total // 1024) > 256:
                self._sync, self._sync_key = None, None
            elif self._sync is None or self._sync_key != lay:
                nb = abi.lib().mcaq_clip_adamw_sync_bytes(total, len(items))
                self._sync = torch.zeros((nb + 7) // 8, dtype=torch.int64, device=items[0][1].device)
                self._sync_key = lay
        mn = self.max_norm if self.max_norm is not None else 0.0
        st = ctypes.c_void_p(torch.cuda.current_stream(items[0][1].device).cuda_stream)
        L = abi.lib()
        if ONE_LAUNCH and self._sync is not None and mn > 0:
            abi.check(L.mcaq_clip_adamw_fused(self._segs, len(items), ctypes.c_void_p(self._hp_t.data_ptr()),
                                              len(self.param_groups), ctypes.c_void_p(self._steps_t.data_ptr()), mn,
                                              ctypes.c_void_p(self._norm_t.data_ptr()),
                                              ctypes.c_void_p(self._sync.data_ptr()), self._sync.numel() * 8, st),
                      "mcaq_clip_adamw_fused")
        else:
            abi.check(L.mcaq_clip_adamw(self._segs, len(items), ctypes.c_void_p(self._hp_t.data_ptr()),
                                        len(self.param_groups), ctypes.c_void_p(self._steps_t.data_ptr()), mn,
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
        for gi, p in items:
            g = self.param_groups[gi]
            st = self.state[p]
            st["step"] += 1
            t = float(st["step"])
            b1, b2 = g["betas"]
            p.mul_(1 - g["lr"] * g["weight_decay"])
            st["exp_avg"].mul_(b1).add_(p.grad, alpha=1 - b1)
            st["exp_avg_sq"].mul_(b2).addcmul_(p.grad, p.grad, value=1 - b2)
            denom = (st["exp_avg_sq"].sqrt() / (1 - b2 ** t) ** 0.5).add_(g["eps"])
            p.addcdiv_(st["exp_avg"], denom, value=-g["lr"] / (1 - b1 ** t))
            if id(p) in self._abs:
                p.abs_()
