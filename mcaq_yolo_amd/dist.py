"""Data parallelism for the hook path: one process per GPU, batch shards,
RCCL over xGMI (torch.distributed backend "nccl"), gloo on CPU for tests.

The reference is single-process (train.py:360, rank=-1); SURVEY 8(e) lists
what sharding the batch needs for the results to equal the single-process
run on the global batch:

* inference: the per-channel batch min/max (quantization.py:650-654) -
  `engine.sync_channel_minmax` / `SpatialAdaptiveQuantization.process_group`;
  detections are all-gathered after NMS (`postprocess.gather_detections`);
* QAT (BASELINE config 5): the quantizer's EMA min/max over the global batch
  (same `process_group`), the bit mapper's train-mode BatchNorm1d statistics
  over the global batch of tiles (bit_allocation.py:126) -
  `sync_mapper_batchnorm`, and the gradient all-reduce - `allreduce_gradients`
  (one flat bucket: the hook parameters are ~8 k floats, one latency-bound
  collective instead of 30).
"""
import torch
import torch.nn as nn


class GroupBatchNorm1d(nn.BatchNorm1d):
    """BatchNorm1d whose train-mode statistics span every rank of a process
    group (sum, sum of squares and count all-reduced once per forward, with
    autograd through the collective); eval mode and the state_dict are plain
    BatchNorm1d's, so reference checkpoints load unchanged.  Works on CPU
    (gloo) as well as on the GPU (RCCL), unlike torch.nn.SyncBatchNorm."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True,
                 process_group=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats)
        self.process_group = process_group

    @classmethod
    def from_bn(cls, bn, process_group):
        new = cls(bn.num_features, bn.eps, bn.momentum, bn.affine, bn.track_running_stats, process_group)
        new.load_state_dict(bn.state_dict())
        new.train(bn.training)      # a swapped-in eval-mode layer stays in eval mode
        return new.to(bn.weight.device if bn.affine else bn.running_mean.device)

    def forward(self, x):
        if not self.training or self.process_group is None:
            return super().forward(x)
        from torch.distributed.nn.functional import all_reduce
        # two passes, as a single-process BatchNorm1d over the global batch:
        # the global mean first (sum and count in one all-reduce), then the
        # sum of squared deviations from it - no E[x^2] - mean^2 cancellation
        # when |mean| >> std
        n_local = torch.tensor([float(x.shape[0])], device=x.device, dtype=x.dtype)
        C = x.shape[1]
        s1 = all_reduce(torch.cat([x.sum(dim=0), n_local]), group=self.process_group)
        n = s1[C]
        mean = s1[:C] / n
        d = x - mean
        var = all_reduce((d * d).sum(dim=0), group=self.process_group) / n
        if self.track_running_stats:
            with torch.no_grad():
                self.num_batches_tracked += 1
                m = self.momentum if self.momentum is not None else 1.0 / float(self.num_batches_tracked)
                unbiased = var.detach() * (n / (n - 1).clamp(min=1.0))
                self.running_mean.mul_(1 - m).add_(m * mean.detach())
                self.running_var.mul_(1 - m).add_(m * unbiased)
        y = d / torch.sqrt(var + self.eps)
        return y * self.weight + self.bias if self.affine else y


def sync_mapper_batchnorm(mapper, process_group):
    """Swap the mapping network's BatchNorm1d layers (bit_allocation.py:126)
    for GroupBatchNorm1d over `process_group`; returns the mapper."""
    net = getattr(mapper, "mapping_network", None)
    if net is None:
        return mapper
    for i, m in enumerate(net):
        if isinstance(m, nn.BatchNorm1d) and not isinstance(m, GroupBatchNorm1d):
            net[i] = GroupBatchNorm1d.from_bn(m, process_group)
    if hasattr(mapper, "_blob"):
        mapper._blob.key = None
    return mapper


from torch.utils.weak import WeakIdKeyDictionary

# per first parameter (by identity; dropped with the model):
# {(group, params): global has-gradient pattern}
_UNUSED_CACHE = WeakIdKeyDictionary()


def _flat_span(grads):
    """The one contiguous fp32 span of storage the gradient views tile exactly
    (no gap, no overlap), or None.  _GradArena lays the hook nets' gradient
    sinks out that way, so their bucket is reduced in place."""
    if not grads or any(g is None or not g.is_contiguous() or g.dtype != torch.float32 for g in grads):
        return None
    base = grads[0].untyped_storage()
    if any(g.untyped_storage().data_ptr() != base.data_ptr() for g in grads):
        return None
    runs = sorted((g.storage_offset(), g.numel()) for g in grads)
    o = runs[0][0]
    for off, n in runs:
        if off != o:
            return None
        o += n
    t = torch.empty(0, dtype=torch.float32, device=grads[0].device)
    t.set_(base, runs[0][0], (o - runs[0][0],))
    return t


def _reduce_in_place(t, process_group, average):
    import torch.distributed as dist
    world = dist.get_world_size(process_group)
    if average and world > 1 and dist.get_backend(process_group) == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG, group=process_group)   # RCCL ncclAvg: no extra launch
        return
    dist.all_reduce(t, group=process_group)
    if average and world > 1:
        t /= world


def allreduce_gradients(params, process_group, average=True, static_pattern=False):
    """Average (or sum) the gradients of `params` over the group as ONE flat
    bucket (train.py:626-641 under DDP).  Afterwards every parameter that had
    a gradient on some rank holds the reduced gradient (a None grad
    contributes zeros), and one whose grad was None on every rank keeps None,
    as DDP leaves globally unused parameters (optimizers then skip them).

    static_pattern=False (default): one flag per parameter rides along in the
    bucket and is read back, so ranks whose has-gradient patterns differ or
    change between calls stay consistent - at the cost of a device-to-host
    read per call (not capturable).

    static_pattern=True: the caller guarantees that the set of parameters
    with a gradient on SOME rank is fixed (a captured step, the hook step of
    dist.shard_hooks).  The pattern is agreed collectively on the first call
    (flags in the bucket, one read-back) and cached per (group, parameters);
    later calls move exactly the cached parameters on every rank, whatever the
    local pattern, so bucket sizes always match across ranks (a local None
    sends zeros; a parameter that became globally unused then ends with a
    zero gradient instead of None).  A local gradient on a parameter the
    cached pattern says no rank uses raises ValueError: call
    reset_unused_cache() on every rank when the model changes.  When the
    gradients tile one contiguous buffer (the hook nets' sinks, _GradArena),
    the bucket is that buffer, reduced in place: no concatenation, no copies,
    no host sync - capturable in a HIP graph with RCCL."""
    import torch.distributed as dist
    ps = [p for p in params if p.requires_grad]
    if not ps:
        return
    has = tuple(p.grad is not None for p in ps)
    key = (id(process_group), tuple(id(p) for p in ps))
    cache = _UNUSED_CACHE.setdefault(ps[0], {})
    any_grad = cache.get(key) if static_pattern else None
    if any_grad is not None:
        for p, h, a in zip(ps, has, any_grad):
            if h and not a:
                raise ValueError("allreduce_gradients(static_pattern=True): a parameter that no rank had a "
                                 "gradient for when the pattern was cached has one now; call "
                                 "dist.reset_unused_cache() on every rank")
        live = [p for p, a in zip(ps, any_grad) if a]
        for p in live:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        span = _flat_span([p.grad for p in live])
        if span is not None:
            _reduce_in_place(span, process_group, average)
            return
        flat = torch.cat([p.grad.reshape(-1) for p in live])
        _reduce_in_place(flat, process_group, average)
        o = 0
        for p in live:
            n = p.numel()
            p.grad.copy_(flat[o:o + n].view_as(p))
            o += n
        return
    # flags ride along; read back to decide None vs reduced on every rank alike
    parts = [(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in ps]
    parts.append(torch.tensor(has, dtype=ps[0].dtype, device=ps[0].device))
    flat = torch.cat(parts)
    dist.all_reduce(flat, group=process_group)
    any_grad = tuple(bool(v) for v in (flat[-len(ps):] > 0).tolist())
    if static_pattern:
        cache[key] = any_grad
    flat = flat[:-len(ps)]
    if average:
        flat /= dist.get_world_size(process_group)
    o = 0
    for p, h_any in zip(ps, any_grad):
        n = p.numel()
        g = flat[o:o + n].view_as(p)
        if not h_any:
            p.grad = None
        elif p.grad is None:
            p.grad = g.clone()
        else:
            p.grad.copy_(g)
        o += n


def reset_unused_cache():
    _UNUSED_CACHE.clear()


def shard_hooks(hooks, process_group, rank, world, local_batch):
    """Configure an MCAQHooks / MCAQYOLO for batch-sharded data parallelism:
    min/max all-reduce in every quantizer, global-batch tile order for the
    fractal regression, synced mapper BatchNorm for QAT.

    The hook parameters' gradients are then this package's to synchronise
    (`allreduce_gradients`, not a DDP reducer): they are marked so the fused
    backwards keep writing them into their flat sinks, and the sinks of the
    complexity MLP, the bit mapper and every soft mask are laid out back to
    back in ONE device buffer (core._GradArena) - the step's gradient bucket,
    reduced in place by allreduce_gradients(..., static_pattern=True)."""
    from . import core
    hooks.process_group = process_group
    hooks.batch_offset, hooks.batch_total = rank * local_batch, world * local_batch
    for q in hooks.quantizers.values():
        q.process_group = process_group
    sync_mapper_batchnorm(hooks.bit_mapper, process_group)
    pairs = []
    an = getattr(hooks, "complexity_analyzer", None)
    if an is not None and hasattr(an, "_gsink"):
        pairs.append((an._gsink, list(an.complexity_mlp.parameters())))
    bm = hooks.bit_mapper
    if hasattr(bm, "_gsink") and hasattr(bm, "mapping_network"):
        pairs.append((bm._gsink, list(bm.mapping_network.parameters())))
    for q in hooks.quantizers.values():
        sm = getattr(q, "soft_mask", None)
        if sm is not None and hasattr(sm, "_gsink"):
            pairs.append((sm._gsink, list(sm.net.parameters())))
    params = [p for _, ps in pairs for p in ps]
    for p in params:
        p._mcaq_dp_manual = True
    if params:
        hooks._grad_arena = core._GradArena(pairs, params[0].device)
    return hooks
