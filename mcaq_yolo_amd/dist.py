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
# {(group, params, local pattern): global pattern}
_UNUSED_CACHE = WeakIdKeyDictionary()


def allreduce_gradients(params, process_group, average=True):
    """Average the gradients of `params` over the group with ONE collective:
    every parameter that requires grad goes into a single flat bucket in the
    order given (a None grad contributes zeros).  Afterwards every parameter
    that had a gradient on some rank holds the averaged gradient, and one
    whose grad was None on every rank keeps None (as DDP leaves globally
    unused parameters: optimizers then skip them).

    Which parameters have a gradient on SOME rank is a property of the model
    and the step, not of the data: it is found once per (parameter list,
    local has-gradient pattern) - one flag per parameter rides along in that
    first all-reduce and is read back on the host - and reused afterwards, so
    a steady-state call issues no device-to-host copy, allocates no host
    tensor and can be captured in a HIP graph with the nccl (RCCL) backend.
    `reset_unused_cache()` forgets the patterns (e.g. after freezing layers)."""
    import torch.distributed as dist
    ps = [p for p in params if p.requires_grad]
    if not ps:
        return
    has = tuple(p.grad is not None for p in ps)
    key = (id(process_group), tuple(id(p) for p in ps), has)
    cache = _UNUSED_CACHE.setdefault(ps[0], {})
    any_grad = cache.get(key)
    parts = [(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in ps]
    if any_grad is None:
        parts.append(torch.tensor(has, dtype=ps[0].dtype, device=ps[0].device))
    flat = torch.cat(parts)
    dist.all_reduce(flat, group=process_group)
    if any_grad is None:
        any_grad = tuple(bool(v) for v in (flat[-len(ps):] > 0).tolist())
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
    fractal regression, synced mapper BatchNorm for QAT."""
    hooks.process_group = process_group
    hooks.batch_offset, hooks.batch_total = rank * local_batch, world * local_batch
    for q in hooks.quantizers.values():
        q.process_group = process_group
    sync_mapper_batchnorm(hooks.bit_mapper, process_group)
    return hooks
