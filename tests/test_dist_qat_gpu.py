"""BASELINE config 5's DDP leg on the GPU: one full QAT step of the three hooks
(train mode) sharded over two ranks (gloo, both ranks on cuda:0, as
test_dist_hooks.py does for inference) against the single-process step on the
global batch.

dist.shard_hooks swaps the mapper's BatchNorm1d layers for GroupBatchNorm1d;
the fused train-mode kernels run the mapper on the GLOBAL batch of tiles (one
all-gather of its inputs with the quantizers' EMA min/max riding along, one
of the bit gradients in the backward: train_step.DP_GLOBAL_MAPPER), and
dist.allreduce_gradients sums the hook parameters' gradients (the ranks'
shares of the mapper's).  The loss is a sum over samples, so the ranks' losses
add up to the single-process loss and the summed gradients must equal its
gradients.

Bits, y, feature gradients and every buffer (EMA and BatchNorm running
statistics) are bit-identical to the single process.  Parameter gradients
are fp32 sums in other orders (the ranks' shares added by the all-reduce):
as test_train_fused_gpu.py
(1e-3 of the tensor's largest magnitude; the Linear layers feeding a
train-mode BatchNorm 1e-4 of the module's largest gradient)."""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import load_weights

pytestmark = pytest.mark.gpu
WORLD = 2
B = 4
SHAPES = ((64, 80), (128, 40), (256, 20))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _hooks(dev):
    from mcaq_yolo_amd.hooks import MCAQHooks
    torch.manual_seed(0)
    h = MCAQHooks(device=dev, bit_mapping="mlp")
    sd = {}
    for k, v in load_weights().items():
        t = torch.from_numpy(np.asarray(v))
        if k.startswith("soft_mask."):
            for idx in (4, 6, 9):
                sd["quantizers.%d.%s" % (idx, k)] = t
        else:
            sd[k] = t
    h.load_state_dict(sd, strict=False)
    return h.train()


def _inputs():
    gen = torch.Generator(device="cpu").manual_seed(21)
    feats, G = [], []
    for c, s in SHAPES:
        lo = torch.randn(B, c, s // 8, s // 8, generator=gen)
        hi = torch.randn(B, c, s, s, generator=gen)
        up = torch.nn.functional.interpolate(lo, size=(s, s), mode="bilinear", align_corners=False)
        feats.append(torch.nn.functional.silu(1.5 * hi + 2 * up))
        G.append(torch.randn(B, c, s, s, generator=gen) * 1e-3)
    from mcaq_yolo_amd.engine import tile_size
    GB = [torch.randn(B, s // tile_size(s, 8), s // tile_size(s, 8), generator=gen) for _, s in SHAPES]
    return feats, G, GB


def _step(h, feats, G, GB, dev, pg=None):
    """forward + backward of one QAT step on `feats` (this rank's shard);
    returns numpy copies of outputs, bits, feature / parameter gradients and
    buffers.  The loss sum_i (y_i g_i) + sum_t (bits_t gb_t) is a sum over
    samples."""
    from mcaq_yolo_amd import core, train_step
    xs = [f.to(dev).requires_grad_(True) for f in feats]
    calls = {"fused": 0}
    orig, orig_m = core._MapperTrainFn.apply, train_step._MapperMulti.apply

    def spy(*a, **k):
        calls["fused"] += 1
        return orig(*a, **k)

    def spy_m(*a, **k):        # one call for every scale (multi-segment launches)
        calls["fused"] += a[3]
        return orig_m(*a, **k)
    core._MapperTrainFn.apply = spy
    train_step._MapperMulti.apply = spy_m
    try:
        outs, aux = h.forward_features(xs, temperature=1.0)
        loss = sum((o * g.to(dev)).sum() for o, g in zip(outs, G)) + \
            sum((a["bit_map"] * gb.to(dev)).sum() for a, gb in zip(aux, GB))
        loss.backward()
    finally:
        core._MapperTrainFn.apply = orig
        train_step._MapperMulti.apply = orig_m
    params = [p for p in h.parameters() if p.requires_grad]
    if pg is not None:
        from mcaq_yolo_amd.dist import allreduce_gradients
        allreduce_gradients(params, pg, average=False)
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().numpy().copy() for k, p in h.named_parameters() if p.grad is not None}
    bufs = {k: b.detach().cpu().numpy().copy() for k, b in h.named_buffers()
            if b is not None and b.dtype.is_floating_point}
    return ([o.detach().cpu().numpy() for o in outs], [a["bit_map"].detach().cpu().numpy() for a in aux],
            [x.grad.detach().cpu().numpy() for x in xs], grads, bufs, calls["fused"])


def _entry(rank, world, port, q):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mcaq_yolo_amd.dist import GroupBatchNorm1d, shard_hooks
        feats, G, GB = _inputs()
        n = B // world
        sl = slice(rank * n, (rank + 1) * n)
        h = shard_hooks(_hooks("cuda:0"), dist.group.WORLD, rank, world, n)
        assert isinstance(h.bit_mapper.mapping_network[1], GroupBatchNorm1d)
        assert h.bit_mapper._fusable(), "the fused kernels must take the process-group BatchNorm"
        q.put((rank, _step(h, [f[sl] for f in feats], [g[sl] for g in G], [gb[sl] for gb in GB], "cuda:0",
                           dist.group.WORLD)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _rel(got, ref, rtol, floor=1e-30, what=""):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = float(np.abs(got - ref).max()) if ref.size else 0.0
    scale = max(float(np.abs(ref).max()) if ref.size else 0.0, floor)
    assert err <= rtol * scale, "%s: max err %g vs scale %g" % (what, err, scale)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_qat_step_equals_single_process(world):
    import torch.multiprocessing as mp
    feats, G, GB = _inputs()
    outs, bits, gx, grads, bufs, nfused = _step(_hooks("cuda:0"), feats, G, GB, "cuda:0")
    assert nfused == 3    # the fused train-mode mapper for each hook scale
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_entry, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = B // world
    gmax = {}
    for k, v in grads.items():
        mod = k.rsplit(".", 2)[0]
        gmax[mod] = max(gmax.get(mod, 0.0), float(np.abs(v).max()))
    for r in range(world):
        r_outs, r_bits, r_gx, r_grads, r_bufs, r_nfused = res[r]
        assert r_nfused == 3, "the sharded step must run the fused mapper kernels"
        sl = slice(r * n, (r + 1) * n)
        # the mapper runs on the global batch (train_step.DP_GLOBAL_MAPPER):
        # bits, y, feature gradients and buffers are the single process's
        for s in range(3):
            assert np.array_equal(r_bits[s], bits[s][sl]), "bits %d" % s
            assert np.array_equal(r_outs[s], outs[s][sl]), "y %d" % s
            assert np.array_equal(r_gx[s], gx[s][sl]), "grad x %d" % s
        assert set(r_grads) == set(grads)
        for k, v in grads.items():
            mod = k.rsplit(".", 2)[0]
            if k.startswith("bit_mapper.") and k.endswith(("0.bias", "3.bias", "6.bias", "0.weight", "3.weight",
                                                           "6.weight")):
                _rel(r_grads[k], v, 1e-4, floor=gmax[mod], what=k)   # see test_train_fused_gpu._cmp_grads
            else:
                _rel(r_grads[k], v, 1e-3, floor=1e-3 * gmax[mod], what=k)
        for k, v in bufs.items():
            assert np.array_equal(r_bufs[k], v), k
