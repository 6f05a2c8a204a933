"""Data-parallel pieces beyond the min/max all-reduce, on CPU with gloo
(world_size 2; the GPU path runs the same code over RCCL):

* postprocess.gather_detections - detections of every rank's shard, in rank
  order (inference.py:213-219 / SURVEY 8(e));
* the quantizer's EMA statistics over the global batch in QAT
  (quantization.py:319-353 with `process_group`): every rank's running
  min/max and its shard of y equal the single-process run on the full batch;
* dist.sync_mapper_batchnorm + dist.allreduce_gradients: the train-mode bit
  mapper (BatchNorm1d over the batch's tiles, bit_allocation.py:126) on two
  shards gives the single-process bits, BN running statistics and parameter
  gradients of the concatenated batch (summation order: rtol 1e-5 / 1e-4).
Unmeasured on multi-GPU hardware here (one-GPU pool); correctness only."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, load_weights


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, world=2, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_entry, args=(fn, r, world, port, q, args)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _entry(fn, rank, world, port, q, args):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, globals()[fn](rank, world, *args)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _sd(prefix):
    W = load_weights()
    return {k[len(prefix):]: torch.from_numpy(np.asarray(v)) for k, v in W.items() if k.startswith(prefix)}


# ---------------------------------------------------------------------------
def _gather_worker(rank, world):
    from mcaq_yolo_amd.postprocess import gather_detections
    g = torch.Generator().manual_seed(rank)
    out = torch.rand(3, 10, 6, generator=g)
    cnt = torch.tensor([rank, 2, 7], dtype=torch.int32)
    go, gc = gather_detections(out, cnt, dist.group.WORLD)
    return go.numpy(), gc.numpy()


def test_gather_detections_two_ranks():
    res = _run("_gather_worker")
    want = np.concatenate([torch.rand(3, 10, 6, generator=torch.Generator().manual_seed(r)).numpy()
                           for r in range(2)])
    for r in range(2):
        go, gc = res[r]
        assert np.array_equal(go, want)
        assert gc.tolist() == [0, 2, 7, 1, 2, 7]


# ---------------------------------------------------------------------------
def _qat_case():
    d = np.load(os.path.join(GOLDEN, "qat_p4_smooth.npz"))
    x = torch.from_numpy(d["x"])
    x = torch.cat([x, torch.flip(x, dims=[0]) * 1.25])        # 4 images
    bits = torch.from_numpy(d["bits"])
    bits = torch.cat([bits, torch.flip(bits, dims=[0])])
    return x, bits


def _qat_ema_run(x, bits, group):
    from mcaq_yolo_amd import core
    q = core.SpatialAdaptiveQuantization()
    q.soft_mask.load_state_dict(_sd("soft_mask."))
    q.process_group = group
    q.train()
    ys = []
    for step in range(3):
        xx = x * (1.0 + 0.1 * step)
        ys.append(q(xx, bits, training=True).detach())
    return q.running_min.numpy(), q.running_max.numpy(), ys[-1].numpy()


def _qat_ema_worker(rank, world):
    x, bits = _qat_case()
    n = x.shape[0] // world
    return _qat_ema_run(x[rank * n:(rank + 1) * n], bits[rank * n:(rank + 1) * n], dist.group.WORLD)


def test_qat_ema_statistics_two_ranks():
    x, bits = _qat_case()
    rmin, rmax, y = _qat_ema_run(x, bits, None)
    res = _run("_qat_ema_worker")
    n = x.shape[0] // 2
    for r in range(2):
        assert np.array_equal(res[r][0], rmin) and np.array_equal(res[r][1], rmax)
        assert np.array_equal(res[r][2], y[r * n:(r + 1) * n])


# ---------------------------------------------------------------------------
def _mapper_run(c, g, group, world):
    from mcaq_yolo_amd import core
    from mcaq_yolo_amd import dist as mdist
    m = core.ComplexityToBitMappingNetwork()
    m.load_state_dict(_sd("bit_mapper."))
    if group is not None:
        mdist.sync_mapper_batchnorm(m, group)
    m.train()
    c = c.clone().requires_grad_(True)
    bits = m(c, 1.0, return_continuous=True)
    # the global loss is the sum of the ranks' losses; the collective's
    # autograd carries every rank's share of the BatchNorm statistics, so the
    # summed (not averaged) parameter gradients equal the single-process ones
    (bits * g).sum().backward()
    if group is not None:
        mdist.allreduce_gradients(m.parameters(), group, average=False)
    grads = {n: p.grad.numpy().copy() for n, p in m.mapping_network.named_parameters()}
    bufs = {n: b.numpy().copy() for n, b in m.mapping_network.named_buffers() if b.dtype.is_floating_point}
    return bits.detach().numpy(), grads, bufs, c.grad.numpy()


def _mapper_case():
    d = np.load(os.path.join(GOLDEN, "train_mapper.npz"))
    return torch.from_numpy(d["t1.c"]), torch.from_numpy(d["t1.gb"])


def _mapper_worker(rank, world):
    c, g = _mapper_case()
    n = c.shape[0] // world
    return _mapper_run(c[rank * n:(rank + 1) * n], g[rank * n:(rank + 1) * n], dist.group.WORLD, world)


def test_mapper_sync_batchnorm_and_grad_allreduce_two_ranks():
    c, g = _mapper_case()
    bits, grads, bufs, gc = _mapper_run(c, g, None, 1)
    res = _run("_mapper_worker")
    n = c.shape[0] // 2
    gmax = max(np.abs(v).max() for v in grads.values())
    for r in range(2):
        rb, rg, rbuf, rgc = res[r]
        np.testing.assert_allclose(rb, bits[r * n:(r + 1) * n], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(rgc, gc[r * n:(r + 1) * n], rtol=1e-4, atol=1e-4 * np.abs(gc).max())
        for k, v in grads.items():
            np.testing.assert_allclose(rg[k], v, rtol=1e-4, atol=1e-4 * gmax, err_msg=k)
        for k, v in bufs.items():
            np.testing.assert_allclose(rbuf[k], v, rtol=1e-5, atol=1e-6, err_msg=k)


# ---------------------------------------------------------------------------
def _none_grad_worker(rank, world):
    from mcaq_yolo_amd import dist as mdist
    a = torch.nn.Parameter(torch.zeros(3))
    b = torch.nn.Parameter(torch.zeros(5))
    c = torch.nn.Parameter(torch.zeros(2))
    # rank 0 leaves b's grad None, rank 1 leaves a's: the buckets still line up
    if rank == 0:
        a.grad, c.grad = torch.full((3,), 1.0), torch.full((2,), 10.0)
    else:
        b.grad, c.grad = torch.full((5,), 2.0), torch.full((2,), 20.0)
    d = torch.nn.Parameter(torch.zeros(4))          # None on every rank
    mdist.allreduce_gradients([a, b, d, c], dist.group.WORLD)
    return a.grad.numpy(), b.grad.numpy(), c.grad.numpy(), d.grad


def test_allreduce_gradients_ranks_disagree_on_none():
    res = _run("_none_grad_worker")
    for r in range(2):
        a, b, c, d = res[r]
        assert d is None        # globally unused: stays None (optimizers skip it), as DDP leaves it
        assert np.array_equal(a, np.full(3, 0.5, np.float32))
        assert np.array_equal(b, np.full(5, 1.0, np.float32))
        assert np.array_equal(c, np.full(2, 15.0, np.float32))


def _bn_large_mean_worker(rank, world):
    from mcaq_yolo_amd.dist import GroupBatchNorm1d
    x = _bn_large_mean_case()
    n = x.shape[0] // world
    bn = GroupBatchNorm1d(x.shape[1], process_group=dist.group.WORLD).train()
    y = bn(x[rank * n:(rank + 1) * n])
    return y.detach().numpy(), bn.running_var.numpy()


def _bn_large_mean_case():
    g = torch.Generator().manual_seed(5)
    return 1e4 + 0.5 * torch.randn(64, 6, generator=g)     # |mean| >> std


def test_group_batchnorm_large_mean_two_ranks():
    """|mean| = 1e4, std 0.5: E[x^2] - mean^2 in fp32 loses the variance; the
    two-pass global statistics match the single-process BatchNorm1d."""
    x = _bn_large_mean_case()
    bn = torch.nn.BatchNorm1d(6).train()
    y = bn(x).detach().numpy()
    res = _run("_bn_large_mean_worker")
    for r in range(2):
        np.testing.assert_allclose(res[r][0], y[r * 32:(r + 1) * 32], rtol=1e-3, atol=2e-3)
        np.testing.assert_allclose(res[r][1], bn.running_var.numpy(), rtol=1e-3)


def _sink_worker(rank, world):
    from mcaq_yolo_amd import core
    p = torch.nn.Parameter(torch.zeros(3))
    r = (core._grads_observed([p]), core._GradSink().target([p]) is None)
    # marked by dist.shard_hooks (this package's own gradient all-reduce, no
    # DDP reducer): the sinks stay on
    q = torch.nn.Parameter(torch.zeros(3))
    q._mcaq_dp_manual = True
    return r + (core._grads_observed([q]), core._GradSink().target([q]) is None)


def test_direct_grad_accumulation_off_under_torch_distributed():
    """with torch.distributed initialised (DDP's reducer hooks every
    parameter's AccumulateGrad) or a parameter hook registered, the fused
    backwards return their gradients to autograd instead of writing .grad."""
    from mcaq_yolo_amd import core
    p = torch.nn.Parameter(torch.zeros(3))
    assert not core._grads_observed([p])
    p.register_hook(lambda g: g)
    assert core._grads_observed([p])
    q = torch.nn.Parameter(torch.zeros(3))
    q.register_post_accumulate_grad_hook(lambda t: None)
    assert core._grads_observed([q])
    res = _run("_sink_worker")
    assert [tuple(res[r]) for r in range(2)] == [(True, True, False, False), (True, True, False, False)]


def test_allreduce_gradients_cached_pattern_no_host_sync():
    """static_pattern=True: second and later calls reuse the global pattern
    agreed on the first: no device-to-host read (.tolist()), so the call can
    sit inside a captured step.  World size 1 (gloo)."""
    import os
    import torch.distributed as dist
    from mcaq_yolo_amd import dist as mdist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = "29611"
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        a = torch.nn.Parameter(torch.ones(3))
        b = torch.nn.Parameter(torch.ones(2))
        a.grad = torch.full((3,), 2.0)
        mdist.allreduce_gradients([a, b], dist.group.WORLD, static_pattern=True)
        assert b.grad is None and torch.equal(a.grad, torch.full((3,), 2.0))
        calls = {"n": 0}
        orig = torch.Tensor.tolist

        def spy(self):
            calls["n"] += 1
            return orig(self)
        torch.Tensor.tolist = spy
        try:
            a.grad = torch.full((3,), 5.0)
            mdist.allreduce_gradients([a, b], dist.group.WORLD, static_pattern=True)
        finally:
            torch.Tensor.tolist = orig
        assert calls["n"] == 0 and b.grad is None and torch.equal(a.grad, torch.full((3,), 5.0))
    finally:
        dist.destroy_process_group()


def _changing_pattern_worker(rank, world, static):
    """rank 1 leaves b's gradient None on the second call only;
    the ranks' buckets must still match (gloo aborts on a size mismatch)."""
    from mcaq_yolo_amd import dist as mdist
    a = torch.nn.Parameter(torch.zeros(3))
    b = torch.nn.Parameter(torch.zeros(2))
    out = []
    for call in range(3):
        a.grad = torch.full((3,), float(rank + 1))
        b.grad = None if (rank == 1 and call == 1) else torch.full((2,), 10.0 * (rank + 1))
        mdist.allreduce_gradients([a, b], dist.group.WORLD, static_pattern=static)
        out.append((a.grad.numpy().copy(), None if b.grad is None else b.grad.numpy().copy()))
    return out


@pytest.mark.parametrize("static", [False, True])
def test_allreduce_gradients_local_pattern_changes(static):
    res = _run("_changing_pattern_worker", 2, static)
    for r in range(2):
        for call in range(3):
            a, b = res[r][call]
            assert np.array_equal(a, np.full(3, 1.5, np.float32))
            # call 1: only rank 0 contributes b (a None sends zeros): (10 + 0) / 2
            assert np.array_equal(b, np.full(2, 5.0 if call == 1 else 15.0, np.float32))


def _static_unused_worker(rank, world):
    from mcaq_yolo_amd import dist as mdist
    a = torch.nn.Parameter(torch.zeros(3))
    b = torch.nn.Parameter(torch.zeros(2))
    a.grad = torch.ones(3)
    mdist.allreduce_gradients([a, b], dist.group.WORLD, static_pattern=True)     # b unused everywhere: cached
    first = b.grad is None
    b.grad = torch.ones(2)
    try:
        mdist.allreduce_gradients([a, b], dist.group.WORLD, static_pattern=True)
        raised = False
    except ValueError:
        raised = True
    return first, raised


def test_allreduce_gradients_static_pattern_rejects_new_gradient():
    res = _run("_static_unused_worker")
    assert [tuple(res[r]) for r in range(2)] == [(True, True), (True, True)]


def test_flat_span_in_place_bucket():
    """Gradients tiling one buffer (the hook nets' sink arena) are reduced in
    place as that buffer; anything else is not a span."""
    from mcaq_yolo_amd.dist import _flat_span
    buf = torch.arange(10, dtype=torch.float32)
    g = [buf[4:10], buf[0:3], buf[3:4]]
    sp = _flat_span(g)
    assert sp is not None and sp.data_ptr() == buf.data_ptr() and sp.numel() == 10
    assert _flat_span([buf[0:3], buf[4:10]]) is None          # gap
    assert _flat_span([buf[0:3], torch.zeros(2)]) is None      # two buffers
    sp.mul_(2)
    assert torch.equal(buf, 2 * torch.arange(10, dtype=torch.float32))
