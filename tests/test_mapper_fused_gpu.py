"""The train-mode bit mapper as ONE launch per direction
(train_step.MAPPER_FUSED: the batch statistics between its layers exchanged
inside the launch as write-through granules, no grid barrier) against the
staged launches (4 + 4, one per statistics barrier), bit for bit: outputs,
bits, complexity, feature and parameter gradients, parameters and buffers
over SGD steps, eager and replayed in a HIP graph, with the soft masks'
reductions riding on the backward launch; segment layouts that change
between calls; through the C ABI the options the hook step does not use;
no exchange timed out (the sync buffer's status word)."""
import pytest
import torch

from test_concurrent_scales_gpu import _feats, _run, _same
from test_train_fused_gpu import _hooks

pytestmark = pytest.mark.gpu


def _with(fused, **kw):
    from mcaq_yolo_amd import train_step
    old = train_step.MAPPER_FUSED
    train_step.MAPPER_FUSED = fused
    try:
        return _run(False, multi=True, **kw)
    finally:
        train_step.MAPPER_FUSED = old


@pytest.mark.parametrize("fused_mq", [False, True])
def test_fused_mapper_equals_staged_eager(fused_mq):
    _same(_with(True, steps=3, fused_mq=fused_mq, budget=fused_mq),
          _with(False, steps=3, fused_mq=fused_mq, budget=fused_mq))


def test_fused_mapper_equals_staged_graph():
    _same(_with(True, steps=3, graph=True, fused_mq=True, budget=True),
          _with(False, steps=4, fused_mq=True, budget=True))


@pytest.mark.parametrize("graph", [False, True])
def test_fused_head_reduction_equals_separate(graph):
    """train_step.HEAD_FUSED: the complexity MLP's parameter reduction inside
    its backward launch (granule exchange) against the separate chain
    reduction launch, bit for bit, eager and graph-replayed; status clear."""
    from mcaq_yolo_amd import train_step
    res = []
    for fused in (True, False):
        old = train_step.HEAD_FUSED
        train_step.HEAD_FUSED = fused
        try:
            res.append(_run(False, multi=True, steps=3, graph=graph, fused_mq=True, budget=True))
        finally:
            train_step.HEAD_FUSED = old
    _same(res[0], res[1])


def test_fused_mapper_one_launch_per_direction_and_layouts():
    """One fused forward and one fused backward call per step (no staged
    call); batches of 4, 2, 4 images (the layout changes, then comes back to a
    buffer with advanced epochs): every value equal to the staged path's and
    the status word clear."""
    from mcaq_yolo_amd import abi, train_step
    L = abi.lib()
    names = ("mcaq_mapper_train_forward_fused", "mcaq_mapper_train_backward_fused",
             "mcaq_mapper_train_forward_multi", "mcaq_mapper_train_backward_multi",
             "mcaq_mapper_train_backward_multi_ride")
    res = {}
    for fused in (True, False):
        calls = {n: 0 for n in names}
        orig = {n: getattr(L, n) for n in names}

        def spy(n):
            def f(*a):
                calls[n] += 1
                return orig[n](*a)
            return f
        for n in names:
            setattr(L, n, spy(n))
        old = train_step.MAPPER_FUSED
        train_step.MAPPER_FUSED = fused
        try:
            h = _hooks()
            out = []
            for B in (4, 2, 4):
                feats, gens = _feats(B=B, seed=11 + B)
                outs, aux = h.forward_features(feats, temperature=1.0)
                sum((o * g).sum() for o, g in zip(outs, gens)).backward()
                torch.cuda.synchronize()
                out += [a["bit_map"].detach().clone() for a in aux] + [o.detach().clone() for o in outs]
                out += [f.grad.clone() for f in feats]
            out += [p.grad.clone() for p in h.bit_mapper.parameters()]
            out += [b.clone() for b in h.bit_mapper.buffers()]
            if fused:
                assert train_step.mapper_sync_status(h.bit_mapper) == 0
                assert train_step.mapper_sync_status(h.complexity_analyzer) == 0
                assert len(h.bit_mapper._mapx) == 2          # two layouts, the first one reused
            res[fused] = out
        finally:
            train_step.MAPPER_FUSED = old
            for n in names:
                setattr(L, n, orig[n])
        if fused:
            assert calls["mcaq_mapper_train_forward_fused"] == 3 and calls["mcaq_mapper_train_backward_fused"] == 3
            assert calls["mcaq_mapper_train_forward_multi"] == 0
            assert calls["mcaq_mapper_train_backward_multi"] + calls["mcaq_mapper_train_backward_multi_ride"] == 0
        else:
            assert calls["mcaq_mapper_train_forward_fused"] == 0 and calls["mcaq_mapper_train_forward_multi"] == 3
    assert len(res[True]) == len(res[False])
    for i, (a, b) in enumerate(zip(res[True], res[False])):
        assert torch.equal(a, b), i


def test_fused_mapper_rejects_too_many_workgroups():
    """The launcher refuses a grid that could not be resident at once (the
    caller then takes the staged launches) and a missing or short buffer."""
    from mcaq_yolo_amd import abi
    L = abi.lib()
    mx = L.mcaq_mapper_fused_max_wg()
    assert mx >= 64
    assert L.mcaq_mapper_sync_bytes(1) == 64 * 4 + 3 * 129 * 8
    dev = torch.device("cuda")
    n = 64 * (mx + 1)
    c = torch.rand(n, device=dev)
    bits = torch.empty(n, device=dev)
    work = torch.empty(L.mcaq_mapper_work_floats(n), device=dev)
    h = _hooks()
    net = h.bit_mapper.mapping_network
    q = abi.MapperParams()
    for k, t in zip(("w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4"),
                    (net[0].weight, net[0].bias, net[3].weight, net[3].bias, net[6].weight, net[6].bias,
                     net[9].weight, net[9].bias)):
        setattr(q, k, t.data_ptr())
    segs = (abi.MapperSeg * 1)()
    segs[0].c, segs[0].bits, segs[0].work, segs[0].n = c.data_ptr(), bits.data_ptr(), work.data_ptr(), n
    sync = torch.zeros((L.mcaq_mapper_sync_bytes(mx + 1) + 7) // 8, dtype=torch.int64, device=dev)
    import ctypes
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    err = L.mcaq_mapper_train_forward_fused(ctypes.byref(q), segs, 1, 2.0, 8.0, 1.0, 0.1, 0, 0,
                                            ctypes.c_void_p(sync.data_ptr()), sync.numel() * 8, st)
    assert err != 0
    segs[0].n = 64
    err = L.mcaq_mapper_train_forward_fused(ctypes.byref(q), segs, 1, 2.0, 8.0, 1.0, 0.1, 0, 0, None, 0, st)
    assert err != 0
    err = L.mcaq_mapper_train_forward_fused(ctypes.byref(q), segs, 1, 2.0, 8.0, 1.0, 0.1, 0, 0,
                                            ctypes.c_void_p(sync.data_ptr()), 100, st)
    assert err != 0
    torch.cuda.synchronize()


def _mapper_struct(net):
    from mcaq_yolo_amd import abi
    q = abi.MapperParams()
    for k, t in zip(("w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4"),
                    (net[0].weight, net[0].bias, net[3].weight, net[3].bias, net[6].weight, net[6].bias,
                     net[9].weight, net[9].bias)):
        setattr(q, k, t.data_ptr())
    for i, j in enumerate((1, 4, 7), 1):
        bn = net[j]
        for k, t in (("g", bn.weight), ("be", bn.bias), ("rm", bn.running_mean), ("rv", bn.running_var),
                     ("nbt", bn.num_batches_tracked)):
            setattr(q, "%s%d" % (k, i), t.data_ptr())
    return q


@pytest.mark.parametrize("opts", [(1, 1, 0.0, (1000,)), (0, 0, 1.7, (130,)), (2, 1, 0.5, (64, 1000, 7)),
                                  (2, 0, 1.0, (4096, 65, 200))])
def test_fused_mapper_abi_options_equal_staged(opts):
    """Through the C ABI, the options the hook step does not use: the in-kernel
    running-statistics update (update_stats 1, one segment), rounded bits,
    no temperature, 1-3 segments of odd tile counts (one workgroup, partial
    last workgroups): bits, work buffers (activations, statistics, deferred
    running statistics), the BatchNorm running buffers, c's gradient and the
    parameter partials of the fused launches equal the staged launches'."""
    import copy
    import ctypes
    from mcaq_yolo_amd import abi, core
    update_stats, round_bits, T, ns = opts
    L = abi.lib()
    dev = torch.device("cuda")
    torch.manual_seed(11)
    base = core.ComplexityToBitMappingNetwork().to(dev).train()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cs = [torch.rand(n, device=dev) * 1.2 - 0.1 for n in ns]          # some outside [0, 1]: the clamp
    gbs = [torch.randn(n, device=dev) for n in ns]
    res = []
    for fused in (True, False):
        mod = copy.deepcopy(base)
        net = mod.mapping_network
        q = _mapper_struct(net)
        segs = (abi.MapperSeg * len(ns))()
        keep = []
        for i, (c, g) in enumerate(zip(cs, gbs)):
            n = c.numel()
            w = torch.zeros(L.mcaq_mapper_work_floats(n), device=dev)
            b = torch.empty(n, device=dev)
            gc = torch.empty(n, device=dev)
            gp = torch.zeros(L.mcaq_mapper_gpart_floats(n), device=dev)
            keep.append((w, b, gc, gp))
            s = segs[i]
            s.c, s.bits, s.work, s.gbits, s.gc, s.gpart, s.n = (c.data_ptr(), b.data_ptr(), w.data_ptr(), g.data_ptr(),
                                                                gc.data_ptr(), gp.data_ptr(), n)
        mom = 0.1
        if fused:
            total = sum((n + 63) // 64 for n in ns)
            sync = torch.zeros((L.mcaq_mapper_sync_bytes(total) + 7) // 8, dtype=torch.int64, device=dev)
            for _ in range(2):       # twice: the second launch runs on advanced epochs
                abi.check(L.mcaq_mapper_train_forward_fused(ctypes.byref(q), segs, len(ns), 2.0, 8.0, T, mom,
                                                            round_bits, update_stats, ctypes.c_void_p(sync.data_ptr()),
                                                            sync.numel() * 8, st), "fwd fused")
                abi.check(L.mcaq_mapper_train_backward_fused(ctypes.byref(q), segs, len(ns), 2.0, 8.0, T, None, 0,
                                                             ctypes.c_void_p(sync.data_ptr()), sync.numel() * 8, st),
                          "bwd fused")
            torch.cuda.synchronize()
            assert int(sync.view(torch.int32)[abi.MAPPER_SYNC_STATUS_WORD].item()) == 0
        else:
            for _ in range(2):
                abi.check(L.mcaq_mapper_train_forward_multi(ctypes.byref(q), segs, len(ns), 2.0, 8.0, T, mom,
                                                            round_bits, update_stats, st), "fwd staged")
                abi.check(L.mcaq_mapper_train_backward_multi(ctypes.byref(q), segs, len(ns), 2.0, 8.0, T, st),
                          "bwd staged")
            torch.cuda.synchronize()
        out = []
        for c, (w, b, gc, gp) in zip(cs, keep):
            n = c.numel()
            out += [b.clone(), gc.clone(), gp.clone()]
            # activations a1..a3, sigmoid output, and the statistics / deferred-statistics blocks
            acts = n * (32 + 64 + 32 + 1)
            out.append(w[:acts].clone())
            nwg = (n + 63) // 64
            stat0 = n * (32 + 64 + 32 + 1 + 64) + 2 * nwg * 128 + nwg
            out.append(w[stat0:stat0 + 3 * 128].clone())
            rst0 = stat0 + 3 * 128 + 2 * nwg * 128 + 64
            out.append(w[rst0:rst0 + 3 * 128].clone())
        out += [t.detach().clone() for t in mod.mapping_network.buffers()]
        res.append(out)
    for i, (a, b) in enumerate(zip(*res)):
        assert torch.equal(a, b), i
