"""The batch-sharded (N > 1) steps as bench.py runs them on the nccl (RCCL)
backend, exercised on the one GPU with a world_size 1 nccl process group on
cuda:0: the collectives really run through RCCL and are captured inside the
step's HIP graph, and on one rank each is the identity, so every value must
equal the unsharded step.

* inference: the statistics as [-min | max] in one buffer, ONE in-place MAX
  all-reduce between the finalize and pass 2 (engine.HookPlan shared_stats),
  for one batch and for a 2-batch launch set; and the MCAQHooks eval path
  with dist.shard_hooks;
* QAT (BASELINE config 5's step): dist.shard_hooks (GroupBatchNorm1d mapper
  statistics all-gathered / all-reduced between the fused stage launches, EMA
  min/max all-reduced) + dist.allreduce_gradients, the whole step captured in
  one HIP graph and replayed, against the unsharded eager step (tolerances of
  test_dist_qat_gpu.py: the staged BatchNorm combines per-rank partials).
The 2-rank value tests stay on gloo (test_dist_hooks.py, test_dist_qat_gpu.py).
"""
import socket

import pytest

from test_launch_set_gpu import CONFIG2, KEYS, _feats, _snap, blobs, dev  # noqa: F401

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl1(dev):
    """A world_size 1 process group on the nccl (RCCL) backend on cuda:0."""
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group is already initialised")
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1,
                            device_id=dev)
    yield dist.group.WORLD
    dist.destroy_process_group()


@pytest.mark.parametrize("nbat", [1, 2])
def test_sharded_step_rccl_allreduce_in_graph(dev, blobs, nccl1, nbat):
    """The batch-sharded step as bench.py runs it with N > 1: the statistics
    as [-min | max] in one buffer, ONE in-place MAX all-reduce over RCCL
    between the finalize and pass 2, all captured in one HIP graph.  On one
    rank it must equal the unsharded step bit for bit (the collective is the
    identity), for every batch of the launch set."""
    import torch
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    W, cm, mm, sm = blobs
    geoms = [ScaleGeom(*s, 8) for s in CONFIG2]
    feats = [_feats(CONFIG2, 500 + k, dev) for k in range(nbat)]
    arg = feats if nbat > 1 else feats[0]
    sh = HookPlan(geoms, dev, batches=nbat)
    sh.prepare(arg, cm, mm, [sm] * 3, shared_stats=True)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        sh.launch(st, nccl1)            # warm-up: communicator setup outside capture
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st, capture_error_mode="thread_local"):
        sh.launch(torch.cuda.current_stream(), nccl1)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    ref = HookPlan(geoms, dev, batches=nbat)
    ref.run(arg, cm, mm, [sm] * 3)
    torch.cuda.synchronize()
    for j in range(len(sh.geoms)):
        a, b = sh.bufs[j], ref.bufs[j]
        for key in ("bits", "complexity", "mt", "y"):
            assert torch.equal(a[key], b[key]), (j, key)
        mn, mx = sh.channel_minmax(j)
        assert torch.equal(mn, b["xmin"]) and torch.equal(mx, b["xmax"])
        assert torch.equal(a["xmin"], -b["xmin"])       # stored negated for the one MAX all-reduce


def test_sharded_hooks_eval_nccl_equals_unsharded(dev, nccl1):
    """MCAQHooks with a process group (dist.shard_hooks, world 1, nccl): the
    eval-mode hook path runs the shared-statistics plan and its all-reduce;
    outputs equal the unsharded hooks'."""
    import torch
    from mcaq_yolo_amd.dist import shard_hooks
    from mcaq_yolo_amd.hooks import MCAQHooks
    import bench
    feats = _feats(CONFIG2, 700, dev)
    outs = []
    for sharded in (False, True):
        torch.manual_seed(0)
        h = MCAQHooks(grid_size=8, bit_mapping="mlp", device=dev)
        h.load_state_dict(bench.hook_state_dict(dev), strict=False)
        h.eval()
        if sharded:
            shard_hooks(h, nccl1, 0, 1, CONFIG2[0][0])
        with torch.no_grad():
            y, aux = h.forward_features(feats)
        torch.cuda.synchronize()
        outs.append(([t.clone() for t in y], [a["bit_map"].clone() for a in aux]))
    for a, b in zip(outs[0][0] + outs[0][1], outs[1][0] + outs[1][1]):
        assert torch.equal(a, b)


def test_sharded_qat_step_nccl_graph_equals_unsharded(dev, nccl1):
    """Config 5's QAT step (forward, backward, gradient all-reduce) with the
    batch-sharding collectives on RCCL, captured in one HIP graph and
    replayed: after the same number of steps the outputs, bit maps, feature
    and parameter gradients and every floating buffer (EMA min/max, mapper
    running statistics) equal the unsharded eager step's."""
    import torch
    from mcaq_yolo_amd.dist import allreduce_gradients, shard_hooks
    from test_dist_qat_gpu import B, _hooks, _inputs, _rel
    feats, G, GB = _inputs()
    G = [g.to(dev) for g in G]
    GB = [g.to(dev) for g in GB]

    def make(sharded):
        h = _hooks(dev)
        if sharded:
            shard_hooks(h, nccl1, 0, 1, B)
        xs = [f.to(dev).requires_grad_(True) for f in feats]
        params = [p for p in h.parameters() if p.requires_grad]
        rec = {}

        def step():
            for p in params:
                p.grad = None
            for x in xs:
                x.grad = None
            outs, aux = h.forward_features(xs, temperature=1.0)
            loss = sum((o * g).sum() for o, g in zip(outs, G)) + sum((a["bit_map"] * gb).sum() for a, gb in zip(aux, GB))
            loss.backward()
            if sharded:
                allreduce_gradients(params, nccl1, average=True, static_pattern=True)
            rec["outs"] = [o.detach() for o in outs]
            rec["bits"] = [a["bit_map"].detach() for a in aux]
            rec["gx"] = [x.grad for x in xs]
            rec["grads"] = {k: p.grad for k, p in h.named_parameters() if p.grad is not None}
        return h, step, rec

    h0, step0, rec0 = make(False)
    for _ in range(3):
        step0()
    h1, step1, rec1 = make(True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step1()                              # lazy state, communicators, the has-grad pattern
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):   # the watchdog thread polls meanwhile
        step1()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    # the mapper runs on the global batch (train_step.DP_GLOBAL_MAPPER): at
    # world 1 the forward values and feature gradients are the unsharded ones
    for k in ("outs", "bits", "gx"):
        for i, (a, b) in enumerate(zip(rec1[k], rec0[k])):
            assert torch.equal(a, b), "%s %d" % (k, i)
    assert set(rec1["grads"]) == set(rec0["grads"])
    for k, v in rec0["grads"].items():
        _rel(rec1["grads"][k].cpu().numpy(), v.cpu().numpy(), 1e-3, floor=1e-3 * float(v.abs().max()) + 1e-30,
             what=k)
    b0 = {k: b for k, b in h0.named_buffers() if b is not None and b.dtype.is_floating_point}
    b1 = {k: b for k, b in h1.named_buffers() if b is not None and b.dtype.is_floating_point}
    assert set(b0) == set(b1)
    for k in b0:
        _rel(b1[k].cpu().numpy(), b0[k].cpu().numpy(), 1e-5, floor=1e-6, what=k)


def test_sharded_qat_step_issues_three_collectives(dev, nccl1):
    """the batch-sharded QAT step (dist.shard_hooks) keeps the
    fused fast path - gradient sinks in one arena, the mapper on the global
    batch - and issues 3 collectives per step: the forward all-gather (mapper
    inputs + EMA min / max), the backward all-gather (bit gradients) and ONE
    in-place gradient all-reduce over the arena (no concatenation)."""
    import torch
    import torch.distributed as dist
    from mcaq_yolo_amd.dist import allreduce_gradients, shard_hooks
    from test_dist_qat_gpu import B, _hooks, _inputs
    feats, G, _ = _inputs()
    G = [g.to(dev) for g in G]
    h = shard_hooks(_hooks(dev), nccl1, 0, 1, B)
    xs = [f.to(dev).requires_grad_(True) for f in feats]
    params = [p for p in h.parameters() if p.requires_grad]
    arena = h._grad_arena.flat

    def step():
        for p in params:
            p.grad = None
        outs, aux = h.forward_features(xs, temperature=1.0)
        torch.autograd.backward(list(outs) + [h.bit_budget_loss(aux, 4.0)],
                                list(G) + [torch.full((), 0.1, device=dev)])
        allreduce_gradients(params, nccl1, static_pattern=True)
    step()
    calls = []
    names = ("all_reduce", "all_gather", "all_gather_into_tensor", "broadcast", "reduce_scatter_tensor")
    orig = {n: getattr(dist, n) for n in names}

    def spy(n):
        def f(t, *a, **k):
            calls.append((n, t))
            return orig[n](t, *a, **k)
        return f
    for n in names:
        setattr(dist, n, spy(n))
    try:
        step()
    finally:
        for n in names:
            setattr(dist, n, orig[n])
    torch.cuda.synchronize()
    assert [c[0] for c in calls] == ["all_gather_into_tensor", "all_gather_into_tensor", "all_reduce"], calls
    red = calls[-1][1]
    assert red.data_ptr() == arena.data_ptr() and red.numel() == arena.numel()
    assert all(p.grad.untyped_storage().data_ptr() == arena.untyped_storage().data_ptr() for p in params)
