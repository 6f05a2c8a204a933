"""Launch sets: several independent batches in ONE launch of each kernel
(engine.HookPlan(batches=k)).

Every batch of a launch set has its own statistics (quantization.py:650-654:
the per-channel min/max is over ITS batch), its own outputs and its own
batch_offset / batch_total, so each must be bit-identical to the same batch
run alone - bits, complexity, m(tile), channel min/max and y - and to the
oracle on its first two images.  Also the batch-sharded form of the step:
statistics as [-min | max] in one buffer, combined by one in-place RCCL
all-reduce captured inside the step's HIP graph (world_size 1 nccl group on
cuda:0), equal to the unsharded step.
"""
import socket

import numpy as np
import pytest

from conftest import load_weights
from oracle import mcaq_oracle as O

pytestmark = pytest.mark.gpu

CONFIG2 = [(32, 64, 80, 80), (32, 128, 40, 40), (32, 256, 20, 20)]


@pytest.fixture(scope="module")
def dev():
    import torch
    from mcaq_yolo_amd import abi
    abi.lib()
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def blobs(dev):
    import torch
    from mcaq_yolo_amd import params
    W = load_weights()
    cm = torch.from_numpy(params.pack_complexity_mlp(params.sub(W, "complexity_analyzer."))).to(dev)
    mm = torch.from_numpy(params.pack_mapper_mlp(params.sub(W, "bit_mapper."))).to(dev)
    sm = torch.from_numpy(params.pack_soft_mask(params.sub(W, "soft_mask."))).to(dev)
    return W, cm, mm, sm


def _feats(shapes, seed, dev):
    import torch
    import torch.nn.functional as F
    g = torch.Generator(device="cpu").manual_seed(seed)
    out = []
    for s in shapes:
        lo = torch.randn(s[0], s[1], s[2] // 8, s[3] // 8, generator=g)
        out.append(F.silu(1.5 * torch.randn(s, generator=g) +
                          2.0 * F.interpolate(lo, size=s[2:], mode="bilinear")).contiguous().to(dev))
    return out


KEYS = ("bits", "complexity", "mt", "y", "xmin", "xmax")


def _snap(bufs):
    return [{k: b[k].clone() for k in KEYS} for b in bufs]


@pytest.mark.parametrize("nbat,band,tiles_batch", [(2, False, False), (3, False, False), (2, True, True)])
def test_launch_set_equals_solo_runs(dev, blobs, monkeypatch, nbat, band, tiles_batch):
    """Config-2 shapes (yolov8n bs32 C3/C4/C5), k independent batches per
    launch: each batch bit-identical to its solo run and, on its first two
    images, to the oracle (with its own batch min/max)."""
    import torch
    from mcaq_yolo_amd import engine
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    monkeypatch.setattr(engine, "BAND_PASS", band)
    monkeypatch.setattr(engine, "TILES_BATCH", tiles_batch)
    W, cm, mm, sm = blobs
    geoms = [ScaleGeom(*s, 8) for s in CONFIG2]
    feats = [_feats(CONFIG2, 100 + k, dev) for k in range(nbat)]
    ls = HookPlan(geoms, dev, batches=nbat)
    assert len(ls.geoms) == 3 * nbat and ls.seg[:2] == [(0, 0), (0, 1)]    # scale-major segments
    ls.run(feats, cm, mm, [sm] * 3)
    torch.cuda.synchronize()
    got = [_snap(ls.batch_bufs(k)) for k in range(nbat)]
    solo = HookPlan(geoms, dev)
    for k in range(nbat):
        want = _snap(solo.run(feats[k], cm, mm, [sm] * 3))
        torch.cuda.synchronize()
        for si in range(3):
            for key in KEYS:
                assert torch.equal(got[k][si][key], want[si][key]), "batch %d scale %d %s" % (k, si, key)
            f = feats[k][si]
            assert torch.equal(got[k][si]["xmin"], f.amin(dim=(0, 2, 3)))
            assert torch.equal(got[k][si]["xmax"], f.amax(dim=(0, 2, 3)))
    for k in range(nbat):
        for si in range(3):
            x2 = feats[k][si][:2].cpu().numpy()
            ref = O.hook_forward(x2, W, 8, xmin=got[k][si]["xmin"].cpu().numpy(),
                                 xmax=got[k][si]["xmax"].cpu().numpy(), batch_total=32)
            assert np.array_equal(got[k][si]["bits"][:2].cpu().numpy(), ref["bits"]), "bits vs oracle"
            assert np.array_equal(got[k][si]["complexity"][:2].cpu().numpy(), ref["complexity"])
            assert np.array_equal(got[k][si]["y"][:2].cpu().numpy(), ref["y"]), "y vs oracle"


def test_launch_set_graph_replay_equals_eager(dev, blobs):
    """A 2-batch launch set captured in a HIP graph and replayed on new inputs
    (copied in place) equals the eager launch set on those inputs."""
    import torch
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    W, cm, mm, sm = blobs
    shapes = [(8, 64, 80, 80), (8, 128, 40, 40), (8, 256, 20, 20)]
    geoms = [ScaleGeom(*s, 8) for s in shapes]
    feats = [_feats(shapes, 300 + k, dev) for k in range(2)]
    ls = HookPlan(geoms, dev, batches=2)
    ls.prepare(feats, cm, mm, [sm] * 3)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        ls.launch(st)
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        ls.launch(torch.cuda.current_stream())
    new = [_feats(shapes, 400 + k, dev) for k in range(2)]
    for fb, nb in zip(feats, new):
        for f, n in zip(fb, nb):
            f.copy_(n)
    g.replay()
    torch.cuda.synchronize()
    got = [_snap(ls.batch_bufs(k)) for k in range(2)]
    ref = HookPlan(geoms, dev, batches=2)
    ref.run(new, cm, mm, [sm] * 3)
    torch.cuda.synchronize()
    for k in range(2):
        for a, b in zip(got[k], _snap(ref.batch_bufs(k))):
            for key in KEYS:
                assert torch.equal(a[key], b[key]), key


def test_launch_set_segment_limit(dev):
    from mcaq_yolo_amd import abi
    from mcaq_yolo_amd.engine import HookPlan, ScaleGeom
    geoms = [ScaleGeom(*s, 8) for s in CONFIG2]
    with pytest.raises(ValueError):
        HookPlan(geoms, dev, batches=abi.MAX_SEGMENTS // 3 + 1)


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
    with torch.cuda.graph(g, stream=st):
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
