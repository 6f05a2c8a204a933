"""Launch sets: several independent batches in ONE launch of each kernel
(engine.HookPlan(batches=k)).

Every batch of a launch set has its own statistics (quantization.py:650-654:
the per-channel min/max is over ITS batch), its own outputs and its own
batch_offset / batch_total, so each must be bit-identical to the same batch
run alone - bits, complexity, m(tile), channel min/max and y - and to the
oracle on its first two images.  (The batch-sharded form of a launch set,
with its RCCL all-reduce inside the HIP graph: tests/test_rccl_graph_gpu.py.)
"""
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
