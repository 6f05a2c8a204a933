"""Value-level test of the batch-sharded hook path: two (and four) ranks,
each running `dist.shard_hooks(MCAQHooks(...))` on its half of a batch, must
give exactly the bits, complexity and quantized y of ONE process running the
whole batch (and of the oracle on the whole batch).

What couples the shards (everything else is per image):
* the per-channel batch min/max of the quantizer (quantization.py:653-654):
  one all-reduce per hook;
* the fractal regression's outer sums over the S box scales (morphology.py:
  614-620): ATen picks the vectorised or the row_sum order of a tile by its
  column in the WHOLE (S, batch * tiles) tensor, so a shard must reduce as if
  it sat at its global position (batch_offset / batch_total).

The case is built so that this order matters: tile 32 (S = 5 scales, where
the two orders differ), 3 x 3 tiles per image and a global batch of 4
(36 columns, tail from column 32) - rank 1's columns 18..35 are all tail
columns in its local (18-column) reduction but only 32..35 are in the global
one.  A channel whose max lives on rank 1 only and one whose min lives on
rank 0 only exercise the all-reduce.

CPU: gloo, the pure-PyTorch path (hooks._run_scale_shard_cpu).  GPU (-m gpu):
gloo, both ranks on cuda:0, the HIP kernels with batch_offset / batch_total
and the min/max all-reduce between the passes."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT

GRID = 3
SHAPES = ((4, 8, 96, 96), (4, 16, 40, 40))     # grid 3: tile 32 (3x3 tiles) and tile 8 (5x5 tiles)
IDX = (4, 6)
WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _feats():
    g = torch.Generator().manual_seed(2024)
    out = []
    for i, (B, C, H, W) in enumerate(SHAPES):
        lo = torch.randn(B, C, H // 8, W // 8, generator=g)
        hi = torch.randn(B, C, H, W, generator=g)
        up = torch.nn.functional.interpolate(lo, size=(H, W), mode="bilinear", align_corners=False)
        x = torch.nn.functional.silu(1.5 * hi + 2.0 * up)
        x[2:, 1] += 3.0          # channel max only in rank 1's images
        x[:2, 2] -= 3.0          # channel min only in rank 0's images
        out.append(x.contiguous())
    return out


def _state_dict():
    w = np.load(os.path.join(GOLDEN, "weights.npz"))
    sd = {}
    for k in w.files:
        t = torch.from_numpy(np.array(w[k]))
        if k.startswith("soft_mask."):
            for idx in IDX:
                sd["quantizers.%d.%s" % (idx, k)] = t
        else:
            sd[k] = t
    return sd


def _hooks(dev):
    from mcaq_yolo_amd.hooks import MCAQHooks
    from oracle.mcaq_oracle import REF_THREADS
    h = MCAQHooks(grid_size=GRID, device=dev, indices=IDX)
    h.load_state_dict(_state_dict(), strict=False)
    h.to(dev).eval()
    h.softmax_threads = REF_THREADS
    return h


def _run_hooks(h, feats, dev):
    with torch.no_grad():
        outs, aux = h.forward_features([f.to(dev) for f in feats])
    if str(dev).startswith("cuda"):
        torch.cuda.synchronize()
    return [(o.cpu().numpy(), a["bit_map"].cpu().numpy(), a["complexity"].cpu().numpy())
            for o, a in zip(outs, aux)]


def _entry(rank, world, port, dev, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from oracle.mcaq_oracle import REF_THREADS
    torch.set_num_threads(REF_THREADS)     # the CPU path's softmax follows ATen's thread partition
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mcaq_yolo_amd.dist import shard_hooks
        if dev != "cpu":
            torch.cuda.set_device(0)
        feats = _feats()
        B = feats[0].shape[0] // world
        h = shard_hooks(_hooks(dev), dist.group.WORLD, rank, world, B)
        q.put((rank, _run_hooks(h, [f[rank * B:(rank + 1) * B].contiguous() for f in feats], dev)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _sharded(dev, world=WORLD):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_entry, args=(r, world, port, dev, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _check(res, full, world=WORLD):
    B = SHAPES[0][0] // world
    for r in range(world):
        sl = slice(r * B, (r + 1) * B)
        for s, ((y, bits, c), (fy, fbits, fc)) in enumerate(zip(res[r], full)):
            assert np.array_equal(bits, fbits[sl]), (r, s)
            assert np.array_equal(c, fc[sl]), (r, s)
            assert np.array_equal(y, fy[sl]), (r, s)


def test_fractal_order_depends_on_global_position():
    """The case really exercises the global column order: the oracle's phi1
    of rank 1's shard reduced at its local position differs from the global
    one for some tile (otherwise the test below would not bite)."""
    from oracle import mcaq_oracle as O
    x = _feats()[0].numpy()
    g = O.phi_tiles(x, GRID)[2:, ..., 0]
    loc = O.phi_tiles(x[2:], GRID)[..., 0]
    glob = O.phi_tiles(x[2:], GRID, batch_offset=2, batch_total=4)[..., 0]
    assert np.array_equal(glob, g)
    assert not np.array_equal(loc, g)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_hooks_cpu_equal_single_process(world):
    full = _run_hooks(_hooks("cpu"), _feats(), "cpu")
    _check(_sharded("cpu", world), full, world)


@pytest.mark.gpu
def test_sharded_hooks_gpu_equal_single_process_and_oracle():
    """Two ranks on the one GPU (gloo): the HIP path on shards equals the HIP
    path on the whole batch, the CPU path on the whole batch and the oracle."""
    from oracle import mcaq_oracle as O
    feats = _feats()
    full = _run_hooks(_hooks("cuda:0"), feats, "cuda:0")
    cpu = _run_hooks(_hooks("cpu"), feats, "cpu")
    W = O.load_weights(os.path.join(GOLDEN, "weights.npz"))
    for (y, bits, c), (cy, cbits, cc), f in zip(full, cpu, feats):
        ref = O.hook_forward(f.numpy(), W, GRID)
        assert np.array_equal(bits, ref["bits"]) and np.array_equal(y, ref["y"])
        assert np.array_equal(bits, cbits) and np.array_equal(y, cy)
    _check(_sharded("cuda:0"), full)


@pytest.mark.gpu
def test_sharded_hooks_gpu_four_ranks():
    """Four ranks (one image each) on the one GPU (gloo): the statistics
    exchange and the global fractal column order at world size 4."""
    full = _run_hooks(_hooks("cuda:0"), _feats(), "cuda:0")
    _check(_sharded("cuda:0", 4), full, 4)
