"""Batch-sharded multi-process path on CPU (gloo, world_size 2): the one
exchange of the hook path - the per-channel batch min/max all-reduce
(engine.sync_channel_minmax) - makes every rank's statistics equal to the
single-process statistics of the global batch (quantization.py:650-654),
which is what lets a rank quantize its shard exactly like the reference run
on the whole batch."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, shards, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mcaq_yolo_amd.engine import sync_channel_minmax
    bufs = []
    for x in shards[rank]:
        t = torch.from_numpy(x)
        bufs.append({"xmin": t.amin(dim=(0, 2, 3)).contiguous(), "xmax": t.amax(dim=(0, 2, 3)).contiguous()})
    sync_channel_minmax(bufs, dist.group.WORLD)
    q.put((rank, [(b["xmin"].numpy(), b["xmax"].numpy()) for b in bufs]))
    dist.barrier()
    dist.destroy_process_group()


def test_channel_minmax_allreduce_two_ranks():
    rng = np.random.default_rng(3)
    shapes = [(4, 16, 8, 8), (4, 32, 4, 4), (4, 64, 2, 2)]
    full = [rng.standard_normal(s).astype(np.float32) * rng.uniform(0.5, 3.0) for s in shapes]
    full[1][2:, 5] += 100.0     # a channel whose max lives on rank 1 only
    full[2][:2, 7] -= 100.0     # a channel whose min lives on rank 0 only
    shards = [[f[:2].copy() for f in full], [f[2:].copy() for f in full]]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, shards, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        for f, (mn, mx) in zip(full, res[r]):
            assert np.array_equal(mn, f.min(axis=(0, 2, 3)))
            assert np.array_equal(mx, f.max(axis=(0, 2, 3)))
