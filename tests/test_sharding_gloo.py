"""Multi-process (world_size 2, gloo, CPU) check of the sharded bench path
(SURVEY §8e): contiguous item blocks per rank, parameters drawn on the
global stream so each item's parameters do not depend on the number of
ranks, backgrounds broadcast from rank 0, max-over-ranks timing."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from image_processor_pipeline_amd import fused


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_global, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, stop = fused.shard_range(n_global, rank, world)
        cfg = fused.PipeConfig(margins=(8, 8, 8, 8))
        plan = fused.plan_pipe((96, 80), stop - start, (64, 72), 3, cfg, seed=5, item_range=(start, stop),
                                n_global=n_global)
        bgs = torch.zeros((3, 64, 72, 3), dtype=torch.uint8)
        if rank == 0:
            bgs.copy_(torch.randint(0, 256, bgs.shape, dtype=torch.uint8, generator=torch.Generator().manual_seed(1)))
        dist.broadcast(bgs, src=0)
        params = [None] * world
        dist.all_gather_object(params, [(p.angle, p.sym, p.bg_index, p.ratio, p.x, p.y) for p in plan.params])
        t = torch.tensor([0.5 + rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            result_q.put((params, int(bgs.sum()), float(t.item())))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    for n in (0, 1, 7, 4096):
        for w in (1, 2, 3, 8):
            rs = [fused.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    with pytest.raises(ValueError):
        fused.shard_range(4, 2, 2)


def test_two_rank_plan_matches_single_process():
    n_global, world = 9, 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _free_port(), n_global, q), nprocs=world, join=True,
                       start_method="spawn")
    params, bg_sum, tmax = q.get()
    single = fused.plan_pipe((96, 80), n_global, (64, 72), 3, fused.PipeConfig(margins=(8, 8, 8, 8)), seed=5)
    exp = [(p.angle, p.sym, p.bg_index, p.ratio, p.x, p.y) for p in single.params]
    assert [tuple(x) for part in params for x in part] == exp
    ref_bg = torch.randint(0, 256, (3, 64, 72, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(1))
    assert bg_sum == int(ref_bg.sum())
    assert tmax == 1.5
