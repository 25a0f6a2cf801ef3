"""Tenant collectives on 2 CPU ranks (gloo): bucketed gradient averaging,
sharded reduce-scatter + all-gather, and the bus-bandwidth formula."""
from __future__ import annotations

import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nos_amd.parallel.collectives import GradBucketer, busbw, measure_allreduce


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        params = [torch.nn.Parameter(torch.zeros(n)) for n in (5, 1000, 7, 300)]
        for i, p in enumerate(params):
            p.grad = torch.full_like(p, float(rank + 1) * (i + 1))
        b = GradBucketer(params, bucket_bytes=2000)  # several buckets
        assert len(b.buckets) >= 2
        b.sync()
        ok = all(torch.allclose(p.grad, torch.full_like(p, 1.5 * (i + 1))) for i, p in enumerate(params))
        # sharded: reduce-scatter, "update" the shard, all-gather back
        for i, p in enumerate(params):
            p.grad = torch.full_like(p, float(rank + 1))
        sb = GradBucketer(params, bucket_bytes=1 << 20, sharded=True)
        shards = sb.sync()
        ok = ok and all(torch.allclose(s, torch.full_like(s, 1.5)) for s in shards)
        sb.all_gather([s * 2 for s in shards])
        ok = ok and all(torch.allclose(p.grad, torch.full_like(p, 3.0)) for p in params)
        r = measure_allreduce(1 << 16, iters=2)
        ok = ok and r["seconds"] > 0
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_grad_bucketer_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    assert res == {0: True, 1: True}


def test_busbw_formula():
    assert busbw(1 << 30, 1.0, 8) == (1 << 30) * 2 * 7 / 8 / 1e9
    assert busbw(100, 1.0, 1) == 0.0
