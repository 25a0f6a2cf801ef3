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


def _overlap_worker(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 32),
                                    torch.nn.ReLU(), torch.nn.Linear(32, 4))
        ref = [p.detach().clone().requires_grad_(True) for p in model.parameters()]
        b = GradBucketer(list(model.parameters()), bucket_bytes=1500, overlap=True).attach()
        ok = len(b.buckets) >= 3
        torch.manual_seed(100 + rank)  # different data per rank
        x = torch.randn(8, 16)
        for step in range(2):  # twice: the hook bookkeeping resets between steps
            model.zero_grad(set_to_none=False)
            model(x).square().mean().backward()
            launched = b.launched_in_backward
            b.finish()
            ok = ok and launched == (step + 1) * len(b.buckets)  # every bucket started inside backward
        # reference: this rank's gradient (functional copy), all-reduced by hand
        w1, b1, w2, b2, w3, b3 = ref
        h = torch.relu(x @ w1.T + b1)
        h = torch.relu(h @ w2.T + b2)
        (h @ w3.T + b3).square().mean().backward()
        for p, r in zip(model.parameters(), ref):
            g = r.grad.clone()
            dist.all_reduce(g)
            ok = ok and torch.allclose(p.grad, g / world, atol=1e-6)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_overlapped_bucketer_matches_allreduced_gradients():
    """Buckets launched from gradient hooks during backward average exactly like a plain all-reduce."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    assert res == {0: True, 1: True}


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


def test_overlapped_bucketer_accumulation_contract():
    """a second backward before finish() used to drop the later
    micro-batches' gradients silently.  Now it raises, and no_sync() gives
    DDP-style accumulation: the buckets carry the sum of every micro-batch."""
    import pytest

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 2))
    b = GradBucketer(list(model.parameters()), bucket_bytes=300, overlap=True).attach()
    xs = [torch.randn(4, 8) for _ in range(3)]
    model(xs[0]).sum().backward()
    with pytest.raises(RuntimeError, match="already launched"):
        model(xs[1]).sum().backward()
    b.finish()
    model.zero_grad(set_to_none=True)
    with b.no_sync():
        for x in xs[:2]:
            model(x).sum().backward()
    model(xs[2]).sum().backward()
    launched = b.launched_in_backward
    b.finish()
    got = [p.grad.clone() for p in model.parameters()]
    model.zero_grad(set_to_none=True)
    b.detach()
    for x in xs:
        model(x).sum().backward()
    assert launched >= len(b.buckets)
    for g, p in zip(got, model.parameters()):
        assert torch.allclose(g, p.grad, atol=1e-6)


def test_allreduce_sweep_tool_launches_under_torchrun(tmp_path):
    """tools/allreduce_sweep.py through the same launcher the GPU sweep uses
    (torch.distributed.run, 2 ranks, 127.0.0.1), gloo on the CPU: one row per
    message size with NCCL-tests busbw, slowest rank's time."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    out = tmp_path / "sweep.json"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        str(repo / "tools" / "allreduce_sweep.py"), "--device", "cpu", "--min-bytes", str(1 << 16),
                        "--max-bytes", str(1 << 18), "--iters", "3", "--warmup", "1", "--out", str(out)],
                       capture_output=True, text=True, timeout=180, cwd=str(repo),
                       env={**__import__("os").environ, "OMP_NUM_THREADS": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(out.read_text())
    assert d["world_size"] == 2 and d["backend"] == "gloo"
    assert [x["bytes"] for x in d["rows"]] == [1 << 16, 1 << 17, 1 << 18]
    for x in d["rows"]:
        assert x["seconds"] > 0 and abs(x["busbw_gbps"] - x["algbw_gbps"] * 2 * 1 / 2) < 1e-9
