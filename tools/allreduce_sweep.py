"""NCCL-tests style all-reduce sweep of the tenant data plane: RCCL over xGMI.

SURVEY.md 2.8 "Tenant collectives": bf16 all-reduce from 1 MiB to 1 GiB at
the launcher's world size (2/4/8 GPUs of one node), one rank per GPU, reported
as algorithm and bus bandwidth (busbw = algbw x 2(n-1)/n, the per-link figure
to hold against xGMI's ~153 GB/s per link), optionally while every rank also
runs bf16 GEMMs on a second stream (``--with-gemm``: slices measured under
compute + collective traffic).

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
      --master-port 29611 tools/allreduce_sweep.py --out gpurun_out/allreduce.json

On a CPU host it runs over gloo (float32) -- the launch-path test.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def sizes(min_bytes: int, max_bytes: int) -> list[int]:
    out, s = [], min_bytes
    while s <= max_bytes:
        out.append(s)
        s *= 2
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--min-bytes", type=int, default=1 << 20)
    ap.add_argument("--max-bytes", type=int, default=1 << 30)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--with-gemm", action="store_true", help="bf16 8192^2 GEMMs on a side stream while timing")
    ap.add_argument("--device", choices=["auto", "cuda", "cpu"], default="auto")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    from nos_amd.parallel.collectives import busbw, init_from_env

    cuda = torch.cuda.is_available() if a.device == "auto" else a.device == "cuda"
    world, rank, local = init_from_env("nccl" if cuda else "gloo")
    dev = torch.device("cuda", local) if cuda else torch.device("cpu")
    dtype = torch.bfloat16 if cuda else torch.float32
    esize = torch.tensor([], dtype=dtype).element_size()
    side = torch.cuda.Stream(dev) if (cuda and a.with_gemm) else None
    gemm = None
    if side is not None:
        g = torch.Generator(device=dev).manual_seed(rank)
        gemm = (torch.randn(8192, 8192, device=dev, dtype=dtype, generator=g),
                torch.randn(8192, 8192, device=dev, dtype=dtype, generator=g))

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    rows = []
    for nbytes in sizes(a.min_bytes, a.max_bytes):
        x = torch.ones(max(1, nbytes // esize), dtype=dtype, device=dev)
        for _ in range(a.warmup):
            dist.all_reduce(x) if world > 1 else None
        sync()
        if world > 1:
            dist.barrier()
        gemms = 0
        if side is not None:
            with torch.cuda.stream(side):
                for _ in range(4):
                    torch.matmul(*gemm)
                    gemms += 1
        t0 = time.perf_counter()
        for _ in range(a.iters):
            if world > 1:
                dist.all_reduce(x)
        sync()
        dt = (time.perf_counter() - t0) / a.iters
        t = torch.tensor([dt], dtype=torch.float64, device=dev if cuda else "cpu")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the slowest rank defines the collective
        dt = float(t.item())
        row = {"bytes": int(x.numel() * esize), "seconds": dt, "algbw_gbps": x.numel() * esize / dt / 1e9 if dt else 0.0,
               "busbw_gbps": busbw(x.numel() * esize, dt, world), "side_gemms": gemms}
        rows.append(row)
        if rank == 0:
            print(json.dumps(row), flush=True)
    out = {"world_size": world, "backend": "nccl" if cuda else "gloo", "dtype": str(dtype).replace("torch.", ""),
           "iters": a.iters, "with_gemm": bool(side is not None), "rows": rows,
           "peak_busbw_gbps": max((r["busbw_gbps"] for r in rows), default=0.0),
           "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES")}
    if rank == 0 and a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(out, indent=1))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
