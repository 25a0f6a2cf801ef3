"""A data-parallel trainer tenant as its own pod process.

The GPU-sharing demo's pods only infer; BASELINE config 5 and SURVEY.md 2.8
add synthetic training tenants so slices are measured under collective
traffic.  This is that tenant as a real pod: its own process, started with the
device plugin's allocation env exactly like :mod:`nos_amd.models.pod`
(``HIP_VISIBLE_DEVICES``, ``ROC_GLOBAL_CU_MASK`` + the CU budget of slice-sized
grids, ``NOS_AMD_MEMORY_LIMIT_GB``), plus the job's rendezvous
(``MASTER_ADDR/PORT``, ``RANK``, ``WORLD_SIZE``: one trainer pod per GPU of the
job).  Every iteration is a forward + backward of a bf16 MLP whose gradient
buckets are all-reduced by RCCL over xGMI from the gradient hooks
(:class:`~nos_amd.models.tenants.CollectiveTenant`), then SGD.

Lockstep stop: each iteration also all-reduces a stop flag (MAX of the
ranks' "orchestrator asked me to stop"), so every rank leaves after the same
iteration and no collective is ever left unmatched.  Before the loop the pod
times a plain all-reduce of one bucket (``bucket_busbw_gbps``, NCCL-tests
formula).  Status protocol, result file and orphan guard: those of
:mod:`nos_amd.models.pod`.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time
from pathlib import Path

from .pod import STATE_DONE, STATE_FAILED, STATE_READY, StatusBoard, _die_with_parent, slice_cu_budget


def run_trainer(status: str, slot: int, out: str, device: str = "cuda", dim: int = 4096, bucket_mb: int = 64,
                warmup: int = 2) -> int:
    orphaned = _die_with_parent()
    board = StatusBoard(status)
    row = board.row(slot)
    row[3] = os.getpid()
    try:
        import torch
        import torch.distributed as dist

        from ..parallel.collectives import measure_allreduce
        from ..utils.memlimit import apply_memory_limit
        from .tenants import CollectiveTenant

        if os.environ.get("NOS_AMD_TRAINER_FAULT") == "init":  # test hook: the job never forms
            raise RuntimeError("injected trainer init fault")
        gpu = device == "cuda"
        world = int(os.environ.get("WORLD_SIZE", "1"))
        backend = os.environ.get("NOS_AMD_TRAINER_BACKEND") or ("nccl" if gpu else "gloo")
        if gpu:
            torch.cuda.set_device(0)  # the allocation leaves exactly this pod's GPU visible
            apply_memory_limit(0)
            budget = slice_cu_budget(os.environ)
            if budget:
                from ..ops import set_cu_budget

                set_cu_budget(budget)
        if world > 1:
            kw = {"timeout": datetime.timedelta(seconds=float(os.environ.get("NOS_AMD_TRAINER_TIMEOUT_S", "300")))}
            if backend == "nccl":
                kw["device_id"] = torch.device("cuda", 0)
            dist.init_process_group(backend, **kw)
        t = CollectiveTenant(dim=dim if gpu else 128, bucket_mb=bucket_mb if gpu else 1, device=0 if gpu else "cpu")
        for _ in range(warmup):
            t.step()
        bb = t.bucketer.buckets[0].flat
        probe = measure_allreduce(bb.numel() * bb.element_size(), iters=5,
                                  device=torch.device("cuda", 0) if gpu else torch.device("cpu"))
        if gpu:
            torch.cuda.synchronize()
        info = {"slot": slot, "pid": os.getpid(), "kind": "trainer", "world_size": world, "backend": backend,
                "rank": int(os.environ.get("RANK", "0")), "dim": t.dim, "layers": t.layers,
                "flops_per_step": t.flops_per_step(), "bucket_bytes": t.bucket_bytes(),
                "buckets": len(t.bucketer.buckets), "bucket_busbw_gbps": round(probe["busbw_gbps"], 2),
                "cu_mask": os.environ.get("ROC_GLOBAL_CU_MASK"),
                "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES"),
                "memory_limit_gb": os.environ.get("NOS_AMD_MEMORY_LIMIT_GB")}
        row[0] = STATE_READY
        info["t_ready"] = time.monotonic()
        times: list[float] = []
        flag = torch.zeros(1, device=t.dev, dtype=torch.float32)
        while True:
            if orphaned():
                print(f"[trainer {slot}] launcher gone: exiting", file=sys.stderr, flush=True)
                return 1
            t.step()
            flag.fill_(1.0 if board.stopped() else 0.0)
            if world > 1:
                dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            stop = flag.item() > 0  # synchronises the iteration
            now = time.monotonic()
            times.append(now)
            row[1] = len(times)
            row[2] = now
            if stop:
                break
        info["launched_in_backward"] = t.bucketer.launched_in_backward
        info["times"] = times
        Path(out, f"pod-{slot}.json").write_text(json.dumps(info))
        if world > 1:
            dist.destroy_process_group()
        row[0] = STATE_DONE
        return 0
    except Exception as e:  # the orchestrator sees the failure in the board and in the file
        Path(out, f"pod-{slot}.json").write_text(json.dumps({"slot": slot, "error": repr(e)}))
        row[0] = STATE_FAILED
        print(f"[trainer {slot}] failed: {e!r}", file=sys.stderr, flush=True)
        return 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="nos-amd DP trainer pod")
    ap.add_argument("--status", required=True)
    ap.add_argument("--slot", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--dim", type=int, default=int(os.environ.get("NOS_AMD_COLL_DIM", "4096")))
    ap.add_argument("--bucket-mb", type=int, default=int(os.environ.get("NOS_AMD_COLL_BUCKET_MB", "64")))
    a, _ = ap.parse_known_args(argv)
    return run_trainer(a.status, a.slot, a.out, a.device, a.dim, a.bucket_mb)


if __name__ == "__main__":
    sys.exit(main())
