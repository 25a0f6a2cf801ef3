"""Collectives of the tenant jobs that load the slices with real traffic
(SURVEY.md 2.8 "Tenant collectives"): one process per GPU (or partition),
``torch.distributed`` with backend ``nccl`` (= RCCL on ROCm) over xGMI, or
``gloo`` on the CPU for tests.

* :class:`GradBucketer` -- DP gradient synchronisation in fixed-size flat
  buckets (all-reduce, or reduce-scatter + all-gather for ZeRO-style
  sharding) on a side stream.  With :meth:`GradBucketer.attach` the buckets
  are built in reverse parameter order (the order backward produces
  gradients) and each bucket's all-reduce is launched from a
  post-accumulate-grad hook the moment its last gradient lands, so the
  collectives overlap the rest of backward; :meth:`GradBucketer.finish`
  waits for them and writes the averaged gradients back.  Bucket size
  defaults to 64 MiB: xGMI is point-to-point (7 links x ~153 GB/s per
  MI355X), a ring all-reduce is per-link bound, and 64 MiB amortises the
  ~20-30 us RCCL launch/latency to < 5 %.
* :func:`busbw` -- NCCL-tests style bus bandwidth of an all-reduce.
* :func:`init_from_env` -- RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* rendezvous
  (127.0.0.1), one rank per GPU.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 64 << 20


def init_from_env(backend: str | None = None) -> tuple[int, int, int]:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def busbw(nbytes: int, seconds: float, world: int) -> float:
    """All-reduce bus bandwidth (GB/s): algbw x 2(n-1)/n."""
    if seconds <= 0 or world <= 1:
        return 0.0
    return nbytes / seconds * 2 * (world - 1) / world / 1e9


@dataclass
class _Bucket:
    params: list[torch.Tensor]
    flat: torch.Tensor
    offsets: list[tuple[int, int]] = field(default_factory=list)


class GradBucketer:
    """Flatten gradients into buckets of ``bucket_bytes`` and average them
    across the process group (optionally sharded: reduce-scatter, then the
    caller's optimizer updates its shard, then :meth:`all_gather`).

    Two ways to drive it: :meth:`sync` after backward (all buckets at once),
    or :meth:`attach` once and :meth:`finish` after every backward (buckets
    launched from gradient hooks while backward still runs)."""

    def __init__(self, params: list[torch.Tensor], bucket_bytes: int = DEFAULT_BUCKET_BYTES, group=None,
                 sharded: bool = False, overlap: bool = False):
        self.group = group
        self.sharded = sharded
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.buckets: list[_Bucket] = []
        # backward produces gradients roughly in reverse parameter order: build
        # the buckets that way so the first buckets complete first
        order = list(reversed(params)) if overlap else list(params)
        cur: list[torch.Tensor] = []
        size = 0
        for p in order:
            nb = p.numel() * p.element_size()
            if cur and size + nb > bucket_bytes:
                self.buckets.append(self._make(cur))
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            self.buckets.append(self._make(cur))
        self.stream = torch.cuda.Stream(device=params[0].device) if (params and params[0].is_cuda) else None
        self.last_seconds = 0.0
        self._where = {id(p): i for i, b in enumerate(self.buckets) for p in b.params}
        self._ready = [0] * len(self.buckets)
        self._works: list = [None] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._sync_enabled = True
        self._hooks: list = []
        self._lock = threading.Lock()  # hooks of different devices run on different autograd threads
        self.launched_in_backward = 0  # bucket collectives started from a gradient hook (all steps)

    def _make(self, params: list[torch.Tensor]) -> _Bucket:
        n = sum(p.numel() for p in params)
        pad = (-n) % max(1, self.world)  # reduce-scatter needs equal shards
        flat = torch.zeros(n + pad, dtype=params[0].dtype, device=params[0].device)
        b = _Bucket(params, flat)
        off = 0
        for p in params:
            b.offsets.append((off, p.numel()))
            off += p.numel()
        return b

    def _pack(self, b: _Bucket) -> None:
        for p, (o, n) in zip(b.params, b.offsets):
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            b.flat[o:o + n].copy_(g.reshape(-1))

    def _unpack(self, b: _Bucket, src: torch.Tensor) -> None:
        for p, (o, n) in zip(b.params, b.offsets):
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.copy_(src[o:o + n].view_as(p))

    # -- overlapped mode -------------------------------------------------
    def attach(self) -> "GradBucketer":
        """Launch each bucket's all-reduce from a post-accumulate-grad hook as
        soon as all of its gradients exist (not sharded).  Collectives start in
        the order the buckets complete; with one device per rank (data
        parallelism) backward runs the same graph on one autograd thread in
        every rank, so that order is the same everywhere, as collectives need."""
        if self.sharded:
            raise ValueError("overlapped bucketing is for all-reduce (sharded=False)")
        for b in self.buckets:
            for p in b.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        return self

    def detach(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def _launch(self, i: int) -> None:
        b = self.buckets[i]
        if self.stream is not None:
            # the gradients were produced on the backward stream of this thread
            self.stream.wait_stream(torch.cuda.current_stream(b.flat.device))
        ctx = torch.cuda.stream(self.stream) if self.stream is not None else _null()
        with ctx:
            self._pack(b)
            self._works[i] = dist.all_reduce(b.flat, group=self.group, async_op=True) if self.world > 1 else None

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation (DDP's ``no_sync``): backward passes inside
        this context only accumulate into ``p.grad``; the next backward outside
        it launches the buckets with the accumulated gradients."""
        prev, self._sync_enabled = self._sync_enabled, False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def _on_grad(self, p: torch.Tensor) -> None:
        if not self._sync_enabled:
            return
        i = self._where[id(p)]
        with self._lock:
            if self._launched[i]:
                # a second backward before finish(): its gradients would be silently
                # dropped (the bucket already holds the first micro-batch's)
                raise RuntimeError(
                    f"GradBucketer: bucket {i} was already launched in this step; call finish() after every "
                    "backward, or run the earlier micro-batches of an accumulation under no_sync()")
            self._ready[i] += 1
            full = self._ready[i] == len(self.buckets[i].params)
            if full:
                self._launched[i] = True
                self.launched_in_backward += 1
        if full:
            self._launch(i)

    def finish(self) -> None:
        """Wait for this step's bucket collectives (launching any bucket whose
        hooks did not all fire, e.g. unused parameters) and write the averaged
        gradients back; the caller's stream then waits for them."""
        t0 = time.perf_counter()
        for i in range(len(self.buckets)):
            if not self._launched[i]:
                self._launched[i] = True
                self._launch(i)
        ctx = torch.cuda.stream(self.stream) if self.stream is not None else _null()
        with ctx:
            for i, b in enumerate(self.buckets):
                w = self._works[i]
                if w is not None:
                    w.wait()  # on the side stream (NCCL) / blocking (gloo)
                if self.world > 1:
                    b.flat.div_(self.world)
                self._unpack(b, b.flat)
        if self.stream is not None:
            torch.cuda.current_stream(self.buckets[0].flat.device).wait_stream(self.stream)
        self._ready = [0] * len(self.buckets)
        self._works = [None] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self.last_seconds = time.perf_counter() - t0

    # -- after-backward mode ---------------------------------------------
    def sync(self) -> list[torch.Tensor]:
        """Average all gradients; returns the local shards when ``sharded``."""
        t0 = time.perf_counter()
        shards = []
        ctx = torch.cuda.stream(self.stream) if self.stream is not None else _null()
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream())
        with ctx:
            for b in self.buckets:
                self._pack(b)
                if self.world > 1:
                    if self.sharded:
                        shard = torch.empty(b.flat.numel() // self.world, dtype=b.flat.dtype, device=b.flat.device)
                        dist.reduce_scatter_tensor(shard, b.flat, group=self.group)
                        shard.div_(self.world)
                        shards.append(shard)
                        continue
                    dist.all_reduce(b.flat, group=self.group)
                    b.flat.div_(self.world)
                elif self.sharded:
                    shards.append(b.flat)
                    continue
                self._unpack(b, b.flat)
        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)
        self.last_seconds = time.perf_counter() - t0
        return shards

    def all_gather(self, shards: list[torch.Tensor]) -> None:
        """ZeRO step 2: gather the updated shards back into every gradient."""
        for b, shard in zip(self.buckets, shards):
            full = torch.empty_like(b.flat)
            if self.world > 1:
                dist.all_gather_into_tensor(full, shard, group=self.group)
            else:
                full.copy_(shard)
            self._unpack(b, full)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def measure_allreduce(nbytes: int, iters: int = 10, device: torch.device | None = None) -> dict:
    """Timed all-reduce of ``nbytes`` (bf16) on the default group."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                     else torch.device("cpu"))
    x = torch.ones(nbytes // 2, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32, device=dev)
    for _ in range(2):
        if world > 1:
            dist.all_reduce(x)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        if world > 1:
            dist.all_reduce(x)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    return {"bytes": nbytes, "seconds": dt, "busbw_gbps": busbw(nbytes, dt, world)}
