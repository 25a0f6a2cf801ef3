"""Synthetic tenant "pods" run inside GPU slices.

* :class:`InferenceTenants` -- N independent YOLOS-small inference pods on one
  GPU, each with its own weights, input, HIP graph and (optionally) CU-masked
  stream: the MI355X version of the reference demo's 7-pod deployment
  (``demos/gpu-sharing-comparison/README.md:41-60``).
* :class:`CollectiveTenant` -- a data-parallel "trainer" pod: forward +
  backward of a bf16 MLP with its gradients averaged in 64 MiB buckets by RCCL
  over xGMI, each bucket's all-reduce launched from the gradient hooks while
  backward still runs (``parallel.collectives.GradBucketer``), then an SGD
  step -- so slices are measured under real collective traffic.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

from .yolos import GraphedTenant, YolosConfig, YolosDetector, make_demo_input


@dataclass
class TenantSpec:
    name: str
    cus: list[int] | None  # logical CU ids of the slice (None = whole GPU, no mask)


class InferenceTenants:
    def __init__(self, specs: list[TenantSpec], num_cus: int, cfg: YolosConfig | None = None,
                 hw: tuple[int, int] | None = None, use_graphs: bool = True, share_weights: bool = False,
                 device: int | None = None):
        from ..ops.streams import CUMaskedStream

        self.cfg = cfg or YolosConfig.small()
        self.specs = specs
        dev = torch.cuda.current_device() if device is None else device
        self.device = dev
        self.streams = [CUMaskedStream(s.cus, num_cus, dev) for s in specs]
        self.tenants: list[GraphedTenant] = []
        shared = None
        for i, s in enumerate(specs):
            if share_weights and shared is not None:
                m = shared
            else:
                m = YolosDetector(self.cfg)
                m.reset_parameters(seed=i)
                m = m.to(f"cuda:{dev}", torch.bfloat16).eval()
                shared = m
            x = make_demo_input(self.cfg, device=f"cuda:{dev}", hw=hw, seed=i)
            self.tenants.append(GraphedTenant(m, self.streams[i].torch, x))
        self.use_graphs = use_graphs

    @torch.no_grad()
    def prepare(self) -> None:
        for t in self.tenants:
            if self.use_graphs:
                t.capture()
            else:
                t.launch()
        self.synchronize()

    def launch_all(self) -> None:
        for t in self.tenants:
            t.launch()

    def synchronize(self) -> None:
        for s in self.streams:
            s.synchronize()

    @torch.no_grad()
    def run(self, steps: int) -> float:
        """Enqueue `steps` inferences per tenant, wait, return wall seconds."""
        t0 = time.perf_counter()
        for _ in range(steps):
            self.launch_all()
        self.synchronize()
        return time.perf_counter() - t0

    def close(self) -> None:
        for s in self.streams:
            s.close()


class CollectiveTenant:
    """DP trainer pod: per step, forward + backward of ``layers`` bf16
    ``dim x dim`` linear layers on a ``batch x dim`` activation, bucketed
    gradient all-reduce overlapped with backward (RCCL over xGMI on GPUs, gloo
    on the CPU rehearsal path), SGD update; one per rank/GPU.  Ranks run in
    LOCKSTEP: every iteration also all-reduces a stop flag, so all ranks leave
    a time-bounded loop after the same iteration and never issue mismatched
    collectives."""

    def __init__(self, dim: int = 4096, bucket_mb: int = 64, device: int | str | None = None, stream=None,
                 layers: int = 4, batch: int | None = None):
        from ..parallel.collectives import GradBucketer

        if device == "cpu":
            self.dev, dt = torch.device("cpu"), torch.float32
        else:
            dev = torch.cuda.current_device() if device is None else device
            self.dev, dt = torch.device("cuda", dev), torch.bfloat16
        g = torch.Generator().manual_seed(0)
        self.batch = batch or dim
        self.x = torch.randn(self.batch, dim, generator=g).to(self.dev, dt)
        self.model = torch.nn.Sequential(*[torch.nn.Linear(dim, dim, bias=False) for _ in range(layers)])
        with torch.no_grad():
            for m in self.model:
                m.weight.copy_(torch.randn(dim, dim, generator=g) * dim ** -0.5)
        self.model.to(self.dev, dt)
        params = list(self.model.parameters())
        self.bucketer = GradBucketer(params, bucket_bytes=max(1, bucket_mb) << 20, overlap=True).attach()
        self.opt = torch.optim.SGD(params, lr=1e-3)
        self.flag = torch.zeros(1, device=self.dev, dtype=torch.float32)
        self.stream = stream if (stream is not None or self.dev.type == "cpu") else torch.cuda.Stream(device=self.dev)
        self.dim = dim
        self.layers = layers
        self.iters = 0

    def _dist(self):
        import torch.distributed as dist

        return dist if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1 else None

    def step(self) -> None:
        ctx = torch.cuda.stream(self.stream) if self.stream is not None else _null()
        with ctx:
            y = self.model(self.x)
            loss = y.float().square().mean()
            loss.backward()  # bucket all-reduces start from the gradient hooks
            self.bucketer.finish()
            self.opt.step()
            self.opt.zero_grad(set_to_none=False)

    def run_until(self, deadline: float, times: list[float] | None = None) -> int:
        """Iterate (train step + stop-flag all-reduce) until every rank has
        passed ``deadline`` (time.monotonic()); completion times of the
        iterations are appended to ``times``."""
        import torch.distributed as dist

        n = 0
        while True:
            self.step()
            ctx = torch.cuda.stream(self.stream) if self.stream is not None else _null()
            with ctx:
                self.flag.fill_(1.0 if time.monotonic() >= deadline else 0.0)
                if self._dist() is not None:
                    dist.all_reduce(self.flag, op=dist.ReduceOp.MAX)
                stop = self.flag.item() > 0  # synchronises this iteration
            n += 1
            self.iters += 1
            if times is not None:
                times.append(time.monotonic())
            if stop:
                return n

    def flops_per_step(self) -> float:
        return 6.0 * self.batch * self.dim * self.dim * self.layers  # forward + backward (dX and dW)

    def bucket_bytes(self) -> int:
        return sum(b.flat.numel() * b.flat.element_size() for b in self.bucketer.buckets)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
