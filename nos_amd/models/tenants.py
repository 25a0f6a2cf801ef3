"""Synthetic tenant "pods" run inside GPU slices.

* :class:`InferenceTenants` -- N independent YOLOS-small inference pods on one
  GPU, each with its own weights, input, HIP graph and (optionally) CU-masked
  stream: the MI355X version of the reference demo's 7-pod deployment
  (``demos/gpu-sharing-comparison/README.md:41-60``).
* :class:`CollectiveTenant` -- a data-parallel "trainer" pod: bf16 GEMMs plus a
  bucketed RCCL all-reduce of its gradient buffer over xGMI, so slices are
  measured under real collective traffic.
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
    """DP trainer tenant: y = x @ W (bf16 GEMMs) then all-reduce of a gradient
    bucket on its own stream; one per rank/GPU."""

    def __init__(self, dim: int = 8192, bucket_mb: int = 64, device: int | None = None, stream=None):
        dev = torch.cuda.current_device() if device is None else device
        self.x = torch.randn(dim, dim, device=f"cuda:{dev}", dtype=torch.bfloat16)
        self.w = torch.randn(dim, dim, device=f"cuda:{dev}", dtype=torch.bfloat16)
        self.grad = torch.randn(bucket_mb * (1 << 20) // 2, device=f"cuda:{dev}", dtype=torch.bfloat16)
        self.stream = stream if stream is not None else torch.cuda.Stream(device=dev)
        self.dim = dim

    def step(self) -> None:
        import torch.distributed as dist

        with torch.cuda.stream(self.stream):
            y = self.x @ self.w
            self.grad[: y.numel() // 64].copy_(y.view(-1)[: y.numel() // 64])
            if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
                dist.all_reduce(self.grad)

    def flops_per_step(self) -> float:
        return 2.0 * self.dim ** 3
