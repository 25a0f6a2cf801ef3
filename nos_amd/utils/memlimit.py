"""Cooperative GPU-memory cap of a fractional pod.

AMD GPUs have no MPS-style hard per-client memory limit, so
the device plugin hands each slice ``NOS_AMD_MEMORY_LIMIT_GB`` and the tenant
runtime enforces it through PyTorch's caching allocator (allocations beyond
the fraction raise an out-of-memory error inside the pod instead of starving
its neighbours).
"""
from __future__ import annotations

import os

from ..api import constants as C


def apply_memory_limit(device: int = 0) -> float | None:
    """Cap this process's allocations on ``device``; returns the fraction set."""
    gb = os.environ.get(C.ENV_MEMORY_LIMIT_GB)
    if not gb:
        return None
    import torch

    total = torch.cuda.get_device_properties(device).total_memory
    frac = min(1.0, float(gb) * (1 << 30) / total)
    torch.cuda.set_per_process_memory_fraction(frac, device)
    return frac
