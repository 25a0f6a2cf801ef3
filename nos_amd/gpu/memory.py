"""GPU-memory resource calculator (``pkg/gpu/util/resource.go:28-86``).

Adds the virtual resource ``nos.nebuly.com/gpu-memory`` (GB) to a pod's
request so elastic quotas can be expressed in GPU memory:

    gpu-memory = amd.com/gpu x amdGpuResourceMemoryGB
               + sum(partition profile GB x qty)     (amd.com/partition-<n>xcd.<gb>gb)
               + sum(CU-mask slice GB x qty)          (amd.com/gpu-<gb>gb)

The reference counted only whole GPUs and MIG profiles -- MPS slices were
not charged; CU-mask slices are charged here.
"""
from __future__ import annotations

import re
from fractions import Fraction

from ..api import constants as C
from ..kube import quantity as q
from ..resource.resource import compute_pod_request

_PART = re.compile(C.REGEX_AMD_PARTITION_RESOURCE)
_SLICE = re.compile(C.REGEX_AMD_SLICE_RESOURCE)
_GB = re.compile(r"(\d+)gb$")


def memory_gb_of_resource(name: str) -> int | None:
    """GB carried by one unit of a partition / slice resource, else None."""
    m = _PART.match(name) or _SLICE.match(name)
    if not m:
        return None
    g = _GB.search(m.group(1))
    return int(g.group(1)) if g else None


class ResourceCalculator:
    def __init__(self, amd_gpu_memory_gb: int = C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB):
        self.amd_gpu_memory_gb = amd_gpu_memory_gb

    def compute_required_gpu_memory_gb(self, rl: dict) -> int:
        total = 0
        for name, v in rl.items():
            n = q.value(v)
            if name == C.RESOURCE_AMD_GPU:
                total += self.amd_gpu_memory_gb * n
                continue
            gb = memory_gb_of_resource(name)
            if gb is not None:
                total += gb * n
        return total

    def compute_pod_request(self, pod: dict) -> dict[str, Fraction]:
        res = compute_pod_request(pod)
        res[C.RESOURCE_GPU_MEMORY] = Fraction(self.compute_required_gpu_memory_gb(res))
        return res
