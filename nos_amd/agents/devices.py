"""Node-local device views and the node labeler.

* :class:`NodeDeviceClient` joins kubelet PodResources (which device ids
  exist / are used) with amd-smi (device uuid -> GPU index), the role of
  ``pkg/gpu/mig/client.go:28-174`` and ``pkg/gpu/slicing/client.go:27-105``;
* :class:`NodeLabeler` publishes ``amd.com/gpu.product|count|memory|xcds|cus``
  and the current partition modes as node labels -- what NVIDIA's GPU feature
  discovery does for the reference (``pkg/constant/constants.go:78-87``).
"""
from __future__ import annotations

import logging

from ..api import constants as C
from ..gpu.core import GpuDevice
from ..gpu.kfd import max_concurrent_processes
from ..kube import objects as ko
from ..resource.client import Client
from ..runtime.manager import Controller, Request, Result
from ..runtime.predicates import MatchingName

log = logging.getLogger("nos_amd.agents")


def device_uuid(device_id: str) -> str:
    """Device ids of the nos-amd device plugin are ``<gpu-uuid>::<suffix>``."""
    return device_id.split("::", 1)[0]


class NodeDeviceClient:
    def __init__(self, smi, lister):
        self.smi = smi
        self.client = Client(lister)

    def _index_by_uuid(self) -> dict[str, int]:
        return {g.uuid: g.index for g in self.smi.gpus()}

    def get_devices(self, prefix: str) -> list[GpuDevice]:
        idx = self._index_by_uuid()
        out = []
        for d in self.client.get_devices(prefix):
            gi = idx.get(device_uuid(d.device_id))
            if gi is None:
                log.debug("device %s not found on any GPU", d.device_id)
                continue
            out.append(GpuDevice(d, gi))
        return sorted(out, key=lambda g: (g.gpu_index, g.device_id))

    def get_used_devices(self, prefix: str) -> list[GpuDevice]:
        return [d for d in self.get_devices(prefix) if d.is_used()]

    def used_gpus(self, prefix: str = C.AMD_RESOURCE_PREFIX) -> set[int]:
        return {d.gpu_index for d in self.get_used_devices(prefix)}


def node_labels(smi, pod_server_tenants: int = 0) -> dict[str, str]:
    gpus = smi.gpus()
    if not gpus:
        return {C.LABEL_AMD_COUNT: "0"}
    g0 = gpus[0]
    extra = {C.LABEL_POD_SERVER_TENANTS: str(pod_server_tenants)} if pod_server_tenants > 0 else {}
    return {**extra, C.LABEL_AMD_PRODUCT: g0.market_name.replace(" ", "-"), C.LABEL_AMD_COUNT: str(len(gpus)),
            C.LABEL_AMD_MEMORY: str(g0.vram_mb), C.LABEL_AMD_XCDS: str(g0.num_xcds), C.LABEL_AMD_CUS: str(g0.num_cus),
            C.LABEL_AMD_COMPUTE_MODE: g0.compute_mode, C.LABEL_AMD_MEMORY_MODE: g0.memory_mode,
            C.LABEL_AMD_MAX_PROCS: str(max_concurrent_processes(smi))}


class NodeLabeler:
    REFRESH_S = 60.0

    def __init__(self, api, node_name: str, smi, pod_server_tenants: int = 0):
        self.api, self.node_name, self.smi = api, node_name, smi
        self.pod_server_tenants = pod_server_tenants  # > 0: the node runs the pod server (MPS analogue)

    def reconcile(self, req: Request) -> Result:
        node = self.api.try_get("Node", self.node_name)
        if node is None:
            return Result()
        want = node_labels(self.smi, self.pod_server_tenants)
        have = ko.labels(node)
        diff: dict = {k: v for k, v in want.items() if have.get(k) != v}
        if self.pod_server_tenants <= 0 and C.LABEL_POD_SERVER_TENANTS in have:
            # the pod server was disabled: without the label the slice model
            # caps slices per GPU at the HWS process slots again (gpu/cumask.py)
            diff[C.LABEL_POD_SERVER_TENANTS] = None
        if diff:
            self.api.patch("Node", self.node_name, {"metadata": {"labels": diff}})
        return Result(requeue_after=self.REFRESH_S)

    def controller(self) -> Controller:
        return Controller(f"labeler-{self.node_name}", self).for_kind("Node", MatchingName(self.node_name))


def publish_node_metrics(node_name: str, status, smi) -> None:
    """Prometheus gauges of the north-star measurement: fractional devices per
    (node, profile) and GPU busy % (amd-smi gfx activity)."""
    from ..observability import metrics

    per_profile: dict[str, int] = {}
    for s in status:
        per_profile[s.profile] = per_profile.get(s.profile, 0) + s.quantity
    for prof, n in per_profile.items():
        metrics.SCHEDULABLE_PODS_PER_NODE.labels(node_name, prof).set(n)
    for g in smi.gpus():
        try:
            metrics.GPU_UTIL.labels(node_name, str(g.index)).set(smi.activity(g.index).get("gfx", 0))
        except Exception:  # activity is best effort (not every backend reports it)
            pass
