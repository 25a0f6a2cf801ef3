"""CU-mask gpuagent: reports the slices of a ``cumask`` node
(``internal/controllers/gpuagent/reporter.go:34-110``, ``cmd/gpuagent``).

Differences from the reference, both deliberate:

* **plan handshake** -- the reference's MPS path never wrote
  ``status-partitioning-plan``, so the partitioner relied on
  a blind 5 s delay.  Here the reporter writes it once the kubelet's
  allocatable devices (PodResources ``GetAllocatableResources``) realise the
  node's spec annotations, i.e. the device plugin has actually loaded the
  plan's slice table;
* **measured slices** -- with a ``probe`` callable the reporter publishes the
  per-slice MFMA TFLOP/s and HBM GB/s measured by the HIP probe kernels on
  the slice's CU mask (``nos.nebuly.com/probe-gpu-<i>-<profile>-tflops|gbps``).
"""
from __future__ import annotations

import logging
from typing import Callable

from ..api import constants as C
from .probe import METRICS as PROBE_METRICS
from ..gpu import cumask as cm
from ..gpu.core import devices_as_status_annotations, parse_node_annotations, spec_matches_status, status_equal
from ..kube import objects as ko
from ..observability import metrics, tracing
from ..runtime.manager import Controller, Request, Result
from ..runtime.predicates import AnnotationsChanged, ExcludeDelete, MatchingName, NodeResourcesChanged, or_
from .devices import NodeDeviceClient, publish_node_metrics

log = logging.getLogger("nos_amd.agents.gpuagent")


def slice_profile_name(resource: str) -> str:
    return cm.profile_of_resource(resource).name


class AnyPartitionedGpuError(RuntimeError):
    """``cmd/gpuagent/gpuagent.go:105-114`` refuses to run on MIG GPUs; CU-mask
    slices assume SPX (one logical device per GPU)."""


def check_spx(smi) -> None:
    bad = [g.index for g in smi.gpus() if g.compute_mode != "SPX"]
    if bad:
        raise AnyPartitionedGpuError(f"GPUs {bad} are not in SPX mode; CU-mask slicing needs SPX")


class CuMaskReporter:
    def __init__(self, api, node_name: str, smi, lister, refresh_s: float = 10.0,
                 probe: Callable[[int, str], dict] | None = None):
        self.api, self.node_name, self.smi = api, node_name, smi
        self.devices = NodeDeviceClient(smi, lister)
        self.refresh_s = refresh_s
        self.probe = probe
        self._probed: dict[tuple[int, str], dict] = {}
        self.reports = 0

    def status_annotations(self):
        devs = self.devices.get_devices(C.AMD_SLICE_RESOURCE_PREFIX)
        return devices_as_status_annotations(devs, slice_profile_name)

    def _probe_annotations(self, status) -> dict[str, str]:
        if self.probe is None:
            return {}
        out = {}
        for s in status:
            k = (s.index, s.profile)
            if k not in self._probed:
                try:
                    self._probed[k] = self.probe(s.index, s.profile)
                except Exception as e:  # a probe failure must not stop reporting
                    log.warning("probe of gpu %d slice %s failed: %s", s.index, s.profile, e)
                    self._probed[k] = {}
            r = self._probed[k]
            for m in PROBE_METRICS:
                if m in r:
                    key = f"{C.ANNOTATION_PROBE_PREFIX}-{s.index}-{s.profile}-{m}"
                    out[key] = f"{r[m]:.1f}" if "tflops" in m else f"{r[m]:.0f}"
            if "gemmtflops" in r or "tflops" in r:
                metrics.SLICE_TFLOPS.labels(self.node_name, str(s.index), s.profile).set(
                    r.get("gemmtflops", r.get("tflops")))
            if "gbps" in r:
                metrics.SLICE_GBPS.labels(self.node_name, str(s.index), s.profile).set(r["gbps"])
        return out

    def reconcile(self, req: Request) -> Result:
        node = self.api.try_get("Node", self.node_name)
        if node is None:
            return Result()
        status = self.status_annotations()
        cur_status, spec = parse_node_annotations(node)
        publish_node_metrics(self.node_name, status, self.smi)
        ann = ko.annotations(node)
        plan = ann.get(C.ANNOTATION_PARTITIONING_PLAN, "")
        reported = ann.get(C.ANNOTATION_REPORTED_PARTITIONING_PLAN, "")
        new_reported = plan if (plan and spec_matches_status(spec, status)) else reported
        probes = self._probe_annotations(status)
        if status_equal(status, cur_status) and new_reported == reported and \
                all(ann.get(k) == v for k, v in probes.items()):
            return Result(requeue_after=self.refresh_s)
        patch: dict[str, str | None] = {k: None for k in ann if k.startswith(C.ANNOTATION_GPU_STATUS_PREFIX)}
        patch.update({s.key(): s.value() for s in status})
        patch.update(probes)
        if new_reported:
            patch[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] = new_reported
        self.api.patch("Node", self.node_name, {"metadata": {"annotations": patch}})
        self.reports += 1
        if new_reported != reported:
            tracing.event("agent.plan_reported", node=self.node_name, plan_id=new_reported, kind="cumask")
        return Result(requeue_after=self.refresh_s)

    def controller(self) -> Controller:
        return Controller(f"gpuagent-reporter-{self.node_name}", self).for_kind(
            "Node", ExcludeDelete(), MatchingName(self.node_name), or_(NodeResourcesChanged(), AnnotationsChanged()))
