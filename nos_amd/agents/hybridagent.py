"""Agent of ``hybrid`` nodes: partition modes + memory slices per partition.

A hybrid node runs the partition agent's :class:`~nos_amd.agents.partagent.
PartitionActuator` (it switches each GPU to the ``spec-mode-gpu-<i>`` the
gpupartitioner wrote, bounded, drain-checked) next to this reporter, which
publishes what the kubelet actually has:

* ``status-gpu-<i>-<N>gb-<free|used>`` from PodResources (the device plugin's
  slice replicas, as on cumask nodes, ``gpuagent/reporter.go:50-96``);
* ``status-mode-gpu-<i>`` from amd-smi (``SWITCHING`` while a switch runs) and
  the actuator's ``status-error-gpu-<i>``;
* ``status-partitioning-plan`` once the slices AND the modes realise the spec
  (the plan handshake of ``partitioner_controller.go:212-232``).

It shares the actuator's :class:`SharedState`, so the actuator never plans
again before a report (``migagent/shared.go``).
"""
from __future__ import annotations

import logging

from ..api import constants as C
from ..gpu.core import devices_as_status_annotations, parse_node_annotations, spec_matches_status, status_equal
from ..kube import objects as ko
from ..observability import tracing
from ..runtime.manager import Controller, Request, Result
from ..runtime.predicates import AnnotationsChanged, ExcludeDelete, MatchingName, NodeResourcesChanged, or_
from .devices import NodeDeviceClient, publish_node_metrics
from .gpuagent import slice_profile_name
from .shared import SharedState

log = logging.getLogger("nos_amd.agents.hybridagent")


class HybridReporter:
    def __init__(self, api, node_name: str, smi, lister, shared: SharedState, refresh_s: float = 10.0):
        self.api, self.node_name, self.smi = api, node_name, smi
        self.devices = NodeDeviceClient(smi, lister)
        self.shared = shared
        self.refresh_s = refresh_s
        self.reports = 0

    def status_annotations(self):
        return devices_as_status_annotations(self.devices.get_devices(C.AMD_SLICE_RESOURCE_PREFIX),
                                             slice_profile_name)

    def reconcile(self, req: Request) -> Result:
        with self.shared.lock:
            node = self.api.try_get("Node", self.node_name)
            if node is None:
                return Result()
            status = self.status_annotations()
            cur_status, spec = parse_node_annotations(node)
            publish_node_metrics(self.node_name, status, self.smi)
            ann = ko.annotations(node)
            gpus = self.smi.gpus()
            modes = {C.ANNOTATION_STATUS_MODE_FORMAT.format(index=g.index):
                     C.MODE_SWITCHING if g.switching else f"{g.compute_mode}/{g.memory_mode}" for g in gpus}
            want = {C.ANNOTATION_STATUS_MODE_FORMAT.format(index=g.index):
                    ann.get(C.ANNOTATION_SPEC_MODE_FORMAT.format(index=g.index)) for g in gpus}
            modes_ok = all(v is None or modes.get(k) == v for k, v in want.items())
            errors = {C.ANNOTATION_STATUS_ERROR_FORMAT.format(index=i): why for i, why in self.shared.failures().items()}
            stale_errors = [k for k in ann if k.startswith(C.ANNOTATION_STATUS_ERROR_PREFIX) and k not in errors]
            plan = ann.get(C.ANNOTATION_PARTITIONING_PLAN, "")
            reported = ann.get(C.ANNOTATION_REPORTED_PARTITIONING_PLAN, "")
            new_reported = plan if (plan and modes_ok and spec_matches_status(spec, status)) else reported
            if (status_equal(status, cur_status) and new_reported == reported and not stale_errors
                    and all(ann.get(k) == v for k, v in {**modes, **errors}.items())):
                self.shared.on_report_done()
                return Result(requeue_after=self.refresh_s)
            patch: dict[str, str | None] = {k: None for k in ann if k.startswith(C.ANNOTATION_GPU_STATUS_PREFIX)}
            patch.update({s.key(): s.value() for s in status})
            patch.update(modes)
            patch.update(errors)
            patch.update({k: None for k in stale_errors})
            if new_reported:
                patch[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] = new_reported
            self.api.patch("Node", self.node_name, {"metadata": {"annotations": patch}})
            self.reports += 1
            if new_reported != reported:
                tracing.event("agent.plan_reported", node=self.node_name, plan_id=new_reported, kind="hybrid")
            self.shared.on_report_done()
            return Result(requeue_after=self.refresh_s)

    def controller(self) -> Controller:
        return Controller(f"hybrid-reporter-{self.node_name}", self).for_kind(
            "Node", ExcludeDelete(), MatchingName(self.node_name), or_(NodeResourcesChanged(), AnnotationsChanged()))


__all__ = ["HybridReporter"]
