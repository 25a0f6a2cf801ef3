"""Partition agent: realises ``amdpart`` plans on one node (the reference's
``migagent``, ``internal/controllers/migagent``).

AMD compute partitions are a per-GPU MODE (SPX/DPX/QPX/CPX x NPS1/NPS2),
not a set of independently created instances like MIG, so the diff planner
is much simpler than ``migagent/plan/plan.go``: per GPU, either the current
mode already yields the spec'd partitions, or the GPU must switch mode -- and
it may switch only when none of its partitions is in use (kubelet
PodResources) and amd-smi lists no process on it (the drain check of
SURVEY.md 5.3).  After a switch the device plugin re-enumerates (the
reference deletes the device-plugin pod and waits for it, ``pkg/gpu/client.go:51-135``;
our plugin is reconfigured in place) and the reporter publishes the new
status.

* :class:`PartitionReporter` -- ``reporter.go:54-109``: status annotations
  ``status-gpu-<i>-<profile>-<free|used>`` + ``status-mode-gpu-<i>`` +
  ``status-partitioning-plan`` (the last plan id the actuator parsed);
* :class:`PartitionActuator` -- ``actuator.go:71-201``: waits for a report
  since its last apply, parses spec vs status, plans, applies.

Every wait on the node's reconfiguration is bounded, as in the reference
(device-plugin restart timeout ``pkg/gpu/client.go:86-135``, per-op errors
``actuator.go:165-198``): a mode switch runs in a worker thread with a
``switch_timeout_s`` deadline and the shared lock is never held across it, so
the reporter keeps reporting (and the plan handshake keeps clearing) while a
switch hangs.  A GPU past its deadline is marked failed
(``status-error-gpu-<i>``) and not planned again until its switch returns;
then it is verified, rolled back if the mode did not take effect, and the
device plugins re-enumerate.
"""
from __future__ import annotations

import logging
import threading
import time
from dataclasses import dataclass, field

from ..api import constants as C
from ..gpu import amdpart as ap
from ..gpu.amdsmi import PARTITIONS_PER_MODE
from ..gpu.core import (devices_as_status_annotations, parse_node_annotations, spec_matches_status,
                        status_equal)
from ..kube import objects as ko
from ..observability import metrics, tracing
from ..runtime.manager import Controller, Request, Result
from ..runtime.predicates import AnnotationsChanged, ExcludeDelete, MatchingName, NodeResourcesChanged, or_
from .devices import NodeDeviceClient, publish_node_metrics
from .shared import SharedState

log = logging.getLogger("nos_amd.agents.partagent")

MODE_BY_PARTS = {v: k for k, v in PARTITIONS_PER_MODE.items()}


def partition_profile_name(resource: str) -> str:
    return ap.profile_of_resource(resource).name


# ====================================================================== plan
@dataclass(frozen=True)
class ModeChange:
    gpu_index: int
    compute: str
    memory: str
    from_compute: str
    from_memory: str


@dataclass
class PartitionPlan:
    changes: list[ModeChange] = field(default_factory=list)
    blocked: dict[int, str] = field(default_factory=dict)   # gpu -> reason

    def is_empty(self) -> bool:
        return not self.changes

    def __eq__(self, other) -> bool:
        return isinstance(other, PartitionPlan) and self.changes == other.changes


def desired_modes(node: dict, gpus, memory_preference: str = "NPS1") -> dict[int, tuple[str, str]]:
    """Per GPU, the (compute, memory) mode the spec annotations ask for.
    ``spec-mode-gpu-<i>`` wins; otherwise it is derived from the single spec
    profile (``<x>xcd.<gb>gb`` -> total_xcds / x partitions)."""
    ann = ko.annotations(node)
    _, spec = parse_node_annotations(node)
    by_gpu: dict[int, list] = {}
    for s in spec:
        if s.quantity:
            by_gpu.setdefault(s.index, []).append(s)
    info = {g.index: g for g in gpus}
    out: dict[int, tuple[str, str]] = {}
    for i, g in info.items():
        mode = ann.get(C.ANNOTATION_SPEC_MODE_FORMAT.format(index=i))
        if mode and "/" in mode:
            c, m = mode.split("/", 1)
            out[i] = (c, m)
            continue
        specs = by_gpu.get(i)
        if not specs:
            continue
        prof = ap.profile(specs[0].profile)
        parts = max(1, (g.num_xcds or 8) // max(1, prof.xcds))
        c = MODE_BY_PARTS.get(parts)
        if c is None:
            continue
        out[i] = (c, memory_preference if parts in (2, 8) else "NPS1")
    return out


def new_partition_plan(node: dict, gpus, used_gpus: set[int], busy_gpus: set[int],
                       memory_preference: str = "NPS1", switching: set[int] = frozenset()) -> PartitionPlan:
    plan = PartitionPlan()
    want = desired_modes(node, gpus, memory_preference)
    for g in sorted(gpus, key=lambda x: x.index):
        if g.index not in want:
            continue
        if g.index in switching or getattr(g, "switching", False):
            plan.blocked[g.index] = "mode switch in progress"
            continue
        c, m = want[g.index]
        if (g.compute_mode, g.memory_mode) == (c, m):
            continue
        if g.index in used_gpus:
            plan.blocked[g.index] = "partitions in use"
            continue
        if g.index in busy_gpus:
            plan.blocked[g.index] = "processes running"
            continue
        plan.changes.append(ModeChange(g.index, c, m, g.compute_mode, g.memory_mode))
    return plan


# ====================================================================== reporter
class PartitionReporter:
    def __init__(self, api, node_name: str, smi, lister, shared: SharedState, refresh_s: float = 10.0):
        self.api, self.node_name, self.smi = api, node_name, smi
        self.devices = NodeDeviceClient(smi, lister)
        self.shared = shared
        self.refresh_s = refresh_s
        self.reports = 0

    def status_annotations(self):
        devs = self.devices.get_devices(C.AMD_PARTITION_RESOURCE_PREFIX)
        return devices_as_status_annotations(devs, partition_profile_name)

    def reconcile(self, req: Request) -> Result:
        with self.shared.lock:
            node = self.api.try_get("Node", self.node_name)
            if node is None:
                return Result()
            status = self.status_annotations()
            cur_status, _ = parse_node_annotations(node)
            publish_node_metrics(self.node_name, status, self.smi)
            ann = ko.annotations(node)
            modes = {C.ANNOTATION_STATUS_MODE_FORMAT.format(index=g.index):
                     C.MODE_SWITCHING if g.switching else f"{g.compute_mode}/{g.memory_mode}"
                     for g in self.smi.gpus()}
            errors = {C.ANNOTATION_STATUS_ERROR_FORMAT.format(index=i): why
                      for i, why in self.shared.failures().items()}
            stale_errors = [k for k in ann if k.startswith(C.ANNOTATION_STATUS_ERROR_PREFIX) and k not in errors]
            plan = self.shared.last_parsed_plan_id
            if (status_equal(status, cur_status) and ann.get(C.ANNOTATION_REPORTED_PARTITIONING_PLAN, "") == plan
                    and all(ann.get(k) == v for k, v in modes.items())
                    and all(ann.get(k) == v for k, v in errors.items()) and not stale_errors):
                self.shared.on_report_done()
                return Result(requeue_after=self.refresh_s)
            patch: dict[str, str | None] = {k: None for k in ann if k.startswith(C.ANNOTATION_GPU_STATUS_PREFIX)}
            patch.update({s.key(): s.value() for s in status})
            patch.update(modes)
            patch.update(errors)
            patch.update({k: None for k in stale_errors})
            if plan:
                patch[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] = plan
            self.api.patch("Node", self.node_name, {"metadata": {"annotations": patch}})
            self.reports += 1
            if plan and ann.get(C.ANNOTATION_REPORTED_PARTITIONING_PLAN, "") != plan:
                tracing.event("agent.plan_reported", node=self.node_name, plan_id=plan, kind="partition")
            self.shared.on_report_done()
            return Result(requeue_after=self.refresh_s)

    def controller(self) -> Controller:
        return Controller(f"partagent-reporter-{self.node_name}", self).for_kind(
            "Node", ExcludeDelete(), MatchingName(self.node_name), NodeResourcesChanged())


# ====================================================================== actuator
class PartitionActuator:
    """``MigActuator`` analogue.  ``device_plugins`` are refreshed after a mode
    switch (the reference restarts the device-plugin pod).  Each switch runs in
    a worker thread bounded by ``switch_timeout_s`` (see the module doc)."""

    def __init__(self, api, node_name: str, smi, lister, shared: SharedState, device_plugins=(),
                 memory_preference: str = "NPS1", switch_timeout_s: float = 120.0):
        self.api, self.node_name, self.smi = api, node_name, smi
        self.switch_timeout_s = switch_timeout_s
        self.failures = 0
        self.timeouts = 0
        self.devices = NodeDeviceClient(smi, lister)
        self.shared = shared
        self.device_plugins = list(device_plugins)
        self.memory_preference = memory_preference
        self.last_applied_plan: PartitionPlan | None = None
        self.last_applied_status = None
        self.applies = 0
        self._ilock = threading.Lock()
        self._inflight: dict[int, dict] = {}   # gpu -> switch still running past its deadline

    def inflight(self) -> set[int]:
        with self._ilock:
            return set(self._inflight)

    def reconcile(self, req: Request) -> Result:
        if not self.shared.at_least_one_report_since_last_apply():
            return Result(requeue_after=1.0)
        with self.shared.lock:  # planning only: the switches run after the lock is released
            node = self.api.try_get("Node", self.node_name)
            if node is None:
                return Result()
            plan_id = ko.annotations(node).get(C.ANNOTATION_PARTITIONING_PLAN, "")
            if plan_id:
                self.shared.last_parsed_plan_id = plan_id
            status, spec = parse_node_annotations(node)
            if spec_matches_status(spec, status) and not self._mode_mismatch(node):
                return Result()
            gpus = self.smi.gpus()
            inflight = self.inflight() | {g.index for g in gpus if g.switching}
            used = self.devices.used_gpus(C.AMD_PARTITION_RESOURCE_PREFIX) | self.devices.used_gpus(
                C.RESOURCE_AMD_GPU)
            busy = {g.index for g in gpus if g.index not in inflight and self.smi.processes(g.index)}
            plan = new_partition_plan(node, gpus, used, busy, self.memory_preference, inflight)
            for gi, why in plan.blocked.items():
                log.info("node %s gpu %d cannot be repartitioned now: %s", self.node_name, gi, why)
            if plan.is_empty():
                if plan.blocked:
                    return Result(requeue_after=10.0)
                return Result()
            if self.last_applied_plan == plan and status_equal(self.last_applied_status or [], status):
                log.info("plan already applied and state unchanged, skipping")
                return Result()
        failures = self.failures
        self.apply(plan, plan_id)
        self.shared.on_apply_done()
        if self.failures > failures:
            # do not remember a plan that did not (fully) apply: retry it
            self.last_applied_plan = None
            return Result(requeue_after=10.0)
        self.last_applied_plan = plan
        self.last_applied_status = status
        return Result(requeue_after=1.0)

    def _mode_mismatch(self, node: dict) -> bool:
        gpus = self.smi.gpus()
        want = desired_modes(node, gpus, self.memory_preference)
        return any((g.compute_mode, g.memory_mode) != want[g.index] for g in gpus if g.index in want)

    def apply(self, plan: PartitionPlan, plan_id: str = "") -> None:
        with tracing.span("partagent.apply", node=self.node_name, plan_id=plan_id, changes=len(plan.changes)):
            for ch in plan.changes:
                t0 = time.perf_counter()
                outcome = self._bounded_switch(ch)
                if outcome == "timeout":
                    self.failures += 1
                    self.timeouts += 1
                    why = (f"switch to {ch.compute}/{ch.memory} still running after {self.switch_timeout_s:.1f}s "
                           f"(deadline); GPU not planned until it returns")
                    self.shared.mark_failed(ch.gpu_index, why)
                    log.error("node %s gpu %d: %s", self.node_name, ch.gpu_index, why)
                    tracing.event("partagent.switch_timeout", node=self.node_name, gpu=ch.gpu_index,
                                  mode=f"{ch.compute}/{ch.memory}")
                    continue
                if not self._finish_switch(ch, outcome):
                    continue
                dt = time.perf_counter() - t0
                metrics.REPARTITION_DURATION.labels(mode=f"{ch.compute}/{ch.memory}").observe(dt)
                log.info("node %s gpu %d: %s/%s -> %s/%s (%.2fs)", self.node_name, ch.gpu_index, ch.from_compute,
                         ch.from_memory, ch.compute, ch.memory, dt)
            self.applies += 1
            self._refresh_plugins()

    def _refresh_plugins(self) -> None:
        for p in self.device_plugins:
            try:
                p.refresh()
            except Exception as e:  # a plugin that cannot re-enumerate now retries on its own poll
                log.error("node %s: device plugin refresh failed: %s", self.node_name, e)

    def _bounded_switch(self, ch: ModeChange):
        """Run the switch + verification in a worker thread; wait at most
        ``switch_timeout_s``.  Returns the worker's outcome dict, or "timeout"
        (the worker keeps running and finishes the GPU itself: _late_done)."""
        entry: dict = {"change": ch, "done": False, "late": False, "t0": time.monotonic()}

        def work():
            out: dict = {}
            try:
                self._switch(ch.gpu_index, ch.compute, ch.memory, ch.from_compute, ch.from_memory)
                out["ok"] = self._verify(ch.gpu_index, ch.compute, ch.memory)
            except Exception as e:  # reported by whoever finishes the switch
                out["error"] = e
            with self._ilock:
                entry["done"] = True
                entry["outcome"] = out
                late = entry["late"]
            if late:
                self._late_done(ch, out, time.monotonic() - entry["t0"])

        t = threading.Thread(target=work, daemon=True, name=f"partagent-switch-{self.node_name}-{ch.gpu_index}")
        t.start()
        t.join(self.switch_timeout_s)
        with self._ilock:
            if not entry["done"]:
                entry["late"] = True
                self._inflight[ch.gpu_index] = entry
                return "timeout"
            return entry["outcome"]

    def _finish_switch(self, ch: ModeChange, outcome: dict) -> bool:
        """Verification result of a switch that returned: True when the GPU is
        in the new mode; otherwise roll back and mark the GPU failed."""
        if outcome.get("ok"):
            self.shared.clear_failed(ch.gpu_index)
            return True
        err = outcome.get("error") or RuntimeError("mode did not take effect")
        log.error("node %s gpu %d: switching to %s/%s failed: %s -- rolling back to %s/%s", self.node_name,
                  ch.gpu_index, ch.compute, ch.memory, err, ch.from_compute, ch.from_memory)
        self.failures += 1
        self.shared.mark_failed(ch.gpu_index, f"switch to {ch.compute}/{ch.memory} failed: {err}")
        self._rollback(ch)
        return False

    def _late_done(self, ch: ModeChange, outcome: dict, took_s: float) -> None:
        """A switch that ran past its deadline has returned (worker thread)."""
        log.warning("node %s gpu %d: switch to %s/%s returned after %.1fs (deadline %.1fs)", self.node_name,
                    ch.gpu_index, ch.compute, ch.memory, took_s, self.switch_timeout_s)
        try:
            if self._finish_switch(ch, outcome):
                metrics.REPARTITION_DURATION.labels(mode=f"{ch.compute}/{ch.memory}").observe(took_s)
            self._refresh_plugins()
        finally:
            with self._ilock:
                self._inflight.pop(ch.gpu_index, None)
            self.last_applied_plan = None  # plan again from the state the late switch left

    def _switch(self, gpu: int, compute: str, memory: str, from_compute: str, from_memory: str) -> None:
        if memory != from_memory:
            self.smi.set_memory_partition(gpu, memory)
        if compute != from_compute:
            self.smi.set_compute_partition(gpu, compute)

    def _verify(self, gpu: int, compute: str, memory: str, retries: int = 3, delay_s: float = 0.2) -> bool:
        """Read the mode back: the driver may report the old mode for a moment
        after a switch (fault ``stale_mode``) or lose the device."""
        for i in range(retries):
            try:
                g = self.smi.gpu(gpu)
            except Exception:
                return False
            if (g.compute_mode, g.memory_mode) == (compute, memory):
                return True
            if i + 1 < retries:
                time.sleep(delay_s)
        return False

    def _rollback(self, ch: ModeChange) -> None:
        """Best effort: put the GPU back in the mode it had, so its old
        partitions (which the status still advertises) stay valid."""
        try:
            g = self.smi.gpu(ch.gpu_index)
            self._switch(ch.gpu_index, ch.from_compute, ch.from_memory, g.compute_mode, g.memory_mode)
        except Exception as e:
            log.error("node %s gpu %d: rollback failed: %s", self.node_name, ch.gpu_index, e)

    def controller(self) -> Controller:
        return Controller(f"partagent-actuator-{self.node_name}", self).for_kind(
            "Node", ExcludeDelete(), MatchingName(self.node_name), or_(AnnotationsChanged(), NodeResourcesChanged()))
