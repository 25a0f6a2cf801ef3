"""gpupartitioner controllers (``internal/controllers/gpupartitioner``).

* :class:`NodeController` -- keeps :class:`ClusterState` nodes current, runs
  the amdpart node initializer on uninitialised partition nodes
  (``node_controller.go:60-117``);
* :class:`PodController` -- keeps pod usage current (``pod_controller.go:47-104``);
* :class:`PartitionerController` -- one per strategy, reconciles every pod
  event: pods that extra resources could help are batched (timeout / idle
  windows); while any node has ``spec-partitioning-plan !=
  status-partitioning-plan`` the batch is reset and the pod requeued after
  10 s (the plan handshake, with a timeout so a dead agent cannot block
  planning forever); when the batch is ready: list pending unscheduled pods,
  snapshot, plan on a clone, apply on a clone (``partitioner_controller.go:81-232``).
  Each controller owns its batcher (the reference shared one between MIG
  and MPS).
"""
from __future__ import annotations

import logging
import time

from ..api import constants as C
from ..gpu.core import get_count, get_model, is_amdpart_enabled, partitioning_kind
from ..kube import objects as ko
from ..observability import metrics, tracing
from ..partitioning.core import Actuator, Planner, is_node_initialized
from ..partitioning.state import ClusterState
from ..runtime.manager import Controller, Request, Result
from ..runtime.predicates import Funcs, HasLabel
from ..utils.batcher import Batcher
from ..utils.pod import extra_resources_could_help_scheduling

log = logging.getLogger("nos_amd.controllers.gpupartitioner")


class NodeController:
    def __init__(self, api, cluster_state: ClusterState, amdpart_initializer=None):
        self.api, self.cs, self.init = api, cluster_state, amdpart_initializer

    def reconcile(self, req: Request) -> Result:
        node = self.api.try_get("Node", req.name)
        if node is None:
            self.cs.delete_node(req.name)
            return Result()
        if partitioning_kind(node) is None:
            self.cs.delete_node(req.name)
            return Result()
        try:
            get_model(node)
            get_count(node)
        except Exception:
            log.debug("node %s has no GPU model/count labels yet", req.name)
            return Result()
        if is_amdpart_enabled(node) and self.init is not None and not is_node_initialized(node):
            self.init.init_node_partitioning(node)
            node = self.api.get("Node", req.name)
        pods = self.api.list("Pod", field_selector=f"{C.POD_NODE_NAME_KEY}={req.name}")
        self.cs.update_node(node, pods)
        return Result()

    def controller(self, name: str = C.CLUSTER_STATE_NODE_CONTROLLER) -> Controller:
        return Controller(name, self, max_concurrent=10).for_kind("Node", HasLabel(C.LABEL_GPU_PARTITIONING))


class PodController:
    def __init__(self, api, cluster_state: ClusterState):
        self.api, self.cs = api, cluster_state

    def reconcile(self, req: Request) -> Result:
        pod = self.api.try_get("Pod", req.name, req.namespace)
        if pod is None:
            try:
                self.cs.delete_pod(req.namespace, req.name)
            except KeyError:
                pass
            return Result()
        nn = ko.pod_node(pod)
        if not nn:
            return Result()
        if self.cs.get_node(nn) is None:
            node = self.api.try_get("Node", nn)
            if node is not None and partitioning_kind(node) is not None:
                self.cs.update_node(node, self.api.list("Pod", field_selector=f"{C.POD_NODE_NAME_KEY}={nn}"))
            return Result()
        self.cs.update_usage(pod)
        return Result()

    def controller(self, name: str = C.CLUSTER_STATE_POD_CONTROLLER) -> Controller:
        return Controller(name, self, max_concurrent=10).for_kind("Pod")


class PartitionerController:
    REQUEUE_WAITING_PLAN_S = 10.0
    REQUEUE_BATCH_OPEN_S = 5.0

    def __init__(self, api, cluster_state: ClusterState, strategy, framework, clock=None,
                 batch_timeout_s: float = 60.0, batch_idle_s: float = 10.0, plan_report_timeout_s: float = 300.0):
        self.api = api
        self.cs = cluster_state
        self.strategy = strategy
        self.kind = strategy.kind
        self.clock = clock or api.clock
        self.planner = Planner(strategy.partition_calculator, strategy.slice_calculator, framework)
        self.actuator = Actuator(api, strategy.partitioner)
        self.batcher: Batcher[dict] = Batcher(batch_timeout_s, batch_idle_s, self.clock)
        self.batcher.start()
        self.current_batch: dict[str, dict] = {}
        self.plan_report_timeout_s = plan_report_timeout_s
        self._plan_seen: dict[str, tuple[str, float]] = {}
        self.plans_applied = 0
        self.last_plan = None

    def reconcile(self, req: Request) -> Result:
        if not self.cs.is_partitioning_enabled(self.kind):
            return Result()
        pod = self.api.try_get("Pod", req.name, req.namespace)
        if pod is None:
            return Result()
        key = ko.key(pod)
        if not extra_resources_could_help_scheduling(pod) or not self._requests_kind(pod):
            if key in self.current_batch:
                del self.current_batch[key]
                if not self.current_batch:
                    self.batcher.reset()
            return Result()
        if self.waiting_any_node_to_report_plan():
            self.batcher.reset()
            self.current_batch.clear()
            return Result(requeue_after=self.REQUEUE_WAITING_PLAN_S)
        if key not in self.current_batch:
            self.batcher.add(pod)
            self.current_batch[key] = pod
        if self.batcher.ready() is not None:
            self.current_batch = {}
            self.process_pending_pods()
            return Result()
        if self.current_batch:
            d = self.batcher.next_deadline()
            return Result(requeue_after=min(self.REQUEUE_BATCH_OPEN_S, max(0.01, d if d is not None else 0.01)))
        self.batcher.reset()
        return Result()

    def _requests_kind(self, pod: dict) -> bool:
        return bool(self.strategy.slice_calculator.get_requested_slices(pod))

    def process_pending_pods(self) -> None:
        pending = [p for p in self.api.list("Pod", field_selector=f"{C.POD_PHASE_KEY}={ko.PENDING}")
                   if not ko.pod_node(p)]
        pods = [p for p in pending if extra_resources_could_help_scheduling(p) and self._requests_kind(p)]
        metrics.PENDING_FRACTIONAL_PODS.set(len(pods))
        if not pods:
            return
        with tracing.span("partitioner.plan", kind=self.kind, pods=len(pods)) as sp:
            t0 = time.perf_counter()
            snapshot = self.strategy.snapshot_taker.take_snapshot(self.cs)
            plan = self.planner.plan(snapshot.clone(), pods)
            metrics.PLAN_DURATION.labels(kind=self.kind).observe(time.perf_counter() - t0)
            sp.set(plan_id=plan.id, placed=self.planner.last_stats.get("placed"))
            applied = self.actuator.apply(snapshot.clone(), plan)
            sp.set(applied=applied)
        self.last_plan = plan
        if applied:
            self.plans_applied += 1
            metrics.PLANS_APPLIED.labels(kind=self.kind).inc()

    def waiting_any_node_to_report_plan(self) -> bool:
        now = self.clock.monotonic()
        for ni in self.cs.get_nodes().values():
            n = ni.node()
            if n is None or partitioning_kind(n) != self.kind:
                continue
            cur = self.api.try_get("Node", ko.name(n)) or n
            ann = ko.annotations(cur)
            plan = ann.get(C.ANNOTATION_PARTITIONING_PLAN)
            if not plan:
                continue
            if ann.get(C.ANNOTATION_REPORTED_PARTITIONING_PLAN) == plan:
                continue
            seen = self._plan_seen.get(ko.name(n))
            if seen is None or seen[0] != plan:
                self._plan_seen[ko.name(n)] = (plan, now)
                return True
            if now - seen[1] < self.plan_report_timeout_s:
                return True
            log.warning("node %s did not report plan %s within %.0fs; planning anyway", ko.name(n), plan,
                        self.plan_report_timeout_s)
        return False

    def controller(self, name: str | None = None) -> Controller:
        name = name or (C.AMDPART_PARTITIONER_CONTROLLER if self.kind == C.PARTITIONING_AMDPART
                        else C.CUMASK_PARTITIONER_CONTROLLER)
        return Controller(name, self).for_kind("Pod", Funcs(delete=lambda ev: False))
