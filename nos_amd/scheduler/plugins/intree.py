"""In-tree scheduler plugins needed by the nos scheduler profiles.

Behavioural equivalents of the upstream kube-scheduler plugins the
reference's tests run against (``capacity_scheduling_test.go:444-466`` uses
QueueSort / NodeResourcesFit / DefaultBinder):

* PrioritySort (queue sort), NodeResourcesFit (PreFilter + Filter + a
  LeastAllocated-style score), NodeUnschedulable, NodeName, NodeAffinity
  (``nodeSelector`` + required node-affinity terms), TaintToleration,
  DefaultBinder, DefaultPreemption (priority-based PostFilter).
"""
from __future__ import annotations

from ...kube import objects as ko
from ...kube import selectors as sel
from ...resource.resource import Resource
from ..framework import (ERROR, SKIP, SUCCESS, UNRESOLVABLE, UNSCHEDULABLE, CycleState, NodeInfo, Plugin,
                         PreFilterResult, Status)


class PrioritySort(Plugin):
    name = "PrioritySort"

    @staticmethod
    def less(a: dict, b: dict) -> bool:
        pa, pb = ko.pod_priority(a), ko.pod_priority(b)
        if pa != pb:
            return pa > pb
        return ko.creation_time(a) < ko.creation_time(b)


_FIT_KEY = "PreFilterNodeResourcesFit"


class NodeResourcesFit(Plugin):
    """Fits pod requests (cpu, memory, ephemeral-storage, pods, scalar) into
    allocatable - requested; scores least-allocated (or most-allocated when
    ``strategy='MostAllocated'``, the bin-packing mode used for GPU slices)."""

    name = "NodeResourcesFit"

    def __init__(self, args: dict | None = None, handle=None):
        args = args or {}
        self.ignored = set(args.get("ignoredResources", []))
        self.strategy = (args.get("scoringStrategy") or {}).get("type", "LeastAllocated")
        self.score_resources = [r["name"] for r in (args.get("scoringStrategy") or {}).get("resources", [])] or \
            ["cpu", "memory"]

    def pre_filter(self, state: CycleState, pod: dict):
        from ..framework import PodInfo

        state.write(_FIT_KEY, PodInfo(pod).request)
        return None, Status.ok()

    def add_pod(self, state, pod, to_add, node_info):
        return Status.ok()

    def remove_pod(self, state, pod, to_remove, node_info):
        return Status.ok()

    def insufficient(self, req: Resource, ni: NodeInfo) -> list[str]:
        out = []
        if ni.allocatable.allowed_pod_number and len(ni.pods) + 1 > ni.allocatable.allowed_pod_number:
            out.append("Too many pods")
        free = ni.allocatable - ni.requested
        if req.milli_cpu and req.milli_cpu > free.milli_cpu:
            out.append("Insufficient cpu")
        if req.memory and req.memory > free.memory:
            out.append("Insufficient memory")
        if req.ephemeral_storage and req.ephemeral_storage > free.ephemeral_storage:
            out.append("Insufficient ephemeral-storage")
        for k, v in req.scalar.items():
            if v == 0 or k in self.ignored:
                continue
            if v > free.scalar.get(k, 0):
                out.append(f"Insufficient {k}")
        return out

    def filter(self, state: CycleState, pod: dict, ni: NodeInfo) -> Status:
        req = state.get(_FIT_KEY)
        if req is None:
            from ..framework import PodInfo

            req = PodInfo(pod).request
        r = self.insufficient(req, ni)
        return Status(UNSCHEDULABLE, r) if r else Status.ok()

    def score(self, state: CycleState, pod: dict, ni: NodeInfo) -> int:
        req = state.get(_FIT_KEY) or Resource()
        total = 0
        n = 0
        for r in self.score_resources:
            cap = ni.allocatable.get(r)
            if cap <= 0:
                continue
            used = ni.requested.get(r) + req.get(r)
            frac = min(1.0, used / cap)
            total += (frac if self.strategy == "MostAllocated" else 1.0 - frac) * 100
            n += 1
        return int(total / n) if n else 0


class NodeUnschedulable(Plugin):
    name = "NodeUnschedulable"

    def filter(self, state, pod, ni: NodeInfo) -> Status:
        node = ni.node() or {}
        if node.get("spec", {}).get("unschedulable"):
            tol = any(t.get("key") == "node.kubernetes.io/unschedulable" for t in pod.get("spec", {}).get("tolerations") or [])
            if not tol:
                return Status(UNRESOLVABLE, ["node(s) were unschedulable"])
        return Status.ok()


class NodeName(Plugin):
    name = "NodeName"

    def filter(self, state, pod, ni: NodeInfo) -> Status:
        want = pod.get("spec", {}).get("nodeName")
        if want and want != ni.name:
            return Status(UNRESOLVABLE, ["node(s) didn't match the requested node name"])
        return Status.ok()


class NodeAffinity(Plugin):
    name = "NodeAffinity"

    def filter(self, state, pod, ni: NodeInfo) -> Status:
        node = ni.node() or {}
        labels = ko.labels(node)
        ns = pod.get("spec", {}).get("nodeSelector") or {}
        if any(labels.get(k) != v for k, v in ns.items()):
            return Status(UNRESOLVABLE, ["node(s) didn't match Pod's node affinity/selector"])
        aff = (((pod.get("spec") or {}).get("affinity") or {}).get("nodeAffinity") or {}) \
            .get("requiredDuringSchedulingIgnoredDuringExecution")
        if aff:
            terms = aff.get("nodeSelectorTerms") or []
            if terms and not any(sel.match_labels(sel.selector_from_object(
                    {"matchExpressions": t.get("matchExpressions") or []}), labels) for t in terms):
                return Status(UNRESOLVABLE, ["node(s) didn't match Pod's node affinity/selector"])
        return Status.ok()


class TaintToleration(Plugin):
    name = "TaintToleration"

    @staticmethod
    def tolerates(tols: list[dict], taint: dict) -> bool:
        for t in tols:
            if t.get("effect") and t["effect"] != taint.get("effect"):
                continue
            if t.get("operator") == "Exists" and (not t.get("key") or t["key"] == taint.get("key")):
                return True
            if t.get("key") == taint.get("key") and t.get("value", "") == taint.get("value", ""):
                return True
        return False

    def filter(self, state, pod, ni: NodeInfo) -> Status:
        node = ni.node() or {}
        tols = pod.get("spec", {}).get("tolerations") or []
        for taint in node.get("spec", {}).get("taints") or []:
            if taint.get("effect") in ("NoSchedule", "NoExecute") and not self.tolerates(tols, taint):
                return Status(UNRESOLVABLE, [f"node(s) had untolerated taint {{{taint.get('key')}: {taint.get('value', '')}}}"])
        return Status.ok()


class DefaultBinder(Plugin):
    name = "DefaultBinder"

    def __init__(self, args=None, handle=None):
        self.handle = handle

    def set_handle(self, h):
        self.handle = h

    def bind(self, state, pod: dict, node_name: str) -> Status:
        api = getattr(self.handle, "api", None)
        if api is None:
            return Status(ERROR, ["no API client"])
        try:
            api.bind(ko.name(pod), ko.namespace(pod), node_name)
        except Exception as e:  # conflict / not found
            return Status(ERROR, [str(e)])
        return Status.ok()


class DefaultPreemption(Plugin):
    """Priority-based preemption (upstream DefaultPreemption): victims are
    lower-priority pods; uses the shared :class:`~nos_amd.scheduler.preemption.Evaluator`."""

    name = "DefaultPreemption"

    def __init__(self, args=None, handle=None):
        self.handle = handle

    def set_handle(self, h):
        self.handle = h

    def post_filter(self, state, pod, statuses):
        from ..preemption import Evaluator, PriorityPreemptor

        ev = Evaluator(self.name, self.handle, state, PriorityPreemptor(self.handle, state))
        return ev.preempt(pod, statuses)


REGISTRY = {
    "PrioritySort": PrioritySort,
    "NodeResourcesFit": NodeResourcesFit,
    "NodeUnschedulable": NodeUnschedulable,
    "NodeName": NodeName,
    "NodeAffinity": NodeAffinity,
    "TaintToleration": TaintToleration,
    "DefaultBinder": DefaultBinder,
    "DefaultPreemption": DefaultPreemption,
}

__all__ = list(REGISTRY) + ["REGISTRY", "SKIP", "SUCCESS", "PreFilterResult"]
