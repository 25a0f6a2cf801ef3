"""Scheduler framework: the kube-scheduler plugin model, in Python.

The reference's elastic-quota plugin is a kube-scheduler out-of-tree plugin
and the gpupartitioner embeds the scheduler framework to simulate scheduling
(``cmd/gpupartitioner/gpupartitioner.go:294-318``,
``internal/partitioning/core/planner.go:178-207``).  This module provides the
same extension points and semantics:

* :class:`Status` codes (Success, Error, Unschedulable,
  UnschedulableAndUnresolvable, Wait, Skip);
* :class:`CycleState` (cloneable per-cycle scratch space);
* :class:`PodInfo` / :class:`NodeInfo` with incremental requested-resource
  accounting and cheap cloning (the planner clones node infos per fork);
* :class:`PodNominator` (nominated pods per node);
* :class:`Framework` with PreFilter(+AddPod/RemovePod extensions), Filter,
  ``run_filter_plugins_with_nominated_pods`` (upstream two-pass logic),
  PostFilter, Score, Reserve/Unreserve, Permit, Bind.
"""
from __future__ import annotations

import copy
import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Iterable, Protocol

from ..kube import objects as ko
from ..resource.resource import Resource, compute_pod_request

SUCCESS, ERROR, UNSCHEDULABLE, UNRESOLVABLE, WAIT, SKIP = (
    "Success", "Error", "Unschedulable", "UnschedulableAndUnresolvable", "Wait", "Skip")


@dataclass
class Status:
    code: str = SUCCESS
    reasons: list[str] = field(default_factory=list)
    plugin: str = ""

    @classmethod
    def ok(cls) -> "Status":
        return cls(SUCCESS)

    @classmethod
    def new(cls, code: str, *reasons: str) -> "Status":
        return cls(code, [r for r in reasons if r])

    def is_success(self) -> bool:
        return self.code == SUCCESS

    def is_unschedulable(self) -> bool:
        return self.code in (UNSCHEDULABLE, UNRESOLVABLE)

    def message(self) -> str:
        return ", ".join(self.reasons)

    def as_error(self) -> Exception:
        return RuntimeError(f"{self.plugin}: {self.code}: {self.message()}")

    def __str__(self) -> str:
        return f"{self.code}({self.plugin}: {self.message()})" if self.reasons else self.code


def as_status(e: BaseException) -> Status:
    return Status(ERROR, [str(e)])


class CycleState:
    def __init__(self):
        self._d: dict[str, Any] = {}
        self.skip_filter_plugins: set[str] = set()

    def write(self, key: str, v: Any) -> None:
        self._d[key] = v

    def read(self, key: str) -> Any:
        if key not in self._d:
            raise KeyError(f"{key} not found in cycle state")
        return self._d[key]

    def get(self, key: str, default=None) -> Any:
        return self._d.get(key, default)

    def clone(self) -> "CycleState":
        c = CycleState()
        for k, v in self._d.items():
            c._d[k] = v.clone() if hasattr(v, "clone") else copy.copy(v)
        c.skip_filter_plugins = set(self.skip_filter_plugins)
        return c


# --------------------------------------------------------------------- infos
class PodInfo:
    __slots__ = ("pod", "_req", "key")

    def __init__(self, pod: dict, request: Resource | None = None):
        self.pod = pod
        self._req = request
        self.key = pod_key(pod)

    @property
    def request(self) -> Resource:
        if self._req is None:
            self._req = Resource.from_list(compute_pod_request(self.pod))
        return self._req


def pod_key(pod: dict) -> str:
    u = ko.uid(pod)
    return u if u else ko.key(pod)


class NodeInfo:
    def __init__(self, node: dict | None = None):
        self._node = node
        self.pods: list[PodInfo] = []
        self.requested = Resource()
        self.allocatable = Resource.from_list((node or {}).get("status", {}).get("allocatable") or {})
        self.generation = 0

    def node(self) -> dict | None:
        return self._node

    @property
    def name(self) -> str:
        return ko.name(self._node) if self._node else ""

    def set_node(self, node: dict) -> None:
        self._node = node
        self.allocatable = Resource.from_list(node.get("status", {}).get("allocatable") or {})
        self.generation += 1

    def add_pod(self, pod: dict | PodInfo) -> None:
        pi = pod if isinstance(pod, PodInfo) else PodInfo(pod)
        self.pods.append(pi)
        self.requested.iadd(pi.request)
        self.requested.allowed_pod_number += 1
        self.generation += 1

    add_pod_info = add_pod

    def remove_pod(self, pod: dict) -> None:
        k = pod_key(pod)
        for i, pi in enumerate(self.pods):
            if pi.key == k:
                self.pods.pop(i)
                self.requested.isub(pi.request)
                self.requested.allowed_pod_number -= 1
                self.generation += 1
                return
        raise KeyError(f"no corresponding pod {ko.key(pod)} in pods of node {self.name}")

    def has_pod(self, pod: dict) -> bool:
        k = pod_key(pod)
        return any(pi.key == k for pi in self.pods)

    def clone(self) -> "NodeInfo":
        n = NodeInfo.__new__(NodeInfo)
        n._node = self._node
        n.pods = list(self.pods)
        n.requested = self.requested.clone()
        n.allocatable = self.allocatable.clone()
        n.generation = self.generation
        return n

    def free(self) -> Resource:
        return self.allocatable - self.requested

    def __repr__(self) -> str:
        return f"NodeInfo({self.name}, pods={len(self.pods)}, req={self.requested}, alloc={self.allocatable})"


class NodeInfoLister(Protocol):
    def list(self) -> list[NodeInfo]: ...

    def get(self, name: str) -> NodeInfo | None: ...


class Snapshot:
    """Immutable-by-convention view of the cluster for one scheduling cycle."""

    def __init__(self, node_infos: Iterable[NodeInfo] = ()):
        self._infos = {ni.name: ni for ni in node_infos}

    def list(self) -> list[NodeInfo]:
        return list(self._infos.values())

    def get(self, name: str) -> NodeInfo | None:
        return self._infos.get(name)

    def set(self, ni: NodeInfo) -> None:
        self._infos[ni.name] = ni

    @classmethod
    def from_objects(cls, pods: Iterable[dict], nodes: Iterable[dict]) -> "Snapshot":
        """``fakeSharedLister``: node infos from static pods/nodes (pkg/test/util/fake.go)."""
        infos = {ko.name(n): NodeInfo(n) for n in nodes}
        for p in pods:
            nn = ko.pod_node(p)
            if nn in infos and not ko.is_terminated(p):
                infos[nn].add_pod(p)
        return cls(infos.values())


class PodNominator:
    """Tracks pods nominated to nodes by preemption (upstream ``PodNominator``)."""

    def __init__(self):
        self._lock = threading.RLock()
        self._by_node: dict[str, list[PodInfo]] = {}
        self._node_of: dict[str, str] = {}

    def add_nominated_pod(self, pod: dict, node_name: str | None = None) -> None:
        nn = node_name or ko.pod_nominated_node(pod)
        if not nn:
            return
        with self._lock:
            self.delete_nominated_pod_if_exists(pod)
            pi = PodInfo(pod)
            self._by_node.setdefault(nn, []).append(pi)
            self._node_of[pi.key] = nn

    def delete_nominated_pod_if_exists(self, pod: dict) -> None:
        k = pod_key(pod)
        with self._lock:
            nn = self._node_of.pop(k, None)
            if nn is not None:
                self._by_node[nn] = [p for p in self._by_node.get(nn, []) if p.key != k]

    def update_nominated_pod(self, old: dict, new: dict) -> None:
        with self._lock:
            nn = ko.pod_nominated_node(new) or self._node_of.get(pod_key(old))
            self.delete_nominated_pod_if_exists(old)
            if nn and not ko.pod_node(new):
                self.add_nominated_pod(new, nn)

    def nominated_pods_for_node(self, node_name: str) -> list[PodInfo]:
        with self._lock:
            return list(self._by_node.get(node_name, []))

    def nominated_node(self, pod: dict) -> str | None:
        return self._node_of.get(pod_key(pod))


# --------------------------------------------------------------------- plugins
class Plugin:
    name = "Plugin"

    def events_to_register(self) -> list[tuple[str, str]]:
        return []


@dataclass
class PreFilterResult:
    node_names: set[str] | None = None


@dataclass
class PostFilterResult:
    nominated_node_name: str = ""


class Framework:
    """Runs plugins at each extension point (``framework.Framework``)."""

    EXTENSION_POINTS = ("queue_sort", "pre_filter", "filter", "post_filter", "pre_score", "score", "reserve",
                        "permit", "pre_bind", "bind", "post_bind")

    def __init__(self, plugins: dict[str, list[Plugin]], snapshot: Snapshot | None = None,
                 nominator: PodNominator | None = None, api=None, profile_name: str = "default-scheduler",
                 score_weights: dict[str, int] | None = None):
        self.plugins = {ep: list(plugins.get(ep, [])) for ep in self.EXTENSION_POINTS}
        self._snapshot = snapshot or Snapshot()
        self.nominator = nominator or PodNominator()
        self.api = api
        self.profile_name = profile_name
        self.score_weights = score_weights or {}
        for ps in self.plugins.values():
            for p in ps:
                if hasattr(p, "set_handle"):
                    p.set_handle(self)

    # ---------------------------------------------------------- handle API
    def snapshot_shared_lister(self) -> Snapshot:
        return self._snapshot

    def set_snapshot(self, s: Snapshot) -> None:
        self._snapshot = s

    def nominated_pods_for_node(self, node_name: str) -> list[PodInfo]:
        return self.nominator.nominated_pods_for_node(node_name)

    def has_filter_plugins(self) -> bool:
        return bool(self.plugins["filter"])

    def list_plugins(self) -> dict[str, list[str]]:
        return {ep: [p.name for p in ps] for ep, ps in self.plugins.items() if ps}

    # ---------------------------------------------------------- pre-filter
    def run_pre_filter_plugins(self, state: CycleState, pod: dict) -> tuple[PreFilterResult | None, Status]:
        result: PreFilterResult | None = None
        for p in self.plugins["pre_filter"]:
            r, s = p.pre_filter(state, pod)
            if s.code == SKIP:
                state.skip_filter_plugins.add(p.name)
                continue
            if not s.is_success():
                s.plugin = s.plugin or p.name
                if s.code == ERROR:
                    s.reasons = [f"running PreFilter plugin {p.name!r}: {s.message()}"]
                return None, s
            if r is not None and r.node_names is not None:
                result = r if result is None or result.node_names is None else \
                    PreFilterResult(result.node_names & r.node_names)
        return result, Status.ok()

    def run_pre_filter_extension_add_pod(self, state: CycleState, pod: dict, to_add: PodInfo,
                                         node_info: NodeInfo) -> Status:
        for p in self.plugins["pre_filter"]:
            if p.name in state.skip_filter_plugins or not hasattr(p, "add_pod"):
                continue
            s = p.add_pod(state, pod, to_add, node_info)
            if not s.is_success():
                return s
        return Status.ok()

    def run_pre_filter_extension_remove_pod(self, state: CycleState, pod: dict, to_remove: PodInfo,
                                            node_info: NodeInfo) -> Status:
        for p in self.plugins["pre_filter"]:
            if p.name in state.skip_filter_plugins or not hasattr(p, "remove_pod"):
                continue
            s = p.remove_pod(state, pod, to_remove, node_info)
            if not s.is_success():
                return s
        return Status.ok()

    # ---------------------------------------------------------- filter
    def run_filter_plugins(self, state: CycleState, pod: dict, node_info: NodeInfo) -> Status:
        for p in self.plugins["filter"]:
            if p.name in state.skip_filter_plugins:
                continue
            s = p.filter(state, pod, node_info)
            if not s.is_success():
                s.plugin = s.plugin or p.name
                return s
        return Status.ok()

    def _add_nominated_pods(self, pod: dict, state: CycleState, node_info: NodeInfo
                            ) -> tuple[bool, CycleState, NodeInfo]:
        nominated = self.nominated_pods_for_node(node_info.name)
        if not nominated:
            return False, state, node_info
        ni = node_info.clone()
        st = state.clone()
        added = False
        prio = ko.pod_priority(pod)
        for pi in nominated:
            if pi.key != pod_key(pod) and ko.pod_priority(pi.pod) >= prio and not ni.has_pod(pi.pod):
                ni.add_pod(pi)
                s = self.run_pre_filter_extension_add_pod(st, pod, pi, ni)
                if not s.is_success():
                    return False, state, node_info
                added = True
        return added, st, ni

    def run_filter_plugins_with_nominated_pods(self, state: CycleState, pod: dict, node_info: NodeInfo) -> Status:
        """Upstream semantics: filter with higher/equal-priority nominated pods
        added, then (if any were added) again without them."""
        status = Status.ok()
        for i in range(2):
            st, ni = state, node_info
            added = False
            if i == 0:
                added, st, ni = self._add_nominated_pods(pod, state, node_info)
            elif not status.is_success():
                break
            status = self.run_filter_plugins(st, pod, ni)
            if not status.is_success():
                break
            if i == 0 and not added:
                break
        return status

    # ---------------------------------------------------------- post-filter
    def run_post_filter_plugins(self, state: CycleState, pod: dict, statuses: dict[str, Status]
                                ) -> tuple[PostFilterResult | None, Status]:
        reasons = []
        for p in self.plugins["post_filter"]:
            r, s = p.post_filter(state, pod, statuses)
            if s.is_success():
                return r, s
            if s.code != UNSCHEDULABLE and s.code != UNRESOLVABLE:
                return None, s
            reasons.extend(s.reasons)
        return None, Status(UNSCHEDULABLE, reasons)

    # ---------------------------------------------------------- score
    def run_score_plugins(self, state: CycleState, pod: dict, nodes: list[NodeInfo]) -> dict[str, int]:
        totals = {n.name: 0 for n in nodes}
        for p in self.plugins["pre_score"]:
            p.pre_score(state, pod, nodes)
        for p in self.plugins["score"]:
            w = self.score_weights.get(p.name, 1)
            scores = {n.name: p.score(state, pod, n) for n in nodes}
            if hasattr(p, "normalize_score"):
                scores = p.normalize_score(state, pod, scores)
            for k, v in scores.items():
                totals[k] += w * v
        return totals

    # ---------------------------------------------------------- reserve / permit / bind
    def run_reserve_plugins_reserve(self, state: CycleState, pod: dict, node_name: str) -> Status:
        for p in self.plugins["reserve"]:
            s = p.reserve(state, pod, node_name)
            if not s.is_success():
                s.plugin = p.name
                return s
        return Status.ok()

    def run_reserve_plugins_unreserve(self, state: CycleState, pod: dict, node_name: str) -> None:
        for p in reversed(self.plugins["reserve"]):
            p.unreserve(state, pod, node_name)

    def run_permit_plugins(self, state: CycleState, pod: dict, node_name: str) -> Status:
        for p in self.plugins["permit"]:
            s = p.permit(state, pod, node_name)
            if not s.is_success():
                return s
        return Status.ok()

    def run_bind_plugins(self, state: CycleState, pod: dict, node_name: str) -> Status:
        for p in self.plugins["pre_bind"]:
            s = p.pre_bind(state, pod, node_name)
            if not s.is_success():
                return s
        for p in self.plugins["bind"]:
            s = p.bind(state, pod, node_name)
            if s.code == SKIP:
                continue
            return s
        return Status(ERROR, ["no bind plugin bound the pod"])

    def run_post_bind_plugins(self, state: CycleState, pod: dict, node_name: str) -> None:
        for p in self.plugins["post_bind"]:
            p.post_bind(state, pod, node_name)


PluginFactory = Callable[[dict | None, Framework | None], Plugin]
