"""Cluster state and partitioning-state types of the gpupartitioner.

* :class:`ClusterState` (``internal/partitioning/state/state.go:29-222``):
  thread-safe in-memory view of nodes (as scheduler NodeInfos counting only
  Running pods), pod -> node bindings and a histogram of partitioning kinds.
  Unlike the reference, ``get_nodes`` returns a copy of the map taken under
  the lock (the reference returned the live map after unlocking,
  ``state.go:65-70``).
* :class:`GPUPartitioning` / :class:`NodePartitioning` /
  :class:`PartitioningState` with order-insensitive equality
  (``partitioning.go:24-56``), extended with the GPU's target compute/memory
  mode for the amdpart strategy.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field

from ..gpu.core import partitioning_kind
from ..kube import objects as ko
from ..scheduler.framework import NodeInfo


@dataclass(frozen=True)
class GPUPartitioning:
    gpu_index: int
    resources: tuple[tuple[str, int], ...]  # sorted (resource name, quantity)
    mode: str = ""                           # e.g. "CPX/NPS2" (amdpart only)

    @classmethod
    def of(cls, gpu_index: int, resources: dict[str, int], mode: str = "") -> "GPUPartitioning":
        return cls(gpu_index, tuple(sorted((k, int(v)) for k, v in resources.items() if v)), mode)

    def resource_dict(self) -> dict[str, int]:
        return dict(self.resources)


@dataclass
class NodePartitioning:
    gpus: list[GPUPartitioning] = field(default_factory=list)

    def equal(self, other: "NodePartitioning | None") -> bool:
        if other is None or len(self.gpus) != len(other.gpus):
            return False
        return sorted(self.gpus, key=repr) == sorted(other.gpus, key=repr)


class PartitioningState(dict):
    """node name -> NodePartitioning"""

    def is_empty(self) -> bool:
        return len(self) == 0

    def equal(self, other: "PartitioningState") -> bool:
        if len(self) != len(other):
            return False
        return all(np.equal(other.get(n)) for n, np in self.items())


class ClusterState:
    def __init__(self):
        self._mtx = threading.RLock()
        self.nodes: dict[str, NodeInfo] = {}
        self.bindings: dict[str, str] = {}
        self.partitioning_kinds: dict[str, int] = {}

    def get_node(self, name: str) -> NodeInfo | None:
        with self._mtx:
            return self.nodes.get(name)

    def get_nodes(self) -> dict[str, NodeInfo]:
        with self._mtx:
            return dict(self.nodes)

    def delete_node(self, name: str) -> None:
        with self._mtx:
            self.nodes.pop(name, None)
            for k in [k for k, n in self.bindings.items() if n == name]:
                del self.bindings[k]
            self._refresh_kinds()

    def update_node(self, node: dict, pods: list[dict]) -> None:
        with self._mtx:
            ni = NodeInfo(node)
            for p in pods:
                if ko.pod_phase(p) == ko.RUNNING:
                    ni.add_pod(p)
            self.nodes[ko.name(node)] = ni
            for k in [k for k, n in self.bindings.items() if n == ko.name(node)]:
                del self.bindings[k]
            for p in pods:
                self.bindings[ko.key(p)] = ko.name(node)
            self._refresh_kinds()

    def delete_pod(self, namespace: str, name: str) -> None:
        key = f"{namespace}/{name}"
        with self._mtx:
            node_name = self.bindings.pop(key, None)
            if node_name is None:
                raise KeyError(f"cannot delete pod {key} from cluster state: pod not found")
            ni = self.nodes.get(node_name)
            if ni is None:
                return
            for pi in ni.pods:
                if ko.key(pi.pod) == key:
                    ni.remove_pod(pi.pod)
                    return

    def update_usage(self, pod: dict) -> None:
        nn = ko.pod_node(pod)
        if not nn:
            return
        with self._mtx:
            ni = self.nodes.get(nn)
            if ni is None:
                return
            key = ko.key(pod)
            cached = self.bindings.get(key)
            running = ko.pod_phase(pod) == ko.RUNNING
            if cached is not None:
                if cached != nn:
                    old = self.nodes.get(cached)
                    if old is not None and old.has_pod(pod):
                        old.remove_pod(pod)
                    if running and not ni.has_pod(pod):
                        ni.add_pod(pod)
                elif not running and ni.has_pod(pod):
                    ni.remove_pod(pod)
                elif running and not ni.has_pod(pod):
                    ni.add_pod(pod)
            elif running:
                ni.add_pod(pod)
            self.bindings[key] = nn

    def _refresh_kinds(self) -> None:
        kinds: dict[str, int] = {}
        for ni in self.nodes.values():
            n = ni.node()
            if n is not None:
                k = partitioning_kind(n)
                if k:
                    kinds[k] = kinds.get(k, 0) + 1
        self.partitioning_kinds = kinds

    def is_partitioning_enabled(self, kind: str) -> bool:
        with self._mtx:
            return self.partitioning_kinds.get(kind, 0) > 0
