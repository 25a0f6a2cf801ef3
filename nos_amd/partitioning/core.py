"""Partitioning core: snapshot / tracker / sorter / planner / actuator.

Same algorithm as the reference's ``internal/partitioning/core``:

* :class:`ClusterSnapshot` with single-level ``fork`` / ``commit`` /
  ``revert`` (deep clone of the partitionable nodes), candidate nodes (free
  capacity, by name), lacking slices of a pod (pod request minus cluster-wide
  free, filtered to GPU slices) -- ``snapshot.go:29-190``.  Fixed gotcha: the
  planner fetches each candidate node from the fork *after* forking, so
  ``revert`` really undoes a geometry change (the reference mutated pre-fork
  node objects);
* :class:`SliceTracker` (``tracker.go:26-88``);
* pod sorter: priority desc, then smaller requested slice first
  (``util.go:34-71``);
* :class:`Planner` (``planner.go:67-207``): greedy node-by-node, per node
  update the geometry for the lacking slices, then try every pod through the
  scheduler framework's PreFilter + Filter; commit if any pod was added;
* :class:`Actuator` (``actuator.go:27-66``): no-op when the desired state
  equals the current one or is empty, else ``Partitioner.apply_partitioning``
  per node with a new plan id.
"""
from __future__ import annotations

import collections
import heapq
import logging
import time
from dataclasses import dataclass, field
from typing import Protocol

from ..kube import objects as ko
from ..resource.resource import Resource, compute_pod_request, request_memo
from ..scheduler.framework import CycleState, Framework, NodeInfo
from .state import NodePartitioning, PartitioningState

log = logging.getLogger("nos_amd.partitioning")


class PartitionableNode(Protocol):
    name: str
    node_info: NodeInfo

    def geometry(self) -> dict: ...

    def has_free_capacity(self) -> bool: ...

    def update_geometry_for(self, slices: dict) -> bool: ...

    def add_pod(self, pod: dict) -> None: ...

    def clone(self) -> "PartitionableNode": ...


class PartitionCalculator(Protocol):
    def get_partitioning(self, node: PartitionableNode) -> NodePartitioning: ...


class Partitioner(Protocol):
    def apply_partitioning(self, node: dict, plan_id: str, partitioning: NodePartitioning) -> None: ...


class SnapshotTaker(Protocol):
    def take_snapshot(self, cluster_state) -> "ClusterSnapshot": ...


class NodeInitializer(Protocol):
    def init_node_partitioning(self, node: dict) -> None: ...


def new_plan_id(clock=None) -> str:
    t = clock.now() if clock is not None else time.time()
    return str(int(t * 1000))


@dataclass
class PartitioningPlan:
    desired_state: PartitioningState
    id: str = ""

    def __post_init__(self):
        if not self.id:
            self.id = new_plan_id()


class ClusterSnapshot:
    def __init__(self, nodes: dict[str, PartitionableNode], partition_calculator: PartitionCalculator,
                 slice_calculator, slice_filter):
        self._data: dict[str, PartitionableNode] = dict(nodes)
        self._forked: dict[str, PartitionableNode] | None = None
        self._cow: set[str] = set()
        # cluster-wide (allocatable, requested) of _data / _forked, kept up to
        # date by add_pod and dropped by set_node: lacking_resources() is
        # called per pod per candidate node, and re-summing every node there
        # made planning O(nodes^2 x pods) (the reference's getLackingResources
        # re-sums too, snapshot.go:132-165)
        self._agg_data: tuple[Resource, Resource] | None = None
        self._agg_fork: tuple[Resource, Resource] | None = None
        self.partition_calculator = partition_calculator
        self.slice_calculator = slice_calculator
        self.slice_filter = slice_filter

    def _d(self) -> dict[str, PartitionableNode]:
        return self._forked if self._forked is not None else self._data

    def fork(self) -> None:
        if self._forked is not None:
            raise RuntimeError("snapshot already forked")
        # copy-on-write: nodes are cloned when first touched inside the fork
        # (get_node / add_pod); a deep copy of every node per candidate node
        # made planning O(nodes^2)
        self._forked = dict(self._data)
        self._cow: set[str] = set()
        self._agg_fork = None if self._agg_data is None else (self._agg_data[0].clone(), self._agg_data[1].clone())

    def commit(self) -> None:
        if self._forked is not None:
            self._data = self._forked
            self._forked = None
            self._agg_data, self._agg_fork = self._agg_fork, None

    def revert(self) -> None:
        self._forked = None
        self._agg_fork = None

    def _aggregates(self) -> tuple[Resource, Resource]:
        agg = self._agg_fork if self._forked is not None else self._agg_data
        if agg is None:
            alloc, requested = Resource(), Resource()
            for n in self.get_nodes().values():
                alloc.iadd(n.node_info.allocatable)
                requested.iadd(n.node_info.requested)
            agg = (alloc, requested)
            if self._forked is not None:
                self._agg_fork = agg
            else:
                self._agg_data = agg
        return agg

    def _invalidate(self) -> None:
        if self._forked is not None:
            self._agg_fork = None
        else:
            self._agg_data = None

    def clone(self) -> "ClusterSnapshot":
        c = ClusterSnapshot({k: v.clone() for k, v in self._data.items()}, self.partition_calculator,
                            self.slice_calculator, self.slice_filter)
        if self._forked is not None:
            c._forked = {k: v.clone() for k, v in self._forked.items()}
            c._cow = set(c._forked)
        return c

    def get_nodes(self) -> dict[str, PartitionableNode]:
        """Read-only view (mutate nodes through get_node / add_pod / set_node)."""
        return self._d()

    def _writable(self, name: str) -> PartitionableNode | None:
        d = self._d()
        n = d.get(name)
        if n is not None and self._forked is not None and name not in self._cow:
            n = n.clone()
            d[name] = n
            self._cow.add(name)
        return n

    def get_node(self, name: str) -> PartitionableNode | None:
        """The node; inside a fork, the fork's own copy (safe to mutate)."""
        return self._writable(name)

    def set_node(self, n: PartitionableNode) -> None:
        self._d()[n.name] = n
        if self._forked is not None:
            self._cow.add(n.name)
        self._invalidate()

    def get_candidate_nodes(self) -> list[str]:
        """Nodes with free capacity in name order (``snapshot.go:93-103``);
        nodes that expose a measured-throughput ``score()`` (cumask placement
        "measured", see partitioning/scoring.py) come first, best score first."""
        def key(n):
            sc = n.score() if hasattr(n, "score") else None
            return (sc is None, -(sc or 0.0), n.name)

        return [n.name for n in sorted((n for n in self._d().values() if n.has_free_capacity()), key=key)]

    def get_partitioning_state(self) -> PartitioningState:
        return PartitioningState({name: self.partition_calculator.get_partitioning(n)
                                  for name, n in self.get_nodes().items()})

    def lacking_resources(self, pod: dict) -> Resource:
        req = Resource.from_list(compute_pod_request(pod))
        alloc, requested = self._aggregates()
        available = alloc.subtract_non_negative(requested)
        diff = available - req
        res = Resource(min(diff.milli_cpu, 0), min(diff.memory, 0), min(diff.ephemeral_storage, 0),
                       min(diff.allowed_pod_number, 0))
        res.scalar = {k: v for k, v in diff.scalar.items() if v < 0}
        return res.abs()

    def get_lacking_slices(self, pod: dict) -> dict:
        return self.slice_filter.extract_slices(self.lacking_resources(pod).scalar)

    def add_pod(self, node_name: str, pod: dict) -> None:
        n = self._writable(node_name)
        if n is None:
            raise KeyError(f"could not find node {node_name} in cluster snapshot")
        before = n.node_info.requested.clone()
        alloc_before = n.node_info.allocatable.clone()
        n.add_pod(pod)
        agg = self._agg_fork if self._forked is not None else self._agg_data
        if agg is not None:
            agg[1].isub(before)
            agg[1].iadd(n.node_info.requested)
            agg[0].isub(alloc_before)
            agg[0].iadd(n.node_info.allocatable)


class SliceTracker:
    def __init__(self, snapshot: ClusterSnapshot, calculator, pods: list[dict]):
        self.calculator = calculator
        self.requested: dict = {}
        self.lacking: dict = {}
        self.lookup: dict[str, dict] = {}
        for pod in pods:
            k = ko.key(pod)
            per = self.lookup.setdefault(k, {})
            for s, n in snapshot.get_lacking_slices(pod).items():
                self.lacking[s] = self.lacking.get(s, 0) + n
                per[s] = per.get(s, 0) + n
            for s, n in calculator.get_requested_slices(pod).items():
                self.requested[s] = self.requested.get(s, 0) + n

    def get_lacking_slices(self) -> dict:
        return self.lacking

    def get_requested_slices(self) -> dict:
        return self.requested

    def remove(self, pod: dict) -> None:
        for s, n in self.calculator.get_requested_slices(pod).items():
            self.requested[s] = self.requested.get(s, 0) - n
            if self.requested[s] <= 0:
                del self.requested[s]
        per = self.lookup.get(ko.key(pod))
        if per:
            for s, n in list(per.items()):
                self.lacking[s] = self.lacking.get(s, 0) - n
                per[s] -= n
                if per[s] <= 0:
                    del per[s]
                if self.lacking[s] <= 0:
                    del self.lacking[s]


def sort_pods(pods: list[dict], slice_calculator) -> list[dict]:
    """Priority desc; equal priority: the pod requesting the smaller slice
    first (``util.go:34-71``).  Requested slices are computed once per pod."""
    import functools

    keyed = [(ko.pod_priority(p), slice_calculator.get_requested_slices(p), p) for p in pods]

    def cmp(a, b):
        pa, pb = a[0], b[0]
        if pa != pb:
            return -1 if pa > pb else 1
        ra, rb = a[1], b[1]
        if not ra or not rb:
            return 0
        sa, sb = min(ra, key=str), min(rb, key=str)
        if sa.smaller_than(sb):
            return -1
        if sb.smaller_than(sa):
            return 1
        return 0

    return [k[2] for k in sorted(keyed, key=functools.cmp_to_key(cmp))]


def is_node_initialized(node: dict) -> bool:
    from ..gpu.core import get_count, parse_node_annotations

    try:
        count = get_count(node)
    except Exception:
        return False
    _, spec = parse_node_annotations(node)
    return count == len({a.index for a in spec})


class Planner:
    def __init__(self, partition_calculator: PartitionCalculator, slice_calculator, framework: Framework):
        self.partition_calculator = partition_calculator
        self.slice_calculator = slice_calculator
        self.framework = framework
        self.last_stats: dict = {}

    def plan(self, snapshot: ClusterSnapshot, candidate_pods: list[dict]) -> PartitioningPlan:
        with request_memo():
            return self._plan(snapshot, candidate_pods)

    def _plan(self, snapshot: ClusterSnapshot, candidate_pods: list[dict]) -> PartitioningPlan:
        t0 = time.perf_counter()
        state = snapshot.get_partitioning_state()
        tracker = SliceTracker(snapshot, self.slice_calculator, candidate_pods)
        placed = 0
        if not tracker.get_lacking_slices():
            self.last_stats = {"placed": 0, "seconds": time.perf_counter() - t0, "lacking": 0}
            return PartitioningPlan(state)
        pods = sort_pods(candidate_pods, self.slice_calculator)
        # pods grouped by (namespace, request) signature, each group an index
        # queue in sort order.  Within one node's pass capacity only shrinks
        # (the geometry is updated once, before the pass), so once a pod of a
        # group fails on the node every later pod of that group would too:
        # the pass walks the groups' heads in sort order (a heap) and drops a
        # group at its first failure -- O((placed + groups) log groups) per
        # node instead of re-simulating every pending pod on every node.
        groups: dict[tuple, collections.deque] = {}
        for i, pod in enumerate(pods):
            sig = (ko.namespace(pod), frozenset(compute_pod_request(pod).items()))
            groups.setdefault(sig, collections.deque()).append(i)
        for name in snapshot.get_candidate_nodes():
            if not tracker.get_lacking_slices() or not groups:
                break
            snapshot.fork()
            n = snapshot.get_node(name)  # the forked copy (fixes the pre-fork mutation gotcha)
            if n.update_geometry_for(dict(tracker.get_lacking_slices())):
                snapshot.set_node(n)
            added: list[tuple[tuple, int]] = []
            heap = [(q[0], k) for k, q in enumerate(groups.values())]
            keys = list(groups)
            heapq.heapify(heap)
            taken: dict[tuple, int] = {}
            while heap:
                i, k = heapq.heappop(heap)
                sig = keys[k]
                if not self._try_add_pod(pods[i], name, snapshot):
                    continue  # the group is done on this node
                state[name] = self.partition_calculator.get_partitioning(snapshot.get_node(name))
                tracker.remove(pods[i])
                added.append((sig, i))
                t = taken.get(sig, 0) + 1
                taken[sig] = t
                q = groups[sig]
                if t < len(q):
                    heapq.heappush(heap, (q[t], k))
            if added:
                snapshot.commit()
                for sig, t in taken.items():
                    q = groups[sig]
                    for _ in range(t):
                        q.popleft()
                    if not q:
                        del groups[sig]
                placed += len(added)
            else:
                snapshot.revert()
        self.last_stats = {"placed": placed, "seconds": time.perf_counter() - t0,
                           "lacking": sum(tracker.get_lacking_slices().values())}
        return PartitioningPlan(state)

    def _try_add_pod(self, pod: dict, node_name: str, snapshot: ClusterSnapshot) -> bool:
        if snapshot.get_lacking_slices(pod):
            return False
        n = snapshot.get_node(node_name)
        if n is None:
            return False
        if not self.can_schedule_pod(pod, n.node_info):
            return False
        try:
            snapshot.add_pod(node_name, pod)
        except Exception:
            return False
        return True

    def can_schedule_pod(self, pod: dict, node_info: NodeInfo) -> bool:
        state = CycleState()
        _, s = self.framework.run_pre_filter_plugins(state, pod)
        if not s.is_success():
            return False
        return self.framework.run_filter_plugins(state, pod, node_info).is_success()


class Actuator:
    def __init__(self, api, partitioner: Partitioner):
        self.api = api
        self.partitioner = partitioner

    def apply(self, snapshot: ClusterSnapshot, plan: PartitioningPlan) -> bool:
        if snapshot.get_partitioning_state().equal(plan.desired_state):
            log.info("current and desired partitioning states are equal, nothing to do")
            return False
        if plan.desired_state.is_empty():
            log.info("desired partitioning state is empty, nothing to do")
            return False
        for node_name, np_ in plan.desired_state.items():
            node = self.api.get("Node", node_name)
            self.partitioner.apply_partitioning(node, plan.id, np_)
        return True


__all__ = ["ClusterSnapshot", "SliceTracker", "Planner", "Actuator", "PartitioningPlan", "sort_pods",
           "is_node_initialized", "new_plan_id", "field"]
