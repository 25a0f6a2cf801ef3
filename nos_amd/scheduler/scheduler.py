"""The scheduler process: cache, scheduling queue and the scheduling cycle.

Equivalent of ``cmd/scheduler`` (kube-scheduler + the CapacityScheduling
plugin, ``cmd/scheduler/scheduler.go:43-59``) running against the in-process
API server:

* a cache of nodes and assigned pods (plus assumed pods between Reserve and
  Bind) fed by watches;
* a priority queue (PrioritySort) with an unschedulable set that is flushed
  back to the active queue on cluster events (pod delete, node add/update,
  ElasticQuota changes -- the plugin's EventsToRegister) and periodically;
* ``schedule_one``: snapshot -> PreFilter -> Filter (with nominated pods) on
  every node -> Score -> Reserve -> Permit -> Bind; on failure PostFilter
  (preemption), nomination (``status.nominatedNodeName``) and the
  ``PodScheduled=False/Unschedulable`` condition that the gpupartitioner
  watches for (``pkg/util/pod/pod.go:41-48``).
"""
from __future__ import annotations

import heapq
import itertools
import logging
import threading
import time
from typing import Any

from ..kube import objects as ko
from .config import Profile, SchedulerConfiguration, build_framework
from .framework import CycleState, Framework, NodeInfo, PodInfo, PodNominator, Snapshot, Status

log = logging.getLogger("nos_amd.scheduler")


class SchedulerCache:
    """Node infos maintained incrementally from informer events (the
    kube-scheduler cache); :meth:`snapshot` clones them per cycle without
    recomputing pod requests."""

    def __init__(self):
        self._lock = threading.RLock()
        self.nodes: dict[str, dict] = {}
        self.pods: dict[str, dict] = {}      # key -> assigned pod
        self.assumed: dict[str, str] = {}    # key -> node
        self._infos: dict[str, NodeInfo] = {}
        self._pod_node: dict[str, str] = {}  # key -> node the pod is accounted on

    def _info(self, node_name: str) -> NodeInfo:
        ni = self._infos.get(node_name)
        if ni is None:
            ni = NodeInfo(self.nodes.get(node_name))
            self._infos[node_name] = ni
        return ni

    def _unaccount(self, k: str) -> None:
        nn = self._pod_node.pop(k, None)
        old = self.pods.get(k)
        if nn is not None and old is not None and nn in self._infos:
            try:
                self._infos[nn].remove_pod(old)
            except KeyError:
                pass

    def _account(self, k: str, p: dict) -> None:
        nn = ko.pod_node(p)
        self.pods[k] = p
        self._pod_node[k] = nn
        self._info(nn).add_pod(p)

    def update_node(self, n: dict) -> None:
        with self._lock:
            name = ko.name(n)
            self.nodes[name] = n
            self._info(name).set_node(n)

    def delete_node(self, n: dict) -> None:
        with self._lock:
            name = ko.name(n)
            self.nodes.pop(name, None)
            ni = self._infos.get(name)
            if ni is not None and not ni.pods:
                del self._infos[name]
            elif ni is not None:
                ni._node = None

    def update_pod(self, p: dict) -> None:
        with self._lock:
            k = ko.key(p)
            self._unaccount(k)
            self.pods.pop(k, None)
            self.assumed.pop(k, None)
            if ko.pod_node(p) and not ko.is_terminated(p):
                self._account(k, p)

    def delete_pod(self, p: dict) -> None:
        with self._lock:
            k = ko.key(p)
            self._unaccount(k)
            self.pods.pop(k, None)
            self.assumed.pop(k, None)

    def assume(self, p: dict, node: str) -> None:
        with self._lock:
            k = ko.key(p)
            q = dict(p)
            q["spec"] = dict(p.get("spec") or {})
            q["spec"]["nodeName"] = node
            self._unaccount(k)
            self._account(k, q)
            self.assumed[k] = node

    def forget(self, p: dict) -> None:
        with self._lock:
            k = ko.key(p)
            if k in self.assumed:
                self.assumed.pop(k)
                self._unaccount(k)
                self.pods.pop(k, None)

    def snapshot(self) -> Snapshot:
        with self._lock:
            return Snapshot(ni.clone() for name, ni in self._infos.items() if name in self.nodes)


class SchedulingQueue:
    def __init__(self, clock, backoff: float = 1.0):
        self.clock = clock
        self._lock = threading.RLock()
        self._heap: list[tuple[int, float, int, str]] = []
        self._pods: dict[str, dict] = {}
        self._unschedulable: dict[str, tuple[dict, float]] = {}
        self._seq = itertools.count()
        self.backoff = backoff

    def add(self, pod: dict) -> None:
        with self._lock:
            k = ko.key(pod)
            self._unschedulable.pop(k, None)
            self._pods[k] = pod
            heapq.heappush(self._heap, (-ko.pod_priority(pod), ko.creation_time(pod), next(self._seq), k))

    def update(self, pod: dict) -> None:
        with self._lock:
            k = ko.key(pod)
            if k in self._pods:
                self._pods[k] = pod
            elif k in self._unschedulable:
                self._unschedulable[k] = (pod, self._unschedulable[k][1])
            else:
                self.add(pod)

    def delete(self, pod: dict) -> None:
        with self._lock:
            k = ko.key(pod)
            self._pods.pop(k, None)
            self._unschedulable.pop(k, None)

    def pop(self) -> dict | None:
        with self._lock:
            while self._heap:
                _, _, _, k = heapq.heappop(self._heap)
                p = self._pods.pop(k, None)
                if p is not None:
                    return p
            return None

    def add_unschedulable(self, pod: dict) -> None:
        with self._lock:
            self._unschedulable[ko.key(pod)] = (pod, self.clock.monotonic())

    def move_all_to_active(self, respect_backoff: bool = True) -> int:
        with self._lock:
            now = self.clock.monotonic()
            moved = 0
            for k, (p, t) in list(self._unschedulable.items()):
                if respect_backoff and now - t < self.backoff:
                    continue
                self._unschedulable.pop(k)
                self.add(p)
                moved += 1
            return moved

    def __len__(self) -> int:
        with self._lock:
            return len(self._pods)

    def unschedulable_count(self) -> int:
        with self._lock:
            return len(self._unschedulable)


class Scheduler:
    def __init__(self, api, config: SchedulerConfiguration | None = None, clock=None,
                 flush_unschedulable_s: float = 30.0):
        from .config import nos_scheduler_config

        self.api = api
        self.clock = clock or api.clock
        self.config = config or nos_scheduler_config()
        self.cache = SchedulerCache()
        self.nominator = PodNominator()
        self.queue = SchedulingQueue(self.clock)
        self.frameworks: dict[str, Framework] = {}
        for prof in self.config.profiles:
            self.frameworks[prof.scheduler_name] = build_framework(prof, api=api, nominator=self.nominator)
        self._watches: list = []
        self._last_flush = self.clock.monotonic()
        self.flush_interval = flush_unschedulable_s
        self.stats = {"attempts": 0, "scheduled": 0, "unschedulable": 0, "errors": 0, "preemptions": 0}
        self._lock = threading.RLock()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    # ------------------------------------------------------------ informers
    def start_informers(self) -> None:
        self._watches.append(self.api.watch("Node", callback=self._node_event))
        self._watches.append(self.api.watch("Pod", callback=self._pod_event))
        for kind in ("ElasticQuota", "CompositeElasticQuota"):
            try:
                self._watches.append(self.api.watch(kind, callback=lambda ev: self.queue.move_all_to_active(False)))
            except Exception:
                pass

    def _responsible(self, pod: dict) -> bool:
        return (pod.get("spec") or {}).get("schedulerName", "default-scheduler") in self.frameworks

    def _node_event(self, ev) -> None:
        if ev.type == "DELETED":
            self.cache.delete_node(ev.object)
        else:
            self.cache.update_node(ev.object)
            self.queue.move_all_to_active(False)

    def _pod_event(self, ev) -> None:
        p = ev.object
        if ev.type == "DELETED":
            self.cache.delete_pod(p)
            self.queue.delete(p)
            self.nominator.delete_nominated_pod_if_exists(p)
            self.queue.move_all_to_active(False)
            return
        if ko.pod_node(p):
            self.cache.update_pod(p)
            self.queue.delete(p)
            self.nominator.delete_nominated_pod_if_exists(p)
            if ko.is_terminated(p):
                self.queue.move_all_to_active(False)
        elif self._responsible(p) and not ko.is_terminated(p):
            if ev.type == "ADDED":
                self.queue.add(p)
            else:
                self.queue.update(p)

    # ------------------------------------------------------------ cycle
    def _framework_for(self, pod: dict) -> Framework | None:
        return self.frameworks.get((pod.get("spec") or {}).get("schedulerName", "default-scheduler"))

    def schedule_one(self) -> bool:
        """One scheduling cycle.  An exception inside the cycle (API error,
        plugin bug) never loses the pod: it goes back to the queue with
        backoff and the loop carries on."""
        pod = self.queue.pop()
        if pod is None:
            return False
        cycle: dict[str, Any] = {}
        try:
            return self._schedule_pod(pod, cycle)
        except Exception:
            log.exception("scheduling cycle of %s failed; requeued with backoff", ko.key(pod))
            self.stats["cycle_errors"] = self.stats.get("cycle_errors", 0) + 1
            reserved = cycle.get("reserved")
            if reserved is not None:  # Reserve succeeded: give back what it took (e.g. quota "used")
                fw, state, rpod, node = reserved
                try:
                    fw.run_reserve_plugins_unreserve(state, rpod, node)
                except Exception:
                    log.exception("unreserve of %s after a failed cycle failed", ko.key(pod))
            try:
                self.cache.forget(pod)
            except Exception:
                pass
            self.queue.add_unschedulable(pod)
            return True

    def _schedule_pod(self, pod: dict, cycle: dict | None = None) -> bool:
        cycle = {} if cycle is None else cycle
        fw = self._framework_for(pod)
        if fw is None:
            return True
        cur = self.api.try_get("Pod", ko.name(pod), ko.namespace(pod))
        if cur is None or ko.pod_node(cur):
            return True
        pod = cur
        self.stats["attempts"] += 1
        snap = self.cache.snapshot()
        fw.set_snapshot(snap)
        state = CycleState()
        _, s = fw.run_pre_filter_plugins(state, pod)
        if not s.is_success():
            self._unschedulable(fw, state, pod, s, {n.name: s for n in snap.list()})
            return True
        statuses: dict[str, Status] = {}
        feasible: list[NodeInfo] = []
        for ni in snap.list():
            st = fw.run_filter_plugins_with_nominated_pods(state, pod, ni)
            if st.is_success():
                feasible.append(ni)
            else:
                statuses[ni.name] = st
        if not feasible:
            self._unschedulable(fw, state, pod, Status("Unschedulable", ["no feasible node"]), statuses)
            return True
        scores = fw.run_score_plugins(state, pod, feasible) if len(feasible) > 1 else {feasible[0].name: 0}
        node = max(feasible, key=lambda n: (scores.get(n.name, 0), -len(n.pods), n.name)).name
        self.cache.assume(pod, node)
        s = fw.run_reserve_plugins_reserve(state, pod, node)
        if not s.is_success():
            fw.run_reserve_plugins_unreserve(state, pod, node)
            self.cache.forget(pod)
            self._unschedulable(fw, state, pod, s, {})
            return True
        cycle["reserved"] = (fw, state, pod, node)
        s = fw.run_permit_plugins(state, pod, node)
        if s.is_success():
            s = fw.run_bind_plugins(state, pod, node)
        if not s.is_success():
            cycle.pop("reserved", None)
            fw.run_reserve_plugins_unreserve(state, pod, node)
            self.cache.forget(pod)
            self.stats["errors"] += 1
            self.queue.add_unschedulable(pod)
            return True
        cycle.pop("reserved", None)  # bound: the reservation is now the pod's real usage
        fw.run_post_bind_plugins(state, pod, node)
        self.nominator.delete_nominated_pod_if_exists(pod)
        self.stats["scheduled"] += 1
        return True

    def _unschedulable(self, fw: Framework, state: CycleState, pod: dict, status: Status,
                       statuses: dict[str, Status]) -> None:
        self.stats["unschedulable"] += 1
        nominated = ""
        if fw.plugins["post_filter"]:
            res, ps = fw.run_post_filter_plugins(state, pod, statuses)
            if ps.is_success() and res is not None and res.nominated_node_name:
                nominated = res.nominated_node_name
                self.stats["preemptions"] += 1
        patch: dict[str, Any] = {"status": {"conditions": _merge_cond(pod, status)}}
        if nominated:
            patch["status"]["nominatedNodeName"] = nominated
            p2 = dict(pod)
            p2["status"] = dict(pod.get("status") or {}, nominatedNodeName=nominated)
            self.nominator.add_nominated_pod(p2, nominated)
        try:
            self.api.patch("Pod", ko.name(pod), patch, ko.namespace(pod), subresource="status")
        except Exception:
            pass
        self.queue.add_unschedulable(pod)

    def resync(self) -> int:
        """Informer resync: reconcile the cache and the queue with a fresh
        list (covers watch events that were lost)."""
        try:
            nodes = self.api.list("Node")
            pods = self.api.list("Pod")
        except Exception as e:
            log.debug("scheduler resync failed: %s", e)
            return 0
        with self._lock:
            for n in nodes:
                self.cache.update_node(n)
            for name in set(self.cache.nodes) - {ko.name(n) for n in nodes}:
                self.cache.delete_node({"metadata": {"name": name}})
            live = set()
            queued = 0
            for p in pods:
                live.add(ko.key(p))
                if ko.pod_node(p):
                    if ko.key(p) not in self.cache.assumed:
                        self.cache.update_pod(p)
                elif self._responsible(p) and not ko.is_terminated(p):
                    self.queue.update(p)
                    queued += 1
            for k in [k for k in self.cache.pods if k not in live]:
                self.cache.delete_pod(self.cache.pods[k])
            return queued

    def run_until_idle(self, max_cycles: int = 100000) -> int:
        n = 0
        while n < max_cycles and self.schedule_one():
            n += 1
        now = self.clock.monotonic()
        if now - self._last_flush >= self.flush_interval:
            self._last_flush = now
            self.resync()
            if self.queue.move_all_to_active() or len(self.queue):
                n += self.run_until_idle(max_cycles - n)
        return n

    def retry_unschedulable(self) -> int:
        self.queue.move_all_to_active(False)
        return self.run_until_idle()

    # ------------------------------------------------------------ threaded mode
    def start(self) -> None:
        if not self._watches:
            self.start_informers()

        def loop():
            while not self._stop.is_set():
                self.heartbeat = time.monotonic()
                try:
                    if self.schedule_one():
                        continue
                    self._stop.wait(0.02)
                    if self.clock.monotonic() - self._last_flush >= self.flush_interval:
                        self._last_flush = self.clock.monotonic()
                        self.resync()
                        self.queue.move_all_to_active()
                except Exception:  # resync against an unreachable API server etc.: back off, keep going
                    log.exception("scheduler loop error")
                    self.stats["loop_errors"] = self.stats.get("loop_errors", 0) + 1
                    self._stop.wait(1.0)

        self.heartbeat = time.monotonic()
        self._thread = threading.Thread(target=loop, daemon=True, name="scheduler")
        self._thread.start()

    def healthy(self, max_stall_s: float = 30.0) -> bool:
        """Liveness: the scheduling thread runs and completed a loop recently."""
        t = self._thread
        return bool(t and t.is_alive() and not self._stop.is_set()
                    and time.monotonic() - getattr(self, "heartbeat", 0.0) < max_stall_s)

    def stop(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=2)
        for w in self._watches:
            w.stop()
        for fw in self.frameworks.values():
            for p in getattr(fw, "instances", {}).values():
                if hasattr(p, "stop"):
                    p.stop()


def _merge_cond(pod: dict, status: Status) -> list[dict]:
    conds = [c for c in ko.pod_conditions(pod) if c.get("type") != "PodScheduled"]
    conds.append({"type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                  "message": status.message() or status.code, "lastTransitionTime": ko.now_rfc3339()})
    return conds


__all__ = ["Scheduler", "SchedulerCache", "SchedulingQueue", "Profile", "PodInfo"]
