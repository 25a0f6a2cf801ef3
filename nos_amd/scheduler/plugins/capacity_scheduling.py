"""``CapacityScheduling`` -- the elastic-quota scheduler plugin.

API-compatible with the reference plugin (name ``CapacityScheduling``, args
``CapacitySchedulingArgs``; ``pkg/scheduler/plugins/capacityscheduling/
capacity_scheduling.go:50-900``):

* PreFilter: snapshot the quota infos, compute the pod request (with
  ``nos.nebuly.com/gpu-memory``), add the requests of nominated pods that are
  subject to the same quota and at least as important (and of pods in other
  quotas that are not over their min), reject when ``used + req > max``
  (only if max is set) or when ``sum(used) + req > sum(min)``;
* PreFilterExtensions AddPod / RemovePod on the cycle's snapshot;
* PostFilter: preemption with over-quota fair-share victim selection using
  guaranteed over-quotas, PDB-aware reprieve;
* Reserve / Unreserve adjust ``used`` under the plugin lock;
* EventsToRegister: pod delete and every ElasticQuota event;
* an informer on ElasticQuota / CompositeElasticQuota (CEQ wins over an EQ
  in the same namespace) and handlers for assigned pods.

Deliberate fix vs. the reference: a victim that still does not fit is
appended to the victim list once (the reference's reprieve could remove and
append the same pod twice, ``:634-673``).
"""
from __future__ import annotations

import logging
import threading

from ...api import constants as C
from ...api import v1alpha1
from ...gpu.memory import ResourceCalculator
from ...kube import objects as ko
from ...resource.resource import Resource
from ..framework import (ERROR, UNRESOLVABLE, UNSCHEDULABLE, CycleState, NodeInfo, Plugin, PodInfo, Status,
                         as_status)
from ..preemption import Evaluator, filter_pods_with_pdb_violation, more_important_pod
from .elasticquotainfo import ElasticQuotaInfo, ElasticQuotaInfos

log = logging.getLogger("nos_amd.scheduler.capacityscheduling")

NAME = "CapacityScheduling"
PRE_FILTER_STATE_KEY = "PreFilter" + NAME
ELASTIC_QUOTA_SNAPSHOT_KEY = "ElasticQuotaSnapshot"


def is_over_quota(pod: dict) -> bool:
    return ko.labels(pod).get(C.LABEL_CAPACITY_INFO) == C.CAPACITY_OVER_QUOTA


class PreFilterState:
    def __init__(self, pod_req: Resource, in_eq: Resource | None = None, total: Resource | None = None):
        self.pod_req = pod_req
        self.nominated_pods_req_in_eq_with_pod_req = in_eq or Resource()
        self.nominated_pods_req_with_pod_req = total or Resource()

    def clone(self) -> "PreFilterState":
        return self  # read-only after PreFilter (as upstream)


class ElasticQuotaSnapshotState:
    def __init__(self, infos: ElasticQuotaInfos):
        self.elastic_quota_infos = infos

    def clone(self) -> "ElasticQuotaSnapshotState":
        return ElasticQuotaSnapshotState(self.elastic_quota_infos.clone())


def info_from_eq(obj: dict, calc) -> ElasticQuotaInfo:
    spec = obj.get("spec") or {}
    ns = set(v1alpha1.namespaces(obj)) if obj.get("kind") == v1alpha1.KIND_CEQ else {ko.namespace(obj)}
    return ElasticQuotaInfo(ko.name(obj), ko.namespace(obj), ns, Resource.from_list(spec.get("min")),
                            Resource.from_list(spec.get("max")), Resource(), spec.get("max") is not None, calc)


class ElasticQuotaInfoInformer:
    """Watches EQ + CEQ and keeps ElasticQuotaInfo objects; EQ events are
    dropped when a CEQ covers the namespace (``informer.go:225-260``)."""

    def __init__(self, api, calculator, on_add, on_update, on_delete):
        self.api, self.calc = api, calculator
        self.on_add, self.on_update, self.on_delete = on_add, on_update, on_delete
        self._eq: dict[str, dict] = {}
        self._ceq: dict[str, dict] = {}
        self._watches = []

    def start(self) -> None:
        self._watches.append(self.api.watch(v1alpha1.KIND_CEQ, callback=self._ceq_event))
        self._watches.append(self.api.watch(v1alpha1.KIND_EQ, callback=self._eq_event))

    def stop(self) -> None:
        for w in self._watches:
            w.stop()

    def _covered_by_ceq(self, ns: str) -> bool:
        return any(ns in v1alpha1.namespaces(c) for c in self._ceq.values())

    def _eq_event(self, ev) -> None:
        obj, k = ev.object, ko.key(ev.object)
        if ev.type == "DELETED":
            old = self._eq.pop(k, None)
            if old is not None and not self._covered_by_ceq(ko.namespace(old)):
                self.on_delete(info_from_eq(old, self.calc))
            return
        old = self._eq.get(k)
        self._eq[k] = obj
        if self._covered_by_ceq(ko.namespace(obj)):
            return
        if old is None:
            self.on_add(info_from_eq(obj, self.calc))
        else:
            self.on_update(info_from_eq(old, self.calc), info_from_eq(obj, self.calc))

    def _ceq_event(self, ev) -> None:
        obj, k = ev.object, ko.key(ev.object)
        if ev.type == "DELETED":
            old = self._ceq.pop(k, None)
            if old is not None:
                self.on_delete(info_from_eq(old, self.calc))
                for e in self._eq.values():  # namespaces released by the CEQ fall back to their EQ
                    if ko.namespace(e) in v1alpha1.namespaces(old) and not self._covered_by_ceq(ko.namespace(e)):
                        self.on_add(info_from_eq(e, self.calc))
            return
        old = self._ceq.get(k)
        self._ceq[k] = obj
        if old is None:
            self.on_add(info_from_eq(obj, self.calc))
        else:
            self.on_update(info_from_eq(old, self.calc), info_from_eq(obj, self.calc))

    def get_associated_composite_elastic_quota(self, namespace: str) -> ElasticQuotaInfo | None:
        for c in self._ceq.values():
            if namespace in v1alpha1.namespaces(c):
                return info_from_eq(c, self.calc)
        return None

    def get_associated_elastic_quota(self, namespace: str) -> ElasticQuotaInfo | None:
        for e in self._eq.values():
            if ko.namespace(e) == namespace:
                return info_from_eq(e, self.calc)
        return None


class CapacityScheduling(Plugin):
    name = NAME

    def __init__(self, args: dict | None = None, handle=None, api=None, start_informers: bool = True):
        args = args or {}
        mem = args.get("amdGpuResourceMemoryGB", args.get("nvidiaGpuResourceMemoryGB"))
        if mem is None:  # the reference's defaulter is empty (default 0); default to one MI355X
            mem = C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB
        self.calculator = ResourceCalculator(int(mem))
        self.fh = handle
        self._lock = threading.RLock()
        self.elastic_quota_infos = ElasticQuotaInfos()
        self.preemption_attempts = 0
        self.api = api or getattr(handle, "api", None)
        self.informer: ElasticQuotaInfoInformer | None = None
        self._pod_watch = None
        if self.api is not None and start_informers:
            self.informer = ElasticQuotaInfoInformer(self.api, self.calculator, self.add_elastic_quota_info,
                                                     self.update_elastic_quota_info,
                                                     self.delete_elastic_quota_info)
            self.informer.start()
            self._pod_watch = self.api.watch("Pod", callback=self._pod_event)

    def set_handle(self, h) -> None:
        self.fh = h
        if self.api is None:
            self.api = getattr(h, "api", None)

    def events_to_register(self):
        return [("Pod", "Delete"), (f"elasticquotas.v1alpha1.{C.GROUP}", "All")]

    # ------------------------------------------------------------ informer handlers
    def add_elastic_quota_info(self, info: ElasticQuotaInfo) -> None:
        with self._lock:
            self.elastic_quota_infos.add(info)
            self._resync_pods(info)

    def update_elastic_quota_info(self, old: ElasticQuotaInfo, new: ElasticQuotaInfo) -> None:
        with self._lock:
            self.elastic_quota_infos.update(old, new)
            self._resync_pods(new)

    def delete_elastic_quota_info(self, info: ElasticQuotaInfo) -> None:
        with self._lock:
            self.elastic_quota_infos.delete(info)

    def _resync_pods(self, info: ElasticQuotaInfo) -> None:
        """Account already-assigned, non-terminated pods of the quota's namespaces
        (the reference relies on the pod informer replaying adds after the EQ sync)."""
        if self.api is None:
            return
        for ns in info.namespaces:
            for p in self.api.list("Pod", ns):
                if ko.pod_node(p) and ko.pod_phase(p) in (ko.RUNNING, ko.PENDING, ""):
                    info.add_pod_if_not_present(p)

    def _pod_event(self, ev) -> None:
        pod = ev.object
        if not ko.pod_node(pod) and not (ev.old is not None and ko.pod_node(ev.old)):
            return
        if ev.type == "ADDED":
            self.add_pod_event(pod)
        elif ev.type == "MODIFIED":
            if ev.old is not None and not ko.pod_node(ev.old) and ko.pod_node(pod):
                self.add_pod_event(pod)  # bound: add (idempotent with Reserve)
            self.update_pod_event(ev.old or pod, pod)
        elif ev.type == "DELETED":
            self.delete_pod_event(pod)

    def get_elastic_quota_info_for_pod(self, pod: dict) -> ElasticQuotaInfo | None:
        info = self.elastic_quota_infos.get(ko.namespace(pod))
        if info is not None:
            return info
        if self.informer is None:
            return None
        return (self.informer.get_associated_composite_elastic_quota(ko.namespace(pod))
                or self.informer.get_associated_elastic_quota(ko.namespace(pod)))

    def add_pod_event(self, pod: dict) -> None:
        with self._lock:
            if ko.is_terminated(pod):
                return
            info = self.get_elastic_quota_info_for_pod(pod)
            if info is not None:
                info.add_pod_if_not_present(pod)

    def update_pod_event(self, old: dict, new: dict) -> None:
        if ko.pod_phase(old) in (ko.SUCCEEDED, ko.FAILED):
            return
        if ko.pod_phase(new) not in (ko.RUNNING, ko.PENDING):
            with self._lock:
                info = self.elastic_quota_infos.get(ko.namespace(new))
                if info is not None:
                    info.delete_pod_if_present(new)

    def delete_pod_event(self, pod: dict) -> None:
        with self._lock:
            info = self.elastic_quota_infos.get(ko.namespace(pod))
            if info is not None:
                info.delete_pod_if_present(pod)

    def snapshot_elastic_quota(self) -> ElasticQuotaSnapshotState:
        with self._lock:
            return ElasticQuotaSnapshotState(self.elastic_quota_infos.clone())

    # ------------------------------------------------------------ PreFilter
    def pre_filter(self, state: CycleState, pod: dict):
        snap = self.snapshot_elastic_quota()
        pod_req = Resource.from_list(self.calculator.compute_pod_request(pod))
        state.write(ELASTIC_QUOTA_SNAPSHOT_KEY, snap)
        infos = snap.elastic_quota_infos
        eq = infos.get(ko.namespace(pod))
        if eq is None:
            state.write(PRE_FILTER_STATE_KEY, PreFilterState(pod_req))
            return None, Status.ok()
        in_eq = Resource()
        total = Resource()
        prio = ko.pod_priority(pod)
        for ni in self.fh.snapshot_shared_lister().list():
            for npi in self.fh.nominated_pods_for_node(ni.name):
                p = npi.pod
                if ko.uid(p) and ko.uid(p) == ko.uid(pod):
                    continue
                ns = ko.namespace(p)
                info = self.elastic_quota_infos.get(ns)
                if info is None:
                    continue
                preq = Resource.from_list(self.calculator.compute_pod_request(p))
                if ns == ko.namespace(pod) and ko.pod_priority(p) >= prio:
                    in_eq.iadd(preq)
                    total.iadd(preq)
                elif ns != ko.namespace(pod) and not info.used_over_min():
                    total.iadd(preq)
        in_eq.iadd(pod_req)
        total.iadd(pod_req)
        state.write(PRE_FILTER_STATE_KEY, PreFilterState(pod_req, in_eq, total))
        if eq.used_over_max_with(in_eq):
            return None, Status(UNSCHEDULABLE, [
                f"Pod {ko.namespace(pod)}/{ko.name(pod)} is rejected in PreFilter because quota "
                f"{eq.resource_namespace}/{eq.resource_name} is more than Max"])
        if infos.aggregated_used_over_min_with(total):
            return None, Status(UNSCHEDULABLE, [
                f"Pod {ko.namespace(pod)}/{ko.name(pod)} is rejected in PreFilter because total quota used "
                "is more than min"])
        return None, Status.ok()

    def add_pod(self, state: CycleState, pod: dict, to_add: PodInfo, node_info: NodeInfo) -> Status:
        try:
            snap: ElasticQuotaSnapshotState = state.read(ELASTIC_QUOTA_SNAPSHOT_KEY)
        except KeyError as e:
            return Status(ERROR, [str(e)])
        info = snap.elastic_quota_infos.get(ko.namespace(to_add.pod))
        if info is not None:
            info.add_pod_if_not_present(to_add.pod)
        return Status.ok()

    def remove_pod(self, state: CycleState, pod: dict, to_remove: PodInfo, node_info: NodeInfo) -> Status:
        try:
            snap: ElasticQuotaSnapshotState = state.read(ELASTIC_QUOTA_SNAPSHOT_KEY)
        except KeyError as e:
            return Status(ERROR, [str(e)])
        info = snap.elastic_quota_infos.get(ko.namespace(to_remove.pod))
        if info is not None:
            info.delete_pod_if_present(to_remove.pod)
        return Status.ok()

    # ------------------------------------------------------------ PostFilter
    def post_filter(self, state: CycleState, pod: dict, statuses):
        try:
            ev = Evaluator(self.name, self.fh, state, CapacityPreemptor(self.fh, state))
            return ev.preempt(pod, statuses)
        finally:
            self.preemption_attempts += 1

    # ------------------------------------------------------------ Reserve
    def reserve(self, state: CycleState, pod: dict, node_name: str) -> Status:
        with self._lock:
            info = self.elastic_quota_infos.get(ko.namespace(pod))
            if info is not None:
                try:
                    info.add_pod_if_not_present(pod)
                except Exception as e:
                    return as_status(e)
        return Status.ok()

    def unreserve(self, state: CycleState, pod: dict, node_name: str) -> None:
        with self._lock:
            info = self.elastic_quota_infos.get(ko.namespace(pod))
            if info is not None:
                info.delete_pod_if_present(pod)

    def stop(self) -> None:
        if self.informer:
            self.informer.stop()
        if self._pod_watch:
            self._pod_watch.stop()


class CapacityPreemptor:
    """The plugin's preemption interface (``capacity_scheduling.go:371-675``)."""

    def __init__(self, fh, state: CycleState):
        self.fh, self.state = fh, state

    def get_offset_and_num_candidates(self, n: int) -> tuple[int, int]:
        return 0, n

    def candidates_to_victims_map(self, cands):
        return {c.name: c for c in cands}

    def pod_eligible_to_preempt_others(self, pod: dict, nominated_status: Status | None) -> tuple[bool, str]:
        if (pod.get("spec") or {}).get("preemptionPolicy") == "Never":
            return False, "not eligible due to preemptionPolicy=Never."
        try:
            pfs: PreFilterState = self.state.read(PRE_FILTER_STATE_KEY)
        except KeyError:
            return False, "not eligible due to failed to read from cycleState"
        nom = ko.pod_nominated_node(pod)
        if not nom:
            return True, ""
        if nominated_status is not None and nominated_status.code == UNRESOLVABLE:
            return True, ""
        try:
            snap: ElasticQuotaSnapshotState = self.state.read(ELASTIC_QUOTA_SNAPSHOT_KEY)
        except KeyError:
            return True, ""
        ni = self.fh.snapshot_shared_lister().get(nom)
        if ni is None:
            return True, ""
        prio = ko.pod_priority(pod)
        infos = snap.elastic_quota_infos
        pinfo = infos.get(ko.namespace(pod))
        if pinfo is not None:
            more_than_min = pinfo.used_over_min_with(pfs.nominated_pods_req_in_eq_with_pod_req)
            for pi in ni.pods:
                p = pi.pod
                if not ko.deletion_timestamp(p):
                    continue
                einfo = infos.get(ko.namespace(p))
                if einfo is None:
                    continue
                if ko.namespace(p) == ko.namespace(pod) and ko.pod_priority(p) < prio:
                    return False, "not eligible due to a terminating pod on the nominated node."
                if ko.namespace(p) != ko.namespace(pod) and not more_than_min and einfo.used_over_min():
                    return False, "not eligible due to a terminating pod on the nominated node."
        else:
            for pi in ni.pods:
                p = pi.pod
                if infos.get(ko.namespace(p)) is not None:
                    continue
                if ko.deletion_timestamp(p) and ko.pod_priority(p) < prio:
                    return False, "not eligible due to a terminating pod on the nominated node."
        return True, ""

    def select_victims_on_node(self, state: CycleState, pod: dict, ni: NodeInfo, pdbs: list[dict]):
        try:
            snap: ElasticQuotaSnapshotState = state.read(ELASTIC_QUOTA_SNAPSHOT_KEY)
            pfs: PreFilterState = state.read(PRE_FILTER_STATE_KEY)
        except KeyError as e:
            return [], 0, Status(UNSCHEDULABLE, [f"Failed to read cycle state: {e}"])
        fh = self.fh
        pod_req = pfs.pod_req

        def remove(pi: PodInfo) -> None:
            ni.remove_pod(pi.pod)
            s = fh.run_pre_filter_extension_remove_pod(state, pod, pi, ni)
            if not s.is_success():
                raise s.as_error()

        def add(pi: PodInfo) -> None:
            ni.add_pod(pi)
            s = fh.run_pre_filter_extension_add_pod(state, pod, pi, ni)
            if not s.is_success():
                raise s.as_error()

        infos = snap.elastic_quota_infos
        prio = ko.pod_priority(pod)
        pinfo = infos.get(ko.namespace(pod))
        # least important first (sort.Slice with !MoreImportantPod)
        ordered = sorted(ni.pods, key=lambda pi: (ko.pod_priority(pi.pod), -_start(pi.pod)))
        potential: list[PodInfo] = []
        in_eq = pfs.nominated_pods_req_in_eq_with_pod_req
        total = pfs.nominated_pods_req_with_pod_req
        try:
            if pinfo is not None:
                more_than_min = pinfo.used_over_min_with(in_eq)
                for pi in ordered:
                    pv = pi.pod
                    pv_info = infos.get(ko.namespace(pv))
                    if pv_info is None:
                        continue
                    if more_than_min:
                        if ko.namespace(pv) == ko.namespace(pod):
                            if ko.pod_priority(pv) < prio:
                                potential.append(pi)
                                remove(pi)
                            continue
                        if not is_over_quota(pv):
                            continue
                        g = infos.get_guaranteed_overquotas(ko.namespace(pod))
                        min_plus_g = g + (pinfo.min or Resource())
                        if pinfo.used_lte_with(min_plus_g, in_eq):
                            pv_g = infos.get_guaranteed_overquotas(ko.namespace(pv))
                            pv_min_plus_g = pv_g + (pv_info.min or Resource())
                            if pv_info.used_over(pv_min_plus_g):
                                potential.append(pi)
                                remove(pi)
                    else:
                        if ko.namespace(pv) != ko.namespace(pod) and pv_info.used_over_min() and is_over_quota(pv):
                            potential.append(pi)
                            remove(pi)
            else:
                for pi in ordered:
                    if infos.get(ko.namespace(pi.pod)) is not None:
                        continue
                    if ko.pod_priority(pi.pod) < prio:
                        potential.append(pi)
                        remove(pi)
        except Exception as e:
            return [], 0, as_status(e)

        if not potential:
            return [], 0, Status(UNRESOLVABLE, [f"No victims found on node {ni.name} for preemptor pod {ko.name(pod)}"])
        s = fh.run_filter_plugins_with_nominated_pods(state, pod, ni)
        if not s.is_success():
            return [], 0, s
        if pinfo is not None:
            if pinfo.used_over_max_with(pod_req):
                return [], 0, Status(UNSCHEDULABLE, ["max quota exceeded"])
            if infos.aggregated_used_over_min_with(pod_req):
                return [], 0, Status(UNSCHEDULABLE, ["total min quota exceeded"])

        potential.sort(key=lambda pi: (-ko.pod_priority(pi.pod), _start(pi.pod)))  # most important first
        violating, non_violating = filter_pods_with_pdb_violation(potential, pdbs)
        victims: list[dict] = []
        nviol = 0

        def reprieve(pi: PodInfo) -> bool:
            add(pi)
            fits = fh.run_filter_plugins_with_nominated_pods(state, pod, ni).is_success()
            quota_violated = pinfo is not None and (pinfo.used_over_max_with(in_eq)
                                                    or infos.aggregated_used_over_min_with(total))
            if not fits or quota_violated:
                remove(pi)
                victims.append(pi.pod)
            return fits and not quota_violated

        try:
            for pi in violating:
                if not reprieve(pi):
                    nviol += 1
            for pi in non_violating:
                reprieve(pi)
        except Exception as e:
            return [], 0, as_status(e)
        return victims, nviol, Status.ok()


def _start(p: dict) -> float:
    st = (p.get("status") or {}).get("startTime")
    return ko.parse_time(st) if st else ko.creation_time(p)


__all__ = ["CapacityScheduling", "CapacityPreemptor", "NAME", "is_over_quota", "more_important_pod"]
