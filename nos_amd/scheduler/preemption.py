"""Preemption evaluator (upstream ``framework/preemption`` semantics).

``Evaluator.preempt``: fetch the latest preemptor, check eligibility, dry-run
victim selection on every node where preemption might help (nodes not
``UnschedulableAndUnresolvable``), pick one candidate
(``pick_one_node_for_preemption``: fewest PDB violations, lowest
highest-victim priority, lowest priority sum, fewest victims, latest start),
then delete its victims and clear the nomination of lower-priority pods
nominated to that node.  The plugin-specific part (eligibility and victim
selection) is an :class:`PreemptorInterface` -- CapacityScheduling plugs its
over-quota fair-share rules in there (``capacity_scheduling.go:378-675``).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field
from typing import Protocol

from ..kube import objects as ko
from ..kube import selectors as sel
from .framework import (UNRESOLVABLE, UNSCHEDULABLE, CycleState, NodeInfo, PodInfo, PostFilterResult, Status,
                        as_status)

log = logging.getLogger("nos_amd.scheduler.preemption")

MAX_INT32 = 2 ** 31 - 1


@dataclass
class Candidate:
    name: str
    victims: list[dict] = field(default_factory=list)
    num_pdb_violations: int = 0


class PreemptorInterface(Protocol):
    def get_offset_and_num_candidates(self, n: int) -> tuple[int, int]: ...

    def candidates_to_victims_map(self, candidates: list[Candidate]) -> dict[str, Candidate]: ...

    def pod_eligible_to_preempt_others(self, pod: dict, nominated_node_status: Status | None) -> tuple[bool, str]: ...

    def select_victims_on_node(self, state: CycleState, pod: dict, node_info: NodeInfo,
                               pdbs: list[dict]) -> tuple[list[dict], int, Status]: ...


def more_important_pod(a: dict, b: dict) -> bool:
    """schedutil.MoreImportantPod: higher priority, then earlier start time."""
    pa, pb = ko.pod_priority(a), ko.pod_priority(b)
    if pa != pb:
        return pa > pb
    return _start_time(a) < _start_time(b)


def _start_time(p: dict) -> float:
    st = (p.get("status") or {}).get("startTime")
    return ko.parse_time(st) if st else ko.creation_time(p)


def filter_pods_with_pdb_violation(pods: list[PodInfo], pdbs: list[dict]) -> tuple[list[PodInfo], list[PodInfo]]:
    """Split victims into PDB-violating / non-violating (capacity_scheduling.go:850-895)."""
    allowed = [int((p.get("status") or {}).get("disruptionsAllowed", 0)) for p in pdbs]
    violating, non_violating = [], []
    for pi in pods:
        pod = pi.pod
        violated = False
        if ko.labels(pod):
            for i, pdb in enumerate(pdbs):
                if ko.namespace(pdb) != ko.namespace(pod):
                    continue
                reqs = sel.selector_from_object((pdb.get("spec") or {}).get("selector"))
                if not reqs or not sel.match_labels(reqs, ko.labels(pod)):
                    continue
                if ko.name(pod) in ((pdb.get("status") or {}).get("disruptedPods") or {}):
                    continue
                allowed[i] -= 1
                if allowed[i] < 0:
                    violated = True
        (violating if violated else non_violating).append(pi)
    return violating, non_violating


def pick_one_node_for_preemption(cands: dict[str, Candidate]) -> str | None:
    if not cands:
        return None
    for name, c in cands.items():
        if not c.victims:
            return name
    names = list(cands)
    # 1. fewest PDB violations
    m = min(cands[n].num_pdb_violations for n in names)
    names = [n for n in names if cands[n].num_pdb_violations == m]
    if len(names) == 1:
        return names[0]

    def highest(n):
        return max(ko.pod_priority(v) for v in cands[n].victims)
    m = min(highest(n) for n in names)
    names = [n for n in names if highest(n) == m]
    if len(names) == 1:
        return names[0]

    def psum(n):
        return sum(ko.pod_priority(v) + MAX_INT32 + 1 for v in cands[n].victims)
    m = min(psum(n) for n in names)
    names = [n for n in names if psum(n) == m]
    if len(names) == 1:
        return names[0]
    m = min(len(cands[n].victims) for n in names)
    names = [n for n in names if len(cands[n].victims) == m]
    if len(names) == 1:
        return names[0]

    def earliest(n):
        hp = highest(n)
        return min(_start_time(v) for v in cands[n].victims if ko.pod_priority(v) == hp)
    latest = max(earliest(n) for n in names)
    for n in names:
        if earliest(n) == latest:
            return n
    return names[0]


class Evaluator:
    def __init__(self, plugin_name: str, handle, state: CycleState, interface: PreemptorInterface):
        self.plugin_name = plugin_name
        self.handle = handle
        self.state = state
        self.iface = interface

    def _latest(self, pod: dict) -> dict:
        api = getattr(self.handle, "api", None)
        if api is None:
            return pod
        p = api.try_get("Pod", ko.name(pod), ko.namespace(pod))
        return p or pod

    def _pdbs(self) -> list[dict]:
        api = getattr(self.handle, "api", None)
        if api is None:
            return list(getattr(self.handle, "pdbs", []) or [])
        try:
            return api.list("PodDisruptionBudget")
        except Exception:
            return []

    def preempt(self, pod: dict, statuses: dict[str, Status]) -> tuple[PostFilterResult | None, Status]:
        pod = self._latest(pod)
        ok, msg = self.iface.pod_eligible_to_preempt_others(pod, statuses.get(ko.pod_nominated_node(pod)))
        if not ok:
            return None, Status(UNSCHEDULABLE, [msg])
        cands, node_status = self.find_candidates(pod, statuses)
        if not cands:
            return None, Status(UNSCHEDULABLE, [f"0/{len(node_status)} nodes are available: preemption: "
                                                "no candidate found"])
        best = self.select_candidate(cands)
        if best is None or not best.name:
            return None, Status(UNSCHEDULABLE, ["no candidate node for preemption"])
        st = self.prepare_candidate(best, pod)
        if not st.is_success():
            return None, st
        return PostFilterResult(best.name), Status.ok()

    def find_candidates(self, pod: dict, statuses: dict[str, Status]) -> tuple[list[Candidate], dict[str, Status]]:
        all_nodes = self.handle.snapshot_shared_lister().list()
        potential = [n for n in all_nodes if statuses.get(n.name, Status(UNSCHEDULABLE)).code != UNRESOLVABLE]
        unresolvable = {n.name: statuses[n.name] for n in all_nodes
                        if n.name in statuses and statuses[n.name].code == UNRESOLVABLE}
        if not potential:
            return [], unresolvable
        pdbs = self._pdbs()
        offset, num = self.iface.get_offset_and_num_candidates(len(potential))
        cands, st = self.dry_run_preemption(pod, potential, pdbs, offset, num)
        st.update(unresolvable)
        return cands, st

    def dry_run_preemption(self, pod: dict, nodes: list[NodeInfo], pdbs: list[dict], offset: int,
                           num_candidates: int) -> tuple[list[Candidate], dict[str, Status]]:
        non_violating: list[Candidate] = []
        violating: list[Candidate] = []
        statuses: dict[str, Status] = {}
        n = len(nodes)
        for i in range(n):
            ni = nodes[(offset + i) % n]
            ni_copy = ni.clone()
            st_copy = self.state.clone()
            try:
                victims, nviol, status = self.iface.select_victims_on_node(st_copy, pod, ni_copy, pdbs)
            except Exception as e:  # a plugin bug must not kill the scheduler
                victims, nviol, status = [], 0, as_status(e)
            if status.is_success() and victims:
                c = Candidate(ni.name, victims, nviol)
                (non_violating if nviol == 0 else violating).append(c)
                if len(non_violating) >= num_candidates:
                    break
            elif status.is_success() and not victims:
                status = Status(UNSCHEDULABLE, [f"expected at least one victim pod on node {ni.name!r}"])
            statuses[ni.name] = status
        return non_violating + violating, statuses

    def select_candidate(self, cands: list[Candidate]) -> Candidate | None:
        if not cands:
            return None
        if len(cands) == 1:
            return cands[0]
        vm = self.iface.candidates_to_victims_map(cands)
        name = pick_one_node_for_preemption(vm)
        for c in cands:
            if c.name == name:
                return c
        return cands[0]

    def prepare_candidate(self, c: Candidate, pod: dict) -> Status:
        api = getattr(self.handle, "api", None)
        for v in c.victims:
            if api is not None:
                try:
                    api.delete("Pod", ko.name(v), ko.namespace(v))
                except Exception as e:
                    if "not found" not in str(e).lower():
                        return as_status(e)
            log.info("preempted %s on %s for %s", ko.key(v), c.name, ko.key(pod))
        # clear the nomination of lower-priority pods nominated to this node
        nominator = getattr(self.handle, "nominator", None)
        if nominator is not None:
            prio = ko.pod_priority(pod)
            for pi in nominator.nominated_pods_for_node(c.name):
                if ko.pod_priority(pi.pod) < prio:
                    nominator.delete_nominated_pod_if_exists(pi.pod)
                    if api is not None:
                        try:
                            api.patch("Pod", ko.name(pi.pod), {"status": {"nominatedNodeName": None}},
                                      ko.namespace(pi.pod), subresource="status")
                        except Exception:
                            pass
        return Status.ok()


class PriorityPreemptor:
    """DefaultPreemption's plugin part: lower-priority pods are victims."""

    def __init__(self, handle, state: CycleState):
        self.fh, self.state = handle, state

    def get_offset_and_num_candidates(self, n: int) -> tuple[int, int]:
        return 0, n

    def candidates_to_victims_map(self, cands):
        return {c.name: c for c in cands}

    def pod_eligible_to_preempt_others(self, pod, nominated_status):
        if (pod.get("spec") or {}).get("preemptionPolicy") == "Never":
            return False, "not eligible due to preemptionPolicy=Never."
        nn = ko.pod_nominated_node(pod)
        if nn:
            if nominated_status is not None and nominated_status.code == UNRESOLVABLE:
                return True, ""
            ni = self.fh.snapshot_shared_lister().get(nn)
            if ni is not None:
                prio = ko.pod_priority(pod)
                for pi in ni.pods:
                    if ko.deletion_timestamp(pi.pod) and ko.pod_priority(pi.pod) < prio:
                        return False, "not eligible due to a terminating pod on the nominated node."
        return True, ""

    def select_victims_on_node(self, state, pod, ni: NodeInfo, pdbs):
        prio = ko.pod_priority(pod)
        potential = [pi for pi in ni.pods if ko.pod_priority(pi.pod) < prio]
        for pi in potential:
            ni.remove_pod(pi.pod)
            s = self.fh.run_pre_filter_extension_remove_pod(state, pod, pi, ni)
            if not s.is_success():
                return [], 0, s
        if not potential:
            return [], 0, Status(UNRESOLVABLE, [f"No victims found on node {ni.name} for preemptor pod {ko.name(pod)}"])
        s = self.fh.run_filter_plugins_with_nominated_pods(state, pod, ni)
        if not s.is_success():
            return [], 0, s
        potential.sort(key=lambda pi: (-ko.pod_priority(pi.pod), _start_time(pi.pod)))
        violating, non_violating = filter_pods_with_pdb_violation(potential, pdbs)
        victims: list[dict] = []
        nviol = 0

        def reprieve(pi) -> bool:
            ni.add_pod(pi)
            self.fh.run_pre_filter_extension_add_pod(state, pod, pi, ni)
            fits = self.fh.run_filter_plugins_with_nominated_pods(state, pod, ni).is_success()
            if not fits:
                ni.remove_pod(pi.pod)
                self.fh.run_pre_filter_extension_remove_pod(state, pod, pi, ni)
                victims.append(pi.pod)
            return fits

        for pi in violating:
            if not reprieve(pi):
                nviol += 1
        for pi in non_violating:
            reprieve(pi)
        return victims, nviol, Status.ok()
