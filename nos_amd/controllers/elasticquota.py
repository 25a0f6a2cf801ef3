"""Elastic-quota operator reconcilers (``internal/controllers/elasticquota``).

``ElasticQuotaReconciler`` / ``CompositeElasticQuotaReconciler``:

1. list the Running pods of the quota's namespace(s) (field index
   ``status.phase``);
2. sort them by creation time, then priority (asc), then request (asc), then
   name, accumulate ``used`` and label each pod
   ``nos.nebuly.com/capacity=in-quota`` while ``used <= min`` (only resources
   present in min are compared), else ``over-quota``
   (``elasticquota.go:38-104``); the scheduler's preemption reads that label;
3. drop from ``used`` every resource not in ``min`` and merge-patch
   ``status.used`` if it changed.

The composite reconciler also deletes every ElasticQuota that overlaps its
namespaces (``compositeelasticquota_controller.go:112-137``).  Pods without
``spec.priority`` are treated as priority 0 (the reference dereferences a nil
pointer there, ``elasticquota.go:87-88``).
"""
from __future__ import annotations

import functools
import logging
from fractions import Fraction

from ..api import constants as C
from ..api import v1alpha1
from ..gpu.memory import ResourceCalculator
from ..kube import objects as ko
from ..kube import quantity as q
from ..runtime.manager import Controller, Request, Result
from ..runtime.predicates import Funcs

log = logging.getLogger("nos_amd.controllers.elasticquota")


def less_than_or_equal(a: dict, b: dict) -> bool:
    """quota.LessThanOrEqual: every key of b present in a satisfies a[k] <= b[k]."""
    return all(q.parse(a[k]) <= q.parse(v) for k, v in b.items() if k in a)


def rl_equals(a: dict, b: dict) -> bool:
    return set(a) == set(b) and all(q.parse(a[k]) == q.parse(b[k]) for k in a)


class PodsReconciler:
    def __init__(self, api, calculator: ResourceCalculator):
        self.api, self.calc = api, calculator

    def sort_pods(self, pods: list[dict]) -> list[dict]:
        reqs = {ko.key(p): self.calc.compute_pod_request(p) for p in pods}

        def cmp(a, b):
            ta, tb = ko.creation_time(a), ko.creation_time(b)
            if ta != tb:
                return -1 if ta < tb else 1
            pa, pb = ko.pod_priority(a), ko.pod_priority(b)
            if pa != pb:
                return -1 if pa < pb else 1
            ra, rb = reqs[ko.key(a)], reqs[ko.key(b)]
            if not rl_equals(ra, rb):
                return -1 if less_than_or_equal(ra, rb) else 1
            return -1 if ko.name(a) < ko.name(b) else (1 if ko.name(a) > ko.name(b) else 0)

        return sorted(pods, key=functools.cmp_to_key(cmp))

    def patch_pods_and_compute_used(self, pods: list[dict], qmin: dict, qmax: dict) -> dict[str, Fraction]:
        used: dict[str, Fraction] = {k: Fraction(0) for k in list(qmin) + list(qmax)}
        for pod in self.sort_pods(pods):
            used = q.rl_add(used, self.calc.compute_pod_request(pod))
            desired = C.CAPACITY_IN_QUOTA if less_than_or_equal(used, qmin) else C.CAPACITY_OVER_QUOTA
            if ko.labels(pod).get(C.LABEL_CAPACITY_INFO) != desired:
                self.api.patch("Pod", ko.name(pod), {"metadata": {"labels": {C.LABEL_CAPACITY_INFO: desired}}},
                               ko.namespace(pod))
        return {k: v for k, v in used.items() if k in qmin}


def _running_pods(api, namespaces: list[str]) -> list[dict]:
    out = []
    for ns in namespaces:
        out.extend(api.list("Pod", ns, field_selector=f"{C.POD_PHASE_KEY}={ko.RUNNING}"))
    return out


def _update_status(api, obj: dict, used: dict) -> None:
    cur = api.get(obj["kind"], ko.name(obj), ko.namespace(obj))
    want = q.rl_fmt(used)
    have = (cur.get("status") or {}).get("used") or {}
    if rl_equals(q.rl_parse(have), used) and set(have) == set(want):
        return
    api.patch(obj["kind"], ko.name(obj), {"status": {"used": {**{k: None for k in have if k not in want}, **want}}},
              ko.namespace(obj), subresource="status")


def _phase_change_predicate() -> Funcs:
    def upd(ev):
        if ev.old is None:
            return False
        changed = ko.pod_phase(ev.obj) != ko.pod_phase(ev.old)
        any_running = ko.RUNNING in (ko.pod_phase(ev.obj), ko.pod_phase(ev.old))
        return changed and any_running
    return Funcs(create=lambda ev: False, update=upd, delete=lambda ev: True, generic=lambda ev: False)


class ElasticQuotaReconciler:
    def __init__(self, api, memory_gb: int = C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB):
        self.api = api
        self.pods = PodsReconciler(api, ResourceCalculator(memory_gb))

    def reconcile(self, req: Request) -> Result:
        eq = self.api.try_get(v1alpha1.KIND_EQ, req.name, req.namespace)
        if eq is None:
            return Result()
        used = self.pods.patch_pods_and_compute_used(_running_pods(self.api, [req.namespace]),
                                                     v1alpha1.spec_min(eq), v1alpha1.spec_max(eq))
        _update_status(self.api, eq, used)
        return Result()

    def find_for_pod(self, pod: dict) -> list[Request]:
        eqs = self.api.list(v1alpha1.KIND_EQ, ko.namespace(pod))
        return [Request(ko.name(e), ko.namespace(e)) for e in eqs]

    def controller(self, name: str = C.ELASTIC_QUOTA_CONTROLLER) -> Controller:
        return (Controller(name, self).for_kind(v1alpha1.KIND_EQ)
                .watches("Pod", self.find_for_pod, _phase_change_predicate()))


class CompositeElasticQuotaReconciler:
    def __init__(self, api, memory_gb: int = C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB):
        self.api = api
        self.pods = PodsReconciler(api, ResourceCalculator(memory_gb))

    def reconcile(self, req: Request) -> Result:
        ceq = self.api.try_get(v1alpha1.KIND_CEQ, req.name, req.namespace)
        if ceq is None:
            return Result()
        nss = v1alpha1.namespaces(ceq)
        for ns in nss:
            for eq in self.api.list(v1alpha1.KIND_EQ, ns):
                log.info("deleting ElasticQuota %s overlapping CompositeElasticQuota %s", ko.key(eq), ko.key(ceq))
                try:
                    self.api.delete(v1alpha1.KIND_EQ, ko.name(eq), ns)
                except Exception:
                    pass
        used = self.pods.patch_pods_and_compute_used(_running_pods(self.api, nss), v1alpha1.spec_min(ceq),
                                                     v1alpha1.spec_max(ceq))
        _update_status(self.api, ceq, used)
        return Result()

    def find_for_pod(self, pod: dict) -> list[Request]:
        for c in self.api.list(v1alpha1.KIND_CEQ):
            if ko.namespace(pod) in v1alpha1.namespaces(c):
                return [Request(ko.name(c), ko.namespace(c))]
        return []

    def controller(self, name: str = C.COMPOSITE_ELASTIC_QUOTA_CONTROLLER) -> Controller:
        return (Controller(name, self).for_kind(v1alpha1.KIND_CEQ)
                .watches("Pod", self.find_for_pod, _phase_change_predicate()))
