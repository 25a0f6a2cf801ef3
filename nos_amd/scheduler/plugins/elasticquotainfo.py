"""Elastic-quota bookkeeping of the CapacityScheduling plugin.

Same math as the reference (``pkg/scheduler/plugins/capacityscheduling/
elasticquotainfo.go:31-361``):

* infos keyed by namespace; a CompositeElasticQuota maps each of its
  namespaces to the same info object;
* ``update`` preserves ``pods`` / ``used``;
* ``aggregated_used_over_min_with``: sum(used) + request > sum(min);
* guaranteed over-quotas: floor(min_i / sum(min) x sum_j max(0, min_j - used_j))
  per resource;
* used-over predicates compare cpu and memory always and scalar resources
  only when present in the limit (``sumGreaterThan`` / ``sumLessThanEqual``);
* pods are added / removed idempotently by pod key.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

from ...kube import objects as ko
from ...resource.resource import Resource


def _pod_key(pod: dict) -> str:
    return f"{ko.namespace(pod)}/{ko.name(pod)}"


def sum_greater_than(x1: Resource, x2: Resource, y: Resource) -> bool:
    if x1.milli_cpu + x2.milli_cpu > y.milli_cpu:
        return True
    if x1.memory + x2.memory > y.memory:
        return True
    for r in set(x1.scalar) | set(x2.scalar) | set(y.scalar):
        if r in y.scalar and x1.scalar.get(r, 0) + x2.scalar.get(r, 0) > y.scalar[r]:
            return True
    return False


def sum_less_than_equal(x1: Resource, x2: Resource, y: Resource) -> bool:
    if x1.milli_cpu + x2.milli_cpu > y.milli_cpu:
        return False
    if x1.memory + x2.memory > y.memory:
        return False
    for r in set(x1.scalar) | set(x2.scalar) | set(y.scalar):
        if r in y.scalar and x1.scalar.get(r, 0) + x2.scalar.get(r, 0) > y.scalar[r]:
            return False
    return True


def greater_than(x: Resource, y: Resource) -> bool:
    return sum_greater_than(x, Resource(), y)


@dataclass
class ElasticQuotaInfo:
    resource_name: str
    resource_namespace: str
    namespaces: set[str]
    min: Resource | None
    max: Resource | None
    used: Resource = field(default_factory=Resource)
    max_enforced: bool = False
    calculator: object = None
    pods: set[str] = field(default_factory=set)

    def reserve(self, req: Resource) -> None:
        self.used.memory += req.memory
        self.used.milli_cpu += req.milli_cpu
        for k, v in req.scalar.items():
            self.used.scalar[k] = self.used.scalar.get(k, 0) + v

    def unreserve(self, req: Resource) -> None:
        self.used.memory -= req.memory
        self.used.milli_cpu -= req.milli_cpu
        for k, v in req.scalar.items():
            self.used.scalar[k] = self.used.scalar.get(k, 0) - v

    def used_over_min_with(self, req: Resource) -> bool:
        return sum_greater_than(req, self.used, self.min or Resource())

    def used_over_max_with(self, req: Resource) -> bool:
        if self.max_enforced:
            return sum_greater_than(req, self.used, self.max or Resource())
        return False

    def used_over_min(self) -> bool:
        return greater_than(self.used, self.min or Resource())

    def used_over(self, r: Resource) -> bool:
        return greater_than(self.used, r)

    def used_lte_with(self, r: Resource, req: Resource) -> bool:
        return sum_less_than_equal(req, self.used, r)

    def clone(self) -> "ElasticQuotaInfo":
        return ElasticQuotaInfo(self.resource_name, self.resource_namespace, set(self.namespaces),
                                self.min.clone() if self.min is not None else None,
                                self.max.clone() if self.max is not None else None,
                                self.used.clone() if self.used is not None else Resource(),
                                self.max_enforced, self.calculator, set(self.pods))

    def _request(self, pod: dict) -> Resource:
        return Resource.from_list(self.calculator.compute_pod_request(pod))

    def add_pod_if_not_present(self, pod: dict) -> None:
        k = _pod_key(pod)
        if k in self.pods:
            return
        self.pods.add(k)
        self.reserve(self._request(pod))

    def delete_pod_if_present(self, pod: dict) -> None:
        k = _pod_key(pod)
        if k not in self.pods:
            return
        self.pods.discard(k)
        self.unreserve(self._request(pod))


class ElasticQuotaInfos(dict):
    """namespace -> ElasticQuotaInfo"""

    def clone(self) -> "ElasticQuotaInfos":
        out = ElasticQuotaInfos()
        seen: dict[int, ElasticQuotaInfo] = {}
        for ns, info in self.items():
            c = seen.get(id(info))
            if c is None:
                c = seen[id(info)] = info.clone()
            out[ns] = c
        return out

    def add(self, info: ElasticQuotaInfo) -> None:
        for ns in info.namespaces:
            self[ns] = info

    def delete(self, info: ElasticQuotaInfo) -> None:
        for ns in info.namespaces:
            self.pop(ns, None)

    def update(self, old: ElasticQuotaInfo, new: ElasticQuotaInfo) -> None:  # type: ignore[override]
        for ns in new.namespaces:
            cur = self.get(ns)
            if cur is not None:
                new.pods = cur.pods
                new.used = cur.used
            self[ns] = new
        for ns in old.namespaces:
            if ns not in new.namespaces:
                self.pop(ns, None)

    def _unique(self) -> list[ElasticQuotaInfo]:
        seen, out = set(), []
        for info in self.values():
            if id(info) not in seen:
                seen.add(id(info))
                out.append(info)
        return out

    def aggregated_min(self) -> Resource:
        total = Resource()
        for info in self._unique():
            if info.min is not None:
                total = total + info.min
        return total

    def aggregated_used(self) -> Resource:
        total = Resource()
        for info in self._unique():
            if info.used is not None:
                total = total + info.used
        return total

    def aggregated_used_over_min_with(self, req: Resource) -> bool:
        used = self.aggregated_used()
        used.iadd(req)
        return greater_than(used, self.aggregated_min())

    def aggregated_overquotas(self) -> Resource:
        total = Resource()
        for info in self._unique():
            total = total + (info.min or Resource()).subtract_non_negative(info.used)
        return total

    def guaranteed_overquotas_percentages(self, info: ElasticQuotaInfo) -> dict[str, float]:
        if info.min is None:
            return {}
        total = self.aggregated_min()
        out = {}
        for r in info.min.names():
            t = total.get(r)
            out[r] = info.min.get(r) / t if t > 0 else 0.0
        return out

    def get_guaranteed_overquotas(self, namespace: str) -> Resource:
        info = self.get(namespace)
        if info is None:
            raise KeyError(f"elastic quota {namespace!r} not present in elastic quota infos")
        pct = self.guaranteed_overquotas_percentages(info)
        agg = self.aggregated_overquotas()
        r = Resource(math.floor(agg.milli_cpu * pct.get("cpu", 0.0)),
                     math.floor(agg.memory * pct.get("memory", 0.0)),
                     math.floor(agg.ephemeral_storage * pct.get("ephemeral-storage", 0.0)),
                     math.floor(agg.allowed_pod_number * pct.get("pods", 0.0)))
        for k, v in agg.scalar.items():
            r.scalar[k] = math.floor(v * pct.get(k, 0.0))
        return r
