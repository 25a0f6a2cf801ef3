"""``nos.nebuly.com/v1alpha1`` CRDs: ElasticQuota and CompositeElasticQuota.

API-compatible with the reference (same group/version/kind, short names,
schema and status subresource: ``pkg/api/nos.nebuly.com/v1alpha1/
elasticquota_types.go:30-71``, ``compositeelasticquota_types.go:29-66``).
Objects are plain dicts; this module provides the CRD definitions (used by
the API server and rendered to ``config/crd``), builders
(``elasticquota_factory.go:25-87``, ``compositeelasticquota_factory.go:25-92``)
and the validating admission webhooks (``elasticquota_webhook.go:48-87``,
``compositeelasticquota_webhook.go:66-89``) plus the ``max >= min`` check the
reference's docs promise but never implemented.
"""
from __future__ import annotations

import copy
from typing import Any

from ..kube import objects as ko
from ..kube import quantity as q
from . import constants as C

KIND_EQ = "ElasticQuota"
KIND_CEQ = "CompositeElasticQuota"


def _resource_list_schema() -> dict:
    return {"type": "object", "additionalProperties": {
        "anyOf": [{"type": "integer"}, {"type": "string"}],
        "pattern": r"^(\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))(([KMGTPE]i)|[numkMGTPE]|([eE](\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))))?$",
        "x-kubernetes-int-or-string": True}}


def crd(kind: str) -> dict:
    """CustomResourceDefinition manifest (apiextensions.k8s.io/v1)."""
    plural = {"ElasticQuota": "elasticquotas", "CompositeElasticQuota": "compositeelasticquotas"}[kind]
    short = {"ElasticQuota": ["eq", "eqs"], "CompositeElasticQuota": ["ceq", "ceqs"]}[kind]
    spec_props: dict[str, Any] = {"min": _resource_list_schema(), "max": _resource_list_schema()}
    required: list[str] = []
    if kind == KIND_CEQ:
        spec_props["namespaces"] = {"type": "array", "items": {"type": "string"}, "minItems": 1}
        required = ["namespaces"]
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{plural}.{C.GROUP}"},
        "spec": {
            "group": C.GROUP,
            "names": {"kind": kind, "listKind": kind + "List", "plural": plural, "singular": kind.lower(),
                      "shortNames": short},
            "scope": "Namespaced",
            "versions": [{
                "name": C.VERSION, "served": True, "storage": True,
                "subresources": {"status": {}},
                "schema": {"openAPIV3Schema": {
                    "type": "object",
                    "properties": {
                        "apiVersion": {"type": "string"}, "kind": {"type": "string"},
                        "metadata": {"type": "object"},
                        "spec": {"type": "object", "properties": spec_props, **({"required": required} if required else {})},
                        "status": {"type": "object", "properties": {"used": _resource_list_schema()}},
                    }}},
            }],
        },
    }


# ------------------------------------------------------------------ accessors
def spec_min(eq: dict) -> dict:
    return q.rl_parse((eq.get("spec") or {}).get("min"))


def spec_max(eq: dict) -> dict:
    return q.rl_parse((eq.get("spec") or {}).get("max"))


def status_used(eq: dict) -> dict:
    return q.rl_parse((eq.get("status") or {}).get("used"))


def namespaces(ceq: dict) -> list[str]:
    return list((ceq.get("spec") or {}).get("namespaces") or [])


# ------------------------------------------------------------------ builders
class _QuotaBuilder:
    def __init__(self, kind: str, namespace: str, name: str):
        self._o: dict[str, Any] = {"apiVersion": C.API_VERSION, "kind": kind,
                                   "metadata": {"name": name, "namespace": namespace},
                                   "spec": {}, "status": {}}

    def with_min(self, rl: dict) -> "_QuotaBuilder":
        self._o["spec"].setdefault("min", {}).update({k: q.fmt(q.parse(v)) for k, v in rl.items()})
        return self

    def with_max(self, rl: dict) -> "_QuotaBuilder":
        self._o["spec"].setdefault("max", {}).update({k: q.fmt(q.parse(v)) for k, v in rl.items()})
        return self

    def with_min_gpu_memory(self, gb: int) -> "_QuotaBuilder":
        return self.with_min({C.RESOURCE_GPU_MEMORY: gb})

    def with_max_gpu_memory(self, gb: int) -> "_QuotaBuilder":
        return self.with_max({C.RESOURCE_GPU_MEMORY: gb})

    def with_min_cpu_milli(self, m: int) -> "_QuotaBuilder":
        self._o["spec"].setdefault("min", {})["cpu"] = f"{m}m"
        return self

    def with_max_cpu_milli(self, m: int) -> "_QuotaBuilder":
        self._o["spec"].setdefault("max", {})["cpu"] = f"{m}m"
        return self

    def with_namespaces(self, *ns: str) -> "_QuotaBuilder":
        self._o["spec"]["namespaces"] = list(ns)
        return self

    def with_used(self, rl: dict) -> "_QuotaBuilder":
        self._o["status"]["used"] = {k: q.fmt(q.parse(v)) for k, v in rl.items()}
        return self

    def get(self) -> dict:
        return copy.deepcopy(self._o)


def build_eq(namespace: str, name: str) -> _QuotaBuilder:
    return _QuotaBuilder(KIND_EQ, namespace, name)


def build_composite_eq(namespace: str, name: str) -> _QuotaBuilder:
    return _QuotaBuilder(KIND_CEQ, namespace, name)


# ------------------------------------------------------------------ webhooks
class ValidationError(Exception):
    pass


def validate_min_max(obj: dict) -> None:
    """New: every resource present in both min and max must satisfy max >= min."""
    mn, mx = spec_min(obj), spec_max(obj)
    for k in set(mn) & set(mx):
        if mx[k] < mn[k]:
            raise ValidationError(f"spec.max[{k}]={q.fmt(mx[k])} is lower than spec.min[{k}]={q.fmt(mn[k])}")


def validate_eq_create(eq: dict, existing_eqs: list[dict], ceqs: list[dict]) -> None:
    ns = ko.namespace(eq)
    others = [e for e in existing_eqs if ko.namespace(e) == ns and ko.name(e) != ko.name(eq)]
    if others:
        raise ValidationError(f"only 1 ElasticQuota per namespace is allowed - ElasticQuota "
                              f"{ko.name(others[0])!r} already exists in namespace {ns!r}")
    for c in ceqs:
        if ns in namespaces(c):
            raise ValidationError(f'the CompositeElasticQuota "{ko.namespace(c)}/{ko.name(c)}" already '
                                  f"defines quotas for namespace {ns!r}")
    validate_min_max(eq)


def validate_ceq(ceq: dict, ceqs: list[dict]) -> None:
    if not namespaces(ceq):
        raise ValidationError("spec.namespaces: at least 1 namespace is required")
    for c in ceqs:
        if ko.key(c) == ko.key(ceq):
            continue
        for ns in namespaces(ceq):
            if ns in namespaces(c):
                raise ValidationError(
                    f"a namespace can belong to only 1 CompositeElasticQuota: namespace {ns!r} already "
                    f'belongs to CompositeElasticQuota "{ko.namespace(c)}/{ko.name(c)}"')
    validate_min_max(ceq)


def register_webhooks(api) -> None:
    """Install the validating admission hooks into an :class:`ApiServer`."""
    from ..sim.apiserver import Forbidden

    def eq_hook(op, new, old, server):
        try:
            if op == "CREATE":
                validate_eq_create(new, server.list(KIND_EQ, ko.namespace(new)), server.list(KIND_CEQ))
            elif op == "UPDATE":
                validate_min_max(new)
        except ValidationError as e:
            raise Forbidden(f"admission webhook velasticquota.kb.io denied the request: {e}") from e

    def ceq_hook(op, new, old, server):
        try:
            if op in ("CREATE", "UPDATE"):
                validate_ceq(new, server.list(KIND_CEQ))
        except ValidationError as e:
            raise Forbidden(f"admission webhook vcompositeelasticquota.kb.io denied the request: {e}") from e

    api.register_admission(KIND_EQ, eq_hook)
    api.register_admission(KIND_CEQ, ceq_hook)


def register_types(api, webhooks: bool = True) -> None:
    from ..sim.apiserver import ResourceType

    api.register_type(ResourceType(C.API_VERSION, KIND_EQ, "elasticquotas"))
    api.register_type(ResourceType(C.API_VERSION, KIND_CEQ, "compositeelasticquotas"))
    if webhooks:
        register_webhooks(api)
