"""Fluent object builders for tests and the simulator.

Mirrors the reference's ``pkg/test/factory/core_factory.go:27-229`` builder API
(``BuildNode().WithLabels(...)``, ``BuildPod(ns, name).WithContainer(...)``,
``BuildContainer(name, image).WithRequests(...)``) with AMD resource helpers
instead of the NVIDIA ones.
"""
from __future__ import annotations

import copy
from typing import Any

from . import objects as ko
from . import quantity as q

AMD_GPU = "amd.com/gpu"


class _Builder:
    def __init__(self, obj: dict):
        self._o = obj

    def get(self) -> dict:
        return copy.deepcopy(self._o)


class NodeBuilder(_Builder):
    def with_labels(self, labels: dict[str, str]) -> "NodeBuilder":
        ko.meta(self._o).setdefault("labels", {}).update(labels)
        return self

    def with_annotations(self, ann: dict[str, str]) -> "NodeBuilder":
        ko.meta(self._o).setdefault("annotations", {}).update(ann)
        return self

    def with_allocatable_resources(self, rl: dict[str, Any]) -> "NodeBuilder":
        st = self._o.setdefault("status", {})
        st["allocatable"] = {k: str(v) for k, v in rl.items()}
        st.setdefault("capacity", dict(st["allocatable"]))
        return self

    def with_capacity(self, rl: dict[str, Any]) -> "NodeBuilder":
        self._o.setdefault("status", {})["capacity"] = {k: str(v) for k, v in rl.items()}
        return self


def build_node(name: str) -> NodeBuilder:
    return NodeBuilder({"apiVersion": "v1", "kind": "Node",
                        "metadata": {"name": name, "labels": {}, "annotations": {}},
                        "spec": {}, "status": {"allocatable": {}, "capacity": {}}})


def build_namespace(name: str) -> _Builder:
    return _Builder({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": name}})


class PodBuilder(_Builder):
    def with_container(self, c: dict) -> "PodBuilder":
        self._o["spec"].setdefault("containers", []).append(copy.deepcopy(c))
        return self

    def with_init_container(self, c: dict) -> "PodBuilder":
        self._o["spec"].setdefault("initContainers", []).append(copy.deepcopy(c))
        return self

    def with_phase(self, phase: str) -> "PodBuilder":
        self._o.setdefault("status", {})["phase"] = phase
        return self

    def with_uid(self, uid: str) -> "PodBuilder":
        ko.meta(self._o)["uid"] = uid
        return self

    def with_label(self, k: str, v: str) -> "PodBuilder":
        ko.set_label(self._o, k, v)
        return self

    def with_annotation(self, k: str, v: str) -> "PodBuilder":
        ko.set_annotation(self._o, k, v)
        return self

    def with_node_name(self, n: str) -> "PodBuilder":
        self._o["spec"]["nodeName"] = n
        return self

    def with_creation_timestamp(self, t: float | str) -> "PodBuilder":
        ko.meta(self._o)["creationTimestamp"] = t if isinstance(t, str) else ko.now_rfc3339(t)
        return self

    def with_priority(self, p: int) -> "PodBuilder":
        self._o["spec"]["priority"] = int(p)
        return self

    def with_owner(self, kind: str, name: str) -> "PodBuilder":
        ko.meta(self._o).setdefault("ownerReferences", []).append(
            {"apiVersion": "apps/v1", "kind": kind, "name": name, "uid": ko.new_uid()})
        return self

    def with_overhead(self, rl: dict[str, Any]) -> "PodBuilder":
        self._o["spec"]["overhead"] = {k: str(v) for k, v in rl.items()}
        return self

    def with_scheduler_name(self, n: str) -> "PodBuilder":
        self._o["spec"]["schedulerName"] = n
        return self

    def with_nominated_node(self, n: str) -> "PodBuilder":
        self._o.setdefault("status", {})["nominatedNodeName"] = n
        return self

    def with_unschedulable_condition(self) -> "PodBuilder":
        ko.set_condition(self._o, "PodScheduled", "False", "Unschedulable", "simulated")
        return self


def build_pod(namespace: str, name: str) -> PodBuilder:
    return PodBuilder({"apiVersion": "v1", "kind": "Pod",
                       "metadata": {"name": name, "namespace": namespace, "uid": ko.new_uid(),
                                    "labels": {}, "annotations": {},
                                    "creationTimestamp": ko.now_rfc3339()},
                       "spec": {"containers": []}, "status": {"phase": ko.PENDING}})


class ContainerBuilder(_Builder):
    def _res(self, which: str) -> dict:
        return self._o.setdefault("resources", {}).setdefault(which, {})

    def with_limits(self, rl: dict[str, Any]) -> "ContainerBuilder":
        self._res("limits").update({k: str(v) for k, v in rl.items()})
        return self

    def with_requests(self, rl: dict[str, Any]) -> "ContainerBuilder":
        self._res("requests").update({k: str(v) for k, v in rl.items()})
        return self

    def with_cpu_milli_limit(self, m: int) -> "ContainerBuilder":
        self._res("limits")["cpu"] = f"{m}m"
        return self

    def with_cpu_milli_request(self, m: int) -> "ContainerBuilder":
        self._res("requests")["cpu"] = f"{m}m"
        return self

    def with_amd_gpu_limit(self, n: int) -> "ContainerBuilder":
        self._res("limits")[AMD_GPU] = str(n)
        return self

    def with_amd_gpu_request(self, n: int) -> "ContainerBuilder":
        self._res("requests")[AMD_GPU] = str(n)
        return self

    def with_scalar_resource_limit(self, name: str, n: int) -> "ContainerBuilder":
        self._res("limits")[name] = str(n)
        return self

    def with_scalar_resource_request(self, name: str, n: int) -> "ContainerBuilder":
        self._res("requests")[name] = str(n)
        return self

    def with_resource_request(self, name: str, quantity: Any) -> "ContainerBuilder":
        self._res("requests")[name] = q.fmt(q.parse(quantity))
        return self

    def with_memory_request(self, quantity: Any) -> "ContainerBuilder":
        self._res("requests")["memory"] = str(quantity)
        return self


def build_container(name: str = "c", image: str = "test") -> ContainerBuilder:
    return ContainerBuilder({"name": name, "image": image, "resources": {}})


def build_configmap(namespace: str, name: str, data: dict[str, str] | None = None) -> dict:
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": namespace},
            "data": dict(data or {})}


def build_pdb(namespace: str, name: str, selector: dict[str, str], min_available: int | None = None,
              max_unavailable: int | None = None, disruptions_allowed: int = 0) -> dict:
    spec: dict[str, Any] = {"selector": {"matchLabels": dict(selector)}}
    if min_available is not None:
        spec["minAvailable"] = min_available
    if max_unavailable is not None:
        spec["maxUnavailable"] = max_unavailable
    return {"apiVersion": "policy/v1", "kind": "PodDisruptionBudget",
            "metadata": {"name": name, "namespace": namespace}, "spec": spec,
            "status": {"disruptionsAllowed": disruptions_allowed}}
