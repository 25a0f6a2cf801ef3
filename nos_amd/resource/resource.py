"""Scheduler resource math (``framework.Resource`` + ``pkg/resource/resource.go:35-146``).

:class:`Resource` holds integer milli-CPU, memory bytes, ephemeral storage,
allowed pod number and scalar (extended) resources -- the same fields as the
kube-scheduler framework type -- with the reference's ``Sum``/``Subtract``/
``SubtractNonNegative``/``Abs`` helpers as methods.

:func:`compute_pod_request` is the pod's effective request: sum of the
containers, element-wise max with every init container, plus pod overhead.
The reference computes the overhead sum and discards it
(``pkg/resource/resource.go:141``); here it is applied.
"""
from __future__ import annotations

import contextlib
import threading

from dataclasses import dataclass, field
from fractions import Fraction
from typing import Protocol

from ..kube import objects as ko
from ..kube import quantity as q

CPU, MEMORY, PODS, EPHEMERAL = "cpu", "memory", "pods", "ephemeral-storage"


def is_scalar_resource_name(name: str) -> bool:
    """Extended (domain-prefixed), hugepages, or prefixed-native resources."""
    return "/" in name or name.startswith("hugepages-") or name.startswith("attachable-volumes-")


@dataclass
class Resource:
    milli_cpu: int = 0
    memory: int = 0
    ephemeral_storage: int = 0
    allowed_pod_number: int = 0
    scalar: dict[str, int] = field(default_factory=dict)

    # ------------------------------------------------------------ conversions
    @classmethod
    def from_list(cls, rl: dict | None) -> "Resource":
        r = cls()
        r.add_list(rl or {})
        return r

    def add_list(self, rl: dict) -> None:
        for name, v in rl.items():
            if name == CPU:
                self.milli_cpu += q.milli_value(v)
            elif name == MEMORY:
                self.memory += q.value(v)
            elif name == PODS:
                self.allowed_pod_number += q.value(v)
            elif name == EPHEMERAL:
                self.ephemeral_storage += q.value(v)
            elif is_scalar_resource_name(name):
                self.scalar[name] = self.scalar.get(name, 0) + q.value(v)

    def to_list(self) -> dict[str, Fraction]:
        out: dict[str, Fraction] = {CPU: q.from_milli(self.milli_cpu), MEMORY: Fraction(self.memory),
                                    PODS: Fraction(self.allowed_pod_number),
                                    EPHEMERAL: Fraction(self.ephemeral_storage)}
        for k, v in self.scalar.items():
            out[k] = Fraction(v)
        return out

    def clone(self) -> "Resource":
        return Resource(self.milli_cpu, self.memory, self.ephemeral_storage, self.allowed_pod_number,
                        dict(self.scalar))

    def set_scalar(self, name: str, v: int) -> None:
        self.scalar[name] = v

    def get(self, name: str) -> int:
        if name == CPU:
            return self.milli_cpu
        if name == MEMORY:
            return self.memory
        if name == PODS:
            return self.allowed_pod_number
        if name == EPHEMERAL:
            return self.ephemeral_storage
        return self.scalar.get(name, 0)

    def names(self) -> set[str]:
        return {CPU, MEMORY, PODS, EPHEMERAL} | set(self.scalar)

    # ------------------------------------------------------------ math
    def _zip(self, other: "Resource", fn) -> "Resource":
        r = Resource(fn(self.milli_cpu, other.milli_cpu), fn(self.memory, other.memory),
                     fn(self.ephemeral_storage, other.ephemeral_storage),
                     fn(self.allowed_pod_number, other.allowed_pod_number))
        for k in set(self.scalar) | set(other.scalar):
            r.scalar[k] = fn(self.scalar.get(k, 0), other.scalar.get(k, 0))
        return r

    def __add__(self, other: "Resource") -> "Resource":  # resource.Sum
        return self._zip(other, lambda a, b: a + b)

    def __sub__(self, other: "Resource") -> "Resource":  # resource.Subtract
        return self._zip(other, lambda a, b: a - b)

    def subtract_non_negative(self, other: "Resource") -> "Resource":
        return self._zip(other, lambda a, b: max(0, a - b))

    def abs(self) -> "Resource":
        r = Resource(abs(self.milli_cpu), abs(self.memory), abs(self.ephemeral_storage),
                     abs(self.allowed_pod_number))
        r.scalar = {k: abs(v) for k, v in self.scalar.items()}
        return r

    def iadd(self, other: "Resource") -> None:
        self.milli_cpu += other.milli_cpu
        self.memory += other.memory
        self.ephemeral_storage += other.ephemeral_storage
        self.allowed_pod_number += other.allowed_pod_number
        for k, v in other.scalar.items():
            self.scalar[k] = self.scalar.get(k, 0) + v

    def isub(self, other: "Resource") -> None:
        self.milli_cpu -= other.milli_cpu
        self.memory -= other.memory
        self.ephemeral_storage -= other.ephemeral_storage
        self.allowed_pod_number -= other.allowed_pod_number
        for k, v in other.scalar.items():
            self.scalar[k] = self.scalar.get(k, 0) - v

    def is_zero(self) -> bool:
        return not (self.milli_cpu or self.memory or self.ephemeral_storage or self.allowed_pod_number
                    or any(self.scalar.values()))

    def __repr__(self) -> str:
        sc = ",".join(f"{k}={v}" for k, v in sorted(self.scalar.items()) if v)
        return f"Resource(cpu={self.milli_cpu}m,mem={self.memory},pods={self.allowed_pod_number}" + \
            (f",{sc}" if sc else "") + ")"


_memo = threading.local()


@contextlib.contextmanager
def request_memo():
    """Memoise :func:`compute_pod_request` per pod object for the duration of
    the block (this thread only).  The planner evaluates the same pods
    thousands of times per plan; their specs do not change inside a plan.
    Keys are object ids, valid because the pods stay referenced by the caller
    for the whole block."""
    prev = getattr(_memo, "d", None)
    _memo.d = {} if prev is None else prev
    try:
        yield
    finally:
        _memo.d = prev


def compute_pod_request(pod: dict) -> dict[str, Fraction]:
    """max(sum(containers) + overhead, max(init containers)) as a ResourceList."""
    memo = getattr(_memo, "d", None)
    if memo is not None:
        hit = memo.get(id(pod))
        if hit is not None and hit[0] is pod:
            return dict(hit[1])
        out = _compute_pod_request(pod)
        memo[id(pod)] = (pod, out)
        return dict(out)
    return _compute_pod_request(pod)


def _compute_pod_request(pod: dict) -> dict[str, Fraction]:
    containers: dict[str, Fraction] = {}
    for c in ko.pod_containers(pod):
        containers = q.rl_add(containers, ko.container_requests(c))
    init: dict[str, Fraction] = {}
    for c in ko.pod_init_containers(pod):
        init = q.rl_max(init, ko.container_requests(c))
    overhead = ko.pod_overhead(pod)
    if overhead:
        containers = q.rl_add(containers, overhead)  # applied (the reference drops it)
    return q.rl_max(containers, init)


def pod_request_resource(pod: dict) -> Resource:
    return Resource.from_list(compute_pod_request(pod))


class Calculator(Protocol):
    """``resource.Calculator`` (pkg/resource/resource.go:30-32)."""

    def compute_pod_request(self, pod: dict) -> dict[str, Fraction]: ...


class DefaultCalculator:
    def compute_pod_request(self, pod: dict) -> dict[str, Fraction]:
        return compute_pod_request(pod)
