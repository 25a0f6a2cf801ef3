"""Event predicates (controller-runtime ``predicate.Funcs`` analogue).

Includes the reference's custom predicates (``pkg/util/predicate/predicates.go:27-76``):
``MatchingName``, ``NodeResourcesChanged``, ``AnnotationsChanged``,
``ExcludeDelete`` -- with the reference bug fixed: its ``NodeResourcesChanged``
returned *false* when the allocatable resources changed (``:51-58``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

from ..kube import objects as ko
from ..kube import quantity as q


@dataclass
class Event:
    type: str          # "create" | "update" | "delete" | "generic"
    obj: dict
    old: dict | None = None


class Predicate:
    def create(self, ev: Event) -> bool:
        return True

    def update(self, ev: Event) -> bool:
        return True

    def delete(self, ev: Event) -> bool:
        return True

    def generic(self, ev: Event) -> bool:
        return True

    def __call__(self, ev: Event) -> bool:
        return getattr(self, ev.type)(ev)


class Funcs(Predicate):
    def __init__(self, create: Callable[[Event], bool] | None = None, update: Callable[[Event], bool] | None = None,
                 delete: Callable[[Event], bool] | None = None, generic: Callable[[Event], bool] | None = None):
        self._c, self._u, self._d, self._g = create, update, delete, generic

    def create(self, ev):
        return self._c(ev) if self._c else True

    def update(self, ev):
        return self._u(ev) if self._u else True

    def delete(self, ev):
        return self._d(ev) if self._d else True

    def generic(self, ev):
        return self._g(ev) if self._g else True


class MatchingName(Predicate):
    def __init__(self, name: str):
        self.name = name

    def _m(self, ev: Event) -> bool:
        return ko.name(ev.obj) == self.name

    create = update = delete = generic = _m


class ExcludeDelete(Predicate):
    def delete(self, ev: Event) -> bool:
        return False


class NodeResourcesChanged(Predicate):
    """Update events pass only when node allocatable/capacity changed (fixed form)."""

    def update(self, ev: Event) -> bool:
        if ev.old is None:
            return True
        return not (q.rl_equal(ko.node_allocatable(ev.old), ko.node_allocatable(ev.obj))
                    and q.rl_equal(ko.node_capacity(ev.old), ko.node_capacity(ev.obj)))


class AnnotationsChanged(Predicate):
    def update(self, ev: Event) -> bool:
        return ev.old is None or ko.annotations(ev.old) != ko.annotations(ev.obj)


class LabelsChanged(Predicate):
    def update(self, ev: Event) -> bool:
        return ev.old is None or ko.labels(ev.old) != ko.labels(ev.obj)


class GenerationChanged(Predicate):
    def update(self, ev: Event) -> bool:
        if ev.old is None:
            return True
        return ev.old.get("metadata", {}).get("generation") != ev.obj.get("metadata", {}).get("generation")


class HasLabel(Predicate):
    def __init__(self, key: str, values: tuple[str, ...] | None = None):
        self.key, self.values = key, values

    def _m(self, ev: Event) -> bool:
        v = ko.labels(ev.obj).get(self.key)
        if v is None and ev.old is not None:
            v = ko.labels(ev.old).get(self.key)
        return v is not None and (self.values is None or v in self.values)

    create = update = delete = generic = _m


def or_(*ps: Predicate) -> Predicate:
    return Funcs(*(lambda ev, n=n: any(getattr(p, n)(ev) for p in ps)
                   for n in ("create", "update", "delete", "generic")))


def and_(*ps: Predicate) -> Predicate:
    return Funcs(*(lambda ev, n=n: all(getattr(p, n)(ev) for p in ps)
                   for n in ("create", "update", "delete", "generic")))
