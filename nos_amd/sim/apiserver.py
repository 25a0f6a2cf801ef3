"""In-process Kubernetes API server (the envtest / kind replacement).

Implements the API-machinery semantics the nos-amd components rely on:

* typed resource registry (core kinds + the nos CRDs), namespaced or not;
* ``resourceVersion`` (one global counter), ``uid``, ``creationTimestamp``,
  ``generation`` (bumped on spec change);
* optimistic concurrency: an update carrying a stale ``resourceVersion``
  fails with 409 Conflict;
* the ``status`` subresource: ``update``/``patch`` ignore status on kinds
  that have one, ``update_status``/``patch(subresource="status")`` change
  only status;
* RFC 7386 JSON merge patch;
* list/watch with label selectors, field selectors and registered field
  indexers (``status.phase``, ``spec.nodeName`` ...), watch streams with
  ADDED/MODIFIED/DELETED events;
* validating admission hooks (the webhooks of ``pkg/api/.../*_webhook.go``);
* pod binding (``pods/binding``) and graceful-delete-free deletion;
* fault injection: forced 409s on write, dropped / delayed watch events;
* JSON snapshot / restore of the whole store (the "API server is the
  checkpoint" design).

Thread-safe (one RLock); watchers receive events on their own queues.
"""
from __future__ import annotations

import collections
import copy
import itertools
import json
import random
import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Iterable

from ..kube import objects as ko
from ..kube import selectors as sel


class ApiError(Exception):
    code = 500
    reason = "InternalError"

    def __init__(self, message: str = ""):
        super().__init__(message or self.reason)


class NotFound(ApiError):
    code, reason = 404, "NotFound"


class AlreadyExists(ApiError):
    code, reason = 409, "AlreadyExists"


class Conflict(ApiError):
    code, reason = 409, "Conflict"


class Invalid(ApiError):
    code, reason = 422, "Invalid"


class Forbidden(ApiError):
    code, reason = 403, "Forbidden"


class Expired(ApiError):
    """410 Gone: a watch asked for a resourceVersion older than the event history."""

    code, reason = 410, "Expired"


ERRORS_BY_REASON = {c.reason: c for c in (NotFound, AlreadyExists, Conflict, Invalid, Forbidden, Expired)}


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, NotFound)


def is_conflict(e: BaseException) -> bool:
    return isinstance(e, Conflict)


@dataclass(frozen=True)
class ResourceType:
    api_version: str
    kind: str
    plural: str
    namespaced: bool = True
    has_status: bool = True


CORE_TYPES = [
    ResourceType("v1", "Pod", "pods"),
    ResourceType("v1", "Node", "nodes", namespaced=False),
    ResourceType("v1", "Namespace", "namespaces", namespaced=False),
    ResourceType("v1", "ConfigMap", "configmaps", has_status=False),
    ResourceType("v1", "Event", "events", has_status=False),
    ResourceType("v1", "Secret", "secrets", has_status=False),
    ResourceType("coordination.k8s.io/v1", "Lease", "leases", has_status=False),
    ResourceType("policy/v1", "PodDisruptionBudget", "poddisruptionbudgets"),
    ResourceType("scheduling.k8s.io/v1", "PriorityClass", "priorityclasses", namespaced=False, has_status=False),
    ResourceType("apps/v1", "DaemonSet", "daemonsets"),
    ResourceType("apiextensions.k8s.io/v1", "CustomResourceDefinition", "customresourcedefinitions",
                 namespaced=False),
]

ADDED, MODIFIED, DELETED = "ADDED", "MODIFIED", "DELETED"


@dataclass
class WatchEvent:
    type: str
    object: dict
    old: dict | None = None


# (operation, new_obj, old_obj, server) -> None or raise Invalid/Forbidden
AdmissionHook = Callable[[str, dict | None, dict | None, "ApiServer"], None]


@dataclass
class Watch:
    kind: str
    namespace: str | None
    label_reqs: list | None
    field_reqs: list
    server: "ApiServer"
    queue: collections.deque = field(default_factory=collections.deque)
    cond: threading.Condition = field(default_factory=threading.Condition)
    closed: bool = False
    callback: Callable[[WatchEvent], None] | None = None

    def matches(self, obj: dict) -> bool:
        if self.namespace and ko.namespace(obj) != self.namespace:
            return False
        if self.label_reqs is not None and not sel.match_labels(self.label_reqs, ko.labels(obj)):
            return False
        return sel.match_fields(self.field_reqs, obj, self.server._indexers.get(self.kind))

    def push(self, ev: WatchEvent) -> None:
        if self.callback is not None:
            self.callback(ev)
            return
        with self.cond:
            self.queue.append(ev)
            self.cond.notify_all()

    def drain(self) -> list[WatchEvent]:
        with self.cond:
            out = list(self.queue)
            self.queue.clear()
            return out

    def next(self, timeout: float | None = None) -> WatchEvent | None:
        with self.cond:
            if not self.queue and not self.closed:
                self.cond.wait(timeout)
            return self.queue.popleft() if self.queue else None

    def stop(self) -> None:
        self.closed = True
        self.server._remove_watch(self)
        with self.cond:
            self.cond.notify_all()


class ApiServer:
    def __init__(self, clock=None, seed: int = 0):
        from ..utils.clock import RealClock

        self.clock = clock or RealClock()
        self._lock = threading.RLock()
        self._types: dict[str, ResourceType] = {}
        self._store: dict[str, dict[str, dict]] = {}
        self._rv = itertools.count(1)
        self._last_rv = 0
        self._watches: list[Watch] = []
        self._hooks: dict[str, list[AdmissionHook]] = collections.defaultdict(list)
        self._indexers: dict[str, dict[str, Callable[[dict], Any]]] = collections.defaultdict(dict)
        self._rng = random.Random(seed)
        self.faults: dict[str, float] = {}  # conflict_on_write, drop_watch_event
        self.request_counts: collections.Counter = collections.Counter()
        # (rv, kind, event) for watches that resume from a resourceVersion
        self._history: collections.deque = collections.deque(maxlen=50000)
        self._history_floor = 0  # events with rv <= floor may have been dropped
        for t in CORE_TYPES:
            self.register_type(t)
        self.register_field_indexer("Pod", "status.phase", ko.pod_phase)
        self.register_field_indexer("Pod", "spec.nodeName", ko.pod_node)
        self.register_field_indexer("Pod", "metadata.name", ko.name)
        self.register_field_indexer("Pod", "metadata.namespace", ko.namespace)

    # ------------------------------------------------------------ registry
    def register_type(self, t: ResourceType) -> None:
        with self._lock:
            self._types[t.kind] = t
            self._store.setdefault(t.kind, {})

    def register_field_indexer(self, kind: str, path: str, fn: Callable[[dict], Any]) -> None:
        self._indexers[kind][path] = fn

    def register_admission(self, kind: str, hook: AdmissionHook) -> None:
        self._hooks[kind].append(hook)

    def type_of(self, kind: str) -> ResourceType:
        t = self._types.get(kind)
        if t is None:
            raise NotFound(f"the server could not find the requested resource kind {kind}")
        return t

    def kinds(self) -> list[str]:
        return list(self._types)

    # ------------------------------------------------------------ helpers
    def _key(self, t: ResourceType, name: str, namespace: str | None) -> str:
        if t.namespaced:
            if not namespace:
                raise Invalid(f"{t.kind} {name}: namespace required")
            return f"{namespace}/{name}"
        return name

    def _next_rv(self) -> str:
        self._last_rv = next(self._rv)
        return str(self._last_rv)

    def _maybe_fault(self, op: str) -> None:
        p = self.faults.get("conflict_on_write", 0.0)
        if p and op in ("update", "patch", "update_status") and self._rng.random() < p:
            raise Conflict("injected conflict")

    def _admit(self, op: str, new: dict | None, old: dict | None, kind: str) -> None:
        for h in self._hooks.get(kind, []):
            h(op, new, old, self)

    def _emit(self, kind: str, etype: str, obj: dict, old: dict | None = None) -> None:
        drop = self.faults.get("drop_watch_event", 0.0)
        # one copy per event, shared read-only by the history and all watchers (informer cache)
        ev = WatchEvent(etype, copy.deepcopy(obj), copy.deepcopy(old) if old else None)
        if len(self._history) == self._history.maxlen:
            self._history_floor = self._history[0][0]
        self._history.append((int(ko.resource_version(obj) or self._last_rv), kind, ev))
        for w in list(self._watches):
            if w.kind != kind or w.closed:
                continue
            if not (w.matches(obj) or (old is not None and w.matches(old))):
                continue
            if drop and self._rng.random() < drop:
                continue
            w.push(ev)

    def _remove_watch(self, w: Watch) -> None:
        with self._lock:
            if w in self._watches:
                self._watches.remove(w)

    # ------------------------------------------------------------ CRUD
    def create(self, obj: dict) -> dict:
        kind = obj.get("kind", "")
        t = self.type_of(kind)
        obj = copy.deepcopy(obj)
        obj.setdefault("apiVersion", t.api_version)
        m = ko.meta(obj)
        if not m.get("name"):
            gn = m.get("generateName")
            if not gn:
                raise Invalid("metadata.name required")
            m["name"] = gn + "%05x" % self._rng.randrange(16 ** 5)
        with self._lock:
            self.request_counts["create"] += 1
            if t.namespaced and not m.get("namespace"):
                m["namespace"] = "default"
            if not t.namespaced:
                m.pop("namespace", None)
            k = self._key(t, m["name"], m.get("namespace"))
            if k in self._store[kind]:
                raise AlreadyExists(f'{kind} "{k}" already exists')
            self._admit("CREATE", obj, None, kind)
            m["uid"] = m.get("uid") or ko.new_uid()
            m.setdefault("creationTimestamp", ko.now_rfc3339(self.clock.now()))
            m["resourceVersion"] = self._next_rv()
            m["generation"] = 1
            m.setdefault("labels", m.get("labels") or {})
            m.setdefault("annotations", m.get("annotations") or {})
            self._store[kind][k] = obj
            self._emit(kind, ADDED, obj)
            return copy.deepcopy(obj)

    def get(self, kind: str, name: str, namespace: str | None = None) -> dict:
        t = self.type_of(kind)
        with self._lock:
            self.request_counts["get"] += 1
            o = self._store[kind].get(self._key(t, name, namespace))
            if o is None:
                raise NotFound(f'{kind} "{namespace + "/" if namespace else ""}{name}" not found')
            return copy.deepcopy(o)

    def try_get(self, kind: str, name: str, namespace: str | None = None) -> dict | None:
        try:
            return self.get(kind, name, namespace)
        except NotFound:
            return None

    def list(self, kind: str, namespace: str | None = None, label_selector: str | dict | None = None,
             field_selector: str | None = None) -> list[dict]:
        t = self.type_of(kind)
        lreqs = self._label_reqs(label_selector)
        freqs = sel.parse_field_selector(field_selector)
        idx = self._indexers.get(kind)
        with self._lock:
            self.request_counts["list"] += 1
            out = []
            for o in self._store[kind].values():
                if t.namespaced and namespace and ko.namespace(o) != namespace:
                    continue
                if lreqs is not None and not sel.match_labels(lreqs, ko.labels(o)):
                    continue
                if freqs and not sel.match_fields(freqs, o, idx):
                    continue
                out.append(copy.deepcopy(o))
            out.sort(key=ko.key)
            return out

    @staticmethod
    def _label_reqs(label_selector):
        if label_selector is None:
            return None
        if isinstance(label_selector, dict):
            if "matchLabels" in label_selector or "matchExpressions" in label_selector:
                return sel.selector_from_object(label_selector)
            return [(k, "=", (v,)) for k, v in label_selector.items()]
        return sel.parse_label_selector(label_selector)

    def _write(self, kind: str, new: dict, status_only: bool, op: str) -> dict:
        t = self.type_of(kind)
        m = ko.meta(new)
        with self._lock:
            self.request_counts[op] += 1
            self._maybe_fault(op)
            k = self._key(t, m.get("name", ""), m.get("namespace"))
            cur = self._store[kind].get(k)
            if cur is None:
                raise NotFound(f'{kind} "{k}" not found')
            rv = m.get("resourceVersion")
            if rv and rv != ko.resource_version(cur):
                raise Conflict(f'Operation cannot be fulfilled on {t.plural} "{k}": the object has been '
                               "modified; please apply your changes to the latest version and try again")
            merged = copy.deepcopy(new)
            if t.has_status:
                if status_only:
                    merged = copy.deepcopy(cur)
                    merged["status"] = copy.deepcopy(new.get("status", {}))
                else:
                    merged["status"] = copy.deepcopy(cur.get("status", {}))
            mm = ko.meta(merged)
            for f in ("uid", "creationTimestamp", "namespace", "name"):
                if f in cur.get("metadata", {}):
                    mm[f] = cur["metadata"][f]
            mm["generation"] = cur["metadata"].get("generation", 1)
            if merged.get("spec") != cur.get("spec"):
                mm["generation"] += 1
            if merged == {**cur, "metadata": {**cur["metadata"], "resourceVersion": mm.get("resourceVersion")}}:
                return copy.deepcopy(cur)  # no-op write: no new resourceVersion, no event
            self._admit("UPDATE", merged, cur, kind)
            mm["resourceVersion"] = self._next_rv()
            self._store[kind][k] = merged
            self._emit(kind, MODIFIED, merged, cur)
            return copy.deepcopy(merged)

    def update(self, obj: dict) -> dict:
        return self._write(obj["kind"], obj, False, "update")

    def update_status(self, obj: dict) -> dict:
        return self._write(obj["kind"], obj, True, "update_status")

    def patch(self, kind: str, name: str, patch: dict, namespace: str | None = None,
              subresource: str | None = None) -> dict:
        with self._lock:
            cur = self.get(kind, name, namespace)
            new = sel.merge_patch(cur, patch)
            ko.meta(new)["resourceVersion"] = ko.resource_version(cur)
            if patch.get("metadata", {}).get("resourceVersion"):
                ko.meta(new)["resourceVersion"] = patch["metadata"]["resourceVersion"]
            return self._write(kind, new, subresource == "status", "patch")

    def delete(self, kind: str, name: str, namespace: str | None = None) -> dict:
        t = self.type_of(kind)
        with self._lock:
            self.request_counts["delete"] += 1
            k = self._key(t, name, namespace)
            cur = self._store[kind].get(k)
            if cur is None:
                raise NotFound(f'{kind} "{k}" not found')
            self._admit("DELETE", None, cur, kind)
            del self._store[kind][k]
            gone = copy.deepcopy(cur)
            ko.meta(gone)["resourceVersion"] = self._next_rv()
            ko.meta(gone)["deletionTimestamp"] = ko.now_rfc3339(self.clock.now())
            self._emit(kind, DELETED, gone)
            if kind == "Namespace":
                for kk, store in self._store.items():
                    if self._types[kk].namespaced:
                        for ok_ in [x for x, o in store.items() if ko.namespace(o) == name]:
                            obj = copy.deepcopy(store.pop(ok_))
                            ko.meta(obj)["resourceVersion"] = self._next_rv()
                            self._emit(kk, DELETED, obj)
            return gone

    def bind(self, pod_name: str, namespace: str, node_name: str) -> dict:
        """pods/binding subresource: sets spec.nodeName once."""
        with self._lock:
            cur = self.get("Pod", pod_name, namespace)
            if ko.pod_node(cur):
                raise Conflict(f"pod {namespace}/{pod_name} is already assigned to node {ko.pod_node(cur)}")
            cur["spec"]["nodeName"] = node_name
            ko.set_condition(cur, "PodScheduled", "True", "", "")
            t = self._types["Pod"]
            k = self._key(t, pod_name, namespace)
            old = self._store["Pod"][k]
            ko.meta(cur)["resourceVersion"] = self._next_rv()
            self._store["Pod"][k] = cur
            self._emit("Pod", MODIFIED, cur, old)
            return copy.deepcopy(cur)

    # ------------------------------------------------------------ watch
    def watch(self, kind: str, namespace: str | None = None, label_selector=None,
              field_selector: str | None = None, send_initial: bool = True,
              callback: Callable[[WatchEvent], None] | None = None,
              resource_version: str | None = None) -> Watch:
        """Open a watch.  With ``resource_version`` the stream resumes after
        that version (events replayed from the history, 410 Expired if they
        were dropped); otherwise ``send_initial`` synthesises ADDED events for
        the current objects, atomically with the registration."""
        self.type_of(kind)
        w = Watch(kind, namespace, self._label_reqs(label_selector), sel.parse_field_selector(field_selector),
                  self, callback=callback)
        with self._lock:
            if resource_version not in (None, ""):  # "0" = from the very beginning (empty store)
                rv = int(resource_version)
                if rv < self._history_floor:
                    raise Expired(f"too old resource version: {rv} ({self._history_floor})")
                for erv, ekind, ev in list(self._history):
                    if erv > rv and ekind == kind and (w.matches(ev.object) or
                                                       (ev.old is not None and w.matches(ev.old))):
                        w.push(ev)
            elif send_initial:
                for o in self.list(kind, namespace, label_selector, field_selector):
                    w.push(WatchEvent(ADDED, o))
            self._watches.append(w)
        return w

    def current_resource_version(self) -> str:
        with self._lock:
            return str(self._last_rv)

    def list_with_version(self, kind: str, namespace: str | None = None, label_selector=None,
                          field_selector: str | None = None) -> tuple[list[dict], str]:
        """List + the resourceVersion to resume a watch from (one atomic step)."""
        with self._lock:
            return self.list(kind, namespace, label_selector, field_selector), str(self._last_rv)

    # ------------------------------------------------------------ checkpoint
    def snapshot(self) -> str:
        with self._lock:
            return json.dumps({"rv": self._last_rv, "store": self._store}, sort_keys=True)

    def restore(self, data: str) -> None:
        d = json.loads(data)
        with self._lock:
            for kind, objs in d["store"].items():
                self._store.setdefault(kind, {}).clear()
                self._store[kind].update(objs)
            self._last_rv = d["rv"]
            self._rv = itertools.count(self._last_rv + 1)

    # ------------------------------------------------------------ convenience
    def apply_all(self, objs: Iterable[dict]) -> list[dict]:
        out = []
        for o in objs:
            try:
                out.append(self.create(o))
            except AlreadyExists:
                cur = self.get(o["kind"], ko.name(o), ko.namespace(o) or None)
                new = copy.deepcopy(o)
                ko.meta(new)["resourceVersion"] = ko.resource_version(cur)
                out.append(self.update(new))
        return out
