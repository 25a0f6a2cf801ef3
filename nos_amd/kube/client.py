"""Kubernetes REST client with the interface of the in-process
:class:`~nos_amd.sim.apiserver.ApiServer`.

Every nos-amd component talks to "an API server" through the same methods
(``get/try_get/list/create/update/update_status/patch/delete/bind/watch``),
so the same controllers run in-process on the simulator or as separate
processes against a real kube-apiserver (in-cluster service account) or the
simulator's HTTP front end (:mod:`nos_amd.sim.http`).

Watches are client-side reflectors: list, then watch from the list's
``resourceVersion``; reconnect from the last seen version; on 410 Gone
re-list and emit the difference.  Like client-go informers they keep a cache
so MODIFIED/DELETED events carry the previous object (``ev.old``), which the
controllers' predicates rely on.
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from pathlib import Path
from typing import Callable

import requests
import yaml

from ..sim.apiserver import (ADDED, CORE_TYPES, DELETED, ERRORS_BY_REASON, MODIFIED, ApiError, Expired, NotFound,
                             ResourceType, WatchEvent)
from ..utils.clock import RealClock
from . import objects as ko
from .rest import path_for

log = logging.getLogger("nos_amd.kube.client")

SA_DIR = Path("/var/run/secrets/kubernetes.io/serviceaccount")


def _nos_types() -> list[ResourceType]:
    from ..api import constants as C

    return [ResourceType(C.API_VERSION, "ElasticQuota", "elasticquotas"),
            ResourceType(C.API_VERSION, "CompositeElasticQuota", "compositeelasticquotas")]


class KubeClient:
    def __init__(self, server: str, token: str | None = None, verify: bool | str = True,
                 cert: tuple[str, str] | None = None, timeout: float = 30.0):
        self.server = server.rstrip("/")
        self.token = token
        self.verify = verify
        self.cert = cert
        self.timeout = timeout
        self.clock = RealClock()
        self._types = {t.kind: t for t in CORE_TYPES + _nos_types()}
        self._local = threading.local()
        self._watches: list[ClientWatch] = []

    # ------------------------------------------------------------ construction
    @classmethod
    def from_env(cls, kubeconfig: str | None = None, server: str | None = None) -> "KubeClient":
        """``server`` / ``$NOS_AMD_API_SERVER`` > in-cluster service account >
        kubeconfig (``--kubeconfig`` / ``$KUBECONFIG`` / ``~/.kube/config``)."""
        server = server or os.environ.get("NOS_AMD_API_SERVER")
        if server:
            return cls(server, token=os.environ.get("NOS_AMD_API_TOKEN"))
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if host and port and (SA_DIR / "token").exists():
            return cls(f"https://{host}:{port}", token=(SA_DIR / "token").read_text().strip(),
                       verify=str(SA_DIR / "ca.crt"))
        path = Path(kubeconfig or os.environ.get("KUBECONFIG") or Path.home() / ".kube" / "config")
        if not path.exists():
            raise RuntimeError("no API server: pass --api-server, run in-cluster or provide a kubeconfig")
        return cls.from_kubeconfig(path)

    @classmethod
    def from_kubeconfig(cls, path: str | Path) -> "KubeClient":
        cfg = yaml.safe_load(Path(path).read_text())
        ctx_name = cfg.get("current-context")
        ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in cfg.get("users", []) if u["name"] == ctx.get("user")), {})
        verify: bool | str = not cluster.get("insecure-skip-tls-verify", False)
        if cluster.get("certificate-authority"):
            verify = cluster["certificate-authority"]
        cert = (user["client-certificate"], user["client-key"]) if user.get("client-certificate") else None
        return cls(cluster["server"], token=user.get("token"), verify=verify, cert=cert)

    # ------------------------------------------------------------ plumbing
    def _session(self) -> requests.Session:
        s = getattr(self._local, "s", None)
        if s is None:
            s = requests.Session()
            s.verify = self.verify
            if self.cert:
                s.cert = self.cert
            if self.token:
                s.headers["Authorization"] = f"Bearer {self.token}"
            self._local.s = s
        return s

    def register_type(self, t: ResourceType) -> None:
        self._types[t.kind] = t

    def register_field_indexer(self, *a, **k) -> None:  # server-side concern
        pass

    def register_admission(self, *a, **k) -> None:  # webhooks run in the API server
        pass

    def type_of(self, kind: str) -> ResourceType:
        t = self._types.get(kind)
        if t is None:
            raise NotFound(f"unknown kind {kind}")
        return t

    def _url(self, kind: str, namespace: str | None = None, name: str | None = None, sub: str | None = None) -> str:
        t = self.type_of(kind)
        ns = (namespace or "default") if (t.namespaced and name) else namespace
        return self.server + path_for(t.api_version, t.plural, t.namespaced, ns, name, sub)

    @staticmethod
    def _raise(resp: requests.Response) -> None:
        if resp.status_code < 400:
            return
        try:
            body = resp.json()
        except ValueError:
            body = {"reason": "InternalError", "message": resp.text}
        cls = ERRORS_BY_REASON.get(body.get("reason", ""), ApiError)
        if cls is ApiError and resp.status_code == 404:
            cls = NotFound
        err = cls(body.get("message", resp.reason))
        err.code = resp.status_code
        raise err

    def _req(self, method: str, url: str, **kw) -> dict:
        r = self._session().request(method, url, timeout=self.timeout, **kw)
        self._raise(r)
        return r.json() if r.content else {}

    # ------------------------------------------------------------ CRUD
    def get(self, kind: str, name: str, namespace: str | None = None) -> dict:
        return self._req("GET", self._url(kind, namespace, name))

    def try_get(self, kind: str, name: str, namespace: str | None = None) -> dict | None:
        try:
            return self.get(kind, name, namespace)
        except NotFound:
            return None

    def list_with_version(self, kind: str, namespace: str | None = None, label_selector=None,
                          field_selector: str | None = None) -> tuple[list[dict], str]:
        params = {}
        if label_selector:
            params["labelSelector"] = label_selector if isinstance(label_selector, str) else \
                ",".join(f"{k}={v}" for k, v in label_selector.items())
        if field_selector:
            params["fieldSelector"] = field_selector
        body = self._req("GET", self._url(kind, namespace), params=params)
        items = body.get("items") or []
        t = self.type_of(kind)
        for o in items:  # list items omit kind/apiVersion on a real server
            o.setdefault("kind", kind)
            o.setdefault("apiVersion", t.api_version)
        return items, (body.get("metadata") or {}).get("resourceVersion", "")

    def list(self, kind: str, namespace: str | None = None, label_selector=None,
             field_selector: str | None = None) -> list[dict]:
        return self.list_with_version(kind, namespace, label_selector, field_selector)[0]

    def create(self, obj: dict) -> dict:
        kind = obj["kind"]
        return self._req("POST", self._url(kind, ko.namespace(obj) or None), json=obj)

    def update(self, obj: dict) -> dict:
        return self._req("PUT", self._url(obj["kind"], ko.namespace(obj) or None, ko.name(obj)), json=obj)

    def update_status(self, obj: dict) -> dict:
        return self._req("PUT", self._url(obj["kind"], ko.namespace(obj) or None, ko.name(obj), "status"), json=obj)

    def patch(self, kind: str, name: str, patch: dict, namespace: str | None = None,
              subresource: str | None = None) -> dict:
        return self._req("PATCH", self._url(kind, namespace, name, subresource), data=json.dumps(patch),
                         headers={"Content-Type": "application/merge-patch+json"})

    def delete(self, kind: str, name: str, namespace: str | None = None) -> dict:
        return self._req("DELETE", self._url(kind, namespace, name))

    def bind(self, pod_name: str, namespace: str, node_name: str) -> dict:
        body = {"apiVersion": "v1", "kind": "Binding", "metadata": {"name": pod_name, "namespace": namespace},
                "target": {"apiVersion": "v1", "kind": "Node", "name": node_name}}
        self._req("POST", self._url("Pod", namespace, pod_name, "binding"), json=body)
        return self.get("Pod", pod_name, namespace)

    # ------------------------------------------------------------ watch
    def watch(self, kind: str, namespace: str | None = None, label_selector=None,
              field_selector: str | None = None, send_initial: bool = True,
              callback: Callable[[WatchEvent], None] | None = None) -> "ClientWatch":
        w = ClientWatch(self, kind, namespace, label_selector, field_selector, send_initial, callback)
        self._watches.append(w)
        w.start()
        return w

    def close(self) -> None:
        for w in self._watches:
            w.stop()


class ClientWatch:
    """A reflector: list + watch with resume, re-list on 410, informer cache."""

    RETRY_S = 1.0
    STREAM_TIMEOUT_S = 300  # server ends each stream after this; the reflector resumes

    def __init__(self, client: KubeClient, kind: str, namespace, label_selector, field_selector, send_initial,
                 callback):
        self.client, self.kind, self.namespace = client, kind, namespace
        self.label_selector, self.field_selector = label_selector, field_selector
        self.send_initial = send_initial
        self.callback = callback
        self.cache: dict[str, dict] = {}
        self.rv = ""
        self.closed = False
        self.synced = threading.Event()
        self._queue: list[WatchEvent] = []
        self._cond = threading.Condition()
        self._thread: threading.Thread | None = None
        self.streams = 0  # watch requests opened (1 + reconnects)

    def start(self) -> None:
        self._relist(initial=True)
        self._thread = threading.Thread(target=self._run, daemon=True, name=f"watch-{self.kind}")
        self._thread.start()

    def _deliver(self, ev: WatchEvent) -> None:
        if self.callback is not None:
            try:
                self.callback(ev)
            except Exception:
                log.exception("watch callback failed (%s)", self.kind)
            return
        with self._cond:
            self._queue.append(ev)
            self._cond.notify_all()

    def _relist(self, initial: bool = False) -> None:
        items, rv = self.client.list_with_version(self.kind, self.namespace, self.label_selector,
                                                  self.field_selector)
        fresh = {ko.key(o): o for o in items}
        events = []
        for k, o in fresh.items():
            old = self.cache.get(k)
            if old is None:
                if not initial or self.send_initial:
                    events.append(WatchEvent(ADDED, o))
            elif ko.resource_version(old) != ko.resource_version(o):
                events.append(WatchEvent(MODIFIED, o, old))
        for k, old in self.cache.items():
            if k not in fresh:
                events.append(WatchEvent(DELETED, old, old))
        self.cache, self.rv = fresh, rv
        for ev in events:
            self._deliver(ev)
        self.synced.set()

    def _run(self) -> None:
        params = {"watch": "true", "allowWatchBookmarks": "true", "timeoutSeconds": str(self.STREAM_TIMEOUT_S)}
        if self.label_selector:
            params["labelSelector"] = self.label_selector if isinstance(self.label_selector, str) else \
                ",".join(f"{k}={v}" for k, v in self.label_selector.items())
        if self.field_selector:
            params["fieldSelector"] = self.field_selector
        while not self.closed:
            try:
                params["resourceVersion"] = self.rv
                r = self.client._session().get(self.client._url(self.kind, self.namespace), params=params,
                                               stream=True, timeout=(self.client.timeout,
                                                                     self.STREAM_TIMEOUT_S + 30))
                self.streams += 1
                if r.status_code == 410:
                    self._relist()
                    continue
                KubeClient._raise(r)
                for line in r.iter_lines():
                    if self.closed:
                        break
                    if not line:
                        continue
                    ev = json.loads(line)
                    if ev.get("type") == "ERROR":
                        if (ev.get("object") or {}).get("code") == 410:
                            self._relist()
                        break
                    self._apply(ev["type"], ev["object"])
            except Expired:
                self._relist()
            except Exception as e:
                if self.closed:
                    break
                log.debug("watch %s interrupted: %s", self.kind, e)
                time.sleep(self.RETRY_S)

    def _apply(self, etype: str, obj: dict) -> None:
        rv = ko.resource_version(obj)
        if etype == "BOOKMARK":
            self.rv = rv or self.rv
            return
        obj.setdefault("kind", self.kind)
        k = ko.key(obj)
        old = self.cache.get(k)
        if etype == DELETED:
            self.cache.pop(k, None)
            ev = WatchEvent(DELETED, obj, old)
        else:
            self.cache[k] = obj
            ev = WatchEvent(MODIFIED if (etype == MODIFIED and old is not None) else etype, obj, old)
        if rv:
            self.rv = rv
        self._deliver(ev)

    # Watch-compatible consumer API
    def next(self, timeout: float | None = None) -> WatchEvent | None:
        with self._cond:
            if not self._queue and not self.closed:
                self._cond.wait(timeout)
            return self._queue.pop(0) if self._queue else None

    def drain(self) -> list[WatchEvent]:
        with self._cond:
            out, self._queue = self._queue, []
            return out

    def stop(self) -> None:
        # the reader thread notices on the next event / heartbeat / stream end
        # (closing the response from here would block on its read lock)
        self.closed = True
        with self._cond:
            self._cond.notify_all()
