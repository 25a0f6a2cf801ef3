"""Kubernetes-compatible HTTP front end for :class:`~nos_amd.sim.apiserver.ApiServer`.

Lets the nos-amd binaries (``python -m nos_amd.cmd.*``) run as separate
processes against the simulator exactly as they would against a real
kube-apiserver -- the same REST client, paths, verbs, status codes, merge
patches, ``status``/``binding`` subresources and chunked watch streams
(``?watch=true&resourceVersion=N``).  This is the "kind cluster" of the
reference's dev loop (``hack/kind/cluster.yaml``) without Kubernetes.

Standard library only (``http.server``): one thread per connection.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

from ..kube import objects as ko
from ..kube.rest import parse_path, status_body
from .apiserver import ApiError, ApiServer, Expired, Invalid, NotFound

log = logging.getLogger("nos_amd.sim.http")


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    disable_nagle_algorithm = True  # headers and body go out as separate writes
    server: "ApiHTTPServer"

    def log_message(self, fmt, *args):  # quiet
        log.debug("%s - " + fmt, self.address_string(), *args)

    # ------------------------------------------------------------ helpers
    def _send(self, code: int, body: dict) -> None:
        data = json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _error(self, e: ApiError) -> None:
        self._send(e.code, status_body(e.code, e.reason, str(e)))

    def _body(self) -> dict:
        n = int(self.headers.get("Content-Length") or 0)
        return json.loads(self.rfile.read(n) or b"{}") if n else {}

    def _resolve(self):
        api: ApiServer = self.server.api
        u = urlparse(self.path)
        plurals = {t.plural for t in api._types.values()}
        r = parse_path(u.path, plurals)
        if r is None:
            raise NotFound(f"no route for {u.path}")
        for t in api._types.values():
            if t.plural == r.plural and t.api_version == r.api_version:
                return t, r, {k: v[-1] for k, v in parse_qs(u.query).items()}
        raise NotFound(f"the server could not find the requested resource {r.api_version}/{r.plural}")

    def _auth(self) -> bool:
        tok = self.server.token
        if tok and self.headers.get("Authorization") != f"Bearer {tok}":
            self._send(401, status_body(401, "Unauthorized", "Unauthorized"))
            return False
        return True

    # ------------------------------------------------------------ verbs
    def do_GET(self):  # noqa: N802
        if self.path in ("/healthz", "/readyz", "/livez"):
            data = b"ok"
            self.send_response(200)
            self.send_header("Content-Length", "2")
            self.end_headers()
            self.wfile.write(data)
            return
        if self.path == "/version":
            self._send(200, {"major": "1", "minor": "29", "gitVersion": "v1.29.0-nos-amd-sim"})
            return
        if not self._auth():
            return
        api: ApiServer = self.server.api
        try:
            t, r, q = self._resolve()
            if r.name:
                self._send(200, api.get(t.kind, r.name, r.namespace))
                return
            if q.get("watch") in ("true", "1"):
                self._watch(t, r, q)
                return
            items, rv = api.list_with_version(t.kind, r.namespace, q.get("labelSelector") or None,
                                              q.get("fieldSelector") or None)
            self._send(200, {"kind": f"{t.kind}List", "apiVersion": t.api_version,
                             "metadata": {"resourceVersion": rv}, "items": items})
        except ApiError as e:
            self._error(e)

    def _watch(self, t, r, q) -> None:
        api: ApiServer = self.server.api
        timeout = float(q.get("timeoutSeconds") or 1800)
        try:
            w = api.watch(t.kind, r.namespace, q.get("labelSelector") or None, q.get("fieldSelector") or None,
                          send_initial=q.get("sendInitialEvents") == "true",
                          resource_version=q.get("resourceVersion") or None)
        except Expired as e:
            self._error(e)
            return
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()
        # wall-clock deadlines: the API clock may be a fake one
        deadline = time.monotonic() + timeout
        last = time.monotonic()
        try:
            while not self.server.stopping.is_set() and time.monotonic() < deadline:
                ev = w.next(timeout=0.5)
                if ev is None:
                    if time.monotonic() - last < self.server.heartbeat_s:
                        continue
                    # BOOKMARK heartbeat: advances the client's resourceVersion and
                    # detects clients that went away
                    body = {"type": "BOOKMARK", "object": {"kind": t.kind, "apiVersion": t.api_version,
                                                           "metadata": {"resourceVersion":
                                                                        api.current_resource_version()}}}
                else:
                    body = {"type": ev.type, "object": ev.object}
                line = json.dumps(body).encode() + b"\n"
                self.wfile.write(b"%x\r\n%s\r\n" % (len(line), line))
                self.wfile.flush()
                last = time.monotonic()
            self.wfile.write(b"0\r\n\r\n")
        except (BrokenPipeError, ConnectionResetError):
            pass
        finally:
            w.stop()
        self.close_connection = True

    def do_POST(self):  # noqa: N802
        if not self._auth():
            return
        api: ApiServer = self.server.api
        try:
            t, r, _ = self._resolve()
            body = self._body()
            if r.name and r.subresource == "binding" and t.kind == "Pod":
                target = (body.get("target") or {}).get("name")
                if not target:
                    raise Invalid("binding target name required")
                api.bind(r.name, r.namespace, target)
                self._send(201, {"kind": "Status", "apiVersion": "v1", "status": "Success", "code": 201})
                return
            if r.name:
                raise Invalid("POST on an item")
            body.setdefault("kind", t.kind)
            body.setdefault("apiVersion", t.api_version)
            if t.namespaced and r.namespace:
                ko.meta(body)["namespace"] = r.namespace
            self._send(201, api.create(body))
        except ApiError as e:
            self._error(e)

    def do_PUT(self):  # noqa: N802
        if not self._auth():
            return
        api: ApiServer = self.server.api
        try:
            t, r, _ = self._resolve()
            body = self._body()
            body.setdefault("kind", t.kind)
            if r.subresource == "status":
                self._send(200, api.update_status(body))
            else:
                self._send(200, api.update(body))
        except ApiError as e:
            self._error(e)

    def do_PATCH(self):  # noqa: N802
        if not self._auth():
            return
        api: ApiServer = self.server.api
        try:
            t, r, _ = self._resolve()
            ctype = (self.headers.get("Content-Type") or "").split(";")[0]
            if ctype not in ("application/merge-patch+json", "application/strategic-merge-patch+json",
                             "application/json"):
                raise Invalid(f"unsupported patch type {ctype}")
            self._send(200, api.patch(t.kind, r.name, self._body(), r.namespace, subresource=r.subresource))
        except ApiError as e:
            self._error(e)

    def do_DELETE(self):  # noqa: N802
        if not self._auth():
            return
        api: ApiServer = self.server.api
        try:
            t, r, _ = self._resolve()
            self._send(200, api.delete(t.kind, r.name, r.namespace))
        except ApiError as e:
            self._error(e)


class ApiHTTPServer(ThreadingHTTPServer):
    daemon_threads = True

    def __init__(self, api: ApiServer, host: str = "127.0.0.1", port: int = 0, token: str | None = None):
        super().__init__((host, port), _Handler)
        self.api = api
        self.token = token
        self.heartbeat_s = 10.0
        self.stopping = threading.Event()
        self._thread: threading.Thread | None = None

    @property
    def url(self) -> str:
        host, port = self.server_address[:2]
        return f"http://{host}:{port}"

    def start(self) -> "ApiHTTPServer":
        self._thread = threading.Thread(target=self.serve_forever, daemon=True, name="apiserver-http")
        self._thread.start()
        return self

    def stop(self) -> None:
        self.stopping.set()
        self.shutdown()
        self.server_close()


def serve(api: ApiServer, host: str = "127.0.0.1", port: int = 0, token: str | None = None) -> ApiHTTPServer:
    return ApiHTTPServer(api, host, port, token).start()
