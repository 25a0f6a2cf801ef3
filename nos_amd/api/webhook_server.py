"""Validating admission webhooks served by the operator
(``pkg/api/nos.nebuly.com/v1alpha1/*_webhook.go``, kubebuilder paths).

``POST /validate-nos-nebuly-com-v1alpha1-elasticquota`` and
``/validate-nos-nebuly-com-v1alpha1-compositeelasticquota`` take an
``admission.k8s.io/v1`` AdmissionReview and answer allowed / denied (403)
with the same rules the in-process API server applies
(:func:`nos_amd.api.v1alpha1.register_webhooks`).  TLS when a cert dir is
given (``tls.crt``/``tls.key``, the cert-manager secret layout).
"""
from __future__ import annotations

import json
import logging
import ssl
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path

from . import v1alpha1

log = logging.getLogger("nos_amd.webhook")

EQ_PATH = "/validate-nos-nebuly-com-v1alpha1-elasticquota"
CEQ_PATH = "/validate-nos-nebuly-com-v1alpha1-compositeelasticquota"


def review(api, path: str, req: dict) -> dict:
    """AdmissionReview request -> response object."""
    r = req.get("request") or {}
    uid = r.get("uid", "")
    op = r.get("operation", "")
    obj = r.get("object") or {}
    allowed, message = True, ""
    try:
        if path == EQ_PATH:
            if op == "CREATE":
                v1alpha1.validate_eq_create(obj, api.list(v1alpha1.KIND_EQ, obj.get("metadata", {}).get("namespace")),
                                            api.list(v1alpha1.KIND_CEQ))
            elif op == "UPDATE":
                v1alpha1.validate_min_max(obj)
        elif path == CEQ_PATH:
            if op in ("CREATE", "UPDATE"):
                v1alpha1.validate_ceq(obj, api.list(v1alpha1.KIND_CEQ))
        else:
            allowed, message = False, f"unknown webhook path {path}"
    except v1alpha1.ValidationError as e:
        allowed, message = False, str(e)
    resp: dict = {"uid": uid, "allowed": allowed}
    if not allowed:
        resp["status"] = {"code": 403, "reason": "Forbidden", "message": message}
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}


class WebhookServer(ThreadingHTTPServer):
    daemon_threads = True

    def __init__(self, api, host: str = "0.0.0.0", port: int = 9443, cert_dir: str | None = None):
        outer = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_POST(self):  # noqa: N802
                n = int(self.headers.get("Content-Length") or 0)
                try:
                    body = json.dumps(review(outer.api, self.path, json.loads(self.rfile.read(n) or b"{}")))
                    code = 200
                except Exception as e:  # malformed review
                    body, code = json.dumps({"error": str(e)}), 400
                data = body.encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

        super().__init__((host, port), H)
        self.api = api
        if cert_dir:
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(str(Path(cert_dir) / "tls.crt"), str(Path(cert_dir) / "tls.key"))
            self.socket = ctx.wrap_socket(self.socket, server_side=True)

    def start(self) -> "WebhookServer":
        threading.Thread(target=self.serve_forever, daemon=True, name="webhook").start()
        return self
