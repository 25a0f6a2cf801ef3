"""Shared plumbing of the nos-amd binaries (``cmd/*/*.go`` main()s of the
reference): flags, config file, API connection, health/readiness and
Prometheus endpoints, signal handling."""
from __future__ import annotations

import argparse
import logging
import os
import signal
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable

log = logging.getLogger("nos_amd.cmd")


def parser(description: str, config_help: str = "component config file (YAML)") -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=description)
    ap.add_argument("--config", default="", help=config_help)
    ap.add_argument("--api-server", default="", help="API server URL (default: in-cluster / kubeconfig)")
    ap.add_argument("--kubeconfig", default="", help="kubeconfig path")
    ap.add_argument("--health-probe-bind-address", default="", help="override health.healthProbeBindAddress")
    ap.add_argument("--metrics-bind-address", default="", help="override metrics.bindAddress ('0' disables)")
    ap.add_argument("--log-level", default="", help="debug|info|warning|error")
    return ap


def setup_logging(level: str) -> None:
    logging.basicConfig(level=getattr(logging, (level or "info").upper(), logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")


def connect(args):
    from ..kube.client import KubeClient

    return KubeClient.from_env(args.kubeconfig or None, args.api_server or None)


def node_name() -> str:
    from ..api import constants as C

    n = os.environ.get(C.ENV_NODE_NAME)
    if not n:
        raise SystemExit(f"{C.ENV_NODE_NAME} environment variable is required")
    return n


def _split(addr: str) -> tuple[str, int]:
    host, _, port = addr.rpartition(":")
    return host or "0.0.0.0", int(port)


def serve_health(addr: str, healthz: Callable[[], bool], readyz: Callable[[], bool]) -> ThreadingHTTPServer | None:
    """``/healthz`` and ``/readyz`` (controller-runtime ``healthz.Ping`` on :8081)."""
    if not addr or addr == "0":
        return None

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):  # noqa: N802
            fn = {"/healthz": healthz, "/readyz": readyz}.get(self.path)
            ok = bool(fn and fn())
            body = b"ok" if ok else b"not ok"
            self.send_response(200 if ok else (404 if fn is None else 500))
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

    srv = ThreadingHTTPServer(_split(addr), H)
    threading.Thread(target=srv.serve_forever, daemon=True, name="health").start()
    log.info("health probes on %s", addr)
    return srv


def serve_metrics(addr: str) -> None:
    if not addr or addr == "0":
        return
    from ..observability.metrics import serve

    host, port = _split(addr)
    serve(port)
    log.info("metrics on :%d", port)


def run_until_signal(stop: Callable[[], None], lost: threading.Event | None = None) -> int:
    """Run until SIGTERM/SIGINT (exit 0) or until ``lost`` fires -- the leader
    lease was lost -- then stop and return 1 so the process exits non-zero
    and its supervisor restarts it as a follower (controller-runtime's
    behaviour; never re-exec in place)."""
    ev = threading.Event()

    def _h(signum, frame):
        log.info("received signal %d, shutting down", signum)
        ev.set()

    signal.signal(signal.SIGTERM, _h)
    signal.signal(signal.SIGINT, _h)
    while not ev.wait(0.5):
        if lost is not None and lost.is_set():
            log.error("leader election lost, exiting")
            stop()
            return 1
    stop()
    return 0


def load_config(path: str, kind: str):
    from ..api import config

    if not path:
        return config.KINDS[kind]()
    return config.load(path, kind)


def apply_overrides(cfg, args) -> None:
    if args.health_probe_bind_address:
        cfg.health.health_probe_bind_address = args.health_probe_bind_address
    if args.metrics_bind_address:
        cfg.metrics.bind_address = args.metrics_bind_address
    setup_logging(args.log_level or cfg.log_level)


def manager_for(api, name: str, cfg):
    from ..runtime.manager import Manager

    le = cfg.leader_election
    return Manager(api, name, leader_election=le.leader_elect, leader_election_id=le.resource_name or name,
                   leader_election_namespace=le.resource_namespace, resync_s=300.0)
