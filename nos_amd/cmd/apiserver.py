"""Simulated Kubernetes API server for local multi-process runs (the
reference's kind cluster, ``hack/kind/cluster.yaml``): the in-process
:class:`~nos_amd.sim.apiserver.ApiServer` (CRDs + validating webhooks
registered) behind its Kubernetes-compatible HTTP front end.  The store can
be checkpointed to a JSON file and restored on start.

python -m nos_amd.cmd.apiserver --port 6443 [--state state.json]
"""
from __future__ import annotations

import argparse
import logging
import threading
from pathlib import Path

from . import common

log = logging.getLogger("nos_amd.cmd.apiserver")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=6443)
    ap.add_argument("--token", default="", help="require this bearer token")
    ap.add_argument("--state", default="", help="JSON checkpoint file (restored on start, saved periodically)")
    ap.add_argument("--save-interval", type=float, default=10.0)
    ap.add_argument("--log-level", default="info")
    args = ap.parse_args(argv)
    common.setup_logging(args.log_level)
    from ..api import constants as C
    from ..api import v1alpha1
    from ..kube import factory as kf
    from ..sim.apiserver import ApiServer
    from ..sim.http import ApiHTTPServer

    api = ApiServer()
    v1alpha1.register_types(api)
    state = Path(args.state) if args.state else None
    if state and state.exists():
        api.restore(state.read_text())
        log.info("restored %s", state)
    for ns in ("default", "kube-system", C.DEFAULT_DEVICE_PLUGIN_CM_NAMESPACE):
        if api.try_get("Namespace", ns) is None:
            api.create(kf.build_namespace(ns).get())
    srv = ApiHTTPServer(api, args.host, args.port, args.token or None).start()
    log.info("API server on %s", srv.url)
    stop = threading.Event()

    def saver():
        while not stop.wait(args.save_interval):
            state.write_text(api.snapshot())

    if state:
        threading.Thread(target=saver, daemon=True).start()

    def shutdown():
        stop.set()
        if state:
            state.write_text(api.snapshot())
        srv.stop()

    common.run_until_signal(shutdown)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
