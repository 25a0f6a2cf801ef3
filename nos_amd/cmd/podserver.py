"""nos-amd pod server (the MPS control daemon's role): one process per GPU that
runs the inferences of every fractional pod the device plugin placed on that
GPU's pod-server slices.  The pods stay CPU-only and reach it through
``<socket-dir>/gpu-<index>.sock`` (nos_amd/podserver/server.py).

python -m nos_amd.cmd.podserver --gpu 0 --socket-dir /run/nos-amd/podserver --lanes 8
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading
from pathlib import Path

MAX_HW_QUEUES = 32


def socket_path(socket_dir: str | os.PathLike, gpu: int) -> Path:
    return Path(socket_dir) / f"gpu-{gpu}.sock"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpu", type=int, default=0, help="host GPU index (HIP_VISIBLE_DEVICES unless already set)")
    ap.add_argument("--socket-dir", default="")
    ap.add_argument("--socket", default="", help="explicit socket path (default <socket-dir>/gpu-<gpu>.sock)")
    ap.add_argument("--lanes", type=int, default=8, help="streams = hardware queues the tenants are served on")
    ap.add_argument("--max-tenants", type=int, default=48)
    ap.add_argument("--memory-gb", type=float, default=0.0, help="slice memory the server admits (0 = the GPU's)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--no-graphs", action="store_true")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    # before anything initialises HIP: the GPU, and one hardware queue per lane
    if args.device == "cuda":
        os.environ.setdefault("HIP_VISIBLE_DEVICES", str(args.gpu))
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(MAX_HW_QUEUES, max(args.lanes, 1)))
    from ..api import constants as C
    from ..podserver.server import PodServer

    path = args.socket or socket_path(args.socket_dir or C.DEFAULT_POD_SERVER_SOCKET_DIR, args.gpu)
    srv = PodServer(path, device=args.device, lanes=args.lanes, max_tenants=args.max_tenants,
                    memory_gb=args.memory_gb or None, graphs=not args.no_graphs).start()
    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    print(f"[podserver] ready on {path} ({srv.info})", file=sys.stderr, flush=True)
    while not stop.wait(1.0):
        pass
    srv.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
