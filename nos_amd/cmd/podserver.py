"""nos-amd pod server (the MPS control daemon's role): one process per GPU that
runs the inferences of every fractional pod the device plugin placed on that
GPU's pod-server slices.  The pods stay CPU-only and reach it through
``<socket-dir>/gpu-<index>/server.sock`` (nos_amd/podserver/server.py) and
register with the allocation token the device plugin gave them; the server
reads the slice from the plugin's record under
``<socket-dir>/.allocations/gpu-<index>/`` (podserver/allocations.py).

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
    """``<socket-dir>/gpu-<i>/server.sock`` (the per-GPU directory is what a
    slice pod mounts; podserver/allocations.py)."""
    from ..podserver.allocations import socket_path as sp

    return sp(socket_dir, gpu)


def _gpu_indices(spec: str, smi=None) -> list[tuple[int, int]]:
    """(amd-smi index, HIP id) of ``all`` GPUs (read without initialising
    HIP) or of a comma list of amd-smi indices.  HIP numbering can differ
    from amd-smi's (enumeration order, partitions): the device plugin
    allocates slices by amd-smi index, so the server of socket gpu-<i> must
    run on GPU i's HIP id (``GpuInfo.hip_id``)."""
    want = None if spec == "all" else [int(v) for v in spec.split(",") if v.strip()]
    try:
        if smi is None:
            from ..gpu.amdsmi import AmdSmi

            smi = AmdSmi.real()
        hip = {g.index: (g.hip_id if g.hip_id >= 0 else g.index) for g in smi.gpus()}
    except Exception:  # no amd-smi (CPU rehearsal): HIP ids = indices
        if want is None:
            raise
        hip = {}
    return [(i, hip.get(i, i)) for i in (sorted(hip) if want is None else want)]


def supervise(gpus: list[tuple[int, int]], argv: list[str], metrics_port: int = 0, restart_s: float = 2.0) -> int:
    """One server process per GPU, restarted when it dies (the DaemonSet pod's
    entry point).  This process never touches the GPU, so starting the
    servers from it is safe.  ``gpus``: (amd-smi index, HIP id) pairs."""
    import subprocess
    import time

    hip_of = dict(gpus)

    def start(g):
        port = ["--metrics-port", str(metrics_port + g)] if metrics_port else []
        return subprocess.Popen([sys.executable, "-m", "nos_amd.cmd.podserver", "--gpu", str(g),
                                 "--hip-id", str(hip_of[g])] + argv + port)

    procs = {g: start(g) for g, _ in gpus}
    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    while not stop.wait(1.0):
        for g, p in list(procs.items()):
            if p.poll() is not None:
                logging.getLogger("nos_amd.podserver").warning("server of GPU %d exited (%s): restarting", g, p.returncode)
                time.sleep(restart_s)
                procs[g] = start(g)
    for p in procs.values():
        p.terminate()
    for p in procs.values():
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            p.kill()
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpu", type=int, default=0, help="amd-smi GPU index (names the socket and the records)")
    ap.add_argument("--hip-id", type=int, default=-1,
                    help="the GPU's HIP id (HIP_VISIBLE_DEVICES; default: --gpu unless HIP_VISIBLE_DEVICES is set)")
    ap.add_argument("--gpus", default="", help="'all' or a comma list: supervise one server per GPU")
    ap.add_argument("--log-level", default="info")
    ap.add_argument("--socket-dir", default="")
    ap.add_argument("--socket", default="", help="explicit socket path (default <socket-dir>/gpu-<gpu>/server.sock)")
    ap.add_argument("--lanes", type=int, default=16, help="streams = hardware queues the tenants are served on")
    ap.add_argument("--priority-lanes", type=int, default=0,
                    help="lanes serving only the latency tenants (stateful decoders); every lane takes latency "
                         "requests first")
    ap.add_argument("--latency-cus", type=int, default=0,
                    help="CUs (multiple of 8, XCD-symmetric) reserved for the priority lanes; the other lanes' streams "
                         "are CU-masked to the rest")
    ap.add_argument("--masked-queues", type=int, default=8,
                    help="with --latency-cus: CU-masked streams (hardware queues) the throughput lanes share")
    ap.add_argument("--max-tenants", type=int, default=48)
    ap.add_argument("--memory-gb", type=float, default=0.0, help="slice memory the server admits (0 = the GPU's)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-solo-graphs", action="store_true",
                    help="no second graph per tenant under the whole-GPU kernel configs (replayed when it runs alone)")
    ap.add_argument("--metrics-port", type=int, default=0,
                    help="Prometheus /metrics of this server (supervisor: port + GPU index; 0 = off)")
    ap.add_argument("--open-admission", action="store_true",
                    help="no allocation tokens: clients declare their slice (tests, bare metal)")
    ap.add_argument("--pod-resources-socket", default="",
                    help="kubelet PodResources socket: evict tenants whose devices no pod holds")
    args = ap.parse_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    if args.gpus:
        rest = ["--socket-dir", args.socket_dir, "--lanes", str(args.lanes), "--priority-lanes",
                str(args.priority_lanes), "--latency-cus", str(args.latency_cus), "--masked-queues", str(args.masked_queues), "--max-tenants", str(args.max_tenants),
                "--memory-gb", str(args.memory_gb), "--device", args.device, "--log-level", args.log_level]
        if args.no_graphs:
            rest.append("--no-graphs")
        if args.no_solo_graphs:
            rest.append("--no-solo-graphs")
        if args.open_admission:
            rest.append("--open-admission")
        if args.pod_resources_socket:
            rest += ["--pod-resources-socket", args.pod_resources_socket]
        return supervise(_gpu_indices(args.gpus), rest, args.metrics_port)
    # before anything initialises HIP: the GPU, and one hardware queue per lane
    if args.device == "cuda":
        if args.hip_id >= 0:
            os.environ["HIP_VISIBLE_DEVICES"] = str(args.hip_id)
        os.environ.setdefault("HIP_VISIBLE_DEVICES", str(args.gpu))
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(MAX_HW_QUEUES, max(args.lanes + args.priority_lanes, 1)))
    from ..api import constants as C
    from ..podserver.allocations import records_dir
    from ..podserver.server import PodServer

    root = args.socket_dir or C.DEFAULT_POD_SERVER_SOCKET_DIR
    path = args.socket or socket_path(root, args.gpu)
    records = None if args.open_admission else records_dir(root, args.gpu)
    lister = None
    if args.pod_resources_socket:
        from ..resource.podresources_grpc import GrpcLister

        lister = GrpcLister(args.pod_resources_socket)
    srv = PodServer(path, device=args.device, lanes=args.lanes, priority_lanes=args.priority_lanes,
                    latency_cus=args.latency_cus, masked_queues=args.masked_queues,
                    max_tenants=args.max_tenants,
                    memory_gb=args.memory_gb or None, graphs=not args.no_graphs,
                    solo_graphs=not args.no_solo_graphs, allocations_dir=records, pod_resources=lister).start()
    if args.metrics_port:
        from ..observability import metrics

        metrics.serve(args.metrics_port)
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
