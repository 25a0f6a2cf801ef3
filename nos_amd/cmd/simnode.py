"""A simulated GPU node for local multi-process runs: registers a Node with
the API server and runs its kubelet (pod admission through the nos-amd device
plugin, PodResources v1 gRPC on a unix socket for the node agents) over an
in-memory amd-smi backend.  The partition agent / gpuagent / device plugin
binaries can then run against it as separate processes, as on a real node.

python -m nos_amd.cmd.simnode --api-server http://127.0.0.1:6443 --name node-0 \
    --kind cumask --gpus 8 --podresources-socket /tmp/node-0/kubelet.sock
"""
from __future__ import annotations

import logging

from . import common

log = logging.getLogger("nos_amd.cmd.simnode")


def main(argv=None) -> int:
    ap = common.parser(__doc__.splitlines()[0])
    ap.add_argument("--name", required=True)
    ap.add_argument("--kind", choices=["cumask", "partition", "none"], default="cumask")
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--podresources-socket", required=True)
    ap.add_argument("--cu-policy", default="proportional")
    args = ap.parse_args(argv)
    common.setup_logging(args.log_level)
    from ..api import constants as C
    from ..deviceplugin.config_watcher import ConfigWatcher
    from ..deviceplugin.plugin import NosAmdDevicePlugin
    from ..gpu.fakesmi import FakeSmi
    from ..kube import factory as kf
    from ..resource import podresources_grpc
    from ..runtime.manager import Manager
    from ..sim.kubelet import Kubelet

    api = common.connect(args)
    kind = None if args.kind == "none" else args.kind
    labels = {"kubernetes.io/hostname": args.name}
    if kind:
        labels[C.LABEL_GPU_PARTITIONING] = kind
    if api.try_get("Node", args.name) is None:
        api.create(kf.build_node(args.name).with_labels(labels).get())
    smi = FakeSmi(gpus=args.gpus, node=args.name)
    plugin = NosAmdDevicePlugin(args.name, smi, mode=kind, cu_policy=args.cu_policy)
    kubelet = Kubelet(api, args.name, [plugin])
    kubelet.sync_node_status()
    mgr = Manager(api, f"simnode-{args.name}")
    mgr.add(kubelet.controller())
    if kind == C.PARTITIONING_CUMASK:
        mgr.add(ConfigWatcher(api, args.name, plugin).controller())
    srv = podresources_grpc.serve(kubelet, args.podresources_socket)
    mgr.start()
    log.info("simulated node %s (%s, %d GPUs) up; PodResources on %s", args.name, kind, args.gpus,
             args.podresources_socket)

    def shutdown():
        mgr.stop()
        srv.stop(grace=0)

    common.run_until_signal(shutdown)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
