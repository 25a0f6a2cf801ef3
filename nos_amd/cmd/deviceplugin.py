"""nos-amd device plugin (replaces the NVIDIA device plugin + MPS daemon the
reference depends on): advertises whole GPUs, compute partitions or CU-mask
slices to the kubelet over the device-plugin v1beta1 gRPC API and follows the
gpupartitioner's slice table (ConfigMap entry named by the node label
``nos.nebuly.com/device-plugin.config``) without restarts.  Every
``rescanSeconds`` it re-enumerates amd-smi (a mode the partition agent
switched is invisible to this process's session until then) and re-reads the
node's ``nos.nebuly.com/gpu-partitioning`` label.

NODE_NAME=<node> python -m nos_amd.cmd.deviceplugin --config device_plugin_config.yaml
"""
from __future__ import annotations

import logging
import threading

from . import common

log = logging.getLogger("nos_amd.cmd.deviceplugin")


def main(argv=None) -> int:
    from ..api import constants as C
    from ..deviceplugin.config_watcher import ConfigWatcher
    from ..deviceplugin.grpc_server import DevicePluginServers
    from ..deviceplugin.plugin import SLICE_MODES, NosAmdDevicePlugin
    from ..gpu.core import partitioning_kind
    from ..partitioning.strategies import DevicePluginConfigRef
    from .partagent import open_lister, open_smi

    ap = common.parser(__doc__.splitlines()[0])
    ap.add_argument("--podresources-socket", default=C.KUBELET_PODRESOURCES_SOCKET)
    ap.add_argument("--kubelet-socket", default="", help="default: <socketDir>/kubelet.sock")
    ap.add_argument("--fake-gpus", type=int, default=0)
    ap.add_argument("--expose-partitions-as-gpu", action="store_true",
                    help="static partition mode: every logical partition is an amd.com/gpu")
    ap.add_argument("--device-env", choices=["container", "host"], default=None,
                    help="HIP_VISIBLE_DEVICES numbering (default: the config's deviceEnv)")
    args = ap.parse_args(argv)
    cfg = common.load_config(args.config, "DevicePluginConfig")
    common.apply_overrides(cfg, args)
    node = common.node_name()
    api = common.connect(args)
    smi = open_smi(args.fake_gpus, False, node)
    mode = partitioning_kind(api.get("Node", node))
    plugin = NosAmdDevicePlugin(node, smi, mode=mode, expose_partitions_as_gpu=args.expose_partitions_as_gpu,
                                cu_policy=cfg.cu_policy, device_env=args.device_env or cfg.device_env,
                                pod_server_dir=cfg.pod_server_socket_dir, adopt_records=True)
    mgr = common.manager_for(api, f"nos-deviceplugin-{node}", cfg)
    ref = DevicePluginConfigRef(cfg.config_map.name, cfg.config_map.namespace)
    watcher = ConfigWatcher(api, node, plugin, ref)  # loads the slice table whenever the node is a cumask node
    mgr.add(watcher.controller())
    lister = open_lister(args.podresources_socket)
    servers = DevicePluginServers(plugin, cfg.socket_dir, args.kubelet_socket or None, podresources=lister)
    stop = threading.Event()

    def rescan():
        # modes change under the plugin (another process switches them) and the
        # node may be relabelled: re-enumerate amd-smi, follow the label
        while not stop.wait(cfg.rescan_seconds):
            try:
                n = api.try_get("Node", node)
                if n is not None and plugin.set_mode(partitioning_kind(n)) and plugin.mode in SLICE_MODES:
                    watcher.reconcile(None)
                plugin.rescan()
            except Exception as e:
                log.warning("rescan failed: %s", e)

    threading.Thread(target=rescan, daemon=True).start()
    common.serve_health(cfg.health.health_probe_bind_address, mgr.healthz, mgr.readyz)
    mgr.start()
    servers.start()
    log.info("device plugin started on %s (mode %s): %s", node, mode, sorted(plugin.resources()))

    def shutdown():
        stop.set()
        servers.stop()
        mgr.stop()

    common.run_until_signal(shutdown)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
