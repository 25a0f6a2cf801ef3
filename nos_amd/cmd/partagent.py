"""nos-amd partition agent (the reference's ``cmd/migagent/migagent.go:56-163``):
per-node DaemonSet on ``nos.nebuly.com/gpu-partitioning=partition`` and
``hybrid`` nodes.  Reports the node's compute/memory partitions (hybrid: the
memory slices on them) and applies the gpupartitioner's plans with amd-smi.

NODE_NAME=<node> python -m nos_amd.cmd.partagent --config partition_agent_config.yaml
"""
from __future__ import annotations

import logging

from . import common

log = logging.getLogger("nos_amd.cmd.partagent")


def open_smi(fake_gpus: int, allow_set: bool, node: str = "node"):
    """amd-smi through libnos_amdsmi, or -- for simulated nodes -- the
    in-memory backend whose GPU uuids match :mod:`nos_amd.cmd.simnode`'s."""
    from ..gpu.amdsmi import AmdSmi

    if fake_gpus:
        from ..gpu.fakesmi import FakeSmi

        return FakeSmi(gpus=fake_gpus, node=node)
    return AmdSmi.real(allow_set=allow_set)


def open_lister(socket: str):
    from ..resource.podresources_grpc import GrpcLister

    return GrpcLister(socket)


def build(api, node: str, cfg, smi, lister, device_plugins, kind: str | None = None):
    from ..agents.devices import NodeLabeler
    from ..agents.hybridagent import HybridReporter
    from ..agents.partagent import PartitionActuator, PartitionReporter
    from ..agents.shared import SharedState
    from ..api import constants as C

    shared = SharedState()
    mgr = common.manager_for(api, f"nos-partagent-{node}", cfg)
    mgr.add(NodeLabeler(api, node, smi).controller())
    reporter = HybridReporter if kind == C.PARTITIONING_HYBRID else PartitionReporter
    mgr.add(reporter(api, node, smi, lister, shared, cfg.report_config_interval_seconds).controller())
    mgr.add(PartitionActuator(api, node, smi, lister, shared, device_plugins, cfg.default_memory_mode,
                              cfg.mode_switch_timeout_seconds).controller())
    return mgr


def main(argv=None) -> int:
    from ..api import constants as C

    ap = common.parser(__doc__.splitlines()[0])
    ap.add_argument("--podresources-socket", default=C.KUBELET_PODRESOURCES_SOCKET)
    ap.add_argument("--fake-gpus", type=int, default=0, help="use the in-memory amd-smi backend with N GPUs")
    ap.add_argument("--no-device-plugin-restart", action="store_true")
    args = ap.parse_args(argv)
    cfg = common.load_config(args.config, "PartitionAgentConfig")
    common.apply_overrides(cfg, args)
    node = common.node_name()
    api = common.connect(args)
    smi = open_smi(args.fake_gpus, cfg.allow_mode_changes, node)
    if not smi.gpus():
        raise SystemExit("no GPU found")  # initAgent: at least one partitionable GPU (migagent.go:165-177)
    lister = open_lister(args.podresources_socket)
    dps = []
    if not args.no_device_plugin_restart:
        from ..agents.dpclient import DevicePluginClient

        dps.append(DevicePluginClient(api, node))
    from ..gpu.core import partitioning_kind

    mgr = build(api, node, cfg, smi, lister, dps, partitioning_kind(api.get("Node", node)))
    common.serve_health(cfg.health.health_probe_bind_address, mgr.healthz, mgr.readyz)
    common.serve_metrics(cfg.metrics.bind_address)
    mgr.start()
    log.info("partition agent started on %s (%d GPUs)", node, len(smi.gpus()))
    return common.run_until_signal(mgr.stop, mgr.lost_leadership)


if __name__ == "__main__":
    raise SystemExit(main())
