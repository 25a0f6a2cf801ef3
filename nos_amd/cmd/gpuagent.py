"""nos-amd gpuagent (``cmd/gpuagent/gpuagent.go:54-143``): per-node DaemonSet on
``nos.nebuly.com/gpu-partitioning=cumask`` nodes.  Reports the node's
CU-mask slices (+ the plan handshake) and, with probes enabled, the measured
per-slice TFLOP/s and GB/s from the gfx950 probe kernels.

NODE_NAME=<node> python -m nos_amd.cmd.gpuagent --config gpu_agent_config.yaml
"""
from __future__ import annotations

import logging

from . import common

log = logging.getLogger("nos_amd.cmd.gpuagent")


def build(api, node: str, cfg, smi, lister, probe=None):
    from ..agents.devices import NodeLabeler
    from ..agents.gpuagent import CuMaskReporter

    mgr = common.manager_for(api, f"nos-gpuagent-{node}", cfg)
    mgr.add(NodeLabeler(api, node, smi, cfg.pod_server_tenants).controller())
    mgr.add(CuMaskReporter(api, node, smi, lister, cfg.report_config_interval_seconds, probe).controller())
    return mgr


def main(argv=None) -> int:
    from ..agents.gpuagent import check_spx
    from ..api import constants as C
    from .partagent import open_lister, open_smi

    ap = common.parser(__doc__.splitlines()[0])
    ap.add_argument("--podresources-socket", default=C.KUBELET_PODRESOURCES_SOCKET)
    ap.add_argument("--fake-gpus", type=int, default=0)
    args = ap.parse_args(argv)
    cfg = common.load_config(args.config, "GpuAgentConfig")
    common.apply_overrides(cfg, args)
    node = common.node_name()
    api = common.connect(args)
    smi = open_smi(args.fake_gpus, False, node)
    check_spx(smi)  # refuses partitioned GPUs, like AnyMigEnabledGpu (gpuagent.go:105-114)
    probe = None
    if cfg.probe_enabled and not args.fake_gpus:
        from ..agents.probe import SliceProber

        probe = SliceProber(smi)
    mgr = build(api, node, cfg, smi, open_lister(args.podresources_socket), probe)
    common.serve_health(cfg.health.health_probe_bind_address, mgr.healthz, mgr.readyz)
    common.serve_metrics(cfg.metrics.bind_address)
    mgr.start()
    log.info("gpuagent started on %s", node)
    return common.run_until_signal(mgr.stop, mgr.lost_leadership)


if __name__ == "__main__":
    raise SystemExit(main())
