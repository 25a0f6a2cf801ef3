"""nos-amd gpupartitioner (``cmd/gpupartitioner/gpupartitioner.go:72-268``):
cluster state controllers + one partitioner controller per AMD strategy
(``partition`` = compute/memory modes, ``cumask`` = CU-mask slices,
``hybrid`` = modes + memory slices per partition), planning
with an embedded scheduler framework built from the scheduler config.

python -m nos_amd.cmd.gpupartitioner --config gpu_partitioner_config.yaml
"""
from __future__ import annotations

import logging

from . import common

log = logging.getLogger("nos_amd.cmd.gpupartitioner")


def build(api, cfg):
    from ..controllers.gpupartitioner import NodeController, PartitionerController, PodController
    from ..gpu import amdpart
    from ..partitioning.state import ClusterState
    from ..partitioning.strategies import DevicePluginConfigRef, amdpart_strategy, cumask_strategy, hybrid_strategy
    from ..scheduler.config import build_framework, load, nos_scheduler_config

    if cfg.known_partition_geometries_file:
        amdpart.set_known_geometries(amdpart.load_known_geometries(cfg.known_partition_geometries_file))
    sched_cfg = load(cfg.scheduler_config_file) if cfg.scheduler_config_file else \
        nos_scheduler_config(cfg.amd_gpu_resource_memory_gb)
    # the reference picks the profile named nos-scheduler, else the first (gpupartitioner.go:320-348)
    prof = next((p for p in sched_cfg.profiles if p.scheduler_name == "nos-scheduler"), sched_cfg.profiles[0])
    fw = build_framework(prof, api=api)
    cs = ClusterState()
    ref = DevicePluginConfigRef(cfg.device_plugin_config_map.name, cfg.device_plugin_config_map.namespace)
    amd = amdpart_strategy(api, None, cfg.reserve_whole_gpus, cfg.preferred_memory_mode)
    cum = cumask_strategy(api, ref, cfg.device_plugin_delay_seconds, None, cfg.cu_policy, cfg.slice_placement,
                          {"isolatedProfiles": cfg.isolated_profiles, "isolatedCuSlots": cfg.isolated_cu_slots})
    hyb = hybrid_strategy(api, ref, cfg.device_plugin_delay_seconds, None)
    mgr = common.manager_for(api, "nos-gpupartitioner", cfg)
    mgr.add(NodeController(api, cs, amd.initializer).controller())
    mgr.add(PodController(api, cs).controller())
    for strat in (amd, cum, hyb):
        mgr.add(PartitionerController(api, cs, strat, fw, None, cfg.batch_window_timeout_seconds,
                                      cfg.batch_window_idle_seconds, cfg.plan_report_timeout_seconds).controller())
    return mgr


def main(argv=None) -> int:
    ap = common.parser(__doc__.splitlines()[0])
    args = ap.parse_args(argv)
    cfg = common.load_config(args.config, "GpuPartitionerConfig")
    common.apply_overrides(cfg, args)
    api = common.connect(args)
    mgr = build(api, cfg)
    common.serve_health(cfg.health.health_probe_bind_address, mgr.healthz, mgr.readyz)
    common.serve_metrics(cfg.metrics.bind_address)
    mgr.start()
    log.info("gpupartitioner started (batch window %.0fs/%.0fs)", cfg.batch_window_timeout_seconds,
             cfg.batch_window_idle_seconds)
    return common.run_until_signal(mgr.stop, mgr.lost_leadership)


if __name__ == "__main__":
    raise SystemExit(main())
