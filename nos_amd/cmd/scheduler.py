"""nos-amd scheduler (``cmd/scheduler/scheduler.go:43-59``): the scheduling
framework with the ``CapacityScheduling`` plugin, configured by a
KubeSchedulerConfiguration (profile ``nos-scheduler`` by default).

python -m nos_amd.cmd.scheduler --config scheduler_config.yaml [--api-server URL]
"""
from __future__ import annotations

import logging

from . import common

log = logging.getLogger("nos_amd.cmd.scheduler")


def main(argv=None) -> int:
    ap = common.parser(__doc__.splitlines()[0], "KubeSchedulerConfiguration file (YAML)")
    args = ap.parse_args(argv)
    common.setup_logging(args.log_level)
    from ..runtime.manager import LeaderElector
    from ..scheduler.config import load, nos_scheduler_config
    from ..scheduler.scheduler import Scheduler

    cfg = load(args.config) if args.config else nos_scheduler_config()
    api = common.connect(args)
    if cfg.leader_elect:
        import socket
        import time

        el = LeaderElector(api, cfg.resource_name, cfg.resource_namespace, socket.gethostname())
        while not el.try_acquire_or_renew():
            time.sleep(2.0)
        log.info("acquired lease %s/%s", cfg.resource_namespace, cfg.resource_name)
    sched = Scheduler(api, cfg)
    sched.start()
    common.serve_health(args.health_probe_bind_address or ":10259", lambda: True, lambda: True)
    common.serve_metrics(args.metrics_bind_address)
    log.info("scheduler started with profiles %s", [p.scheduler_name for p in cfg.profiles])
    common.run_until_signal(sched.stop)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
