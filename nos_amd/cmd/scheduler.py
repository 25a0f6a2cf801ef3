"""nos-amd scheduler (``cmd/scheduler/scheduler.go:43-59``): the scheduling
framework with the ``CapacityScheduling`` plugin, configured by a
KubeSchedulerConfiguration (profile ``nos-scheduler`` by default).

python -m nos_amd.cmd.scheduler --config scheduler_config.yaml [--api-server URL]
"""
from __future__ import annotations

import logging
import os
import signal
import socket
import threading

from . import common

log = logging.getLogger("nos_amd.cmd.scheduler")


def main(argv=None) -> int:
    ap = common.parser(__doc__.splitlines()[0], "KubeSchedulerConfiguration file (YAML)")
    args = ap.parse_args(argv)
    common.setup_logging(args.log_level)
    from ..scheduler.config import load, nos_scheduler_config

    cfg = load(args.config) if args.config else nos_scheduler_config()
    api = common.connect(args)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    got = start_scheduler(api, cfg, f"{socket.gethostname()}-{os.getpid()}", stop)
    if got is None:
        return 0
    sched, keeper, lost = got
    common.serve_health(args.health_probe_bind_address or ":10259", sched.healthy,
                        lambda: sched.healthy() and not lost.is_set())
    common.serve_metrics(args.metrics_bind_address)
    log.info("scheduler started with profiles %s", [p.scheduler_name for p in cfg.profiles])

    def shutdown():
        sched.stop()
        if keeper:
            keeper.stop(release=not lost.is_set())

    return common.run_until_signal(shutdown, lost)


def start_scheduler(api, cfg, identity: str, stop: threading.Event | None = None, lease_duration: float = 15.0):
    """Start the scheduler -- as leader when ``cfg.leader_elect``: block until
    the Lease is acquired, then renew it; on loss the binder stops at once and
    ``lost`` fires (the binary then exits 1).  Returns (scheduler, keeper,
    lost) or None when ``stop`` fired before the lease was acquired."""
    from ..runtime.manager import LeaderElector, LeaseKeeper
    from ..scheduler.scheduler import Scheduler

    lost = threading.Event()
    sched = Scheduler(api, cfg)
    keeper = None
    if cfg.leader_elect:
        el = LeaderElector(api, cfg.resource_name, cfg.resource_namespace, identity, lease_duration=lease_duration)
        keeper = LeaseKeeper(el, on_lost=lambda: (sched.stop(), lost.set()))
        if not keeper.acquire(stop or threading.Event(), poll_s=min(2.0, lease_duration / 5)):
            return None
        log.info("%s acquired lease %s/%s", identity, cfg.resource_namespace, cfg.resource_name)
    sched.start()
    if keeper:
        keeper.start()
    return sched, keeper, lost


if __name__ == "__main__":
    raise SystemExit(main())
