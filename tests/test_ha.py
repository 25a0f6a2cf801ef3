"""High availability: leader election with renewal, lease loss, and at most
one active reconciler / binder at any time (controller-runtime semantics the
reference relies on: config/gpupartitioner/manager/gpu_partitioner_config.yaml:9-11,
config/scheduler/deployment/scheduler_config.yaml:3-6)."""
from __future__ import annotations

import threading
import time

from nos_amd.kube import factory as kf
from nos_amd.runtime.manager import Controller, LeaderElector, LeaseKeeper, Manager, Request, Result
from nos_amd.sim.apiserver import ApiServer
from nos_amd.utils.clock import FakeClock


class Recorder:
    def __init__(self, name: str, log: list, clock):
        self.name, self.log, self.clock = name, log, clock

    def reconcile(self, req: Request) -> Result:
        self.log.append((self.clock.now(), self.name, req.name))
        return Result()


def _cm(name: str) -> dict:
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": "default"}, "data": {}}


def _mgr(api, name: str, log: list) -> Manager:
    m = Manager(api, name, leader_election=True, leader_election_id="ha-test", identity=name)
    m.add(Controller(f"rec-{name}", Recorder(name, log, api.clock)).for_kind("ConfigMap"))
    return m


def test_two_managers_one_active_reconciler_through_lease_loss():
    clock = FakeClock()
    api = ApiServer(clock)
    log: list = []
    m1, m2 = _mgr(api, "m1", log), _mgr(api, "m2", log)
    for m in (m1, m2):
        m.setup()
    api.create(_cm("a"))
    for _ in range(5):
        m1.step()
        m2.step()
        clock.advance(1.0)
    assert m1.is_leader and not m2.is_leader
    assert {who for _, who, _ in log} == {"m1"}

    # m1 hangs (no steps) past the lease: m2 takes over and reconciles
    clock.advance(20.0)
    api.create(_cm("b"))
    for _ in range(3):
        m2.step()
        clock.advance(1.0)
    t_takeover = min(t for t, who, _ in log if who == "m2")
    assert m2.is_leader and ("m2" in {who for _, who, _ in log})

    # m1 wakes up: its renewal is refused (m2 holds a live lease) -> lost, never reconciles again
    api.create(_cm("c"))
    for _ in range(5):
        m1.step()
        m2.step()
        clock.advance(1.0)
    assert m1.lost_leadership.is_set() and not m1.is_leader and not m1.healthz()
    assert all(who == "m2" for t, who, _ in log if t >= t_takeover)
    assert any(name == "c" and who == "m2" for _, who, name in log)
    # exactly one holder at every reconcile instant
    holders = {t: {w for tt, w, _ in log if tt == t} for t, _, _ in log}
    assert all(len(h) == 1 for h in holders.values())


def test_renew_errors_past_deadline_lose_the_lease():
    clock = FakeClock()
    api = ApiServer(clock)
    el = LeaderElector(api, "x", "nos-system", "me", lease_duration=15.0)
    lost = []
    k = LeaseKeeper(el, on_lost=lambda: lost.append(clock.now()))
    assert k.acquire()
    broken = {"on": False}
    real = el.try_acquire_or_renew

    def flaky():
        if broken["on"]:
            raise ConnectionError("api server unreachable")
        return real()

    el.try_acquire_or_renew = flaky
    for _ in range(5):
        clock.advance(2.0)
        assert k.tick()
    broken["on"] = True
    t0 = clock.now()
    for _ in range(20):
        clock.advance(2.0)
        if not k.tick():
            break
    assert lost and 10.0 - 2.0 <= lost[0] - t0 <= 10.0 + 2.0  # renew deadline = 2/3 of 15 s
    assert not k.tick()  # once lost, never leads again


def test_threaded_managers_failover_and_exit_code():
    from nos_amd.cmd import common

    api = ApiServer()
    log: list = []

    def mk(name):
        m = Manager(api, name, leader_election=True, leader_election_id="ha-thr", identity=name)
        m.elector.duration = 2.0
        m.lease = LeaseKeeper(m.elector, on_lost=m._on_lease_lost)
        m.add(Controller(f"rec-{name}", Recorder(name, log, api.clock)).for_kind("ConfigMap"))
        return m

    m1, m2 = mk("t1"), mk("t2")
    threading.Thread(target=m1.start, daemon=True).start()
    time.sleep(0.3)
    threading.Thread(target=m2.start, daemon=True).start()
    api.create(_cm("a"))
    time.sleep(0.8)
    assert m1.is_leader and not m2.is_leader
    # a third party steals the lease (e.g. m1 was partitioned and its lease expired elsewhere)
    lease = api.get("Lease", "ha-thr", "nos-system")
    lease["spec"]["holderIdentity"] = "intruder"
    lease["spec"]["renewTime"] = lease["spec"]["renewTime"]
    api.update(lease)
    deadline = time.time() + 5
    while time.time() < deadline and not m1.lost_leadership.is_set():
        time.sleep(0.05)
    assert m1.lost_leadership.is_set()
    rc = common.run_until_signal(m1.stop, m1.lost_leadership)
    assert rc == 1
    m2.stop()


def test_scheduler_loop_survives_cycle_errors():
    from nos_amd.scheduler.config import nos_scheduler_config
    from nos_amd.scheduler.scheduler import Scheduler

    from nos_amd.api import v1alpha1

    api = ApiServer()
    v1alpha1.register_types(api)
    s = Scheduler(api, nos_scheduler_config())
    calls = {"n": 0}
    real = s._schedule_pod

    def boom(pod):
        calls["n"] += 1
        if calls["n"] == 1:
            raise RuntimeError("plugin bug")
        return real(pod)

    s._schedule_pod = boom
    s.start()
    try:
        api.create(kf.build_pod("default", "p").with_scheduler_name("nos-scheduler").get())
        deadline = time.time() + 5
        while time.time() < deadline and calls["n"] < 1:
            time.sleep(0.02)
        time.sleep(0.2)
        assert s.healthy()
        assert s.stats.get("cycle_errors") == 1
        assert len(s.queue._unschedulable) == 1  # the pod was requeued, not lost
    finally:
        s.stop()
    assert not s.healthy()


def test_two_schedulers_one_binder_at_a_time():
    from nos_amd.api import v1alpha1
    from nos_amd.cmd.scheduler import start_scheduler
    from nos_amd.scheduler.config import nos_scheduler_config
    from nos_amd.sim.cluster import SimCluster

    from nos_amd.utils.clock import RealClock

    cl = SimCluster(clock=RealClock())  # API server + a node to bind to (its own scheduler is not started)
    cl.add_node("n1", None, gpus=1)
    api = cl.api
    cfg = nos_scheduler_config()
    cfg.leader_elect = True
    events: list = []
    out = {}

    def run(ident):
        got = start_scheduler(api, cfg, ident, lease_duration=1.5)
        out[ident] = got
        events.append((time.monotonic(), ident, "leading"))

    ta = threading.Thread(target=run, args=("A",), daemon=True)
    ta.start()
    ta.join(5)
    tb = threading.Thread(target=run, args=("B",), daemon=True)
    tb.start()
    for i in range(3):
        api.create(kf.build_pod("default", f"p{i}").with_scheduler_name("nos-scheduler").get())
    time.sleep(0.5)
    sa, ka, lost_a = out["A"]
    assert "B" not in out and sa.stats["scheduled"] == 3
    # A's API connection breaks: renewals fail; past the renew deadline A stops binding
    ka.elector.try_acquire_or_renew = lambda: (_ for _ in ()).throw(ConnectionError("down"))
    assert lost_a.wait(5)
    events.append((time.monotonic(), "A", "lost"))
    a_done = sa.stats["scheduled"]
    tb.join(10)
    sb, kb, _ = out["B"]
    for i in range(3, 6):
        api.create(kf.build_pod("default", f"p{i}").with_scheduler_name("nos-scheduler").get())
    deadline = time.time() + 5
    while time.time() < deadline and sb.stats["scheduled"] < 3:
        time.sleep(0.05)
    assert sb.stats["scheduled"] == 3 and sa.stats["scheduled"] == a_done
    lost_t = next(t for t, w, e in events if w == "A" and e == "lost")
    lead_b = next(t for t, w, e in events if w == "B" and e == "leading")
    assert lead_b >= lost_t - 0.5 and not sa.healthy()
    sb.stop()
    kb.stop()
