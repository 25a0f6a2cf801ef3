"""Controller runtime, API-server semantics, quantities, selectors, batcher,
component configs, webhooks, metrics exporter and the native amd-smi fake."""
from __future__ import annotations

import json
import threading
from fractions import Fraction

import pytest

from nos_amd.api import config as cfgmod
from nos_amd.api import constants as C
from nos_amd.api import v1alpha1
from nos_amd.api.webhook_server import CEQ_PATH, EQ_PATH, review
from nos_amd.kube import factory as kf
from nos_amd.kube import objects as ko
from nos_amd.kube import quantity as q
from nos_amd.kube import selectors as sel
from nos_amd.runtime.manager import Controller, LeaderElector, Manager, Request, Result
from nos_amd.runtime.workqueue import WorkQueue
from nos_amd.sim.apiserver import AlreadyExists, ApiServer, Conflict, Expired, Invalid
from nos_amd.utils.batcher import Batcher
from nos_amd.utils.clock import FakeClock


# ------------------------------------------------------------------ quantities & selectors
@pytest.mark.parametrize("s,v", [("100m", Fraction(1, 10)), ("2", 2), ("1Gi", 2 ** 30), ("1k", 1000),
                                 ("1.5", Fraction(3, 2)), (3, 3), ("288", 288), ("1e3", 1000)])
def test_quantity_parse(s, v):
    assert q.parse(s) == v


def test_quantity_roundtrip_and_rl_math():
    assert q.fmt(q.parse("500m")) == "500m"
    a = q.rl_parse({"cpu": "1", "memory": "1Gi"})
    b = q.rl_parse({"cpu": "500m", "amd.com/gpu": "1"})
    s = q.rl_add(a, b)
    assert s["cpu"] == Fraction(3, 2) and s["amd.com/gpu"] == 1
    assert q.rl_max({"cpu": 1}, {"cpu": 2})["cpu"] == 2


def test_label_and_field_selectors_and_merge_patch():
    reqs = sel.parse_label_selector("app=web,tier!=db,env in (prod,stage),!legacy")
    assert sel.match_labels(reqs, {"app": "web", "tier": "fe", "env": "prod"})
    assert not sel.match_labels(reqs, {"app": "web", "env": "dev"})
    assert not sel.match_labels(reqs, {"app": "web", "env": "prod", "legacy": "1"})
    obj = {"status": {"phase": "Running"}}
    assert sel.match_fields(sel.parse_field_selector("status.phase=Running"), obj)
    assert not sel.match_fields(sel.parse_field_selector("status.phase!=Running"), obj)
    assert sel.merge_patch({"a": {"b": 1, "c": 2}}, {"a": {"b": None, "d": 3}}) == {"a": {"c": 2, "d": 3}}


# ------------------------------------------------------------------ API server semantics
def test_apiserver_generation_status_and_conflicts():
    api = ApiServer()
    p = api.create(kf.build_pod("ns", "p").with_container(kf.build_container().get()).get())
    assert p["metadata"]["generation"] == 1
    p2 = api.patch("Pod", "p", {"spec": {"priority": 5}}, "ns")
    assert p2["metadata"]["generation"] == 2
    p3 = api.patch("Pod", "p", {"status": {"phase": "Running"}}, "ns", subresource="status")
    assert p3["metadata"]["generation"] == 2 and ko.pod_phase(p3) == "Running"
    with pytest.raises(Conflict):
        api.update(p2)
    with pytest.raises(AlreadyExists):
        api.create(kf.build_pod("ns", "p").get())
    with pytest.raises(Invalid):
        api.create({"kind": "Pod", "metadata": {}})
    # no-op write: same resourceVersion, no event
    rv = ko.resource_version(api.get("Pod", "p", "ns"))
    api.patch("Pod", "p", {"metadata": {"labels": {}}}, "ns")
    assert ko.resource_version(api.get("Pod", "p", "ns")) == rv


def test_apiserver_watch_resume_and_expiry():
    api = ApiServer()
    api.create(kf.build_node("a").get())
    _, rv = api.list_with_version("Node")
    api.create(kf.build_node("b").get())
    w = api.watch("Node", resource_version=rv)
    assert [(e.type, ko.name(e.object)) for e in w.drain()] == [("ADDED", "b")]
    api._history_floor = int(rv) + 5
    with pytest.raises(Expired):
        api.watch("Node", resource_version=rv)


def test_apiserver_snapshot_restore_and_namespace_cascade():
    api = ApiServer()
    api.create(kf.build_namespace("t").get())
    api.create(kf.build_pod("t", "p").get())
    snap = api.snapshot()
    api.delete("Namespace", "t")
    assert api.try_get("Pod", "p", "t") is None
    api.restore(snap)
    assert api.try_get("Pod", "p", "t") is not None


def test_conflict_fault_injection_is_retried_by_controllers():
    api = ApiServer(clock=FakeClock())
    api.faults["conflict_on_write"] = 0.5
    api.create(kf.build_node("n").get())
    done = []

    class R:
        def reconcile(self, req):
            api.patch("Node", req.name, {"metadata": {"labels": {"x": "1"}}})
            done.append(1)
            return Result()

    mgr = Manager(api, clock=api.clock)
    mgr.add(Controller("c", R()).for_kind("Node"))
    mgr.run_until_idle(max_time=60)
    assert done and ko.labels(api.get("Node", "n"))["x"] == "1"


# ------------------------------------------------------------------ runtime
def test_workqueue_dedup_dirty_and_delay():
    clk = FakeClock()
    wq = WorkQueue(clk)
    wq.add("a")
    wq.add("a")
    assert wq.get_nowait() == "a"
    wq.add("a")  # while processing: marked dirty, re-queued on done
    assert wq.get_nowait() is None
    wq.done("a")
    assert wq.get_nowait() == "a"
    wq.done("a")
    wq.add_after("b", 5)
    assert wq.get_nowait() is None
    clk.advance(5)
    assert wq.get_nowait() == "b"


def test_leader_election_lease_handover():
    clk = FakeClock()
    api = ApiServer(clock=clk)
    a = LeaderElector(api, "lease", "kube-system", "a", lease_duration=10, clock=clk)
    b = LeaderElector(api, "lease", "kube-system", "b", lease_duration=10, clock=clk)
    assert a.try_acquire_or_renew() and not b.try_acquire_or_renew()
    clk.advance(11)
    assert b.try_acquire_or_renew()
    assert not a.try_acquire_or_renew()
    b.release()
    assert a.try_acquire_or_renew()


def test_manager_requeue_after_with_fake_clock():
    clk = FakeClock()
    api = ApiServer(clock=clk)
    api.create(kf.build_node("n").get())
    calls = []

    class R:
        def reconcile(self, req: Request):
            calls.append(clk.now())
            return Result(requeue_after=10) if len(calls) < 3 else Result()

    mgr = Manager(api, clock=clk)
    mgr.add(Controller("c", R()).for_kind("Node"))
    mgr.run_until_idle(max_time=100)
    assert len(calls) == 3 and calls[2] - calls[0] >= 20


def test_batcher_idle_and_timeout_windows():
    clk = FakeClock()
    b = Batcher(timeout_s=10, idle_s=2, clock=clk)
    assert not b.add(1)  # not started: dropped
    b.start()
    b.add(1)
    clk.advance(1)
    b.add(2)
    clk.advance(1.5)
    assert b.ready() is None  # idle window restarted by item 2
    clk.advance(1)
    assert b.ready() == [1, 2]
    b.add(3)
    for _ in range(10):
        clk.advance(1)
        b.add(4)
    assert b.ready() is not None  # the timeout fires although items keep arriving
    b.reset()
    assert b.ready() is None


# ------------------------------------------------------------------ configs & webhooks
def test_component_configs_and_aliases(tmp_path):
    p = tmp_path / "gp.yaml"
    p.write_text("kind: GpuPartitionerConfig\nbatchWindowTimeoutSeconds: 30\nknownMigGeometriesFile: /x\n"
                 "nvidiaGpuResourceMemoryGB: 80\ndevicePluginConfigMap: {name: '', namespace: ''}\n")
    c = cfgmod.load(p)
    assert c.batch_window_timeout_seconds == 30 and c.known_partition_geometries_file == "/x"
    assert c.amd_gpu_resource_memory_gb == 80
    assert c.device_plugin_config_map.name == C.DEFAULT_DEVICE_PLUGIN_CM_NAME  # defaulted
    p.write_text("kind: GpuPartitionerConfig\nbatchWindowIdleSeconds: 0\n")
    with pytest.raises(ValueError):
        cfgmod.load(p)
    p.write_text("kind: MigAgentConfig\nreportConfigIntervalSeconds: 3\n")
    assert cfgmod.load(p).report_config_interval_seconds == 3
    with pytest.raises(ValueError):
        cfgmod.parse({"kind": "Nope"})


def test_admission_review_responses():
    api = ApiServer()
    v1alpha1.register_types(api, webhooks=False)
    api.create(kf.build_namespace("a").get())
    api.create(v1alpha1.build_eq("a", "q1").with_min({"cpu": "1"}).get())
    eq2 = v1alpha1.build_eq("a", "q2").with_min({"cpu": "1"}).get()
    r = review(api, EQ_PATH, {"request": {"uid": "u1", "operation": "CREATE", "object": eq2}})
    assert r["response"]["uid"] == "u1" and r["response"]["allowed"] is False
    assert r["response"]["status"]["code"] == 403
    bad = v1alpha1.build_eq("b", "q").with_min({"cpu": "2"}).with_max({"cpu": "1"}).get()
    assert review(api, EQ_PATH, {"request": {"uid": "u", "operation": "UPDATE", "object": bad}})["response"][
        "allowed"] is False
    ceq = v1alpha1.build_composite_eq("x", "c").with_namespaces("a", "b").get()
    assert review(api, CEQ_PATH, {"request": {"uid": "u", "operation": "CREATE", "object": ceq}})["response"][
        "allowed"] is True


def test_metrics_exporter_schema(tmp_path, capsys):
    from nos_amd.cmd import metricsexporter

    p = tmp_path / "m.yaml"
    p.write_text("installationUUID: abc\nnodes: [{name: n1, capacity: {amd.com/gpu: '8'}}]\n"
                 "components: {nosScheduler: true}\n")
    assert metricsexporter.main(["--metrics-file", str(p)]) == 0
    doc = json.loads(capsys.readouterr().out)
    assert doc["installationUUID"] == "abc" and doc["components"]["nosScheduler"] is True
    assert doc["nodes"][0]["capacity"]["amd.com/gpu"] == "8"
    assert metricsexporter.main(["--metrics-file", str(tmp_path / "missing.yaml")]) == 0


# ------------------------------------------------------------------ native amd-smi fake (C++ library)
def test_native_amdsmi_fake_backend():
    from nos_amd.gpu.amdsmi import AmdSmi, AmdSmiError

    smi = AmdSmi.fake(gpus=2)
    try:
        g = smi.gpu(0)
        assert g.num_xcds == 8 and g.memory_gb == 288 and g.compute_mode == "SPX"
        smi.set_compute_partition(0, "CPX")
        assert smi.gpu(0).compute_mode == "CPX" and smi.gpu(0).num_partitions == 8
        smi.fake_add_process(1, 123)
        with pytest.raises(AmdSmiError):
            smi.set_compute_partition(1, "DPX")  # busy GPU
        smi.inject("fail_set_compute")
        with pytest.raises(AmdSmiError):
            smi.set_compute_partition(0, "SPX")
        smi.inject("clear")
        assert smi.link(0, 1)["type"] == "xgmi"
    finally:
        smi.close()


def test_threaded_manager_smoke():
    api = ApiServer()
    seen = threading.Event()

    class R:
        def reconcile(self, req):
            seen.set()
            return Result()

    mgr = Manager(api)
    mgr.add(Controller("c", R()).for_kind("Node"))
    mgr.start()
    try:
        api.create(kf.build_node("n").get())
        assert seen.wait(5)
    finally:
        mgr.stop()
