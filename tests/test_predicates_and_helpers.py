"""Small pieces the controllers and agents lean on: event predicates (with
the reference's inverted NodeResourcesChanged fixed,
pkg/util/predicate/predicates.go:51-58), the device-plugin restart client
(pkg/gpu/client.go:51-135), the device-plugin ConfigMap watcher and the
per-process memory cap."""
from __future__ import annotations

import threading
import time

import pytest

from nos_amd.agents.dpclient import DevicePluginClient
from nos_amd.api import constants as C
from nos_amd.kube import factory as kf
from nos_amd.kube import objects as ko
from nos_amd.runtime import predicates as P
from nos_amd.sim.apiserver import ApiServer


def _node(alloc: dict, ann: dict | None = None) -> dict:
    n = {"kind": "Node", "metadata": {"name": "n1", "annotations": dict(ann or {}), "labels": {}},
         "status": {"allocatable": dict(alloc), "capacity": dict(alloc)}}
    return n


def test_node_resources_changed_passes_exactly_on_resource_changes():
    p = P.NodeResourcesChanged()
    a = _node({"cpu": "8", "amd.com/gpu-36gb": "8"})
    b = _node({"cpu": "8", "amd.com/gpu-36gb": "4"})
    assert p(P.Event("update", b, a))          # the reference returned false here
    assert not p(P.Event("update", a, _node({"cpu": "8000m", "amd.com/gpu-36gb": "8"})))  # same quantity
    assert p(P.Event("create", a)) and p(P.Event("delete", a))


def test_simple_predicates_and_combinators():
    a = _node({}, {"x": "1"})
    b = _node({}, {"x": "2"})
    assert P.AnnotationsChanged()(P.Event("update", b, a))
    assert not P.AnnotationsChanged()(P.Event("update", a, a))
    assert P.MatchingName("n1")(P.Event("create", a)) and not P.MatchingName("n2")(P.Event("create", a))
    assert not P.ExcludeDelete()(P.Event("delete", a)) and P.ExcludeDelete()(P.Event("update", b, a))
    both = P.and_(P.MatchingName("n1"), P.AnnotationsChanged())
    either = P.or_(P.MatchingName("n2"), P.AnnotationsChanged())
    assert both(P.Event("update", b, a)) and not both(P.Event("update", a, a))
    assert either(P.Event("update", b, a)) and not either(P.Event("update", a, a))
    labelled = {"kind": "Node", "metadata": {"name": "n1", "labels": {C.LABEL_GPU_PARTITIONING: "cumask"}}}
    assert P.HasLabel(C.LABEL_GPU_PARTITIONING, ("cumask",))(P.Event("create", labelled))
    assert not P.HasLabel(C.LABEL_GPU_PARTITIONING, ("amdpart",))(P.Event("create", labelled))


def _plugin_pod(name: str, phase: str = ko.RUNNING) -> dict:
    k, v = C.DEFAULT_DEVICE_PLUGIN_DS_LABEL
    return kf.build_pod("nos-system", name).with_label(k, v).with_node_name("n1").with_phase(phase).get()


def test_device_plugin_restart_waits_for_the_replacement_pod():
    api = ApiServer()
    api.create(_plugin_pod("dp-old"))
    other = _plugin_pod("dp-other-node")
    other["spec"]["nodeName"] = "n2"
    api.create(other)
    c = DevicePluginClient(api, "n1", poll_s=0.01, timeout_s=5)

    def daemonset():  # the DaemonSet controller recreates the pod, Pending then Running
        time.sleep(0.05)
        api.create(_plugin_pod("dp-new", ko.PENDING))
        time.sleep(0.05)
        p = api.get("Pod", "dp-new", "nos-system")
        p["status"]["phase"] = ko.RUNNING
        api.update_status(p)  # phase lives in the status subresource

    t = threading.Thread(target=daemonset)
    t.start()
    c.restart()
    t.join()
    names = {ko.name(p) for p in api.list("Pod", "nos-system")}
    assert names == {"dp-new", "dp-other-node"}  # only this node's plugin pod was deleted


def test_device_plugin_restart_times_out_without_a_replacement():
    api = ApiServer()
    api.create(_plugin_pod("dp-old"))
    with pytest.raises(TimeoutError):
        DevicePluginClient(api, "n1", poll_s=0.01, timeout_s=0.1).restart()
    DevicePluginClient(api, "n1", poll_s=0.01, timeout_s=0.05).refresh()  # logs, never raises


class _Plugin:
    mode = C.PARTITIONING_CUMASK  # the watcher only loads slice tables on cumask nodes

    def __init__(self):
        self.config_key, self.config, self.loaded = None, None, []

    def set_config(self, key, data):
        self.config_key, self.config = key, data
        self.loaded.append(key)


def test_config_watcher_follows_the_node_label():
    from nos_amd.deviceplugin.config_watcher import ConfigWatcher
    from nos_amd.runtime.manager import Request

    api = ApiServer()
    api.create({"kind": "Node", "metadata": {"name": "n1", "labels": {}}})
    plugin = _Plugin()
    w = ConfigWatcher(api, "n1", plugin)
    assert not w.reconcile(Request("n1", "")).requeue_after and plugin.loaded == []  # no label yet
    node = api.get("Node", "n1")
    ko.set_label(node, C.LABEL_DEVICE_PLUGIN_CONFIG, "n1-p1")
    api.update(node)
    assert w.reconcile(Request("n1", "")).requeue_after == 1.0  # ConfigMap entry not written yet
    api.create({"kind": "ConfigMap", "metadata": {"name": w.cm_ref.name, "namespace": w.cm_ref.namespace},
                "data": {"n1-p1": "{}"}})
    w.reconcile(Request("n1", ""))
    w.reconcile(Request("n1", ""))  # already loaded: no reload
    assert plugin.loaded == ["n1-p1"] and w.loads == 1


def test_memory_limit_is_a_no_op_without_the_env(monkeypatch):
    from nos_amd.utils.memlimit import apply_memory_limit

    monkeypatch.delenv(C.ENV_MEMORY_LIMIT_GB, raising=False)
    assert apply_memory_limit(0) is None
