"""REST client <-> HTTP front end of the simulator: the wire path the
multi-process deployment uses (same verbs/paths/status codes as a real
kube-apiserver)."""
from __future__ import annotations

import time

import pytest

from nos_amd.api import v1alpha1
from nos_amd.kube import factory as kf
from nos_amd.kube import objects as ko
from nos_amd.kube.client import KubeClient
from nos_amd.kube.rest import parse_path, path_for
from nos_amd.sim.apiserver import AlreadyExists, ApiServer, Conflict, Forbidden, NotFound
from nos_amd.sim.http import serve


@pytest.fixture()
def remote():
    api = ApiServer()
    v1alpha1.register_types(api)
    srv = serve(api, token="s3cret")
    cl = KubeClient(srv.url, token="s3cret")
    yield api, cl
    cl.close()
    srv.stop()


def _wait(pred, timeout=5.0):
    end = time.time() + timeout
    while time.time() < end:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_paths_roundtrip():
    plurals = {"pods", "nodes", "elasticquotas", "leases"}
    p = path_for("v1", "pods", True, "ns1", "p0", "status")
    assert p == "/api/v1/namespaces/ns1/pods/p0/status"
    r = parse_path(p, plurals)
    assert (r.api_version, r.plural, r.namespace, r.name, r.subresource) == ("v1", "pods", "ns1", "p0", "status")
    r = parse_path("/apis/nos.nebuly.com/v1alpha1/namespaces/a/elasticquotas", plurals)
    assert (r.api_version, r.plural, r.namespace, r.name) == ("nos.nebuly.com/v1alpha1", "elasticquotas", "a", None)
    r = parse_path("/api/v1/namespaces/foo", plurals | {"namespaces"})
    assert (r.plural, r.name, r.namespace) == ("namespaces", "foo", None)


def test_crud_and_errors(remote):
    api, cl = remote
    cl.create(kf.build_namespace("team").get())
    p = cl.create(kf.build_pod("team", "p0").with_container(kf.build_container().get()).get())
    assert ko.uid(p) and ko.resource_version(p)
    with pytest.raises(AlreadyExists):
        cl.create(kf.build_pod("team", "p0").get())
    with pytest.raises(NotFound):
        cl.get("Pod", "nope", "team")
    assert cl.try_get("Pod", "nope", "team") is None
    # stale resourceVersion -> 409
    p2 = cl.patch("Pod", "p0", {"metadata": {"labels": {"a": "b"}}}, "team")
    stale = dict(p)
    stale["metadata"] = dict(p["metadata"], labels={"x": "y"})
    with pytest.raises(Conflict):
        cl.update(stale)
    # status subresource only changes status
    cl.patch("Pod", "p0", {"status": {"phase": "Running"}, "metadata": {"labels": {"ignored": "1"}}}, "team",
             subresource="status")
    got = cl.get("Pod", "p0", "team")
    assert ko.pod_phase(got) == "Running" and "ignored" not in ko.labels(got) and ko.labels(got)["a"] == "b"
    assert int(ko.resource_version(got)) > int(ko.resource_version(p2))
    # selectors
    assert [ko.name(x) for x in cl.list("Pod", "team", label_selector="a=b")] == ["p0"]
    assert cl.list("Pod", "team", field_selector="status.phase=Pending") == []
    # binding
    cl.create(kf.build_node("n1").get())
    cl.bind("p0", "team", "n1")
    assert ko.pod_node(cl.get("Pod", "p0", "team")) == "n1"
    cl.delete("Pod", "p0", "team")
    assert api.try_get("Pod", "p0", "team") is None


def test_crd_and_webhook_over_http(remote):
    _, cl = remote
    cl.create(kf.build_namespace("a").get())
    cl.create(v1alpha1.build_eq("a", "q1").with_min({"cpu": "1"}).with_max({"cpu": "2"}).get())
    with pytest.raises(Forbidden):  # at most one EQ per namespace (elasticquota_webhook.go:43)
        cl.create(v1alpha1.build_eq("a", "q2").with_min({"cpu": "1"}).get())
    assert [ko.name(e) for e in cl.list(v1alpha1.KIND_EQ, "a")] == ["q1"]


def test_unauthorized():
    api = ApiServer()
    srv = serve(api, token="t")
    try:
        with pytest.raises(Exception):
            KubeClient(srv.url, token="wrong").list("Pod")
    finally:
        srv.stop()


def test_watch_delivers_old_objects_and_resumes(remote):
    api, cl = remote
    api.create(kf.build_node("n0").get())
    events = []
    from nos_amd.kube.client import ClientWatch

    ClientWatch.STREAM_TIMEOUT_S = 1  # streams end every second: exercise resume
    w = cl.watch("Node", callback=events.append)
    assert _wait(lambda: len(events) == 1) and events[0].type == "ADDED"
    api.patch("Node", "n0", {"metadata": {"labels": {"k": "v"}}})
    assert _wait(lambda: len(events) == 2)
    assert events[1].type == "MODIFIED" and events[1].old is not None and "k" not in ko.labels(events[1].old)
    # let the stream end: the reflector reconnects from its last resourceVersion without losing events
    assert _wait(lambda: w.streams >= 2)
    api.create(kf.build_node("n1").get())
    api.delete("Node", "n0")
    assert _wait(lambda: [e.type for e in events][2:] == ["ADDED", "DELETED"])
    assert ko.name(events[3].object) == "n0"
    w.stop()
    ClientWatch.STREAM_TIMEOUT_S = 300


def test_controller_manager_over_rest(remote):
    from nos_amd.runtime.manager import Controller, Manager, Result

    api, cl = remote
    seen = []

    class R:
        def reconcile(self, req):
            seen.append(req.name)
            return Result()

    mgr = Manager(cl, "remote-mgr")
    mgr.add(Controller("c", R()).for_kind("Node"))
    mgr.start()
    try:
        api.create(kf.build_node("a").get())
        api.create(kf.build_node("b").get())
        assert _wait(lambda: {"a", "b"} <= set(seen))
    finally:
        mgr.stop()
