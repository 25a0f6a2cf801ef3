"""Elastic-quota operator + CapacityScheduling end to end on the in-process cluster.

Scenarios of the reference's envtest suites, re-stated for SimCluster:
* internal/controllers/elasticquota/elasticquota_controller_int_test.go:38-427
  (status.used, over-quota labels, label flips when quota frees up or min changes);
* internal/controllers/elasticquota/compositeelasticquota_controller_int_test.go:37-351
  (CEQ status aggregated over namespaces, borrowing, deletion of overlapping EQs :292);
* BASELINE config 1: over-quota borrowing between 2 namespaces, then reclaim by
  preemption through the real Scheduler (CapacityScheduling PostFilter evicts).
"""
from __future__ import annotations

import pytest

from nos_amd.api import constants as C
from nos_amd.api import v1alpha1
from nos_amd.kube import objects as ko
from nos_amd.sim.cluster import SimCluster

GPU_MEM = "nos.nebuly.com/gpu-memory"


def _ns(cl, *names):
    for n in names:
        cl.api.create({"kind": "Namespace", "metadata": {"name": n}})


def _eq(cl, ns, mn, mx, name="q"):
    return cl.api.create(v1alpha1.build_eq(ns, name).with_min({GPU_MEM: mn, "cpu": "16", "memory": "64Gi"})
                         .with_max({GPU_MEM: mx, "cpu": "64", "memory": "1Ti"}).get())


def _labels(cl, ns):
    return {ko.name(p): ko.labels(p).get(C.LABEL_CAPACITY_INFO) for p in cl.pods(ns)
            if ko.pod_phase(p) == ko.RUNNING}


def _cluster(gpus=1, lender_min=40):
    """A GPU node plus an idle "lender" namespace whose unused min others can
    borrow (CapacityScheduling admits over-min pods only while the SUM of all
    quotas' used stays within the sum of their mins)."""
    cl = SimCluster()
    cl.add_node("n1", C.PARTITIONING_CUMASK, gpus=gpus)
    if lender_min:
        _ns(cl, "lender")
        _eq(cl, "lender", lender_min, 100)
    return cl


def _submit(cl, ns, names, res="amd.com/gpu-10gb", priority=None):
    for n in names:
        cl.submit_pod(n, {res: 1}, namespace=ns, priority=priority)
        cl.clock.advance(1)
    cl.settle(600, until=lambda: not cl.pending_pods())
    cl.settle(30)


def test_eq_status_and_labels_flip_when_quota_frees_up():
    cl = _cluster()
    _ns(cl, "team-a")
    _eq(cl, "team-a", 20, 100)
    cl.settle(30)
    _submit(cl, "team-a", ["p0", "p1", "p2"])
    assert _labels(cl, "team-a") == {"p0": "in-quota", "p1": "in-quota", "p2": "over-quota"}
    assert cl.api.get(v1alpha1.KIND_EQ, "q", "team-a")["status"]["used"][GPU_MEM] == "30"
    # an in-quota pod stops: the oldest over-quota pod becomes in-quota, used drops
    cl.api.delete("Pod", "p0", "team-a")
    cl.settle(60)
    assert _labels(cl, "team-a") == {"p1": "in-quota", "p2": "in-quota"}
    assert cl.api.get(v1alpha1.KIND_EQ, "q", "team-a")["status"]["used"][GPU_MEM] == "20"


def test_eq_min_update_relabels_pods():
    cl = _cluster()
    _ns(cl, "team-a")
    _eq(cl, "team-a", 10, 100)
    cl.settle(30)
    _submit(cl, "team-a", ["p0", "p1", "p2"])
    assert sorted(_labels(cl, "team-a").values()) == ["in-quota", "over-quota", "over-quota"]
    eq = cl.api.get(v1alpha1.KIND_EQ, "q", "team-a")
    eq["spec"]["min"][GPU_MEM] = "30"
    cl.api.update(eq)
    cl.settle(60)
    assert set(_labels(cl, "team-a").values()) == {"in-quota"}


def test_ceq_takes_over_the_namespace_of_an_elastic_quota():
    """A CEQ created over a namespace that has an EQ: the EQ is deleted and the
    namespace's pods are accounted and labelled by the CEQ from then on."""
    from nos_amd.controllers.elasticquota import CompositeElasticQuotaReconciler, ElasticQuotaReconciler

    cl = _cluster()
    _ns(cl, "team-a")
    _eq(cl, "team-a", 10, 100)
    cl.settle(30)
    _submit(cl, "team-a", ["p0", "p1"])
    assert _labels(cl, "team-a") == {"p0": "in-quota", "p1": "over-quota"}
    cl.api.create(v1alpha1.build_composite_eq("default", "ceq").with_namespaces("team-a")
                  .with_min({GPU_MEM: 30, "cpu": "16", "memory": "64Gi"})
                  .with_max({GPU_MEM: 100, "cpu": "64", "memory": "1Ti"}).get())
    cl.settle(60)
    assert cl.api.list(v1alpha1.KIND_EQ, "team-a") == []
    assert _labels(cl, "team-a") == {"p0": "in-quota", "p1": "in-quota"}
    assert cl.api.get(v1alpha1.KIND_CEQ, "ceq", "default")["status"]["used"][GPU_MEM] == "20"
    pod = cl.api.get("Pod", "p0", "team-a")
    assert ElasticQuotaReconciler(cl.api).find_for_pod(pod) == []
    assert [r.name for r in CompositeElasticQuotaReconciler(cl.api).find_for_pod(pod)] == ["ceq"]


def test_ceq_aggregates_status_over_namespaces_and_labels_pods():
    cl = _cluster()
    _ns(cl, "ns-1", "ns-2")
    cl.api.create(v1alpha1.build_composite_eq("default", "ceq").with_namespaces("ns-1", "ns-2")
                  .with_min({GPU_MEM: 30, "cpu": "16", "memory": "64Gi"})
                  .with_max({GPU_MEM: 100, "cpu": "64", "memory": "1Ti"}).get())
    cl.settle(30)
    _submit(cl, "ns-1", ["a0", "a1"])
    _submit(cl, "ns-2", ["b0", "b1"])
    ceq = cl.api.get(v1alpha1.KIND_CEQ, "ceq", "default")
    assert ceq["status"]["used"][GPU_MEM] == "40"
    labels = {**_labels(cl, "ns-1"), **_labels(cl, "ns-2")}
    # oldest first across both namespaces: 30 GB in quota, the 4th pod over quota
    assert labels == {"a0": "in-quota", "a1": "in-quota", "b0": "in-quota", "b1": "over-quota"}


def test_ceq_creation_deletes_overlapping_elastic_quotas():
    cl = _cluster()
    _ns(cl, "ns-1", "ns-2", "ns-3")
    for ns in ("ns-1", "ns-2", "ns-3"):
        _eq(cl, ns, 10, 100)
    cl.settle(30)
    cl.api.create(v1alpha1.build_composite_eq("default", "ceq").with_namespaces("ns-1", "ns-2")
                  .with_min({GPU_MEM: 30, "cpu": "16", "memory": "64Gi"})
                  .with_max({GPU_MEM: 100, "cpu": "64", "memory": "1Ti"}).get())
    cl.settle(30)
    left = {ko.namespace(e) for e in cl.api.list(v1alpha1.KIND_EQ)}
    assert left == {"ns-3", "lender"}


def test_ceq_pod_borrowing_from_an_elastic_quota_is_over_quota():
    cl = _cluster(lender_min=0)
    _ns(cl, "ns-1", "ns-2", "other")
    cl.api.create(v1alpha1.build_composite_eq("default", "ceq").with_namespaces("ns-1", "ns-2")
                  .with_min({GPU_MEM: 10, "cpu": "16", "memory": "64Gi"})
                  .with_max({GPU_MEM: 100, "cpu": "64", "memory": "1Ti"}).get())
    _eq(cl, "other", 40, 100)
    cl.settle(30)
    _submit(cl, "ns-1", ["a0"])
    _submit(cl, "ns-2", ["b0", "b1"])  # borrows the unused min of "other"
    assert _labels(cl, "ns-2") == {"b0": "over-quota", "b1": "over-quota"}
    assert _labels(cl, "ns-1") == {"a0": "in-quota"}


def test_baseline_config1_borrow_then_reclaim_by_preemption():
    """BASELINE config 1: team-a borrows team-b's unused min; when team-b
    submits, the real Scheduler's CapacityScheduling PostFilter evicts team-a's
    over-quota pods (never in-quota ones) and team-b's pods bind."""
    cl = SimCluster()
    # CPU-only node with a fake extended resource (no GPU on the node)
    cl.add_node("n1", None, gpus=0, node_resources={"cpu": "8", "memory": "64Gi", "pods": "110",
                                                   "example.com/fake": "8"})
    _ns(cl, "team-a", "team-b")
    for ns, mn in (("team-a", "2"), ("team-b", "6")):
        cl.api.create(v1alpha1.build_eq(ns, "q").with_min({"cpu": mn, "memory": "64Gi", "example.com/fake": mn})
                      .with_max({"cpu": "8", "memory": "1Ti", "example.com/fake": "8"}).get())
    cl.settle(30)
    for i in range(8):
        cl.submit_pod(f"a{i}", {"example.com/fake": 1}, namespace="team-a", cpu_milli=1000)
        cl.clock.advance(1)
    cl.settle(600, until=lambda: not cl.pending_pods())
    cl.settle(30)
    la = _labels(cl, "team-a")
    assert len(la) == 8 and sorted(la.values()).count("in-quota") == 2  # borrowing 6 over min
    in_quota = {n for n, v in la.items() if v == "in-quota"}
    for i in range(4):
        cl.submit_pod(f"b{i}", {"example.com/fake": 1}, namespace="team-b", cpu_milli=1000)
        cl.clock.advance(1)
    cl.settle(1200, until=lambda: all(ko.pod_phase(p) == ko.RUNNING for p in cl.pods("team-b")))
    cl.settle(60)
    lb = _labels(cl, "team-b")
    assert len(lb) == 4 and set(lb.values()) == {"in-quota"}
    la = _labels(cl, "team-a")
    assert len(la) == 4 and in_quota <= set(la)  # only over-quota pods were preempted
    assert cl.scheduler.stats["preemptions"] >= 1


def test_cycle_exception_after_reserve_gives_the_quota_back():
    """an exception escaping the cycle after Reserve (here: a
    permit plugin bug) must run Unreserve, or CapacityScheduling keeps the pod
    in its ElasticQuota "used" and admission drifts until a resync."""
    cl = _cluster(lender_min=0)
    _ns(cl, "team-a")
    _eq(cl, "team-a", 20, 20)
    cl.settle(30)
    fw = next(iter(cl.scheduler.frameworks.values()))
    calls = {"n": 0}
    real_permit = fw.run_permit_plugins

    def boom(state, pod, node):
        calls["n"] += 1
        if calls["n"] == 1:  # the pod goes away while its cycle fails: only Unreserve can give its quota back
            cl.api.delete("Pod", ko.name(pod), ko.namespace(pod))
            raise RuntimeError("permit plugin bug")
        return real_permit(state, pod, node)

    fw.run_permit_plugins = boom
    cs = next(p for p in fw.plugins["reserve"] if p.name == "CapacityScheduling")
    _submit(cl, "team-a", ["gone"])
    assert calls["n"] == 1 and cl.scheduler.stats.get("cycle_errors") == 1
    assert cs.elastic_quota_infos.get("team-a").used.scalar.get(GPU_MEM, 0) == 0
    # two 10 GB pods fit the 20 GB max: nothing leaked from the failed cycle
    _submit(cl, "team-a", ["p0", "p1"])
    assert not cl.pending_pods()
    assert cs.elastic_quota_infos.get("team-a").used.scalar.get(GPU_MEM, 0) == 20
