"""ClusterState: the gpupartitioner's in-memory view of nodes, pod bindings and
partitioning kinds (nos_amd/partitioning/state.py).  Behaviours follow the
reference's state tests (/root/reference/internal/partitioning/state/
state_test.go:31-678: GetNode, deleteNode, deletePod, updateNode, updateUsage,
IsPartitioningEnabled) plus the order-insensitive partitioning-state equality
(/root/reference/internal/partitioning/state/partitioning_test.go)."""
from __future__ import annotations

import threading

import pytest

from nos_amd.api import constants as C
from nos_amd.kube import factory as F
from nos_amd.kube import objects as ko
from nos_amd.partitioning.state import ClusterState, GPUPartitioning, NodePartitioning, PartitioningState


def _node(name: str, kind: str | None = None, cpu: int = 8) -> dict:
    b = F.build_node(name).with_allocatable_resources({"cpu": cpu, "memory": "32Gi", "pods": 110})
    if kind:
        b = b.with_labels({C.LABEL_GPU_PARTITIONING: kind})
    return b.get()


def _pod(name: str, node: str | None = None, phase: str = ko.RUNNING, cpu_m: int = 1000, ns: str = "ns") -> dict:
    # a pod keeps its uid across updates (the state keys running pods by uid)
    b = (F.build_pod(ns, name).with_uid(f"uid-{ns}-{name}").with_phase(phase)
         .with_container(F.build_container().with_cpu_milli_request(cpu_m).get()))
    if node:
        b = b.with_node_name(node)
    return b.get()


def _names(ni) -> list[str]:
    return sorted(ko.name(pi.pod) for pi in ni.pods)


# ------------------------------------------------------------------ get / delete node
def test_get_node_missing_and_present():
    s = ClusterState()
    assert s.get_node("n0") is None
    s.update_node(_node("n0"), [])
    assert s.get_node("n0").name == "n0"
    assert set(s.get_nodes()) == {"n0"}


def test_get_nodes_is_a_snapshot_not_the_live_map():
    s = ClusterState()
    s.update_node(_node("n0"), [])
    view = s.get_nodes()
    s.update_node(_node("n1"), [])
    assert set(view) == {"n0"} and set(s.get_nodes()) == {"n0", "n1"}


def test_delete_missing_node_is_a_no_op():
    s = ClusterState()
    s.update_node(_node("n0"), [_pod("a", "n0")])
    s.delete_node("nope")
    assert set(s.get_nodes()) == {"n0"} and s.bindings == {"ns/a": "n0"}


def test_delete_node_with_pods_cleans_the_binding_table():
    s = ClusterState()
    s.update_node(_node("n0"), [_pod("a", "n0"), _pod("b", "n0")])
    s.update_node(_node("n1"), [_pod("c", "n1")])
    s.delete_node("n0")
    assert set(s.get_nodes()) == {"n1"}
    assert s.bindings == {"ns/c": "n1"}


# ------------------------------------------------------------------ delete pod
def test_delete_unknown_pod_raises():
    s = ClusterState()
    s.update_node(_node("n0"), [])
    with pytest.raises(KeyError, match="pod not found"):
        s.delete_pod("ns", "ghost")


def test_delete_pod_whose_node_is_gone_only_drops_the_binding():
    s = ClusterState()
    s.update_node(_node("n0"), [_pod("a", "n0")])
    s.nodes.pop("n0")  # node vanished between events
    s.delete_pod("ns", "a")
    assert "ns/a" not in s.bindings


def test_delete_pod_frees_its_requests_on_the_node():
    s = ClusterState()
    s.update_node(_node("n0"), [_pod("a", "n0", cpu_m=1500), _pod("b", "n0", cpu_m=500)])
    assert s.get_node("n0").requested.milli_cpu == 2000
    s.delete_pod("ns", "a")
    ni = s.get_node("n0")
    assert _names(ni) == ["b"] and ni.requested.milli_cpu == 500 and ni.requested.allowed_pod_number == 1


# ------------------------------------------------------------------ update node
def test_update_node_counts_only_running_pods_but_binds_all():
    s = ClusterState()
    pods = [_pod("run", "n0"), _pod("pend", "n0", phase=ko.PENDING), _pod("done", "n0", phase=ko.SUCCEEDED)]
    s.update_node(_node("n0"), pods)
    ni = s.get_node("n0")
    assert _names(ni) == ["run"] and ni.requested.milli_cpu == 1000
    assert set(s.bindings) == {"ns/run", "ns/pend", "ns/done"}


def test_update_node_replaces_the_previous_pods_and_bindings():
    s = ClusterState()
    s.update_node(_node("n0"), [_pod("a", "n0"), _pod("b", "n0")])
    s.update_node(_node("n0", cpu=16), [_pod("c", "n0")])
    ni = s.get_node("n0")
    assert _names(ni) == ["c"] and ni.allocatable.milli_cpu == 16000
    assert s.bindings == {"ns/c": "n0"}


# ------------------------------------------------------------------ update usage
def test_update_usage_of_an_unassigned_pod_changes_nothing():
    s = ClusterState()
    s.update_node(_node("n0"), [])
    s.update_usage(_pod("a"))
    assert _names(s.get_node("n0")) == [] and s.bindings == {}


def test_update_usage_for_a_node_not_in_the_state_changes_nothing():
    s = ClusterState()
    s.update_node(_node("n0"), [])
    s.update_usage(_pod("a", "elsewhere"))
    assert s.bindings == {} and _names(s.get_node("n0")) == []


def test_update_usage_adds_a_newly_running_pod_once():
    s = ClusterState()
    s.update_node(_node("n0"), [])
    p = _pod("a", "n0")
    s.update_usage(p)
    s.update_usage(p)  # idempotent
    ni = s.get_node("n0")
    assert _names(ni) == ["a"] and ni.requested.milli_cpu == 1000 and s.bindings == {"ns/a": "n0"}


def test_update_usage_binds_but_does_not_count_a_pending_pod():
    s = ClusterState()
    s.update_node(_node("n0"), [])
    s.update_usage(_pod("a", "n0", phase=ko.PENDING))
    assert _names(s.get_node("n0")) == [] and s.bindings == {"ns/a": "n0"}
    s.update_usage(_pod("a", "n0"))  # now running
    assert _names(s.get_node("n0")) == ["a"]


def test_update_usage_removes_a_pod_that_stopped_running():
    s = ClusterState()
    s.update_node(_node("n0"), [_pod("a", "n0")])
    s.update_usage(_pod("a", "n0", phase=ko.SUCCEEDED))
    ni = s.get_node("n0")
    assert _names(ni) == [] and ni.requested.milli_cpu == 0 and s.bindings == {"ns/a": "n0"}


def test_update_usage_moves_a_pod_between_nodes():
    s = ClusterState()
    s.update_node(_node("n0"), [_pod("a", "n0")])
    s.update_node(_node("n1"), [])
    s.update_usage(_pod("a", "n1"))
    assert _names(s.get_node("n0")) == [] and _names(s.get_node("n1")) == ["a"]
    assert s.bindings == {"ns/a": "n1"}


# ------------------------------------------------------------------ partitioning kinds
def test_partitioning_kinds_follow_node_labels():
    s = ClusterState()
    assert not s.is_partitioning_enabled(C.PARTITIONING_AMDPART)
    s.update_node(_node("n0", C.PARTITIONING_AMDPART), [])
    s.update_node(_node("n1", C.PARTITIONING_CUMASK), [])
    s.update_node(_node("n2"), [])
    s.update_node(_node("n3", "some-other-kind"), [])  # unknown kinds are ignored
    assert s.is_partitioning_enabled(C.PARTITIONING_AMDPART) and s.is_partitioning_enabled(C.PARTITIONING_CUMASK)
    assert not s.is_partitioning_enabled(C.PARTITIONING_HYBRID)
    assert s.partitioning_kinds == {C.PARTITIONING_AMDPART: 1, C.PARTITIONING_CUMASK: 1}
    s.update_node(_node("n0", C.PARTITIONING_HYBRID), [])  # relabelled
    assert not s.is_partitioning_enabled(C.PARTITIONING_AMDPART) and s.is_partitioning_enabled(C.PARTITIONING_HYBRID)
    s.delete_node("n1")
    assert not s.is_partitioning_enabled(C.PARTITIONING_CUMASK)


# ------------------------------------------------------------------ concurrency
def test_concurrent_updates_keep_requests_consistent():
    """Many threads bind, run and finish pods on four nodes; at the end every
    node's requested CPU equals the sum over the pods it holds."""
    s = ClusterState()
    for i in range(4):
        s.update_node(_node(f"n{i}"), [])

    def worker(t: int) -> None:
        for j in range(50):
            node = f"n{(t + j) % 4}"
            p = _pod(f"p{t}-{j}", node, cpu_m=100 + t)
            s.update_usage(p)
            if j % 3 == 0:
                s.update_usage(_pod(f"p{t}-{j}", node, phase=ko.SUCCEEDED, cpu_m=100 + t))
            if j % 5 == 0:
                s.get_nodes()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    total = 0
    for ni in s.get_nodes().values():
        want = sum(pi.request.milli_cpu for pi in ni.pods)
        assert ni.requested.milli_cpu == want
        total += len(ni.pods)
    assert total == 8 * (50 - 17)  # j % 3 == 0 finished: 17 of 50 per worker
    assert len(s.bindings) == 8 * 50


# ------------------------------------------------------------------ partitioning state
def test_node_partitioning_equality_ignores_gpu_order_and_zero_quantities():
    a = NodePartitioning([GPUPartitioning.of(0, {"amd.com/gpu-10gb": 2, "amd.com/gpu-20gb": 0}),
                          GPUPartitioning.of(1, {"amd.com/gpu-36gb": 1})])
    b = NodePartitioning([GPUPartitioning.of(1, {"amd.com/gpu-36gb": 1}),
                          GPUPartitioning.of(0, {"amd.com/gpu-10gb": 2})])
    assert a.equal(b) and b.equal(a)
    assert not a.equal(None)
    assert not a.equal(NodePartitioning([GPUPartitioning.of(0, {"amd.com/gpu-10gb": 2})]))
    c = NodePartitioning([GPUPartitioning.of(0, {"amd.com/gpu-10gb": 2}, mode="CPX/NPS2"),
                          GPUPartitioning.of(1, {"amd.com/gpu-36gb": 1})])
    assert not a.equal(c)  # the target mode is part of a GPU's partitioning


def test_partitioning_state_equality():
    n0 = NodePartitioning([GPUPartitioning.of(0, {"amd.com/gpu-10gb": 1})])
    n1 = NodePartitioning([GPUPartitioning.of(0, {"amd.com/gpu-20gb": 1})])
    s1 = PartitioningState({"a": n0, "b": n1})
    assert s1.equal(PartitioningState({"b": n1, "a": n0}))
    assert not s1.equal(PartitioningState({"a": n0}))
    assert not s1.equal(PartitioningState({"a": n0, "c": n1}))
    assert PartitioningState().is_empty() and not s1.is_empty()
    assert GPUPartitioning.of(3, {"x": 2, "y": 1}).resource_dict() == {"x": 2, "y": 1}
