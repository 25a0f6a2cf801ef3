"""End-to-end control-plane scenarios on the in-process cluster (the
reference's envtest integration suites): pending fractional pods
-> partitioner plan -> agent / device plugin -> kubelet -> Running."""
from __future__ import annotations

from collections import Counter

import pytest

from nos_amd.api import constants as C
from nos_amd.api import v1alpha1
from nos_amd.api.config import GpuPartitionerConfig
from nos_amd.bench_support import control_plane_plan, cus_from_hex
from nos_amd.gpu.fakesmi import FakeSmi
from nos_amd.gpu.topology import xcd_of
from nos_amd.kube import objects as ko
from nos_amd.sim.cluster import SimCluster


def _envs(node):
    return [rc.envs for conts in node.kubelet.running_containers().values() for rc in conts]


@pytest.mark.parametrize("max_procs,pods,first", [(32, 30, 28), (8, 10, 8)])
def test_cumask_pack_places_all_pods_first_fit(max_procs, pods, first):
    from nos_amd.gpu.fakesmi import FakeSmi

    cl = SimCluster()
    nd = cl.add_node("n1", C.PARTITIONING_CUMASK, smi=FakeSmi(gpus=2, node="n1", max_procs=max_procs))
    cl.settle(30)
    for i in range(pods):
        cl.submit_pod(f"p{i}", {"amd.com/gpu-10gb": 1})
    cl.settle(600, until=lambda: not cl.pending_pods())
    assert len(cl.running_pods()) == pods
    ann = ko.annotations(cl.api.get("Node", "n1"))
    assert ko.labels(cl.api.get("Node", "n1"))[C.LABEL_AMD_MAX_PROCS] == str(max_procs)
    # first fit: GPU 0 is filled before GPU 1 -- by memory (28 x 10 GB <= 288 GB, 28 <= 32 masks) or by the
    # HWS concurrent-process limit (8: more would be time-sliced)
    assert ann["nos.nebuly.com/spec-gpu-0-10gb"] == str(first)
    assert ann["nos.nebuly.com/spec-gpu-1-10gb"] == str(pods - first)
    assert ann[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] == ann[C.ANNOTATION_PARTITIONING_PLAN]
    envs = _envs(nd)
    assert Counter(e[C.ENV_VISIBLE_DEVICES] for e in envs) == {"0": first, "1": pods - first}


def test_cumask_spread_masks_are_xcd_symmetric_and_disjoint():
    cfg = GpuPartitionerConfig(slicePlacement="spread")
    cl = SimCluster(partitioner_config=cfg)
    nd = cl.add_node("n1", C.PARTITIONING_CUMASK, gpus=4)
    cl.settle(30)
    for i in range(16):  # proportional CU policy: a 72 GB slice owns a quarter of every XCD
        cl.submit_pod(f"p{i}", {"amd.com/gpu-72gb": 1})
    cl.settle(600, until=lambda: not cl.pending_pods())
    envs = _envs(nd)
    assert Counter(e[C.ENV_VISIBLE_DEVICES] for e in envs) == {str(g): 4 for g in range(4)}
    for g in range(4):
        masks = [cus_from_hex(e[C.ENV_CU_MASK]) for e in envs if e[C.ENV_VISIBLE_DEVICES] == str(g)]
        seen: set[int] = set()
        for m in masks:
            per_xcd = Counter(xcd_of(c) for c in m)
            assert len(per_xcd) == 8 and len(set(per_xcd.values())) == 1, per_xcd
            assert not (seen & set(m))
            seen |= set(m)
        assert len(seen) == 256  # the 4 slices own the whole GPU


@pytest.mark.parametrize("max_procs,expect", [(64, 32), (8, 8)])
def test_cumask_capacity_is_min_of_memory_masks_and_processes(max_procs, expect):
    from nos_amd.gpu.fakesmi import FakeSmi

    cl = SimCluster()
    cl.add_node("n1", C.PARTITIONING_CUMASK, smi=FakeSmi(gpus=1, node="n1", max_procs=max_procs))
    cl.settle(30)
    for i in range(40):
        cl.submit_pod(f"p{i}", {"amd.com/gpu-8gb": 1})
    cl.settle(300)
    # 288 GB / 8 GB = 36 by memory, 32 XCD-symmetric masks per GPU, and the HWS process limit
    assert len(cl.running_pods()) == expect


def test_amdpart_switches_modes_and_exposes_logical_devices():
    cl = SimCluster()
    nd = cl.add_node("n1", C.PARTITIONING_AMDPART, gpus=2)
    cl.settle(30)
    node = cl.api.get("Node", "n1")
    assert ko.node_allocatable(node)["amd.com/partition-8xcd.288gb"] == 2
    for i in range(8):
        cl.submit_pod(f"s{i}", {"amd.com/partition-1xcd.36gb": 1})
    cl.submit_pod("big", {"amd.com/partition-4xcd.144gb": 1})
    cl.settle(600, until=lambda: not cl.pending_pods())
    assert len(cl.running_pods()) == 9
    assert sorted(zip(nd.smi.compute, nd.smi.memory)) == [("CPX", "NPS1"), ("DPX", "NPS1")]
    vis = sorted(int(e[C.ENV_VISIBLE_DEVICES]) for e in _envs(nd))
    # CPX GPU 0 -> logical 0..7; DPX GPU 1 -> logical 8, 9
    assert vis[:8] == list(range(8)) and vis[8] in (8, 9)
    ann = ko.annotations(cl.api.get("Node", "n1"))
    assert ann[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] == ann[C.ANNOTATION_PARTITIONING_PLAN]


def test_amdpart_never_repartitions_a_busy_gpu():
    cl = SimCluster()
    nd = cl.add_node("n1", C.PARTITIONING_AMDPART, gpus=1)
    cl.settle(30)
    cl.submit_pod("whole", {"amd.com/partition-8xcd.288gb": 1})
    cl.settle(120, until=lambda: not cl.pending_pods())
    assert len(cl.running_pods()) == 1
    cl.submit_pod("small", {"amd.com/partition-1xcd.36gb": 1})
    cl.settle(300)
    assert nd.smi.compute == ["SPX"] and nd.smi.switches == 0
    assert [ko.name(p) for p in cl.pending_pods()] == ["small"]
    # the GPU drains -> the pending pod's plan can be realised
    nd.kubelet.complete_pod("default", "whole")
    cl.settle(600, until=lambda: not cl.pending_pods())
    assert nd.smi.compute == ["CPX"]
    assert [ko.name(p) for p in cl.running_pods()] == ["small"]


def test_amdpart_blocked_by_foreign_process():
    cl = SimCluster()
    smi = FakeSmi(gpus=1, node="n1")
    cl.add_node("n1", C.PARTITIONING_AMDPART, smi=smi)
    cl.settle(30)
    smi.fake_add_process(0, 4242)
    cl.submit_pod("small", {"amd.com/partition-1xcd.36gb": 1})
    cl.settle(200)
    assert smi.compute == ["SPX"]
    smi.fake_remove_process(0, 4242)
    cl.settle(600, until=lambda: not cl.pending_pods())
    assert smi.compute == ["CPX"] and len(cl.running_pods()) == 1


def test_elastic_quota_labels_running_pods():
    cl = SimCluster()
    cl.add_node("n1", C.PARTITIONING_CUMASK, gpus=1)
    # as in the reference, min/max always bound cpu and memory (elasticquotainfo.go:319-326),
    # so quotas must state them; team-a can borrow team-b's unused min
    for ns, mn in (("team-a", 20), ("team-b", 40)):
        cl.api.create({"kind": "Namespace", "metadata": {"name": ns}})
        cl.api.create(v1alpha1.build_eq(ns, "q")
                      .with_min({"nos.nebuly.com/gpu-memory": mn, "cpu": "8", "memory": "64Gi"})
                      .with_max({"nos.nebuly.com/gpu-memory": 100, "cpu": "64", "memory": "1Ti"}).get())
    cl.settle(30)
    for i in range(4):
        cl.submit_pod(f"p{i}", {"amd.com/gpu-10gb": 1}, namespace="team-a")
        cl.clock.advance(1)
    cl.settle(600, until=lambda: not cl.pending_pods())
    cl.settle(30)
    labels = {ko.name(p): ko.labels(p).get(C.LABEL_CAPACITY_INFO) for p in cl.pods("team-a")}
    assert labels == {"p0": "in-quota", "p1": "in-quota", "p2": "over-quota", "p3": "over-quota"}
    eq = cl.api.get(v1alpha1.KIND_EQ, "q", "team-a")
    assert eq["status"]["used"]["nos.nebuly.com/gpu-memory"] == "40"


@pytest.mark.parametrize("n_gpus", [1, 2])
def test_bench_control_plane_plan(n_gpus):
    masks, info = control_plane_plan(n_gpus=n_gpus, pods_per_gpu=4, slice_gb=72, num_cus=256, local_gpu=0)
    assert len(masks) == 4
    assert info["placed_pods"] == 4 * n_gpus and info["pending_pods"] == 0
    assert info["schedulable_fractional_pods_per_node"] == 4 * n_gpus  # 288 GB / 72 GB
    assert info["plan_reported"]
    assert sorted(c for m in masks for c in m) == list(range(256))


def test_baseline_config3_eight_gpus_dynamic_spx_cpx_repartitioning():
    """BASELINE config 3: one 8 x MI355X node, mixed pending partition requests
    drive SPX/DPX/QPX/CPX switches; when the small pods finish, whole-GPU
    requests switch the drained GPUs back to SPX."""
    cl = SimCluster()
    nd = cl.add_node("n1", C.PARTITIONING_AMDPART, gpus=8)
    cl.settle(30)
    want = {"amd.com/partition-1xcd.36gb": 16, "amd.com/partition-4xcd.144gb": 3,
            "amd.com/partition-2xcd.72gb": 2, "amd.com/partition-8xcd.288gb": 2}
    n = 0
    for res, k in want.items():
        for _ in range(k):
            cl.submit_pod(f"p{n}", {res: 1})
            n += 1
            cl.clock.advance(0.5)
    cl.settle(1200, until=lambda: not cl.pending_pods())
    assert len(cl.running_pods()) == n
    modes = Counter(nd.smi.compute)
    assert modes["CPX"] == 2 and modes["DPX"] == 2 and modes["QPX"] >= 1 and modes["SPX"] >= 2
    ann = ko.annotations(cl.api.get("Node", "n1"))
    assert ann[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] == ann[C.ANNOTATION_PARTITIONING_PLAN]
    # the CPX pods finish; whole-GPU demand takes the drained GPUs back to SPX
    for i in range(16):
        nd.kubelet.complete_pod("default", f"p{i}")
    for j in range(3):
        cl.submit_pod(f"w{j}", {"amd.com/partition-8xcd.288gb": 1})
        cl.clock.advance(0.5)
    cl.settle(1200, until=lambda: not cl.pending_pods())
    assert {ko.name(p) for p in cl.running_pods()} >= {"w0", "w1", "w2"}
    assert Counter(nd.smi.compute)["CPX"] == 0
    assert Counter(nd.smi.compute)["SPX"] >= 5
