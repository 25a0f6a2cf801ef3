"""Node agents in isolation (the reference's ``internal/controllers/migagent``
actuator/reporter/plan tests and ``gpuagent/reporter_int_test.go``): partition
plan from spec annotations, drain checks, reporter annotations and the
CU-mask plan handshake."""
from __future__ import annotations

from nos_amd.agents.devices import NodeDeviceClient, node_labels
from nos_amd.agents.gpuagent import AnyPartitionedGpuError, CuMaskReporter, check_spx
from nos_amd.agents.partagent import (PartitionActuator, PartitionReporter, desired_modes,
                                      new_partition_plan)
from nos_amd.agents.shared import SharedState
from nos_amd.api import constants as C
from nos_amd.gpu.fakesmi import FakeSmi
from nos_amd.kube import factory as kf
from nos_amd.kube import objects as ko
from nos_amd.resource.client import ContainerDevices, ContainerResources, PodResources
from nos_amd.runtime.manager import Request
from nos_amd.sim.apiserver import ApiServer

import pytest


class FakeLister:
    def __init__(self, allocatable: dict[str, list[str]] | None = None, used: dict[str, list[str]] | None = None):
        self.allocatable = allocatable or {}
        self.used = used or {}

    def list(self):
        return [PodResources("p", "ns", [ContainerResources("c", [ContainerDevices(r, ids)
                                                                   for r, ids in self.used.items()])])]

    def get_allocatable_resources(self):
        return [ContainerDevices(r, ids) for r, ids in self.allocatable.items()]


def _api_with_node(ann: dict | None = None) -> ApiServer:
    api = ApiServer()
    api.create(kf.build_node("n1").with_labels({C.LABEL_GPU_PARTITIONING: "partition"})
               .with_annotations(ann or {}).get())
    return api


def test_desired_modes_from_spec_profiles_and_mode_annotation():
    smi = FakeSmi(gpus=3, node="n1")
    node = kf.build_node("n1").with_annotations({
        "nos.nebuly.com/spec-gpu-0-1xcd.36gb": "8",
        "nos.nebuly.com/spec-gpu-1-4xcd.144gb": "2",
        "nos.nebuly.com/spec-gpu-2-2xcd.72gb": "4",
        "nos.nebuly.com/spec-mode-gpu-2": "QPX/NPS1"}).get()
    assert desired_modes(node, smi.gpus()) == {0: ("CPX", "NPS1"), 1: ("DPX", "NPS1"), 2: ("QPX", "NPS1")}
    assert desired_modes(node, smi.gpus(), "NPS2")[0] == ("CPX", "NPS2")


def test_partition_plan_blocks_used_and_busy_gpus():
    smi = FakeSmi(gpus=3, node="n1")
    node = kf.build_node("n1").with_annotations({f"nos.nebuly.com/spec-gpu-{i}-1xcd.36gb": "8"
                                                 for i in range(3)}).get()
    plan = new_partition_plan(node, smi.gpus(), used_gpus={0}, busy_gpus={1})
    assert [c.gpu_index for c in plan.changes] == [2]
    assert plan.blocked == {0: "partitions in use", 1: "processes running"}
    assert not plan.is_empty()


def test_actuator_applies_then_waits_for_report():
    api = _api_with_node({"nos.nebuly.com/spec-gpu-0-1xcd.36gb": "8",
                          C.ANNOTATION_PARTITIONING_PLAN: "42"})
    smi = FakeSmi(gpus=1, node="n1")
    shared = SharedState()
    refreshed = []

    class DP:
        def refresh(self):
            refreshed.append(1)

    act = PartitionActuator(api, "n1", smi, FakeLister(), shared, [DP()])
    act.reconcile(Request("n1"))
    assert smi.compute == ["CPX"] and refreshed == [1] and act.applies == 1
    assert shared.last_parsed_plan_id == "42"
    # no report since the apply: the actuator must not plan again
    res = act.reconcile(Request("n1"))
    assert res.requeue_after == 1.0 and act.applies == 1


def test_reporter_publishes_status_and_plan():
    api = _api_with_node()
    smi = FakeSmi(gpus=1, compute="CPX", node="n1")
    ids = [f"{smi.gpu(0).uuid}::p{k}" for k in range(8)]
    lister = FakeLister({"amd.com/partition-1xcd.36gb": ids}, {"amd.com/partition-1xcd.36gb": ids[:3]})
    shared = SharedState()
    shared.last_parsed_plan_id = "7"
    rep = PartitionReporter(api, "n1", smi, lister, shared)
    rep.reconcile(Request("n1"))
    ann = ko.annotations(api.get("Node", "n1"))
    assert ann["nos.nebuly.com/status-gpu-0-1xcd.36gb-used"] == "3"
    assert ann["nos.nebuly.com/status-gpu-0-1xcd.36gb-free"] == "5"
    assert ann[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] == "7"
    assert ann["nos.nebuly.com/status-mode-gpu-0"] == "CPX/NPS1"
    rv = ko.resource_version(api.get("Node", "n1"))
    rep.reconcile(Request("n1"))  # unchanged: no write
    assert ko.resource_version(api.get("Node", "n1")) == rv and shared.at_least_one_report_since_last_apply()


def test_cumask_reporter_handshake_only_when_realised():
    api = ApiServer()
    api.create(kf.build_node("n1").with_annotations({"nos.nebuly.com/spec-gpu-0-10gb": "2",
                                                     C.ANNOTATION_PARTITIONING_PLAN: "p1"}).get())
    smi = FakeSmi(gpus=1, node="n1")
    uuid = smi.gpu(0).uuid
    lister = FakeLister({"amd.com/gpu-10gb": [f"{uuid}::10gb::0"]})
    rep = CuMaskReporter(api, "n1", smi, lister, probe=lambda g, p: {"tflops": 300.0, "gbps": 1600.0})
    rep.reconcile(Request("n1"))
    ann = ko.annotations(api.get("Node", "n1"))
    assert C.ANNOTATION_REPORTED_PARTITIONING_PLAN not in ann  # only 1 of the 2 spec'd slices exists
    assert ann["nos.nebuly.com/probe-gpu-0-10gb-tflops"] == "300.0"
    lister.allocatable["amd.com/gpu-10gb"].append(f"{uuid}::10gb::1")
    rep.reconcile(Request("n1"))
    assert ko.annotations(api.get("Node", "n1"))[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] == "p1"


def test_gpuagent_refuses_partitioned_gpus():
    check_spx(FakeSmi(gpus=2))
    with pytest.raises(AnyPartitionedGpuError):
        check_spx(FakeSmi(gpus=2, compute="CPX"))


def test_device_client_maps_uuids_and_labels():
    smi = FakeSmi(gpus=2, node="n1")
    u1 = smi.gpu(1).uuid
    dc = NodeDeviceClient(smi, FakeLister({"amd.com/gpu-10gb": [f"{u1}::10gb::0", "GPU-unknown::x"]},
                                          {"amd.com/gpu-10gb": [f"{u1}::10gb::0"]}))
    devs = dc.get_devices("amd.com/gpu-")
    assert [(d.gpu_index, d.status) for d in devs] == [(1, "used")]
    assert dc.used_gpus() == {1}
    lab = node_labels(smi)
    assert lab[C.LABEL_AMD_COUNT] == "2" and lab[C.LABEL_AMD_PRODUCT] == "AMD-Instinct-MI355X"


def test_actuator_rolls_back_a_switch_that_does_not_take_effect():
    api = _api_with_node({"nos.nebuly.com/spec-gpu-0-1xcd.36gb": "8"})
    smi = FakeSmi(gpus=1, node="n1")
    smi.inject("stale_mode")
    act = PartitionActuator(api, "n1", smi, FakeLister(), SharedState())
    act._verify = lambda *a, **k: PartitionActuator._verify(act, *a, retries=2, delay_s=0)
    act.reconcile(Request("n1"))
    assert act.failures == 1 and smi.compute == ["SPX"]
    smi.inject("clear")


def test_actuator_survives_device_lost_after_switch():
    api = _api_with_node({"nos.nebuly.com/spec-gpu-0-1xcd.36gb": "8"})
    smi = FakeSmi(gpus=1, node="n1")
    smi.inject("lose_after_switch")
    act = PartitionActuator(api, "n1", smi, FakeLister(), SharedState())
    act._verify = lambda *a, **k: PartitionActuator._verify(act, *a, retries=1, delay_s=0)
    act.reconcile(Request("n1"))
    assert act.failures == 1 and smi.count() == 0  # reported as failed, no crash


def test_plan_report_latency_from_spans():
    from nos_amd.observability import tracing

    tracing.clear()
    with tracing.span("partitioner.plan", kind="cumask") as s:
        s.set(plan_id="p9")
    tracing.event("agent.plan_reported", plan_id="p9", node="n1")
    lat = tracing.plan_report_latencies()
    assert set(lat) == {"p9"} and lat["p9"] >= 0
