"""Fault injection on the simulated cluster: dropped watch
events, 409 conflicts on writes, an agent restart mid-flight, a GPU that
fails to switch.  Level-triggered reconciles + periodic requeues must still
converge: every placeable pod Running, no used device ever removed."""
from __future__ import annotations

import pytest

from nos_amd.api import constants as C
from nos_amd.kube import objects as ko
from nos_amd.sim.cluster import SimCluster


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_cumask_converges_under_dropped_events_and_conflicts(seed):
    cl = SimCluster(resync_s=60)  # lost events are recovered by informer resync
    cl.api._rng.seed(seed)
    cl.add_node("n1", C.PARTITIONING_CUMASK, gpus=2)
    cl.settle(30)
    cl.api.faults.update({"drop_watch_event": 0.2, "conflict_on_write": 0.2})
    for i in range(12):
        cl.submit_pod(f"p{i}", {"amd.com/gpu-20gb": 1})
    cl.settle(1800, until=lambda: not cl.pending_pods())
    cl.api.faults.clear()
    cl.settle(120, until=lambda: not cl.pending_pods())
    assert len(cl.running_pods()) == 12
    # no device handed out twice
    envs = [rc.envs.get(C.ENV_CU_MASK, "all") + rc.envs[C.ENV_VISIBLE_DEVICES]
            for conts in cl.nodes["n1"].kubelet.running_containers().values() for rc in conts]
    assert len(envs) == len(set(envs))


def test_partition_agent_restart_keeps_state_consistent():
    from nos_amd.agents.partagent import PartitionActuator, PartitionReporter
    from nos_amd.agents.shared import SharedState

    cl = SimCluster()
    nd = cl.add_node("n1", C.PARTITIONING_AMDPART, gpus=2)
    cl.settle(30)
    for i in range(4):
        cl.submit_pod(f"s{i}", {"amd.com/partition-1xcd.36gb": 1})
    cl.settle(600, until=lambda: not cl.pending_pods())
    assert len(cl.running_pods()) == 4
    # "restart" the agent: a fresh reporter/actuator (in-memory state lost) on the same node
    nd.manager.stop()
    from nos_amd.runtime.manager import Manager

    mgr = Manager(cl.api, "node-n1-restarted", cl.clock)
    shared = SharedState()
    mgr.add(nd.kubelet.controller())
    mgr.add(PartitionReporter(cl.api, "n1", nd.smi, nd.kubelet, shared).controller())
    mgr.add(PartitionActuator(cl.api, "n1", nd.smi, nd.kubelet, shared, [nd.plugin]).controller())
    nd.manager = mgr
    switches = nd.smi.switches
    cl.settle(120)
    # the restarted agent re-derives everything from the API server and amd-smi: no spurious switch
    assert nd.smi.switches == switches and len(cl.running_pods()) == 4
    cl.submit_pod("big", {"amd.com/partition-4xcd.144gb": 1})
    cl.settle(600, until=lambda: not cl.pending_pods())
    assert ko.pod_phase(cl.api.get("Pod", "big", "default")) == ko.RUNNING
    assert sorted(nd.smi.compute) == ["CPX", "DPX"]


def test_failed_switch_leaves_pod_pending_then_recovers():
    cl = SimCluster()
    nd = cl.add_node("n1", C.PARTITIONING_AMDPART, gpus=1)
    cl.settle(30)
    nd.smi.inject("fail_set_compute")
    cl.submit_pod("s", {"amd.com/partition-1xcd.36gb": 1})
    cl.settle(300)
    assert nd.smi.compute == ["SPX"] and [ko.name(p) for p in cl.pending_pods()] == ["s"]
    nd.smi.inject("clear")
    cl.settle(900, until=lambda: not cl.pending_pods())
    assert nd.smi.compute == ["CPX"] and len(cl.running_pods()) == 1


def test_hung_mode_switch_is_bounded_and_the_reporter_keeps_reporting():
    """a switch that takes longer than ``switch_timeout_s``
    (fault ``switch_delay_ms``) must not stall the node.  The actuator stops
    waiting at the deadline and marks the GPU failed; the reporter keeps
    patching status (the switch does not hold the shared lock), so the plan
    handshake clears while the pod stays Pending; when the switch finally
    returns it is verified, the device plugin re-enumerates, the error clears
    and the pod runs (reference: actuator.go:71-123, pkg/gpu/client.go:86-135)."""
    import time

    cl = SimCluster()
    nd = cl.add_node("n1", C.PARTITIONING_AMDPART, gpus=1)
    cl.settle(30)
    act, rep = nd.agents["actuator"], nd.agents["reporter"]
    act.switch_timeout_s = 0.2
    nd.smi.inject("switch_delay_ms=1500")
    cl.submit_pod("s", {"amd.com/partition-1xcd.36gb": 1})
    t0 = time.monotonic()
    while act.timeouts == 0 and time.monotonic() - t0 < 10:
        cl.settle(20)
    assert act.timeouts == 1 and act.inflight() == {0}
    reports = rep.reports
    plan0 = ko.annotations(cl.api.get("Node", "n1"))[C.ANNOTATION_PARTITIONING_PLAN]
    cl.settle(60)
    ann = ko.annotations(cl.api.get("Node", "n1"))
    assert rep.reports > reports  # still reporting while the switch hangs
    assert "deadline" in ann[C.ANNOTATION_STATUS_ERROR_FORMAT.format(index=0)]
    assert ann[C.ANNOTATION_STATUS_MODE_FORMAT.format(index=0)] == C.MODE_SWITCHING
    # the plan handshake keeps clearing: plans written after the hang began get reported
    assert int(ann[C.ANNOTATION_REPORTED_PARTITIONING_PLAN]) >= int(plan0)
    cl.settle(60, until=lambda: ko.annotations(cl.api.get("Node", "n1")).get(C.ANNOTATION_REPORTED_PARTITIONING_PLAN)
              == ko.annotations(cl.api.get("Node", "n1")).get(C.ANNOTATION_PARTITIONING_PLAN))
    ann = ko.annotations(cl.api.get("Node", "n1"))
    assert ann[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] == ann[C.ANNOTATION_PARTITIONING_PLAN]
    assert [ko.name(p) for p in cl.pending_pods()] == ["s"]
    while cl.pending_pods() and time.monotonic() - t0 < 20:  # the switch returns after 1.5 s (real time)
        cl.settle(30)
        time.sleep(0.05)
    assert not cl.pending_pods() and len(cl.running_pods()) == 1
    cl.settle(30)
    ann = ko.annotations(cl.api.get("Node", "n1"))
    assert C.ANNOTATION_STATUS_ERROR_FORMAT.format(index=0) not in ann
    assert ann[C.ANNOTATION_STATUS_MODE_FORMAT.format(index=0)] == "CPX/NPS1"
    assert not act.inflight() and nd.smi.compute == ["CPX"]


def test_failed_switch_is_reported_on_the_node_until_it_succeeds():
    cl = SimCluster()
    nd = cl.add_node("n1", C.PARTITIONING_AMDPART, gpus=1)
    cl.settle(30)
    nd.smi.inject("fail_set_compute")
    cl.submit_pod("s", {"amd.com/partition-1xcd.36gb": 1})
    cl.settle(120)
    key = C.ANNOTATION_STATUS_ERROR_FORMAT.format(index=0)
    assert "failed" in ko.annotations(cl.api.get("Node", "n1"))[key]
    nd.smi.inject("clear")
    cl.settle(900, until=lambda: not cl.pending_pods())
    cl.settle(30)
    assert key not in ko.annotations(cl.api.get("Node", "n1"))
