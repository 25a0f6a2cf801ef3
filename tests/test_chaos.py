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
