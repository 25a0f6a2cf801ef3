"""Measured-throughput placement and xGMI-aware device choice
(nos_amd/partitioning/scoring.py; north star in BASELINE.json: the
partitioner's scoring sees real per-slice throughput).

The reference has no equivalent: candidate nodes are walked in name order
(``internal/partitioning/core/snapshot.go:93-103``) and slices are placed first
fit (``pkg/gpu/slicing/gpu.go:162-220``); these tests also pin that the
default placement keeps exactly that behaviour."""
from __future__ import annotations

from collections import Counter

from nos_amd.api import constants as C
from nos_amd.api.config import GpuPartitionerConfig
from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin
from nos_amd.gpu.cumask import SliceNode, SliceProfile
from nos_amd.gpu.fakesmi import FakeSmi
from nos_amd.kube import factory as kf
from nos_amd.kube import objects as ko
from nos_amd.partitioning import scoring
from nos_amd.partitioning.core import ClusterSnapshot
from nos_amd.partitioning.strategies import CuMaskPartitionCalculator
from nos_amd.gpu.cumask import SliceCalculator, SliceFilter
from nos_amd.scheduler.framework import NodeInfo
from nos_amd.sim.cluster import SimCluster

M = "AMD-Instinct-MI355X"
P10 = SliceProfile("10gb")


def _probe_ann(tf: dict[int, float], profile: str = "10gb") -> dict[str, str]:
    out = {}
    for gi, v in tf.items():
        out[C.ANNOTATION_SLICE_TFLOPS_FORMAT.format(index=gi, profile=profile)] = str(v)
        out[C.ANNOTATION_SLICE_GBPS_FORMAT.format(index=gi, profile=profile)] = "1000"
    return out


def _node(name: str, count: int, ann: dict | None = None, placement: str = "measured") -> SliceNode:
    n = kf.build_node(name).with_labels({"amd.com/gpu.product": M, "amd.com/gpu.count": str(count),
                                         "amd.com/gpu.memory": "294912",
                                         "nos.nebuly.com/gpu-partitioning": "cumask"}) \
        .with_annotations(ann or {}).get()
    sn = SliceNode.from_node_info(NodeInfo(n))
    sn.placement = placement
    return sn


def test_probe_table_and_capacities():
    ann = _probe_ann({0: 300.0, 1: 150.0})
    ann["nos.nebuly.com/probe-gpu-0-20gb-tflops"] = "600"
    ann["nos.nebuly.com/status-gpu-0-10gb-used"] = "2"   # not a probe key
    ann["nos.nebuly.com/probe-gpu-2-10gb-tflops"] = "garbage"
    t = scoring.probe_table(ann)
    assert t[0]["10gb"] == {"tflops": 300.0, "gbps": 1000.0} and t[0]["20gb"] == {"tflops": 600.0}
    assert 2 not in t
    caps = scoring.gpu_capacities(t, {0: {"10gb": 2, "20gb": 1}, 1: {}})
    assert caps == {0: 2 * 300.0 + 600.0, 1: 150.0}   # empty slice table: per-slice rate as lower bound
    filled = scoring.fill_unmeasured(caps, [0, 1, 3])
    assert filled[3] == (1200.0 + 150.0) / 2
    assert scoring.fill_unmeasured({}, [0, 1]) == {0: 1.0, 1: 1.0}
    assert scoring.node_score({0: 100.0, 1: 90.0}, {0: 3, 1: 0}, lambda g: True) == 90.0
    assert scoring.node_score({0: 100.0, 1: 90.0}, {0: 3, 1: 0}, lambda g: g == 0) == 25.0


def test_measured_placement_avoids_the_slow_gpu():
    # 4 GPUs, each with 2 x 10 GB slices; GPU 1 measured at a third of the others
    ann = {f"nos.nebuly.com/status-gpu-{g}-10gb-free": "2" for g in range(4)}
    ann.update(_probe_ann({0: 300.0, 1: 100.0, 2: 300.0, 3: 300.0}))
    n = _node("a", 4, ann)
    assert n.measured and n.capacity[1] == 200.0 and n.capacity[0] == 600.0
    # 4 more slices beyond the 8 free ones: none should land on GPU 1
    assert n.update_geometry_for({P10: 12})
    assert [g.num_slices() for g in n.gpus] == [4, 2, 3, 3]  # shares 200,200,200 then 150 (ties: lower index)
    # the same node under "spread" ignores the measurement
    s = _node("a", 4, ann, placement="spread")
    assert s.update_geometry_for({P10: 12})
    assert [g.num_slices() for g in s.gpus] == [3, 3, 3, 3]
    # pods go to the free slice with the best expected share
    pod = kf.build_pod("ns", "p").with_container(kf.build_container().with_scalar_resource_request(
        "amd.com/gpu-10gb", 1).get()).get()
    n2 = _node("b", 2, {"nos.nebuly.com/status-gpu-0-10gb-free": "1", "nos.nebuly.com/status-gpu-1-10gb-free": "1",
                        **_probe_ann({0: 100.0, 1: 300.0})})
    n2.add_pod(pod)
    assert n2.gpus[1].used.get(P10) == 1 and not n2.gpus[0].used


def test_candidate_nodes_by_measured_headroom_and_name_order_by_default():
    fast = _node("z-fast", 2, {"nos.nebuly.com/status-gpu-0-10gb-free": "1", **_probe_ann({0: 400.0})})
    slow = _node("a-slow", 2, {"nos.nebuly.com/status-gpu-0-10gb-free": "1", **_probe_ann({0: 100.0, 1: 100.0})})
    unmeasured = _node("m-none", 2)
    snap = ClusterSnapshot({n.name: n for n in (fast, slow, unmeasured)}, CuMaskPartitionCalculator(),
                           SliceCalculator(), SliceFilter())
    assert snap.get_candidate_nodes() == ["z-fast", "a-slow", "m-none"]
    for n in (fast, slow, unmeasured):
        n.placement = "pack"
    assert snap.get_candidate_nodes() == ["a-slow", "m-none", "z-fast"]  # the reference's name order


class _RingSmi(FakeSmi):
    """8 GPUs whose amd-smi link weights make GPUs i and i+1 (mod 8) neighbours."""

    def link(self, i, j):
        d = min((i - j) % 8, (j - i) % 8)
        return {"type": "xgmi", "hops": 1, "weight": 15 * d}


def _plugin(smi, allocation="pack", weights=None, gpus=8, slices=4):
    p = NosAmdDevicePlugin("n", smi, mode=C.PARTITIONING_CUMASK)
    cfg = {"cuPolicy": "even", "allocation": allocation,
           "gpus": [{"index": g, "slices": [{"profile": "10gb", "memoryGB": 10, "replicas": slices}]}
                    for g in range(gpus)]}
    if weights:
        cfg["gpuWeights"] = weights
    p.set_config("k", cfg)
    return p


def test_plugin_measured_allocation_uses_gpu_weights():
    p = _plugin(FakeSmi(gpus=2), "measured", {0: 100.0, 1: 300.0}, gpus=2)
    res = "amd.com/gpu-10gb"
    picks = []
    for i in range(4):
        ids = [d.id for d in p.list_devices(res) if d.id not in p.allocated]
        got = p.preferred_allocation(res, ids, [], 1)
        p.allocate(res, got, owner=f"pod{i}")
        picks.append(p.devices[got[0]].gpu_index)
    # shares: 300/1 > 300/2 > 100/1 = 300/3 (tie -> lower index) ...
    assert picks[:2] == [1, 1] and Counter(picks)[1] >= 2 and 0 in picks


def test_plugin_multi_device_requests_are_xgmi_aware():
    smi = _RingSmi(gpus=8)
    p = _plugin(smi, "pack")
    res = "amd.com/gpu-10gb"
    avail = [d.id for d in p.list_devices(res)]
    got = p.preferred_allocation(res, avail, [], 4)
    gpus = [p.devices[d].gpu_index for d in got]
    assert len(set(gpus)) == 4                       # one device per GPU
    assert gpus[:2] == [0, 1]                         # then the lowest link weight to the chosen set
    p.allocate(res, got, owner="tenant-a")
    # a second 2-GPU tenant avoids the GPUs whose links tenant-a already loads
    avail = [d.id for d in p.list_devices(res) if d.id not in p.allocated]
    got2 = p.preferred_allocation(res, avail, [], 2)
    assert not ({p.devices[d].gpu_index for d in got2} & set(gpus))
    # must_include is honoured
    inc = [d for d in avail if p.devices[d].gpu_index == 0][:1]
    got3 = p.preferred_allocation(res, avail, inc, 2)
    assert got3[0] == inc[0] and p.devices[got3[1]].gpu_index != 0


def test_sim_cluster_measured_placement_end_to_end():
    """Probe on GPU 1 reports a third of the others: once the gpuagent has
    published its measurements, new fractional pods are placed away from it."""
    def probe(gi, profile):
        return {"tflops": 100.0 if gi == 1 else 300.0, "gbps": 1000.0}

    cfg = GpuPartitionerConfig(slicePlacement="measured")
    cl = SimCluster(partitioner_config=cfg)
    nd = cl.add_node("n1", C.PARTITIONING_CUMASK, gpus=4, probe=probe)
    cl.settle(30)
    for i in range(4):
        cl.submit_pod(f"a{i}", {"amd.com/gpu-10gb": 1})
    cl.settle(600, until=lambda: not cl.pending_pods())
    cl.settle(30)  # the reporter publishes probe annotations for the new slices
    ann = ko.annotations(cl.api.get("Node", "n1"))
    assert any(k.startswith(C.ANNOTATION_PROBE_PREFIX) for k in ann)
    for i in range(8):
        cl.submit_pod(f"b{i}", {"amd.com/gpu-10gb": 1})
    cl.settle(600, until=lambda: not cl.pending_pods())
    assert len(cl.running_pods()) == 12
    per_gpu = Counter(e[C.ENV_VISIBLE_DEVICES]
                      for conts in nd.kubelet.running_containers().values() for e in (rc.envs for rc in conts))
    assert per_gpu["1"] < min(per_gpu[g] for g in ("0", "2", "3")), per_gpu
