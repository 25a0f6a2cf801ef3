"""Hybrid partitioning: compute/memory modes AND memory
slices per logical partition, the MI355X way past the 8 concurrent processes
of one logical GPU (the reference's declared-but-unused ``hybrid`` kind,
pkg/gpu/partitioning.go:87-91; slice memory rule pkg/gpu/slicing/gpu.go:67-97).

Hardware parity is unpinned: the pool cannot switch modes (no root), so these
run on the simulated node with the real scheduler, partitioner, agents and
device plugin."""
from __future__ import annotations

import pytest

from nos_amd.api import constants as C
from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin
from nos_amd.gpu.amdpart import get_allowed_geometries
from nos_amd.gpu.cumask import SliceProfile
from nos_amd.gpu.fakesmi import FakeSmi
from nos_amd.gpu.hybrid import HybridGPU, pack
from nos_amd.kube import objects as ko
from nos_amd.sim.cluster import SimCluster

G10 = SliceProfile.of(10)
G36 = SliceProfile.of(36)
G100 = SliceProfile.of(100)


def _gpu(mode="SPX/NPS1", used=None, free=None):
    modes = get_allowed_geometries("AMD Instinct MI355X")
    m = next(x for x in modes if x.id() == mode)
    return HybridGPU("AMD Instinct MI355X", 0, 288, modes, m, dict(used or {}), dict(free or {}))


def test_capacity_per_mode_is_min_memory_and_hws_slots_per_partition():
    g = _gpu()
    cap = {m.id(): g.capacity(G10, m) for m in g.modes}
    assert cap["SPX/NPS1"] == 8 and cap["DPX/NPS1"] == 16 and cap["QPX/NPS1"] == 28 and cap["CPX/NPS1"] == 24


def test_pack_respects_partition_memory_and_slots():
    assert pack({G36: 2, G10: 3}, 2, 144, 8) is not None
    assert pack({G100: 2}, 2, 144, 8) is not None and pack({G100: 3}, 2, 144, 8) is None
    assert pack({G10: 9}, 1, 288, 8) is None  # 9 processes on one logical GPU


def test_idle_gpu_switches_to_the_mode_hosting_most_of_the_demand():
    g = _gpu()
    assert g.update_geometry_for({G10: 24})
    assert g.mode.id() == "QPX/NPS1" and g.free == {G10: 24}  # QPX (4 partitions) ties CPX, fewer parts win
    g = _gpu()
    g.update_geometry_for({G10: 6})
    assert g.mode.id() == "SPX/NPS1"  # fits as is: no switch


def test_used_slices_pin_the_mode():
    g = _gpu(used={G10: 2})
    assert not g.can_switch()
    g.update_geometry_for({G10: 20})
    assert g.mode.id() == "SPX/NPS1" and g.free == {G10: 6}


def test_big_slice_demand_keeps_big_partitions():
    g = _gpu()
    g.update_geometry_for({G100: 2})
    assert g.mode.id() == "SPX/NPS1" and g.free == {G100: 2}
    g = _gpu("CPX/NPS1")
    g.update_geometry_for({G100: 2})  # a 100 GB slice does not fit a 36 GB CPX partition
    assert g.mode.id() in ("SPX/NPS1", "DPX/NPS1") and g.free == {G100: 2}


def test_device_plugin_places_slices_on_partitions_after_the_switch():
    smi = FakeSmi(gpus=1, node="n")
    plugin = NosAmdDevicePlugin("n", smi, mode=C.PARTITIONING_HYBRID, device_env="container")
    plugin.set_config("n-1", {"gpus": [{"index": 0, "mode": "CPX/NPS1",
                                        "slices": [{"profile": "10gb", "memoryGB": 10, "replicas": 24}]}]})
    devs = plugin.list_devices("amd.com/gpu-10gb")
    assert len(devs) == 24 and not any(d.healthy for d in devs)  # still SPX: nothing advertised
    smi.set_compute_partition(0, "CPX")
    plugin.refresh()
    devs = plugin.list_devices("amd.com/gpu-10gb")
    assert all(d.healthy for d in devs)
    per_part = {}
    for d in devs:
        per_part[d.partition] = per_part.get(d.partition, 0) + 1
    assert per_part == {p: 3 for p in range(8)}  # 36 GB partitions: 3 x 10 GB each
    d = next(x for x in devs if x.partition == 5)
    a = plugin.allocate("amd.com/gpu-10gb", [d.id], owner="p")
    assert a.envs[C.ENV_VISIBLE_DEVICES] == "0" and C.ENV_CU_MASK not in a.envs
    assert a.devices[1] == f"/dev/dri/renderD{smi.partitions(0)[5].drm_render}"
    assert a.envs[C.ENV_MEMORY_LIMIT_GB] == "10"


def _run(cl, n, res="amd.com/gpu-10gb", prefix="p"):
    for i in range(n):
        cl.submit_pod(f"{prefix}{i}", {res: 1})
    last = -1
    for _ in range(40):
        cl.settle(90)
        r = len(cl.running_pods())
        if r == last:
            break
        last = r
    return len(cl.running_pods())


def test_hybrid_node_runs_28_ten_gb_pods_per_gpu_vs_8_on_cumask():
    """2 simulated MI355X: hybrid places min(memory, 8 x partitions) 10 GB pods
    per GPU (QPX: 4 x 7 = 28), cumask (one logical GPU, 8 HWS process slots)
    places 8."""
    cl = SimCluster()
    nd = cl.add_node("h", C.PARTITIONING_HYBRID, gpus=2)
    cl.settle(30)
    assert _run(cl, 70) == 56
    assert nd.smi.compute == ["QPX", "QPX"]
    ann = ko.annotations(cl.api.get("Node", "h"))
    assert ann[C.ANNOTATION_REPORTED_PARTITIONING_PLAN] == ann[C.ANNOTATION_PARTITIONING_PLAN]
    assert ann[C.ANNOTATION_STATUS_MODE_FORMAT.format(index=0)] == "QPX/NPS1"
    # every running pod got a partition of its own GPU and at most 8 pods share a partition
    envs = [rc.envs for conts in nd.kubelet.running_containers().values() for rc in conts]
    per_dev = {}
    for e in envs:
        per_dev[e[C.ENV_VISIBLE_DEVICES]] = per_dev.get(e[C.ENV_VISIBLE_DEVICES], 0) + 1
    assert len(per_dev) == 8 and max(per_dev.values()) <= 8

    cl2 = SimCluster()
    cl2.add_node("c", C.PARTITIONING_CUMASK, gpus=2)
    cl2.settle(30)
    assert _run(cl2, 70) == 16


@pytest.mark.parametrize("first", ["36gb", "10gb"])
def test_mixed_slice_sizes_on_a_hybrid_node(first):
    cl = SimCluster()
    cl.add_node("h", C.PARTITIONING_HYBRID, gpus=1)
    cl.settle(30)
    sizes = ["amd.com/gpu-36gb"] * 4 + ["amd.com/gpu-10gb"] * 10
    if first == "10gb":
        sizes.reverse()
    for i, r in enumerate(sizes):
        cl.submit_pod(f"m{i}", {r: 1})
    cl.settle(1800, until=lambda: not cl.pending_pods())
    cl.settle(60)
    # 4 x 36 + 10 x 10 = 244 GB on one 288 GB GPU: every pod fits some mode
    assert len(cl.running_pods()) >= 12
