"""CU-mask slice model (the reference's ``pkg/gpu/slicing/gpu_test.go`` and
``node_test.go`` behaviours) plus the MI355X-specific mask limit."""
from __future__ import annotations

import pytest

from nos_amd.gpu.core import GenericError, Geometry
from nos_amd.gpu.cumask import SliceGPU, SliceNode, SliceProfile
from nos_amd.gpu.topology import CUSlice, pack_slices, split_even, xcd_of
from nos_amd.kube import factory as kf
from nos_amd.scheduler.framework import NodeInfo

M = "AMD-Instinct-MI355X"


def P(s: str) -> SliceProfile:
    return SliceProfile(s)


def geo(d: dict[str, int]) -> dict:
    return {P(k): v for k, v in d.items()}


@pytest.mark.parametrize("mem,used,free,ok", [
    (40, {"10gb": 5}, {"20gb": 1}, False),   # profiles exceed memory
    (30, {"10gb": 2}, {"10gb": 1}, True),    # exactly fills memory
    (30, {"0gb": 2}, {"10gb": 2}, False),    # used profile below the 1 GB minimum
    (30, {"10gb": 2}, {"0gb": 2}, False),    # free profile below the minimum
])
def test_new_gpu_validation(mem, used, free, ok):
    mk = lambda: SliceGPU.new(M, 0, mem, geo(used), geo(free))  # noqa: E731
    if ok:
        g = mk()
        assert dict(g.geometry()) == geo({"10gb": 3})
    else:
        with pytest.raises((GenericError, ValueError)):
            mk()


@pytest.mark.parametrize("name,mem,used,free,required,updated,expected", [
    ("no slices required", 40, {"10gb": 2}, {"20gb": 1}, {}, False, {"10gb": 2, "20gb": 1}),
    ("already provides", 40, {}, {"20gb": 2}, {"20gb": 2}, False, {"20gb": 2}),
    ("gpu full", 40, {"20gb": 2}, {}, {"10gb": 1, "20gb": 1}, False, {"20gb": 2}),
    ("spare capacity, keep existing", 60, {"10gb": 1}, {}, {"10gb": 1, "20gb": 2}, True, {"10gb": 2, "20gb": 2}),
    ("never exceed memory", 40, {}, {}, {"10gb": 5}, True, {"10gb": 4}),
    ("smaller first", 40, {}, {}, {"20gb": 2, "10gb": 2, "5gb": 2}, True, {"5gb": 2, "10gb": 2}),
    ("delete free to make room", 40, {"20gb": 1}, {"10gb": 2}, {"20gb": 1}, True, {"20gb": 2}),
    ("free kept if room", 40, {"10gb": 2}, {}, {"20gb": 1}, True, {"10gb": 2, "20gb": 1}),
    ("delete mixed free sizes", 45, {"20gb": 1}, {"10gb": 1, "15gb": 1}, {"20gb": 1}, True, {"20gb": 2}),
    ("unchanged when impossible", 45, {"20gb": 1}, {"10gb": 1, "15gb": 1}, {"30gb": 1, "31gb": 2, "32gb": 2},
     False, {"20gb": 1, "10gb": 1, "15gb": 1}),
])
def test_update_geometry_for(name, mem, used, free, required, updated, expected):
    g = SliceGPU.new(M, 0, mem, geo(used), geo(free))
    assert g.update_geometry_for(geo(required)) is updated, name
    assert dict(g.geometry()) == geo(expected), name


def test_xcd_symmetric_mask_limit_caps_slices():
    g = SliceGPU.new(M, 0, 288, {}, {})
    g.update_geometry_for(geo({"1gb": 40}))
    assert g.num_slices() == 32  # 32 CUs per XCD -> at most 32 XCD-symmetric masks
    with pytest.raises(GenericError):
        SliceGPU.new(M, 0, 288, {}, geo({"1gb": 33}))


def test_clone_is_deep():
    g = SliceGPU.new(M, 0, 100, geo({"20gb": 1, "10gb": 2}), geo({"10gb": 1, "15gb": 1}))
    c = g.clone()
    c.free[P("10gb")] = 0
    assert g.free[P("10gb")] == 1


def test_add_pod_consumes_free_slice():
    g = SliceGPU.new(M, 0, 40, {}, geo({"10gb": 2}))
    pod = kf.build_pod("ns", "p").with_container(kf.build_container().with_scalar_resource_request(
        "amd.com/gpu-10gb", 1).get()).get()
    g.add_pod(pod)
    assert g.used[P("10gb")] == 1 and g.free[P("10gb")] == 1
    g.add_pod(pod)
    with pytest.raises(GenericError):
        g.add_pod(pod)


def _node(count: int, annotations: dict | None = None) -> SliceNode:
    n = kf.build_node("n").with_labels({"amd.com/gpu.product": M, "amd.com/gpu.count": str(count),
                                        "amd.com/gpu.memory": "294912",
                                        "nos.nebuly.com/gpu-partitioning": "cumask"}) \
        .with_annotations(annotations or {}).get()
    return SliceNode.from_node_info(NodeInfo(n))


def test_node_from_annotations_and_pack_vs_spread():
    n = _node(2, {"nos.nebuly.com/status-gpu-0-10gb-used": "2", "nos.nebuly.com/status-gpu-0-20gb-free": "1"})
    assert dict(n.gpus[0].used) == geo({"10gb": 2}) and dict(n.gpus[0].free) == geo({"20gb": 1})
    assert n.gpus[1].num_slices() == 0
    pack = _node(2)
    assert pack.update_geometry_for(geo({"10gb": 4}))
    assert [g.num_slices() for g in pack.gpus] == [4, 0]
    spread = _node(2)
    spread.placement = "spread"
    assert spread.update_geometry_for(geo({"10gb": 4}))
    assert [g.num_slices() for g in spread.gpus] == [2, 2]
    assert spread.node_info.allocatable.scalar["amd.com/gpu-10gb"] == 4


def test_topology_slices_are_xcd_symmetric():
    for n in (1, 2, 3, 4, 7, 8, 16, 32):
        slices = split_even(n)
        cus = [c for s in slices for c in s.cus()]
        assert sorted(cus) == list(range(256))  # every CU owned exactly once
        for s in slices:
            per_xcd = {}
            for c in s.cus():
                per_xcd[xcd_of(c)] = per_xcd.get(xcd_of(c), 0) + 1
            assert len(per_xcd) == 8 and len(set(per_xcd.values())) == 1
    assert pack_slices([4, 8]) == [CUSlice(0, 4), CUSlice(4, 8)]
    with pytest.raises(ValueError):
        pack_slices([30, 4])
    assert isinstance(Geometry({P("10gb"): 1}).id(), str)
