"""Planner scenarios (the reference's ``internal/partitioning/core/planner_test.go``)
for both AMD strategies, with a stub scheduler framework whose PreFilter /
Filter verdicts are programmable, plus the actuator and plan-id rules."""
from __future__ import annotations

from nos_amd.api import constants as C
from nos_amd.gpu import amdpart as ap
from nos_amd.gpu import cumask as cm
from nos_amd.kube import factory as kf
from nos_amd.partitioning.core import ClusterSnapshot, Planner, sort_pods
from nos_amd.partitioning.strategies import AmdPartPartitionCalculator, CuMaskPartitionCalculator
from nos_amd.scheduler.framework import NodeInfo, Status

M = "AMD-Instinct-MI355X"


class StubFramework:
    def __init__(self, pre=Status.ok(), flt=Status.ok()):
        self.pre, self.flt = pre, flt

    def run_pre_filter_plugins(self, state, pod):
        return None, self.pre

    def run_filter_plugins(self, state, pod, ni):
        return self.flt


def _pod(name: str, res: str, n: int = 1, prio: int | None = None) -> dict:
    b = kf.build_pod("ns", name).with_container(kf.build_container().with_cpu_milli_request(100)
                                                .with_scalar_resource_request(res, n).get())
    if prio is not None:
        b = b.with_priority(prio)
    return b.get()


def _node(name: str, kind: str, count: int = 1, ann: dict | None = None, alloc: dict | None = None) -> dict:
    return kf.build_node(name).with_labels({"amd.com/gpu.product": M, "amd.com/gpu.count": str(count),
                                            "amd.com/gpu.memory": "294912",
                                            C.LABEL_GPU_PARTITIONING: kind}) \
        .with_annotations(ann or {}).with_allocatable_resources({"cpu": "64", "memory": "512Gi", "pods": "110",
                                                                 **(alloc or {})}).get()


def _cumask_snapshot(nodes: list[dict], placement: str = "pack") -> ClusterSnapshot:
    sn = {}
    for n in nodes:
        s = cm.SliceNode.from_node_info(NodeInfo(n))
        s.placement = placement
        sn[n["metadata"]["name"]] = s
    return ClusterSnapshot(sn, CuMaskPartitionCalculator(), cm.SliceCalculator(), cm.SliceFilter())


def _amd_snapshot(nodes: list[dict]) -> ClusterSnapshot:
    sn = {n["metadata"]["name"]: ap.PartitionNode.from_node_info(NodeInfo(n)) for n in nodes}
    return ClusterSnapshot(sn, AmdPartPartitionCalculator(), ap.PartitionSliceCalculator(), ap.PartitionSliceFilter())


def _cumask_planner(fw=None) -> Planner:
    return Planner(CuMaskPartitionCalculator(), cm.SliceCalculator(), fw or StubFramework())


def _amd_planner(fw=None) -> Planner:
    return Planner(AmdPartPartitionCalculator(), ap.PartitionSliceCalculator(), fw or StubFramework())


def _res(plan, node: str) -> list[dict]:
    return [g.resource_dict() for g in sorted(plan.desired_state[node].gpus, key=lambda g: g.gpu_index)]


def test_empty_snapshot():
    plan = _cumask_planner().plan(_cumask_snapshot([]), [_pod("p", "amd.com/gpu-10gb")])
    assert plan.desired_state.is_empty()


def test_pods_without_slices_leave_state_unchanged():
    snap = _cumask_snapshot([_node("n1", "cumask", ann={"nos.nebuly.com/status-gpu-0-10gb-free": "1"})])
    plan = _cumask_planner().plan(snap, [kf.build_pod("ns", "cpu-only").get()])
    assert _res(plan, "n1") == [{"amd.com/gpu-10gb": 1}]


def test_cumask_creates_slices_on_free_capacity():
    snap = _cumask_snapshot([_node("n1", "cumask", count=2)])
    pods = [_pod(f"p{i}", "amd.com/gpu-20gb") for i in range(3)] + [_pod("q", "amd.com/gpu-10gb")]
    plan = _cumask_planner().plan(snap, pods)
    assert _res(plan, "n1") == [{"amd.com/gpu-10gb": 1, "amd.com/gpu-20gb": 3}, {}]


def test_cumask_groups_small_free_slices_into_larger():
    # 288 GB GPU: 1 used 100gb + 18 free 10gb slices (full); a 150gb pod needs the free ones dropped
    snap = _cumask_snapshot([_node("n1", "cumask", ann={"nos.nebuly.com/status-gpu-0-100gb-used": "1",
                                                        "nos.nebuly.com/status-gpu-0-10gb-free": "18"})])
    plan = _cumask_planner().plan(snap, [_pod("big", "amd.com/gpu-150gb")])
    # the original free slices are re-created all-or-nothing per profile (slicing/gpu.go:213-216):
    # 18 x 10 GB no longer fit next to 100 + 150 GB, so none come back
    assert _res(plan, "n1") == [{"amd.com/gpu-100gb": 1, "amd.com/gpu-150gb": 1}]


def test_prefilter_or_filter_failure_changes_nothing():
    for fw in (StubFramework(pre=Status.new("Unschedulable", "quota")),
               StubFramework(flt=Status.new("Unschedulable", "taint"))):
        snap = _cumask_snapshot([_node("n1", "cumask")])
        plan = _cumask_planner(fw).plan(snap, [_pod("p", "amd.com/gpu-10gb")])
        assert _res(plan, "n1") == [{}]


def test_spread_placement_balances_gpus():
    snap = _cumask_snapshot([_node("n1", "cumask", count=4)], placement="spread")
    plan = _cumask_planner().plan(snap, [_pod(f"p{i}", "amd.com/gpu-10gb") for i in range(8)])
    assert _res(plan, "n1") == [{"amd.com/gpu-10gb": 2}] * 4


def test_amdpart_switches_idle_gpu_to_cpx():
    snap = _amd_snapshot([_node("n1", "partition", count=2,
                                ann={"nos.nebuly.com/status-gpu-0-8xcd.288gb-used": "1",
                                     "nos.nebuly.com/status-gpu-1-8xcd.288gb-free": "1"})])
    plan = _amd_planner().plan(snap, [_pod(f"s{i}", "amd.com/partition-1xcd.36gb") for i in range(3)])
    gpus = sorted(plan.desired_state["n1"].gpus, key=lambda g: g.gpu_index)
    assert gpus[0].resource_dict() == {"amd.com/partition-8xcd.288gb": 1}  # in use: untouched
    assert gpus[1].resource_dict() == {"amd.com/partition-1xcd.36gb": 8} and gpus[1].mode == "CPX/NPS1"


def test_amdpart_prefers_geometry_providing_most_lacking():
    snap = _amd_snapshot([_node("n1", "partition", count=1,
                                ann={"nos.nebuly.com/status-gpu-0-8xcd.288gb-free": "1"})])
    plan = _amd_planner().plan(snap, [_pod("a", "amd.com/partition-4xcd.144gb"),
                                      _pod("b", "amd.com/partition-4xcd.144gb")])
    g = plan.desired_state["n1"].gpus[0]
    assert g.resource_dict() == {"amd.com/partition-4xcd.144gb": 2} and g.mode == "DPX/NPS1"


def test_sort_pods_priority_then_smaller_slice_first():
    pods = [_pod("big", "amd.com/gpu-40gb"), _pod("small", "amd.com/gpu-10gb"),
            _pod("vip", "amd.com/gpu-80gb", prio=100)]
    assert [p["metadata"]["name"] for p in sort_pods(pods, cm.SliceCalculator())] == ["vip", "small", "big"]


def test_snapshot_fork_revert_is_isolated():
    snap = _cumask_snapshot([_node("n1", "cumask")])
    snap.fork()
    n = snap.get_node("n1")
    n.update_geometry_for({cm.SliceProfile("10gb"): 2})
    snap.set_node(n)
    snap.revert()
    assert snap.get_node("n1").gpus[0].num_slices() == 0


def _fresh_lacking(snap: ClusterSnapshot, pod: dict):
    """lacking_resources recomputed from scratch (no cached aggregates)."""
    from nos_amd.resource.resource import Resource, compute_pod_request

    req = Resource.from_list(compute_pod_request(pod))
    alloc, requested = Resource(), Resource()
    for n in snap.get_nodes().values():
        alloc.iadd(n.node_info.allocatable)
        requested.iadd(n.node_info.requested)
    diff = alloc.subtract_non_negative(requested) - req
    return {k: -v for k, v in diff.scalar.items() if v < 0}


def test_snapshot_cached_aggregates_track_fork_add_commit_revert():
    nodes = [_node(f"n{i}", C.PARTITIONING_CUMASK, 2, alloc={"amd.com/gpu-10gb": "2"},
                   ann={"nos.nebuly.com/status-gpu-0-10gb-free": "2"}) for i in range(3)]
    snap = _cumask_snapshot(nodes)
    probe = _pod("probe", "amd.com/gpu-10gb", 5)
    assert snap.lacking_resources(probe).scalar == _fresh_lacking(snap, probe)
    snap.fork()
    snap.add_pod("n0", _pod("a", "amd.com/gpu-10gb"))
    assert snap.lacking_resources(probe).scalar == _fresh_lacking(snap, probe)
    snap.revert()
    assert snap.lacking_resources(probe).scalar == _fresh_lacking(snap, probe)
    snap.fork()
    n = snap.get_node("n1")
    assert n.update_geometry_for({cm.SliceProfile("10gb"): 6})
    snap.set_node(n)
    snap.add_pod("n1", _pod("b", "amd.com/gpu-10gb"))
    assert snap.lacking_resources(probe).scalar == _fresh_lacking(snap, probe)
    snap.commit()
    assert snap.lacking_resources(probe).scalar == _fresh_lacking(snap, probe)
    snap.add_pod("n2", _pod("c", "amd.com/gpu-10gb"))
    assert snap.lacking_resources(probe).scalar == _fresh_lacking(snap, probe)


def test_planner_scales_linearly_enough():
    """Guard for the O(nodes^2 x pods) regression the cached aggregates fixed
    (tools/planner_bench.py, profiles/r01_planner_bench.json)."""
    import time

    import tools.planner_bench as pb

    t0 = time.perf_counter()
    r = pb.run_one(C.PARTITIONING_CUMASK, 100, 500)
    assert r["placed"] == 500
    assert time.perf_counter() - t0 < 20.0


# ------------------------------------------- amdpart scenarios (planner_test.go:43-508 analogue)
def _modes(plan, node):
    return [g.mode for g in sorted(plan.desired_state[node].gpus, key=lambda g: g.gpu_index)]


ONE = "amd.com/partition-1xcd.36gb"
HALF = "amd.com/partition-4xcd.144gb"
WHOLE = "amd.com/partition-8xcd.288gb"


def test_amdpart_mixed_busy_idle_gpus_over_nodes():
    """n1: GPU0 busy (SPX used), GPU1 idle SPX; n2: CPX GPU with 3 free 1xcd.
    Five 1xcd pods: the free partitions of n2 are used first and only n1's IDLE
    GPU is switched; the busy GPU is never touched."""
    n1 = _node("n1", "partition", count=2, ann={"nos.nebuly.com/status-gpu-0-8xcd.288gb-used": "1",
                                                "nos.nebuly.com/status-gpu-1-8xcd.288gb-free": "1"})
    n2 = _node("n2", "partition", count=1, ann={"nos.nebuly.com/status-gpu-0-1xcd.36gb-used": "5",
                                                "nos.nebuly.com/status-gpu-0-1xcd.36gb-free": "3"})
    snap = _amd_snapshot([n1, n2])
    plan = _amd_planner().plan(snap, [_pod(f"s{i}", ONE) for i in range(5)])
    assert _res(plan, "n2") == [{ONE: 8}]
    r1 = _res(plan, "n1")
    assert r1[0] == {WHOLE: 1}
    assert r1[1] == {ONE: 8}


def test_amdpart_used_partitions_block_a_mode_switch():
    n1 = _node("n1", "partition", count=2, ann={"nos.nebuly.com/status-gpu-0-1xcd.36gb-used": "2",
                                                "nos.nebuly.com/status-gpu-0-1xcd.36gb-free": "6",
                                                "nos.nebuly.com/status-gpu-1-8xcd.288gb-free": "1"})
    plan = _amd_planner().plan(_amd_snapshot([n1]), [_pod("h", HALF)])
    assert _res(plan, "n1") == [{ONE: 8}, {HALF: 2}]
    assert _modes(plan, "n1")[1] == "DPX/NPS1"


def test_amdpart_steers_to_already_split_gpu_before_whole_gpu():
    """GPU0 idle SPX, GPU1 idle DPX: 1xcd demand re-splits GPU1 (already
    fractional) and keeps GPU0 whole."""
    n1 = _node("n1", "partition", count=2, ann={"nos.nebuly.com/status-gpu-0-8xcd.288gb-free": "1",
                                                "nos.nebuly.com/status-gpu-1-4xcd.144gb-free": "2"})
    plan = _amd_planner().plan(_amd_snapshot([n1]), [_pod(f"s{i}", ONE) for i in range(4)])
    assert _res(plan, "n1") == [{WHOLE: 1}, {ONE: 8}]


def test_amdpart_reserve_keeps_whole_gpus_for_whole_gpu_pods():
    n1 = _node("n1", "partition", count=2, ann={"nos.nebuly.com/status-gpu-0-8xcd.288gb-free": "1",
                                                "nos.nebuly.com/status-gpu-1-8xcd.288gb-free": "1"})
    pods = [_pod(f"s{i}", ONE) for i in range(12)]
    snap = _amd_snapshot([n1])
    for n in snap.get_nodes().values():
        n.reserve_whole_gpus = 1
    plan = _amd_planner().plan(snap, pods)
    assert sorted(map(str, _res(plan, "n1"))) == sorted(map(str, [{WHOLE: 1}, {ONE: 8}]))
    # without the reserve both GPUs are split for the 12 small pods
    plan = _amd_planner().plan(_amd_snapshot([n1]), pods)
    assert _res(plan, "n1") == [{ONE: 8}, {ONE: 8}]


def test_amdpart_memory_mode_preference():
    n1 = _node("n1", "partition", count=1, ann={"nos.nebuly.com/status-gpu-0-8xcd.288gb-free": "1"})
    for nps, want in (("NPS1", "CPX/NPS1"), ("NPS2", "CPX/NPS2")):
        snap = _amd_snapshot([n1])
        for n in snap.get_nodes().values():
            n.set_memory_mode_preference(nps)
        plan = _amd_planner().plan(snap, [_pod("s", ONE)])
        assert _modes(plan, "n1") == [want]


def test_amdpart_unsatisfiable_request_changes_nothing():
    n1 = _node("n1", "partition", count=1, ann={"nos.nebuly.com/status-gpu-0-8xcd.288gb-used": "1"})
    plan = _amd_planner().plan(_amd_snapshot([n1]), [_pod("s", ONE)])
    assert _res(plan, "n1") == [{WHOLE: 1}]


def test_amdpart_geometry_from_labels_in_planner():
    """A node whose GPUs report 256 GB plans 1xcd.32gb partitions."""
    n = _node("n1", "partition", count=1, ann={"nos.nebuly.com/status-gpu-0-8xcd.256gb-free": "1"})
    n["metadata"]["labels"]["amd.com/gpu.memory"] = "262144"
    plan = _amd_planner().plan(_amd_snapshot([n]), [_pod("s", "amd.com/partition-1xcd.32gb")])
    assert _res(plan, "n1") == [{"amd.com/partition-1xcd.32gb": 8}]


def test_amdpart_switch_puts_back_demand_its_free_partitions_covered():
    """GPU0 DPX with 2 free 4xcd partitions, GPU1 idle SPX; one
    4xcd pod and one 1xcd pod pending.  Switching GPU0 to CPX for the 1xcd pod
    destroys the free 4xcd partitions counted for the other pod, so that demand
    is lacking again and GPU1 is split to DPX: both pods are placed
    (mig/node.go:145-177 counts free devices after each GPU's update)."""
    n1 = _node("n1", "partition", count=2, ann={"nos.nebuly.com/status-gpu-0-4xcd.144gb-free": "2",
                                                "nos.nebuly.com/status-gpu-1-8xcd.288gb-free": "1"})
    plan = _amd_planner().plan(_amd_snapshot([n1]), [_pod("h", HALF), _pod("s", ONE)])
    res = _res(plan, "n1")
    total = {}
    for r in res:
        for k, v in r.items():
            total[k] = total.get(k, 0) + v
    assert total.get(HALF, 0) >= 1 and total.get(ONE, 0) >= 1, res


def test_slice_tracker_counts_lacking_and_requested_slices_and_forgets_removed_pods():
    """The reference's ``tracker_test.go``: per-pod lacking slices are summed,
    requested slices counted for every pod, and removing a pod gives back
    exactly what it added (a removed pod's lacking entries disappear at 0)."""
    from nos_amd.partitioning.core import SliceTracker

    snap = _cumask_snapshot([_node("n1", "cumask", ann={"nos.nebuly.com/status-gpu-0-10gb-free": "1"},
                                   alloc={"amd.com/gpu-10gb": "1"})])
    fits = _pod("fits", "amd.com/gpu-10gb")
    big = _pod("big", "amd.com/gpu-20gb", 2)
    more = _pod("more", "amd.com/gpu-20gb", 1)
    t = SliceTracker(snap, cm.SliceCalculator(), [fits, big, more])
    req = {str(k): v for k, v in t.get_requested_slices().items()}
    lack = {str(k): v for k, v in t.get_lacking_slices().items()}
    assert req == {"10gb": 1, "20gb": 3}
    assert lack == {"20gb": 3}  # the free 10gb slice covers "fits"
    t.remove(big)
    assert {str(k): v for k, v in t.get_lacking_slices().items()} == {"20gb": 1}
    assert {str(k): v for k, v in t.get_requested_slices().items()} == {"10gb": 1, "20gb": 1}
    t.remove(more)
    t.remove(fits)
    assert t.get_lacking_slices() == {} and t.get_requested_slices() == {}
    t.remove(_pod("never-tracked", "amd.com/gpu-20gb"))  # unknown pods: requested may not go negative
    assert t.get_lacking_slices() == {} and t.get_requested_slices() == {}
