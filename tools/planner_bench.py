"""Planner scalability benchmark (the reference's BenchmarkPlanner_Plan is
commented out, ``internal/partitioning/core/planner_test.go:857-910``; SURVEY.md
4, weakness 5).

Builds a cluster snapshot of N nodes x 8 MI355X (cumask: empty slice tables;
amdpart: every GPU idle in SPX) and P pending pods, then times one
``Planner.plan`` with the real nos-scheduler framework (CapacityScheduling +
NodeResourcesFit, as the gpupartitioner runs it).

python tools/planner_bench.py [--nodes 10,100,1000] [--pods 10,100,1000,10000] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import random
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from nos_amd.api import constants as C  # noqa: E402
from nos_amd.api import v1alpha1  # noqa: E402
from nos_amd.gpu import amdpart as ap  # noqa: E402
from nos_amd.gpu import cumask as cm  # noqa: E402
from nos_amd.kube import factory as kf  # noqa: E402
from nos_amd.partitioning.core import ClusterSnapshot, Planner  # noqa: E402
from nos_amd.partitioning.strategies import AmdPartPartitionCalculator, CuMaskPartitionCalculator  # noqa: E402
from nos_amd.scheduler.config import build_framework, nos_scheduler_config  # noqa: E402
from nos_amd.scheduler.framework import NodeInfo  # noqa: E402
from nos_amd.sim.apiserver import ApiServer  # noqa: E402
from nos_amd.utils.clock import FakeClock  # noqa: E402

M = "AMD-Instinct-MI355X"
SLICES = ["10gb", "20gb", "40gb", "80gb"]
PARTS = ["1xcd.36gb", "2xcd.72gb", "4xcd.144gb"]


def _node(i: int, kind: str) -> dict:
    return kf.build_node(f"node-{i:05d}").with_labels({
        "amd.com/gpu.product": M, "amd.com/gpu.count": "8", "amd.com/gpu.memory": "294912",
        C.LABEL_GPU_PARTITIONING: kind}).with_allocatable_resources(
        {"cpu": "256", "memory": "2048Gi", "pods": "1000"}).get()


def _pod(i: int, res: str, rng: random.Random) -> dict:
    return kf.build_pod("bench", f"p{i:06d}").with_container(
        kf.build_container().with_cpu_milli_request(100).with_scalar_resource_request(res, 1).get()) \
        .with_priority(rng.choice([0, 0, 0, 10])).get()


def snapshot(kind: str, n_nodes: int) -> ClusterSnapshot:
    nodes = [_node(i, kind) for i in range(n_nodes)]
    if kind == C.PARTITIONING_CUMASK:
        sn = {n["metadata"]["name"]: cm.SliceNode.from_node_info(NodeInfo(n)) for n in nodes}
        return ClusterSnapshot(sn, CuMaskPartitionCalculator(), cm.SliceCalculator(), cm.SliceFilter())
    sn = {n["metadata"]["name"]: ap.PartitionNode.from_node_info(NodeInfo(n)) for n in nodes}
    return ClusterSnapshot(sn, AmdPartPartitionCalculator(), ap.PartitionSliceCalculator(), ap.PartitionSliceFilter())


def run_one(kind: str, n_nodes: int, n_pods: int, seed: int = 0) -> dict:
    rng = random.Random(seed)
    api = ApiServer(FakeClock())
    v1alpha1.register_types(api)
    fw = build_framework(nos_scheduler_config(C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB).profiles[0], api=api)
    prefix = C.AMD_SLICE_RESOURCE_PREFIX if kind == C.PARTITIONING_CUMASK else C.AMD_PARTITION_RESOURCE_PREFIX
    names = SLICES if kind == C.PARTITIONING_CUMASK else PARTS
    pods = [_pod(i, prefix + rng.choice(names), rng) for i in range(n_pods)]
    t0 = time.perf_counter()
    snap = snapshot(kind, n_nodes)
    t1 = time.perf_counter()
    planner = (Planner(CuMaskPartitionCalculator(), cm.SliceCalculator(), fw) if kind == C.PARTITIONING_CUMASK
               else Planner(AmdPartPartitionCalculator(), ap.PartitionSliceCalculator(), fw))
    plan = planner.plan(snap, pods)
    t2 = time.perf_counter()
    return {"kind": kind, "nodes": n_nodes, "gpus": 8 * n_nodes, "pods": n_pods,
            "snapshot_s": round(t1 - t0, 4), "plan_s": round(t2 - t1, 4),
            "placed": planner.last_stats.get("placed"), "lacking_after": planner.last_stats.get("lacking"),
            "nodes_in_plan": len(plan.desired_state.items())}


def main() -> int:
    ap_ = argparse.ArgumentParser()
    ap_.add_argument("--nodes", default="10,100,1000")
    ap_.add_argument("--pods", default="10,100,1000,10000")
    ap_.add_argument("--kinds", default="cumask,amdpart")
    ap_.add_argument("--max-cells", type=int, default=2_000_000, help="skip nodes x pods above this")
    ap_.add_argument("--out", default="")
    a = ap_.parse_args()
    res = []
    for kind in a.kinds.split(","):
        for n in map(int, a.nodes.split(",")):
            for p in map(int, a.pods.split(",")):
                if n * p > a.max_cells:
                    continue
                r = run_one(kind, n, p)
                print(json.dumps(r), flush=True)
                res.append(r)
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
