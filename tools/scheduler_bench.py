"""nos-scheduler throughput benchmark: scheduling cycles per second of the
CapacityScheduling profile over N nodes and P pending pods spread over Q
namespaces that each own an ElasticQuota (min/max on CPU and GPU memory),
including over-quota borrowing.

python tools/scheduler_bench.py [--nodes 10,100] [--pods 100,1000] [--quotas 4] [--out f.json]
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
from nos_amd.kube import factory as kf  # noqa: E402
from nos_amd.kube import objects as ko  # noqa: E402
from nos_amd.scheduler.config import nos_scheduler_config  # noqa: E402
from nos_amd.scheduler.scheduler import Scheduler  # noqa: E402
from nos_amd.sim.apiserver import ApiServer  # noqa: E402
from nos_amd.utils.clock import FakeClock  # noqa: E402


def run_one(n_nodes: int, n_pods: int, n_quotas: int, seed: int = 0) -> dict:
    rng = random.Random(seed)
    api = ApiServer(FakeClock())
    v1alpha1.register_types(api)
    for i in range(n_nodes):
        api.create(kf.build_node(f"node-{i:05d}").with_allocatable_resources(
            {"cpu": "128", "memory": "1024Gi", "pods": "500", "amd.com/gpu-10gb": "28"}).get())
    for q in range(n_quotas):
        ns = f"team-{q}"
        api.create(kf.build_namespace(ns).get())
        api.create(v1alpha1.build_eq(ns, "quota").with_min({"cpu": "50", C.RESOURCE_GPU_MEMORY: str(40 * n_nodes)})
                   .with_max({"cpu": "400", C.RESOURCE_GPU_MEMORY: str(200 * n_nodes)}).get())
    cfg = nos_scheduler_config(C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB)
    sched_name = cfg.profiles[0].scheduler_name
    sched = Scheduler(api, cfg)
    sched.start_informers()
    for i in range(n_pods):
        ns = f"team-{rng.randrange(n_quotas)}"
        api.create(kf.build_pod(ns, f"p{i:06d}").with_scheduler_name(sched_name).with_container(
            kf.build_container().with_cpu_milli_request(500).with_scalar_resource_request("amd.com/gpu-10gb", 1)
            .get()).get())
    t0 = time.perf_counter()
    cycles = sched.run_until_idle()
    dt = time.perf_counter() - t0
    bound = sum(1 for p in api.list("Pod") if ko.pod_node(p))
    return {"nodes": n_nodes, "pods": n_pods, "quotas": n_quotas, "cycles": cycles, "bound": bound,
            "seconds": round(dt, 3), "cycles_per_s": round(cycles / dt, 1) if dt else None}


def main() -> int:
    a = argparse.ArgumentParser()
    a.add_argument("--nodes", default="10,100")
    a.add_argument("--pods", default="100,1000")
    a.add_argument("--quotas", type=int, default=4)
    a.add_argument("--out", default="")
    args = a.parse_args()
    res = []
    for n in map(int, args.nodes.split(",")):
        for p in map(int, args.pods.split(",")):
            r = run_one(n, p, args.quotas)
            print(json.dumps(r), flush=True)
            res.append(r)
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
