"""Control-plane half of ``bench.py``: place the fractional pods with the real
nos-amd control plane and hand the data plane their CU masks.

Runs in-process (simulated cluster, :mod:`nos_amd.sim.cluster`) and is not
timed by the bench.  Two runs on a fresh cluster with one ``cumask`` node of
``n_gpus`` MI355X GPUs:

1. **capacity probe** -- submit far more ``amd.com/gpu-<slice>gb`` pods than
   can fit and count how many reach Running: the node's *schedulable
   fractional pods* (north-star metric, BASELINE.json);
2. **placement** -- submit ``pods_per_gpu x n_gpus`` pods; the scheduler binds
   them, the cumask partitioner writes the slice table, the device plugin
   loads it and the kubelet admits each pod with its ``ROC_GLOBAL_CU_MASK``.
   The masks of the pods the device plugin put on GPU ``local_gpu`` are what
   that rank's tenants run with.
"""
from __future__ import annotations

import re
import time

from .api import constants as C
from .api.config import GpuPartitionerConfig
from .gpu.fakesmi import FakeSmi
from .kube import objects as ko
from .sim.cluster import SimCluster


def cus_from_hex(mask: str) -> list[int]:
    v = int(mask, 16)
    out, i = [], 0
    while v:
        if v & 1:
            out.append(i)
        v >>= 1
        i += 1
    return out


def _cluster(n_gpus: int, num_cus: int, placement: str, cu_policy: str, kind: str = C.PARTITIONING_CUMASK,
             pod_server_tenants: int = 0, pod_server_dir: str = C.DEFAULT_POD_SERVER_SOCKET_DIR) -> SimCluster:
    cfg = GpuPartitionerConfig(slicePlacement=placement, cuPolicy=cu_policy)
    cl = SimCluster(partitioner_config=cfg)
    cl.add_node("mi355x-0", kind, smi=FakeSmi(gpus=n_gpus, cus=num_cus, node="mi355x-0"),
                pod_server_tenants=pod_server_tenants, pod_server_dir=pod_server_dir)
    cl.settle(30)
    return cl


def schedulable_pods(n_gpus: int, slice_gb: int, num_cus: int = 256, placement: str = "spread",
                     per_gpu_attempt: int = 40, kind: str = C.PARTITIONING_CUMASK, pod_server_tenants: int = 0
                     ) -> dict:
    """Submit ``per_gpu_attempt`` x GPUs slice pods to a fresh simulated node of
    ``kind`` and count how many reach Running through the real scheduler,
    partitioner, agents and device plugin (cumask: one logical GPU per MI355X,
    8 HWS process slots, or ``pod_server_tenants`` when the pod server hosts
    the slices; hybrid: the partitioner also picks each GPU's compute/memory
    mode, 8 slots per partition)."""
    import tempfile

    # allocation records of the probe's pod-server slices go to a scratch dir
    scratch = tempfile.TemporaryDirectory(prefix="nos_cap_") if pod_server_tenants else None
    cl = _cluster(n_gpus, num_cus, placement, "even", kind, pod_server_tenants,
                  scratch.name if scratch else C.DEFAULT_POD_SERVER_SOCKET_DIR)
    total = n_gpus * per_gpu_attempt
    for i in range(total):
        cl.submit_pod(f"cap-{i}", {f"{C.AMD_SLICE_RESOURCE_PREFIX}{slice_gb}gb": 1})
    t0 = time.perf_counter()
    sim_s, last = 0.0, -1
    while sim_s < 3600:  # until the running count is stable over a full batch window
        sim_s += cl.settle(90)
        running = len(cl.running_pods())
        if running == last:
            break
        last = running
    out = {"schedulable_fractional_pods_per_node": len(cl.running_pods()),
           "capacity_probe_sim_seconds": round(sim_s, 3), "capacity_probe_wall_seconds":
               round(time.perf_counter() - t0, 3)}
    if kind == C.PARTITIONING_HYBRID:
        node = cl.nodes["mi355x-0"]
        out["modes"] = [f"{c}/{m}" for c, m in zip(node.smi.compute, node.smi.memory)]
    if scratch is not None:
        scratch.cleanup()
    return out


def _gpu_of(env: dict) -> str:
    """Host GPU of an allocation: its HIP id, or the pod server's socket name."""
    if env.get(C.ENV_VISIBLE_DEVICES):
        return env[C.ENV_VISIBLE_DEVICES]
    sock = env.get(C.ENV_POD_SERVER, "")
    m = re.search(r"gpu-(\d+)/server\.sock$", sock.split(",")[0])
    return m.group(1) if m else ""


def control_plane_plan(n_gpus: int, pods_per_gpu: int, slice_gb: int, num_cus: int, local_gpu: int = 0,
                       placement: str = "spread", cu_policy: str = "proportional", capacity_probe: bool = True,
                       pod_server_tenants: int = 0, pod_server_dir: str = C.DEFAULT_POD_SERVER_SOCKET_DIR
                       ) -> tuple[list[list[int] | None], dict]:
    """Masks of the pods placed on ``local_gpu`` (None = unmasked) and the
    control-plane facts; ``info["envs"]`` holds each of those pods' full
    device-plugin environment (what its container is started with).
    ``pod_server_tenants`` > 0: the node's slices are pod-server slices
    (sockets under ``pod_server_dir``)."""
    info = schedulable_pods(n_gpus, slice_gb, num_cus, placement, pod_server_tenants=pod_server_tenants) \
        if capacity_probe else {}
    cl = _cluster(n_gpus, num_cus, placement, cu_policy, pod_server_tenants=pod_server_tenants,
                  pod_server_dir=pod_server_dir)
    res = f"{C.AMD_SLICE_RESOURCE_PREFIX}{slice_gb}gb"
    for i in range(n_gpus * pods_per_gpu):
        cl.submit_pod(f"yolos-{i}", {res: 1})
    t0 = time.perf_counter()
    sim_s = cl.settle(3600, until=lambda: not cl.pending_pods())
    wall = time.perf_counter() - t0
    node = cl.nodes["mi355x-0"]
    masks: list[list[int] | None] = []
    envs: list[dict[str, str]] = []
    per_gpu: dict[str, int] = {}
    for _key, conts in sorted(node.kubelet.running_containers().items()):
        for rc in conts:
            env = rc.envs
            gpu = _gpu_of(env)
            per_gpu[gpu] = per_gpu.get(gpu, 0) + 1
            if gpu == str(local_gpu):  # no mask env: the slice runs on every CU (cuPolicy shared)
                mask = env.get(C.ENV_CU_MASK) or env.get(C.ENV_POD_CU_MASK)
                masks.append(cus_from_hex(mask) if mask else None)
                envs.append({k: str(v) for k, v in env.items()})
    ann = ko.annotations(cl.api.get("Node", "mi355x-0"))
    info.update({"placed_pods": len(cl.running_pods()), "pending_pods": len(cl.pending_pods()),
                 "pods_per_gpu_placed": per_gpu, "time_to_running_sim_seconds": round(sim_s, 3),
                 "control_plane_wall_seconds": round(wall, 3),
                 "plan_id": ann.get(C.ANNOTATION_PARTITIONING_PLAN),
                 "plan_reported": ann.get(C.ANNOTATION_REPORTED_PARTITIONING_PLAN) ==
                 ann.get(C.ANNOTATION_PARTITIONING_PLAN),
                 "slice_resource": res, "cus_per_pod": len(masks[0]) if masks and masks[0] else num_cus, "cu_policy": cu_policy, "envs": envs})
    return masks, info
