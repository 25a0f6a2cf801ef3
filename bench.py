"""nos-amd headline benchmark: fractional-GPU pods per node and aggregate GPU
utilisation on MI355X, measured with the pods running as separate processes.

Metric (BASELINE.json): "aggregate GPU util % + schedulable fractional
pods/node".  The reference's only published benchmark is the GPU-sharing
demo (``demos/gpu-sharing-comparison``): YOLOS-small inference pods, each
requesting a GPU slice, inferring back to back in fp32; the table reports the
average inference time over a steady-state window (README.md:53-71).

What one run does, per GPU (one rank per GPU, RCCL for the rank barrier):

1. control plane (untimed, CPU): the nos-amd scheduler, cumask partitioner
   and device plugin (in-process simulated cluster) place ``--pods-per-gpu``
   pods requesting ``amd.com/gpu-<slice>gb`` on an N-GPU node.  Each pod
   gets the device plugin's allocation env: ``NOS_AMD_POD_SERVER`` (the
   GPU's server socket) + ``NOS_AMD_MEMORY_LIMIT_GB`` in server mode,
   otherwise ``HIP_VISIBLE_DEVICES``, ``NOS_AMD_MEMORY_LIMIT_GB`` and, for
   ``--mode cumask``, ``ROC_GLOBAL_CU_MASK``.  The node's schedulable capacity
   for the slice size is also counted by the simulator
   (``schedulable_fractional_pods_per_node_sim``);
2. data plane: in server mode one pod server per rank (its GPU,
   ``--server-lanes`` streams); each pod is started as its own process with
   its env (:mod:`nos_amd.models.pod`), YOLOS-small fp32 (the reference's
   precision), random-init weights, a synthetic 800x1066 image;
3. once every pod is warm, ``--warmup`` then ``--steps`` slices of
   ``--step-s`` wall seconds are timed (barrier + synchronize on both
   sides); amd-smi gfx activity of the GPU is sampled at 50 Hz throughout.
   A pod counts as running concurrently when it completed inferences all
   through the window (no gap > 25 % of it).

value = fractional pods observed running concurrently on the node (all GPUs).
Default ``--mode server``: the pods' slices are served by the GPU's pod server
(nos_amd/podserver, the MPS analogue).  Every pod is its own CPU-only client
process, and its inferences run as HIP-graph replays in one server process per
GPU.  Separate GPU processes are bounded by the amdgpu hardware scheduler,
which runs at most 8 GPU processes per logical GPU at once
(hws_max_conc_proc; more are time-sliced at a ~50 ms quantum and aggregate
throughput falls: profiles/r02_pods_vs_throughput_hwqueues.json).  The server
is ONE such process, so as with the reference's MPS only memory bounds the
slices: 28 x 10 GB pods per 288 GB MI355X, the reference's 10 GB slice size.
``--mode shared|cumask`` runs each pod as its own GPU process (8 x 36 GB
slices, the HWS bound; node label amd.com/gpu.max-concurrent-processes,
nos_amd/gpu/kfd.py).  vs_baseline =
value / (8 x GPUs): 8 is the reference's schedulable 10 GB fractional pods per
A100-80GB (MPS).  gpu_util_pct is the mean amd-smi gfx activity over the window.
aggregate_inf_per_s (fp32) is compared with 21.89 inf/s per GPU (the
reference's best aggregate, 7 MPS pods on one A100).

Also in the JSON: one whole-GPU pod's rate (``--ref-pod-s``), a bf16 fleet on
the gfx950 kernels (``--extra-bf16-s``), the reference demo's latency table
(1/3/5/7 pods: pod-server, shared and CU-mask slices; default on single-GPU runs,
``--table``), and with WORLD_SIZE > 1 a data-parallel trainer pod per GPU
(slot 0: its own pod process with its device-plugin env, CU mask included,
nos_amd/models/trainer_pod.py -- bf16 MLP forward + backward with bucketed
RCCL all-reduces over xGMI launched from the gradient hooks, the trainer pods
of all GPUs one job in lockstep), so slices are measured under collective
traffic.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

BASELINE_PODS_PER_GPU = 8           # 80 GB / 10 GB MPS slices on A100-80GB
BASELINE_INF_PER_S_PER_GPU = 21.89  # 7 / 0.3198 s, MPS 7 pods, A100-80GB
BASELINE_SINGLE_POD_INF_PER_S = 11.37  # 1 / 0.0880 s, 1 pod owning the A100
METRIC = "aggregate GPU util % + schedulable fractional pods/node at 1/2/4/8 MI355X"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--step-s", type=float, default=0.6, help="wall seconds per timed step")
    ap.add_argument("--pods-per-gpu", type=int, default=0,
                    help="default: 28 in server mode (10 GB slices fill 288 GB), else 8 (the HWS process limit)")
    ap.add_argument("--slice-gb", type=int, default=0, help="GPU memory per fractional pod (default 10 / 36)")
    ap.add_argument("--mode", choices=["server", "shared", "cumask"], default="server",
                    help="server: slices served by the GPU's pod server (nos_amd/podserver, the MPS analogue: "
                         "pods are CPU-only client processes, their inferences run in one HIP context); "
                         "shared: each pod its own GPU process, memory-capped, kernels on all CUs; "
                         "cumask: each pod its own GPU process with exclusive XCD-symmetric CUs")
    ap.add_argument("--server-lanes", type=int, default=16,
                    help="pod server lanes (streams, one hardware queue each) the tenants' graphs run on; 16 with "
                         "the h3 kernels: 712.7 vs 702.3 (12) / 673.5 (8) / 628.4 (20) inf/s at 28 tenants "
                         "(profiles/r04_h3_lanes_ab.json)")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--ref-pod-s", type=float, default=4.0,
                    help="window of the single full-GPU pod reference run (0 = skip)")
    ap.add_argument("--extra-bf16-s", type=float, default=4.0,
                    help="window of an extra bf16 (gfx950 kernels) fleet run (0 = skip)")
    ap.add_argument("--hw-queues", type=int, default=0, help="GPU_MAX_HW_QUEUES per pod (0 = HIP default)")
    ap.add_argument("--bursty", default="", metavar="ON_S:OFF_S",
                    help="bursty tenants: every pod infers for ON_S seconds then idles OFF_S, out of phase "
                         "with the others (utilisation under statistical multiplexing)")
    ap.add_argument("--collective", choices=["auto", "on", "off"], default="auto",
                    help="one of each GPU's pods is a DP trainer (bf16 GEMM + RCCL all-reduce over xGMI, in "
                         "lockstep across ranks); auto: on when WORLD_SIZE > 1")
    ap.add_argument("--coll-dim", type=int, default=4096)
    ap.add_argument("--coll-bucket-mb", type=int, default=64)
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: rehearsal of the whole launch path without a GPU (tiny pods, gloo)")
    ap.add_argument("--table", default="auto",
                    help="also measure the reference demo's latency table: comma list of pod counts per GPU "
                         "(e.g. 1,3,5,7), one aligned window per (mode, count), reported as latency_table; "
                         "auto = 1,3,5,7 on single-GPU runs, none on multi-GPU runs; '' = none")
    ap.add_argument("--table-modes", default="shared,cumask")
    ap.add_argument("--table-window-s", type=float, default=5.0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--tenant-mix", default="", metavar="FAMILY:N,...",
                    help="server mode: a mixed fleet of model families, e.g. yolos:16,resnet:6,llama:6 "
                         "(pods of the other families ship prebuilt programs; per-family throughput in 'mix')")
    ap.add_argument("--isolate-team-b", action="store_true",
                    help="with --quota --composed: team-b's tenants on an isolated CU pool (cuPolicy split), "
                         "measured alone and while team-a bursts on the shared pool")
    ap.add_argument("--composed", action="store_true",
                    help="with --quota: BASELINE config 5 composed -- DP trainer pods, bursty team-a waves, a "
                         "simulated amdpart repartition, then preemption (quotabench.ComposedScenario)")
    ap.add_argument("--quota", action="store_true",
                    help="BASELINE config 5 instead of the headline: two namespaces' ElasticQuotas on the GPU's "
                         "pod-server slices, borrowing then fair-share preemption acting on running tenants "
                         "(nos_amd/quotabench.py); prints its own JSON line")
    return ap.parse_args(argv)


def log(rank: int, msg: str) -> None:
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


POD_SERVER_TENANTS = 48  # per GPU, MPS's client limit; memory bounds it first (28 x 10 GB)


def plan(args, world: int, local: int, slice_gb: int, pods: int, mode: str) -> tuple[list[dict], dict]:
    from nos_amd.bench_support import control_plane_plan

    _, info = control_plane_plan(n_gpus=world, pods_per_gpu=pods, slice_gb=slice_gb, num_cus=256, local_gpu=local,
                                 cu_policy="proportional" if mode == "cumask" else "shared", capacity_probe=True,
                                 pod_server_tenants=POD_SERVER_TENANTS if mode == "server" else 0,
                                 pod_server_dir=getattr(args, "pod_server_dir", "/tmp/nos_ps"))
    envs = info.pop("envs")
    if os.environ.get("NOS_AMD_BENCH_FOLD_GPUS") == "1":
        # rehearsal of the multi-rank path on fewer GPUs than ranks (gloo between
        # the ranks, which RCCL cannot do on a shared GPU): rank r's pods go to
        # GPU r % visible GPUs, as the rank itself does (Dist.init_gpu)
        import torch

        # may initialise HIP (when amdsmi is unusable): main() starts the pod
        # launcher before the first plan(), so no pod is forked from a GPU process
        gpu = str(local % max(1, torch.cuda.device_count()))
        envs = [{**e, "HIP_VISIBLE_DEVICES": gpu} for e in envs]
    return envs, info


class Dist:
    """Rank-level barrier/reductions: RCCL when every rank owns a GPU."""

    def __init__(self, device: str = "cuda"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.cuda = device == "cuda"
        self.backend = os.environ.get("NOS_AMD_BENCH_BACKEND", "nccl" if self.cuda else "gloo")
        self.dist = None
        self.device = self.local

    def init_gpu(self) -> None:
        import torch
        import torch.distributed as dist

        if not self.cuda:
            if self.world > 1:
                dist.init_process_group("gloo")
                self.dist = dist
            return
        dev = self.local if self.backend == "nccl" else self.local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev)
        self.device = dev
        if self.world > 1:
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            else:
                dist.init_process_group(self.backend)
            self.dist = dist

    def barrier_sync(self) -> None:
        import torch

        if self.cuda:
            torch.cuda.synchronize()
        if self.dist:
            self.dist.barrier()
        if self.cuda:
            torch.cuda.synchronize()

    def reduce(self, vals: list[float], op: str) -> list[float]:
        if not self.dist:
            return list(vals)
        import torch

        dev = "cuda" if (self.cuda and self.backend == "nccl") else "cpu"
        t = torch.tensor(vals, dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return t.tolist()

    def gather(self, obj) -> list:
        """Every rank's ``obj`` (picklable), in rank order."""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self) -> None:
        if self.dist:
            self.dist.destroy_process_group()


class UtilSampler:
    """amd-smi gfx activity of this rank's GPU at a fixed period; windows are
    cut out of the sample stream by timestamp."""

    def __init__(self, hip_id: int, period_s: float = 0.02, smi=None):
        """``hip_id``: this rank's GPU as HIP numbers it; amd-smi is asked by
        ITS index (the two orders can differ on a node)."""
        self.samples: list[tuple[float, int]] = []
        self.umc: list[tuple[float, int]] = []      # memory-controller (HBM) activity %, same stream
        self.clocks: list[tuple[float, int]] = []
        self.err = None
        self._stop = threading.Event()
        self.period = period_s
        try:
            if smi is None:
                from nos_amd.gpu.amdsmi import AmdSmi

                smi = AmdSmi.real()
            self.smi = smi
            ids = {g.hip_id: g.index for g in self.smi.gpus()}
            self.index = ids.get(hip_id, hip_id)
        except Exception as e:  # amd-smi unusable here: util unreported
            self.smi, self.err = None, repr(e)
        self._t = threading.Thread(target=self._run, daemon=True)
        if self.smi is not None:
            self._t.start()

    def _run(self) -> None:
        nxt = time.monotonic()
        k = 0
        while not self._stop.is_set():
            try:
                a = self.smi.activity(self.index)
                now = time.monotonic()
                self.samples.append((now, a["gfx"]))
                self.umc.append((now, a["umc"]))
                if k % 5 == 0:  # GFX clock at 10 Hz: tells DVFS apart from contention
                    self.clocks.append((time.monotonic(), self.smi.clock(self.index)["sclk_mhz"]))
            except Exception as e:
                self.err = repr(e)
            k += 1
            nxt += self.period
            self._stop.wait(max(0.0, nxt - time.monotonic()))

    def mean(self, t0: float, t1: float) -> tuple[float | None, int]:
        v = [u for t, u in self.samples if t0 <= t <= t1]
        return (sum(v) / len(v) if v else None), len(v)

    def mean_umc(self, t0: float, t1: float) -> float | None:
        v = [u for t, u in self.umc if t0 <= t <= t1]
        return round(sum(v) / len(v), 1) if v else None

    def mean_sclk(self, t0: float, t1: float) -> float | None:
        v = [u for t, u in self.clocks if t0 <= t <= t1]
        return round(sum(v) / len(v)) if v else None

    def close(self) -> None:
        self._stop.set()
        if self._t.is_alive():
            self._t.join(timeout=2)


def fleet_window(d: Dist, fleet, warmup: int, steps: int, step_s: float, sampler: UtilSampler | None):
    """Warm-up then timed steps of ``step_s`` wall seconds with every pod running."""
    t_end = time.monotonic() + warmup * step_s
    last_log = time.monotonic()
    while time.monotonic() < t_end:
        time.sleep(0.05)
        if time.monotonic() - last_log > 30:  # long reference-style warm-ups: show progress
            last_log = time.monotonic()
            log(d.rank, f"warm-up: {t_end - last_log:.0f} s left")
            fleet.check_alive()
    fleet.check_alive()
    d.barrier_sync()
    t0 = time.monotonic()
    for k in range(steps):
        deadline = t0 + (k + 1) * step_s
        while True:
            now = time.monotonic()
            if now >= deadline:
                break
            time.sleep(min(0.05, deadline - now))
        fleet.check_alive()
        if time.monotonic() - last_log > 30:
            last_log = time.monotonic()
            log(d.rank, f"window: step {k + 1}/{steps}")
    d.barrier_sync()
    t1 = time.monotonic()
    util = sampler.mean(t0, t1) if sampler else (None, 0)
    if sampler:
        fleet.sclk_mhz = sampler.mean_sclk(t0, t1)
        fleet.umc_pct = sampler.mean_umc(t0, t1)
    return t0, t1, util


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


TENANT_FAMILIES = ("yolos", "resnet", "llama")


def assign_tenant_mix(args, envs: list[dict]) -> list[str]:
    """``--tenant-mix yolos:16,resnet:6,llama:6``: build the non-YOLOS
    programs once (ResNet-18 at 224x224 via torch.fx, a random-init Llama
    decoder at seq 512), write them under the pod-server directory, and point
    pod slots at them (NOS_AMD_POD_PROGRAM), interleaved so each family is
    spread over the fleet.  Returns the family of every pod slot."""
    from nos_amd.podserver.program import save_program

    want = []
    for part in args.tenant_mix.split(","):
        fam, n = part.split(":")
        if fam not in TENANT_FAMILIES:
            raise SystemExit(f"--tenant-mix: family must be one of {TENANT_FAMILIES}, got {fam!r}")
        want += [fam] * int(n)
    if len(want) != len(envs):
        raise SystemExit(f"--tenant-mix names {len(want)} pods, the fleet has {len(envs)}")
    # interleave: slot i takes the family furthest behind its share
    order, cnt = [], {f: 0 for f in TENANT_FAMILIES}
    tot = {f: want.count(f) for f in TENANT_FAMILIES}
    for i in range(len(want)):
        f = min((f for f in TENANT_FAMILIES if cnt[f] < tot[f]), key=lambda f: (cnt[f] + 1) / tot[f])
        cnt[f] += 1
        order.append(f)
    small = args.device == "cuda"
    built = {}
    for fam in set(order) - {"yolos"}:
        prefix = os.path.join(args.pod_server_dir, f"program-{fam}")
        if fam == "resnet":
            from nos_amd.models.resnet import resnet_tenant

            save_program(prefix, *resnet_tenant(args.dtype, 0, small=small))
        else:
            from nos_amd.models.llama_program import llama_tenant

            save_program(prefix, *llama_tenant(args.dtype, 0, small=small))
        built[fam] = prefix
    for e, fam in zip(envs, order):
        if fam in built:
            e["NOS_AMD_POD_PROGRAM"] = built[fam]
    args.extra_bf16_s, args.table, args.ref_pod_s = 0.0, "", 0.0
    return order


def mix_stats(w, families: list[str]) -> dict:
    """Per-family inferences/s and mean latency of a mixed fleet window."""
    out = {}
    for p in w.inference_pods:
        fam = families[p.slot] if p.slot < len(families) else "?"
        f = out.setdefault(fam, {"pods": 0, "completed": 0.0, "running": 0, "program": p.info.get("program")})
        f["pods"] += 1
        f["completed"] += p.completed
        f["running"] += int(p.running)
    for f in out.values():
        f["inf_per_s"] = round(f.pop("completed") / w.window_s, 2) if w.window_s else 0.0
        f["mean_latency_s"] = round(f["pods"] / f["inf_per_s"], 5) if f["inf_per_s"] else None
    return out


def with_trainer(d: Dist, envs: list[dict], args) -> list[dict]:
    """Pod slot 0 of every GPU becomes the DP trainer pod: the same device-plugin
    env plus the job's rendezvous (rank 0 picks a fresh port, every rank learns
    it through the bench's own group).  Collective call: all ranks, same order.
    On a pod-server slice the trainer is still its own GPU process (RCCL needs
    its own context): it gets the GPU instead of the server socket."""
    port = int(d.reduce([float(_free_port()) if d.rank == 0 else 0.0], "max")[0])
    e0 = dict(envs[0])
    if e0.pop("NOS_AMD_POD_SERVER", None) is not None:
        e0["HIP_VISIBLE_DEVICES"] = args.gpu_env
    t = {**e0, "NOS_AMD_POD_KIND": "trainer", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
         "RANK": str(d.rank), "WORLD_SIZE": str(d.world), "LOCAL_RANK": "0",
         "NOS_AMD_COLL_DIM": str(args.coll_dim), "NOS_AMD_COLL_BUCKET_MB": str(args.coll_bucket_mb),
         # a job that cannot form fails within 2 minutes: every rank then measures without it
         "NOS_AMD_TRAINER_TIMEOUT_S": os.environ.get("NOS_AMD_TRAINER_TIMEOUT_S", "120")}
    if not d.cuda or os.environ.get("NOS_AMD_BENCH_FOLD_GPUS") == "1":
        t["NOS_AMD_TRAINER_BACKEND"] = "gloo"  # several ranks' trainers on one GPU: RCCL refuses that
    return [t] + list(envs[1:])


def trainer_stats(w) -> dict | None:
    """This rank's trainer pod over the window: iterations, GEMM TFLOP/s,
    gradient bytes all-reduced per second, and its one-bucket busbw probe."""
    tps = w.trainer_pods
    if not tps:
        return None
    p = tps[0]
    i = p.info
    n_it = p.completed
    return {"iterations": round(n_it, 2), "running": p.running, "max_gap_s": round(p.max_gap_s, 3),
            "gemm_tflops": round(n_it * (i.get("flops_per_step") or 0) / w.window_s / 1e12, 2),
            "buckets": i.get("buckets"), "buckets_launched_in_backward": i.get("launched_in_backward"),
            "allreduce_gb_per_s": round(n_it * (i.get("bucket_bytes") or 0) / w.window_s / 1e9, 4)
            if (i.get("world_size") or 1) > 1 else 0.0,
            "bucket_busbw_gbps": i.get("bucket_busbw_gbps"), "backend": i.get("backend"),
            "cu_mask": i.get("cu_mask"), "pid": i.get("pid")}


class FleetStartError(RuntimeError):
    """Pods of some rank failed to start; raised on EVERY rank (the flag is reduced)."""


GPU_PROCS = {"max": 0, "runs": []}  # GPU processes per GPU in every fleet run (HWS bound: hws_max_conc_proc)


def gpu_processes(envs: list[dict], server_alive: bool) -> int:
    """GPU processes on this rank's GPU while ``envs`` run: this rank, the pod
    server, and every pod that is not a pod-server client (process pods, the
    DP trainer)."""
    from nos_amd.api import constants as C

    return 1 + int(server_alive) + sum(1 for e in envs if not e.get(C.ENV_POD_SERVER))


def run_fleet(d: Dist, launcher, envs, dtype, graphs, extra_env, warmup, steps, step_s, sampler, device="cuda",
              server_alive: bool = False):
    from nos_amd.podbench import PodFleet

    n = gpu_processes(envs, server_alive)
    GPU_PROCS["max"] = max(GPU_PROCS["max"], n)
    GPU_PROCS["runs"].append(n)

    fleet = PodFleet(envs, dtype=dtype, graphs=graphs, extra_env=extra_env, launcher=launcher, device=device)
    try:
        err = None
        try:
            fleet.start()
            ready_s = fleet.wait_ready(timeout_s=900,
                                       progress_cb=lambda n, t: log(d.rank, f"{dtype} pods ready {n}/{t}"))
        except Exception as e:  # every rank learns of it below instead of waiting at a barrier
            err = e
        failed, = d.reduce([1.0 if err else 0.0], "max")
        if err:
            raise FleetStartError(f"{dtype} pods failed to start: {err!r}") from err
        if failed:
            raise FleetStartError(f"pods of another rank failed to start ({dtype})")
        d.barrier_sync()
        t0, t1, (util, n_util) = fleet_window(d, fleet, warmup, steps, step_s, sampler)
        fleet.stop()
        w = fleet.window(t0, t1)
        w.sclk_mhz = getattr(fleet, "sclk_mhz", None)
        w.umc_pct = getattr(fleet, "umc_pct", None)
    finally:
        fleet.close()
    return w, util, n_util, ready_s, trainer_stats(w)


class PodServerProc:
    """This rank's pod server (nos_amd/cmd/podserver.py), started by the clean
    launcher like the pods, on the rank's GPU."""

    def __init__(self, launcher, args, gpu_env: str, workdir: str):
        import subprocess

        from nos_amd.podbench import REPO

        from nos_amd.podserver.allocations import socket_path

        self.path = str(socket_path(args.pod_server_dir, args.local_gpu))
        env = {k: v for k, v in os.environ.items()
               if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                            "ROC_GLOBAL_CU_MASK", "CUDA_VISIBLE_DEVICES") and not k.startswith("TORCHELASTIC_")}
        env.update({"HIP_VISIBLE_DEVICES": gpu_env, "PYTHONPATH": str(REPO) + os.pathsep + env.get("PYTHONPATH", "")})
        # the server reads the slices from the records the (simulated) device
        # plugin wrote when it allocated them (tokens; podserver/allocations.py)
        cmd = [sys.executable, "-u", "-m", "nos_amd.cmd.podserver", "--gpu", str(args.local_gpu), "--hip-id",
               gpu_env, "--socket-dir", args.pod_server_dir,
               # a CPU rehearsal's lanes are threads on the host's cores: a few serve every tenant
               "--lanes", str(args.server_lanes if args.device == "cuda" else min(args.server_lanes, 4)),
               "--max-tenants", str(POD_SERVER_TENANTS), "--device", args.device]
        self.log = os.path.join(workdir, "podserver.log")
        self.proc = launcher.spawn(cmd, env, self.log, str(REPO))
        self._timeout = subprocess.TimeoutExpired

    def wait_ready(self, timeout_s: float = 300.0) -> float:
        t0 = time.monotonic()
        while not os.path.exists(self.path):
            if self.proc.poll() is not None:
                raise RuntimeError(f"pod server exited ({self.proc.poll()}): {open(self.log).read()[-2000:]}")
            if time.monotonic() - t0 > timeout_s:
                raise TimeoutError(f"pod server not ready after {timeout_s} s")
            time.sleep(0.1)
        return time.monotonic() - t0

    def info(self) -> dict:
        from nos_amd.podserver.client import PodClient

        c = PodClient(self.path, connect_timeout_s=5)
        try:
            st = c.stats()
        finally:
            c.close()
        return {"pid": st.get("pid"), **{k: st["server"].get(k) for k in ("lanes", "hw_queues", "device")}}

    def close(self) -> None:
        if self.proc.poll() is None:
            self.proc.kill()


def _normalise_table(table: list[dict]) -> None:
    """Per row: latency over the same mode's 1-pod row, raw and at the 1-pod
    row's GFX clock (latency scales as 1/clock): under load the MI355X clock
    drops (DVFS), which the raw ratio mixes with contention between pods."""
    solo = {r["mode"]: r for r in table if r["pods"] == 1 and r.get("mean_latency_s")}
    for r in table:
        s1 = solo.get(r["mode"])
        if not s1 or not r.get("mean_latency_s"):
            continue
        r["latency_vs_solo"] = round(r["mean_latency_s"] / s1["mean_latency_s"], 3)
        if r.get("sclk_mhz") and s1.get("sclk_mhz"):
            r["latency_vs_solo_at_solo_clock"] = round(r["mean_latency_s"] * r["sclk_mhz"] / s1["sclk_mhz"]
                                                       / s1["mean_latency_s"], 3)


def _close_server(server: "PodServerProc") -> dict:
    try:
        info = server.info()
    except Exception as e:  # reported, not fatal: the pods' own records are the measurement
        info = {"error": repr(e)}
    server.close()
    return info


def _hws_limit() -> int:
    from nos_amd.gpu.kfd import hws_max_concurrent_processes

    return hws_max_concurrent_processes()


def run_quota(args) -> int:
    """``--quota``: config 5 on this GPU -- the real control plane with
    ElasticQuotas, the kubelet starting every admitted pod as a pod process
    against this GPU's pod server, borrowing, then CapacityScheduling
    preemption stopping the borrowers' tenants."""
    import shutil
    import tempfile

    from nos_amd.podbench import PodLauncher
    from nos_amd.quotabench import ProcessRuntime, scenario_for

    launcher = PodLauncher()  # before anything here touches the GPU
    args.pod_server_dir = tempfile.mkdtemp(prefix="nos_q_", dir="/tmp")
    work = tempfile.mkdtemp(prefix="nos_q_pods_")
    args.local_gpu = 0
    slices = args.pods_per_gpu or 28
    server = PodServerProc(launcher, args, "0", work)
    if args.composed:
        from nos_amd.quotabench import composed_for

        def server_stats():
            from nos_amd.podserver.client import PodClient

            c = PodClient(server.path, connect_timeout_s=5)
            try:
                return c.stats()
            finally:
                c.close()

        def part_env(key: str) -> dict:
            """A pod of the (simulated) repartitioned node as a real tenant of
            this GPU's pod server: an allocation record of a 2 GB slice on the
            shared CUs, as the device plugin writes one, and its pod env."""
            from nos_amd.api import constants as C
            from nos_amd.podserver.allocations import AllocationStore, new_token, socket_path

            tok = new_token()
            AllocationStore(args.pod_server_dir).write(0, tok, {"memory_gb": 2, "cu_mask": None,
                                                                "device_ids": [f"part::{key}"], "owner": key,
                                                                "resource": "partition"})
            return {C.ENV_POD_SERVER: str(socket_path(args.pod_server_dir, 0)), C.ENV_POD_TOKEN: tok,
                    C.ENV_MEMORY_LIMIT_GB: "2"}

        # 36 GB of the GPU for the trainer pod, the rest in 10 GB tenant slices
        sc = composed_for(1, args.pods_per_gpu or 25, args.slice_gb or 10, pod_server_dir=args.pod_server_dir,
                          live=True, server_stats=server_stats, isolate_team_b=args.isolate_team_b,
                          part_tenants=None if args.isolate_team_b else part_env)
    else:
        sc = scenario_for(slices, args.slice_gb or 10, pod_server_dir=args.pod_server_dir, live=True)
    sampler = None
    try:
        log(0, f"pod server ready in {server.wait_ready():.1f} s")
        if args.device == "cuda":
            import torch

            torch.cuda.set_device(0)
            sampler = UtilSampler(0)
        rt = ProcessRuntime(launcher, work, dtype=args.dtype, device=args.device,
                            extra_env={"NOS_AMD_POD_DUTY": sc.duty} if args.composed else None)
        try:
            res = sc.run(rt, phase_timeout_s=900, sampler=sampler)
        finally:
            rt.close()
        try:
            res["pod_server"] = server.info()
        except Exception as e:
            res["pod_server"] = {"error": repr(e)}
    finally:
        if sampler:
            sampler.close()
        server.close()
        launcher.close()
        shutil.rmtree(work, ignore_errors=True)
        shutil.rmtree(args.pod_server_dir, ignore_errors=True)
    metric = ("config5 composed: DP trainer pods + bursty ElasticQuota tenants on a pod-server node, a simulated "
              "amdpart repartition, CapacityScheduling preemption" if args.composed else
              "config5: ElasticQuota borrowing + CapacityScheduling preemption on running pod-server tenants (1 node)")
    line = json.dumps({"metric": metric, "dtype": args.dtype, "device": args.device,
                       "data": "synthetic (random-init YOLOS-small programs)", **res})
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")
    return 0


def main(argv=None) -> int:
    args = parse_args(argv)
    if args.quota:
        return run_quota(args)
    server_mode = args.mode == "server"
    args.pods_per_gpu = args.pods_per_gpu or (28 if server_mode else 8)
    args.slice_gb = args.slice_gb or (10 if server_mode else 36)
    import tempfile

    # short: a Unix socket path has at most 107 bytes
    args.pod_server_dir = tempfile.mkdtemp(prefix="nos_ps_", dir="/tmp")
    args.local_gpu = int(os.environ.get("LOCAL_RANK", "0"))
    from nos_amd.podbench import PodLauncher

    # first of all: pods are forked by this launcher, which must never come
    # from a process that has touched the GPU (plan() may count devices)
    launcher = PodLauncher()
    d = Dist(args.device)
    world, rank, local = d.world, d.rank, d.local
    if world != args.gpus:
        log(rank, f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}")
    # control plane first (CPU only): the GPU is initialised by the pods, then by this rank
    envs, cp = plan(args, world, local, args.slice_gb, args.pods_per_gpu, args.mode)
    from nos_amd.api import constants as C
    from nos_amd.bench_support import schedulable_pods

    cp10 = {}
    if args.slice_gb != 10:
        cp10 = schedulable_pods(world, 10)
    # hybrid partitioning (modes + memory slices per partition): simulated only --
    # the pool cannot switch compute/memory modes (needs root), parity unpinned
    hyb10 = schedulable_pods(world, 10, kind=C.PARTITIONING_HYBRID)
    extra_env = {"GPU_MAX_HW_QUEUES": str(args.hw_queues)} if args.hw_queues else {}
    if args.device == "cpu":
        extra_env["OMP_NUM_THREADS"] = "1"
    fleet_env = {**extra_env, **({"NOS_AMD_POD_DUTY": args.bursty} if args.bursty else {})}
    log(rank, f"control plane placed {cp.get('placed_pods')} pods; local envs {envs[:2]}...")
    if args.table == "auto":
        args.table = "1,3,5,7" if world == 1 and args.device == "cuda" else ""
    if server_mode and "server" not in args.table_modes.split(","):
        args.table_modes = "server," + args.table_modes
    # table rows: the main run's slice size for server rows, 36 GB process slices otherwise
    table_plans = [(mode, n, plan(args, world, local, args.slice_gb if mode == "server" else 36, n, mode)[0])
                   for mode in args.table_modes.split(",") if args.table
                   for n in map(int, args.table.split(","))]
    args.gpu_env = envs[0].get("HIP_VISIBLE_DEVICES", str(local))  # this rank's GPU (folded runs: shared)
    families = assign_tenant_mix(args, envs) if args.tenant_mix else None

    d.init_gpu()
    sampler = UtilSampler(d.device) if d.cuda else None
    use_coll = args.collective == "on" or (args.collective == "auto" and world > 1)
    # pod slot 0 of every GPU is the DP trainer pod (its own process; a fresh job per fleet)
    fleet_envs = (lambda e: with_trainer(d, e, args)) if use_coll else (lambda e: e)
    pod_envs = envs

    ref = None
    if args.ref_pod_s > 0:  # one pod owning the whole GPU (no slice env but the device)
        env1 = [{"HIP_VISIBLE_DEVICES": envs[0].get("HIP_VISIBLE_DEVICES", str(local))}]
        w1, u1, _, _, _ = run_fleet(d, launcher, env1, args.dtype, not args.no_graphs, extra_env, 2, 1,
                                    args.ref_pod_s, sampler, device=args.device)
        ref = {"inf_per_s": round(w1.throughput, 3), "latency_s": w1.mean_latency_s, "gpu_util_pct": u1}

    server = None
    server_socket = None
    if server_mode or any(m == "server" for m, _, _ in table_plans):
        server = PodServerProc(launcher, args, args.gpu_env, args.pod_server_dir)
        server_socket = server.path
        log(rank, f"pod server ready in {server.wait_ready():.1f} s on {server.path}")
    trainer_error = None
    srv = server is not None
    try:
        w, util, n_util, ready_s, tr = run_fleet(d, launcher, fleet_envs(pod_envs), args.dtype, not args.no_graphs,
                                                 fleet_env, args.warmup, args.steps, args.step_s, sampler,
                                                 device=args.device, server_alive=srv)
    except FleetStartError as e:
        if not use_coll:
            raise
        # the trainer job could not form (e.g. RCCL refused the pods' transport):
        # every rank saw the same flag, so every rank measures the inference fleet
        # alone and the line says why there is no trainer row
        trainer_error = str(e)[:400]
        log(rank, f"trainer pods failed to start, measuring without them: {trainer_error}")
        use_coll, fleet_envs = False, (lambda e: e)
        w, util, n_util, ready_s, tr = run_fleet(d, launcher, pod_envs, args.dtype, not args.no_graphs,
                                                 fleet_env, args.warmup, args.steps, args.step_s, sampler,
                                                 device=args.device, server_alive=srv)
    mix = mix_stats(w, families) if families else None
    bf = None
    if args.extra_bf16_s > 0 and args.dtype != "bf16" and d.cuda and not families:
        wb, ub, _, _, _ = run_fleet(d, launcher, fleet_envs(pod_envs), "bf16", not args.no_graphs, extra_env, 2, 1,
                                    args.extra_bf16_s, sampler, server_alive=srv)
        bf = {"inf_per_s": round(wb.throughput, 2), "mean_latency_s": wb.mean_latency_s,
              "concurrent_pods": wb.concurrent, "gpu_util_pct": ub}
    table = []
    server_info = None
    for mode, n, tenvs in table_plans:  # the reference demo's latency-vs-pods rows (README.md:63-71)
        if mode != "server" and server is not None:
            # process-pod rows: the server's GPU process would be one HWS slot
            # more than the pods and this rank (7 + 2 > 8: time-sliced)
            server_info = _close_server(server)
            server = None
        wt, ut, _, _, _ = run_fleet(d, launcher, tenvs, args.dtype, not args.no_graphs, extra_env, 1, 1,
                                    args.table_window_s, sampler, device=args.device,
                                    server_alive=server is not None)
        table.append({"mode": mode, "pods": n, "concurrent": wt.concurrent, "inf_per_s": round(wt.throughput, 2),
                      "mean_latency_s": wt.mean_latency_s, "gpu_util_pct": ut, "sclk_mhz": wt.sclk_mhz,
                      "umc_util_pct": getattr(wt, "umc_pct", None),
                      "pods_over_latency": round(n / wt.mean_latency_s, 2) if wt.mean_latency_s else None,
                      "cu_mask": (wt.pods[0].info.get("cu_mask") if wt.pods else None)})
        log(rank, f"table {table[-1]}")
    if server is not None:
        server_info = _close_server(server)
    _normalise_table(table)
    if sampler:
        sampler.close()
    launcher.close()

    # whole-job aggregates (window = slowest rank's)
    elapsed, gp_max = d.reduce([w.window_s, float(GPU_PROCS["max"])], "max")
    sockets = d.gather(server_socket) if server_mode else None
    running = w.concurrent  # inference pods and the trainer pod alike
    sums = d.reduce([w.completed, float(running), util if util is not None else -1e9, float(len(w.inference_pods)),
                     ref["inf_per_s"] if ref else 0.0, bf["inf_per_s"] if bf else 0.0,
                     tr["gemm_tflops"] if tr else 0.0, tr["allreduce_gb_per_s"] if tr else 0.0,
                     float(len(envs))], "sum")
    completed, concurrent, util_sum, pods_total, ref_sum, bf_sum, tr_tf, tr_gbs, placed = sums
    agg = completed / elapsed
    util_mean = util_sum / world if util_sum >= 0 else None
    lat = pods_total * elapsed / completed if completed > 0 else None
    from nos_amd.models.yolos import YolosConfig, demo_input_hw, flops_per_image, seq_len

    cfg, hw = YolosConfig.small(), demo_input_hw()
    value = int(concurrent)
    kc = next((p.info.get("kernel_config") for p in w.inference_pods if p.info.get("kernel_config")), None) or {}
    f32_math = kc.get("f32_math") if args.dtype == "fp32" else None
    # matrix-pipe FLOPs per model FLOP and the pipe's FLOP per clock per SIMD
    pipe_flops_per_flop, pipe_rate = ({"x6": 6, "h3": 3}[f32_math], 1024) if f32_math in ("x6", "h3") else \
        (1, 64 if args.dtype == "fp32" else 1024)
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "fractional pods/node (observed concurrently running)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (BASELINE_PODS_PER_GPU * world), 3),
        "dtype": args.dtype,
        "data": "synthetic (random-init YOLOS-small weights, random 800x1066 image per pod)",
        "config": {"model": "YOLOS-small (hustvl/yolos-small architecture) inference pods",
                   "global_batch": int(pods_total), "seq_len": seq_len(cfg, hw), "device": args.device,
                   "parallelism": f"{args.mode} fractional slices, {args.pods_per_gpu} pod processes/GPU, "
                                  f"{world} GPU(s)",
                   "pods_per_gpu": args.pods_per_gpu, "slice_gb": args.slice_gb, "mode": args.mode,
                   "pod_execution": ("one CPU-only client process per pod with its device-plugin env (pod-server "
                                     "socket + allocation token); the pod ships its model as a program (op graph + "
                                     "weights, nos_amd/podserver/program.py) and its inferences run as HIP-graph "
                                     f"replays in the GPU's pod server process ({args.server_lanes} lanes; the MPS "
                                     "architecture)")
                   if server_mode else "one GPU process per pod with its device-plugin env",
                   "graphs": not args.no_graphs,
                   "collective_tenant": use_coll, "step_s": args.step_s, "bursty": args.bursty or None,
                   "pods_placed_per_node": int(placed)},
        "gpu_util_pct": None if util_mean is None else round(util_mean, 1),
        "gpu_util_samples": n_util,
        "rank0_sclk_mhz": w.sclk_mhz,
        "rank0_umc_util_pct": getattr(w, "umc_pct", None),
        "schedulable_fractional_pods_per_node": value,
        # what bounds it on this node: the amdgpu hardware scheduler's concurrent
        # processes per logical GPU (VMIDs), read from the driver
        "hws_max_concurrent_processes_per_gpu": _hws_limit(),
        # the most GPU processes any GPU held in any window (rank + pod server +
        # process pods / trainer): must stay within the HWS limit above
        "max_gpu_processes_per_gpu": int(gp_max),
        "pod_server_sockets": sockets,
        # server mode: the GPU processes are the pod server (+ the trainer pod),
        # so the HWS bound does not apply to the pods; memory does (28 x 10 GB)
        "pod_server": None if not server_mode else {**(server_info or {}), "tenants_per_gpu_max": POD_SERVER_TENANTS},
        "schedulable_fractional_pods_per_node_sim": cp.get("schedulable_fractional_pods_per_node"),
        "schedulable_10gb_pods_per_node_sim": cp10.get("schedulable_fractional_pods_per_node",
                                                       cp.get("schedulable_fractional_pods_per_node")),
        # the same 10 GB pods on a simulated HYBRID node of this many MI355X (the
        # partitioner picks each GPU's compute/memory mode; 8 HWS process slots per
        # partition): simulation, not hardware -- the pool cannot switch modes
        "schedulable_10gb_pods_per_node_hybrid_sim": hyb10["schedulable_fractional_pods_per_node"],
        "hybrid_sim_modes": hyb10.get("modes"),
        "aggregate_inf_per_s": round(agg, 3),
        "aggregate_inf_per_s_vs_baseline": round(agg / (BASELINE_INF_PER_S_PER_GPU * world), 2),
        "mean_latency_s": None if lat is None else round(lat, 5),
        "window_s": round(elapsed, 3),
        "achieved_tflops": round(agg * flops_per_image(cfg, hw) / 1e12, 2),
        # how the fp32 pods multiply: "h3" = fp16x3 split (two fp16 pieces per
        # operand on power-of-two scales, three products per product on the
        # fp16 MFMA), "x6" = bf16x6 split (three exact bf16 pieces, six
        # products on the bf16 MFMA) -- both with errors vs fp64 <= the
        # exact-f32 MFMA's (tests/test_gemm_h3_gpu.py, test_kernels_gpu.py) --
        # "exact" = v_mfma_f32_32x32x2_f32
        "f32_math": f32_math,
        # the share of the matrix pipes' peak at the measured clock that the
        # executed MFMAs use (256 CUs x 4 SIMDs x 64 fp32 / 1024 bf16 FLOP per
        # clock; an x6 fp32 FLOP costs six bf16 FLOPs, an h3 one three fp16
        # FLOPs at the same rate): amd-smi's gfx activity
        # reads 100 % whenever any kernel runs, this does not
        "matrix_pipe_util_pct": (round(100.0 * agg * flops_per_image(cfg, hw) * pipe_flops_per_flop /
                                       (world * 256 * 4 * pipe_rate * w.sclk_mhz * 1e6), 1)
                                 if d.cuda and w.sclk_mhz else None),
        "single_pod_inf_per_s": round(ref_sum, 3) if ref else None,
        "aggregate_vs_single_pod": round(agg / ref_sum, 3) if ref and ref_sum > 0 else None,
        "baseline": {"pods_per_gpu": BASELINE_PODS_PER_GPU, "inf_per_s_per_gpu": BASELINE_INF_PER_S_PER_GPU,
                     "aggregate_vs_single_pod_mps": 1.93, "aggregate_vs_single_pod_mig": 1.79},
        "bf16_gfx950_kernels": None if bf is None else {**bf, "inf_per_s_node": round(bf_sum, 2)},
        "trainer_error": trainer_error,
        "trainer_pods": None if tr is None else {"per_node_gemm_tflops": round(tr_tf, 2),
                                                 "per_node_allreduce_gb_per_s": round(tr_gbs, 4),
                                                 "rank0": tr, "bucket_mb": args.coll_bucket_mb,
                                                 "gemm_dim": args.coll_dim,
                                                 "step": "bf16 MLP (4 x dim^2 layers, batch dim) forward + backward, "
                                                         "bucketed all-reduce launched from the gradient hooks "
                                                         "(overlaps backward), SGD",
                                                 "execution": "one pod process per GPU with its device-plugin env "
                                                              "(models/trainer_pod.py), RCCL job across the GPUs",
                                                 "allreduce_gb_per_s": "gradient bytes all-reduced per second "
                                                                       "(payload); rank0.bucket_busbw_gbps = one "
                                                                       "bucket's all-reduce, NCCL-tests busbw"},
        "rank0_window": w.as_dict(),
        "latency_table": table or None,
        "tenant_mix": mix,
        "rank0_ref_pod": ref,
        "pods_ready_s": round(ready_s, 1),
        "control_plane": cp,
    }
    if sampler and sampler.err:
        result["gpu_util_error"] = sampler.err
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    d.close()
    import shutil

    shutil.rmtree(args.pod_server_dir, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
