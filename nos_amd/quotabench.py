"""BASELINE config 5: elastic quotas and GPU partitioning acting on running tenants.

The reference's elastic quota (``pkg/scheduler/plugins/capacityscheduling/
capacity_scheduling.go:468-675`` for victim selection,
``internal/controllers/elasticquota/elasticquota.go:38-72`` for
``status.used`` and the ``in-quota`` / ``over-quota`` pod labels) lets a
namespace borrow other namespaces' unused ``min`` and takes it back by
preempting the borrower's over-quota pods when the lender needs it.  This
harness runs that flow end to end on one node with the real control plane
(scheduler + CapacityScheduling, operator, cumask partitioner, device plugin,
kubelet) and REAL tenants behind the kubelet:

1. two namespaces with ElasticQuotas on ``nos.nebuly.com/gpu-memory``, each
   ``min`` = half the node's slice memory, ``max`` = all of it;
2. team-a submits more 10 GB slice pods than its ``min``: they all run, the
   ones past ``min`` borrowing team-b's unused quota (``over-quota``);
3. team-b submits its ``min`` worth of pods: the node is full, so
   CapacityScheduling's PostFilter preempts team-a's over-quota pods; the
   kubelet stops each victim's tenant (its process ends, the device plugin
   releases the slice and deletes the allocation record, the pod server
   evicts the tenant if it is still registered) and the preemptor's pod
   starts on the freed slice.

The kubelet's ``runtime`` / ``on_stop`` hooks are the data plane: a
:class:`RecordingRuntime` for the CPU rehearsal (tests) or a
:class:`ProcessRuntime` that starts every admitted pod as a real pod process
with its device-plugin env (``models/pod.py`` against the GPU's pod server).
The simulated cluster's clock follows the wall clock while tenants run.

Reported: preemptions, the time from a victim's stop to the preemptor's
first inference, concurrently running tenants, EQ ``status.used`` and pod
labels checked against the tenants actually running, and (GPU) amd-smi
utilisation per phase.
"""
from __future__ import annotations

import os
import shutil
import sys
import tempfile
import threading
import time
from dataclasses import dataclass, field
from pathlib import Path

from .api import constants as C
from .api import v1alpha1
from .api.config import GpuPartitionerConfig
from .kube import objects as ko

GPU_MEM = C.RESOURCE_GPU_MEMORY


@dataclass
class Tenant:
    key: str
    env: dict
    t_start: float
    t_ready: float | None = None
    t_stop: float | None = None
    handle: object = None


class RecordingRuntime:
    """CPU rehearsal: a tenant is 'running' from its container start to its
    stop, 'ready' (first inference) at once."""

    def __init__(self):
        self.tenants: dict[str, Tenant] = {}
        self.lock = threading.Lock()

    def start(self, key: str, env: dict) -> None:
        now = time.monotonic()
        with self.lock:
            self.tenants[key] = Tenant(key, env, now, now)

    def stop(self, key: str) -> None:
        with self.lock:
            t = self.tenants.get(key)
            if t is not None and t.t_stop is None:
                t.t_stop = time.monotonic()

    def poll(self) -> None:
        pass

    def running(self) -> set[str]:
        with self.lock:
            return {k for k, t in self.tenants.items() if t.t_stop is None}

    def ready(self) -> set[str]:
        with self.lock:
            return {k for k, t in self.tenants.items() if t.t_stop is None and t.t_ready is not None}

    def progress(self, key: str) -> int | None:
        """Completions (inferences / training steps) of a live tenant; None:
        not measured (the CPU rehearsal)."""
        return None

    def close(self) -> None:
        pass


class ProcessRuntime(RecordingRuntime):
    """Every admitted pod is a real pod process (``models/pod.py``) with its
    device-plugin env; 'ready' = its first inference completed (status
    board).  Stopping a tenant sets its board's stop flag (graceful: the pod
    closes its pod-server connection) and kills it after ``grace_s``."""

    def __init__(self, launcher, workdir: str, dtype: str = "fp32", device: str = "cuda", grace_s: float = 10.0,
                 extra_env: dict | None = None):
        super().__init__()
        self.launcher, self.dir, self.dtype, self.device, self.grace = launcher, Path(workdir), dtype, device, grace_s
        self.extra_env = dict(extra_env or {})   # e.g. NOS_AMD_POD_DUTY for bursty tenants
        self._n = 0

    def start(self, key: str, env: dict) -> None:
        from .models.pod import StatusBoard
        from .podbench import REPO

        self._n += 1
        d = self.dir / f"t{self._n:03d}"
        d.mkdir(parents=True, exist_ok=True)
        board = StatusBoard(d / "status.bin", pods=1)
        penv = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                                                 "HIP_VISIBLE_DEVICES", "ROC_GLOBAL_CU_MASK")}
        trainer = env.get("NOS_AMD_POD_KIND") == "trainer"
        if not trainer:
            penv.update(self.extra_env)
        penv.update({k: str(v) for k, v in env.items()})
        penv["PYTHONPATH"] = str(REPO) + os.pathsep + penv.get("PYTHONPATH", "")
        penv["NOS_AMD_POD_NAME"] = key  # the server's tenant name: footprints map back to pods
        if trainer:  # the DP trainer tenant: its own GPU process (models/trainer_pod.py)
            cmd = [sys.executable, "-u", "-m", "nos_amd.models.trainer_pod", "--status", str(board.path), "--slot",
                   "0", "--out", str(d), "--device", self.device]
        else:
            cmd = [sys.executable, "-u", "-m", "nos_amd.models.pod", "--status", str(board.path), "--slot", "0",
                   "--out", str(d), "--dtype", self.dtype, "--seed", str(self._n), "--device", self.device]
        proc = self.launcher.spawn(cmd, penv, str(d / "pod.err"), str(REPO))
        with self.lock:
            self.tenants[key] = Tenant(key, env, time.monotonic(), handle=(proc, board, d))

    def stop(self, key: str) -> None:
        with self.lock:
            t = self.tenants.get(key)
            if t is None or t.t_stop is not None:
                return
            t.t_stop = time.monotonic()
        proc, board, _ = t.handle
        board.stop()

        def reap():
            try:
                proc.wait(timeout=self.grace)
            except Exception:
                proc.kill()

        threading.Thread(target=reap, daemon=True).start()

    def poll(self) -> None:
        from .models.pod import STATE_FAILED

        with self.lock:
            ts = [t for t in self.tenants.values() if t.t_ready is None and t.t_stop is None]
        for t in ts:
            proc, board, d = t.handle
            if board.counts()[0] >= 1:
                t.t_ready = float(board.row(0)[2])  # CLOCK_MONOTONIC of its first completion
            elif board.states()[0] == STATE_FAILED or proc.poll() is not None:
                err = (d / "pod.err").read_text()[-1500:] if (d / "pod.err").exists() else ""
                raise RuntimeError(f"tenant {t.key} failed:\n{err}")

    def progress(self, key: str) -> int | None:
        with self.lock:
            t = self.tenants.get(key)
        return None if t is None else int(t.handle[1].counts()[0])

    def close(self) -> None:
        with self.lock:
            keys = [k for k, t in self.tenants.items() if t.t_stop is None]
        for k in keys:
            self.stop(k)
        deadline = time.monotonic() + self.grace + 5
        for t in list(self.tenants.values()):
            proc = t.handle[0]
            try:
                proc.wait(timeout=max(0.5, deadline - time.monotonic()))
            except Exception:
                proc.kill()


@dataclass
class QuotaScenario:
    gpus: int = 1
    slice_gb: int = 10
    team_a_pods: int = 20
    team_b_pods: int = 14
    min_gb: int = 140                 # per team
    max_gb: int = 280
    pod_server_dir: str = ""
    tenants_per_gpu: int = 48         # the pod server's tenant cap (memory bounds 10 GB slices at 28 first)
    live: bool = False                # sim clock follows the wall clock (real tenants)
    batch_window_s: float = 2.0
    events: list = field(default_factory=list)

    def build(self, runtime):
        from .gpu.fakesmi import FakeSmi
        from .sim.cluster import SimCluster

        self.runtime = runtime
        cl = self.cl = SimCluster(partitioner_config=self._partitioner_config())
        cl.add_node("mi355x-0", C.PARTITIONING_CUMASK, smi=FakeSmi(gpus=self.gpus, node="mi355x-0"),
                    pod_server_tenants=self.tenants_per_gpu, pod_server_dir=self.pod_server_dir,
                    runtime=lambda pod, conts: self._start(pod, conts), on_stop=lambda pod, conts: self._stop(pod))
        for ns in ("team-a", "team-b"):
            cl.api.create({"kind": "Namespace", "metadata": {"name": ns}})
            # CapacityScheduling always compares cpu and memory (the reference's
            # usedOverWith); the pods' 100m / 0 stay far inside these
            cl.api.create(v1alpha1.build_eq(ns, "quota").with_min({GPU_MEM: self.min_gb, "cpu": "32", "memory": "256Gi"})
                          .with_max({GPU_MEM: self.max_gb, "cpu": "64", "memory": "1Ti"}).get())
        self._settle(30)
        return cl

    def _partitioner_config(self) -> GpuPartitionerConfig:
        return GpuPartitionerConfig(cuPolicy="shared", batchWindowTimeoutSeconds=int(max(1, self.batch_window_s * 2)),
                                    batchWindowIdleSeconds=int(max(1, self.batch_window_s)))

    # ------------------------------------------------------------ kubelet hooks
    def _start(self, pod: dict, conts) -> None:
        env = {}
        for rc in conts:
            env.update(rc.envs)
        key = ko.key(pod)
        self.runtime.start(key, env)
        self.events.append(("start", key, time.monotonic()))

    def _stop(self, pod: dict) -> None:
        key = ko.key(pod)
        self.runtime.stop(key)
        self.events.append(("stop", key, time.monotonic()))

    # ------------------------------------------------------------ driving
    def _settle(self, sim_s: float, until=None) -> None:
        self.cl.settle(sim_s, until=until)

    def drive(self, until, timeout_s: float, tick_s: float = 0.05) -> bool:
        """Run the control plane until ``until()``: in live mode the sim
        clock follows the wall clock and the runtime is polled."""
        if not self.live:
            self.cl.settle(timeout_s, until=until)
            return until()
        w0, s0 = time.monotonic(), self.cl.clock.now()
        last = w0
        while True:
            if time.monotonic() - last > 10:  # progress for long live phases
                last = time.monotonic()
                print(f"[quota] {last - w0:.0f} s: {len(self.runtime.ready())} tenants ready, "
                      f"{len(self.runtime.running())} running, {len(self.cl.pending_pods())} pods pending",
                      file=sys.stderr, flush=True)
            self.cl.settle(tick_s, until=until)
            target = s0 + (time.monotonic() - w0)
            if self.cl.clock.now() < target:
                self.cl.clock.advance(target - self.cl.clock.now())
            self.runtime.poll()
            if until():
                return True
            if time.monotonic() - w0 > timeout_s:
                return False
            time.sleep(tick_s)

    def submit(self, ns: str, n: int, prefix: str) -> list[str]:
        keys = []
        for i in range(n):
            self.cl.submit_pod(f"{prefix}-{i}", {f"{C.AMD_SLICE_RESOURCE_PREFIX}{self.slice_gb}gb": 1}, namespace=ns)
            keys.append(f"{ns}/{prefix}-{i}")
            if not self.live:
                self.cl.clock.advance(1)
        return keys

    # ------------------------------------------------------------ observations
    def labels(self, ns: str) -> dict[str, str | None]:
        return {ko.key(p): ko.labels(p).get(C.LABEL_CAPACITY_INFO) for p in self.cl.pods(ns)
                if ko.pod_phase(p) == ko.RUNNING}

    def used_gb(self, ns: str) -> float:
        eq = self.cl.api.get(v1alpha1.KIND_EQ, "quota", ns)
        return float(((eq.get("status") or {}).get("used") or {}).get(GPU_MEM, 0))

    def _gb(self, ns: str) -> int:
        """The slice profile (GB) of a namespace's tenants."""
        return getattr(self, "team_b_gb", 0) or self.slice_gb if ns == "team-b" else self.slice_gb

    def snapshot(self) -> dict:
        run = self.runtime.running()
        out = {}
        for ns in ("team-a", "team-b"):
            lab = self.labels(ns)
            mine = {k for k in run if k.startswith(ns + "/")}
            out[ns] = {"running_pods": len(lab), "tenants_running": len(mine),
                       "in_quota": sum(1 for v in lab.values() if v == "in-quota"),
                       "over_quota": sum(1 for v in lab.values() if v == "over-quota"),
                       "status_used_gb": self.used_gb(ns), "tenant_gb": len(mine) * self._gb(ns),
                       "pods_match_tenants": set(lab) == mine}
        return out

    def run(self, runtime, phase_timeout_s: float = 600.0, sampler=None) -> dict:
        """Both phases; returns the measurements."""
        self.build(runtime)
        res: dict = {"config": {"gpus": self.gpus, "slice_gb": self.slice_gb, "team_a_pods": self.team_a_pods,
                                "team_b_pods": self.team_b_pods, "min_gb": self.min_gb, "max_gb": self.max_gb}}
        t0 = time.monotonic()
        a = self.submit("team-a", self.team_a_pods, "a")
        ok = self.drive(lambda: set(a) <= self.runtime.ready() and self._labels_settled(), phase_timeout_s)
        res["phase_a"] = {"ok": ok, "seconds": round(time.monotonic() - t0, 2), **self.snapshot()}
        if sampler is not None:
            res["phase_a"]["gpu_util_pct"] = sampler.mean(t0, time.monotonic())[0]
        t1 = time.monotonic()
        over_a = {k for k, v in self.labels("team-a").items() if v == "over-quota"}
        p0 = self.cl.scheduler.stats.get("preemptions", 0)
        b = self.submit("team-b", self.team_b_pods, "b")
        ok = self.drive(lambda: set(b) <= self.runtime.ready() and self._labels_settled(), phase_timeout_s)
        t2 = time.monotonic()
        stops = sorted(t for kind, k, t in self.events if kind == "stop" and t >= t1)
        b_ready = sorted(self.runtime.tenants[k].t_ready for k in b if k in self.runtime.tenants
                         and self.runtime.tenants[k].t_ready is not None)
        # each victim's stop frees one slice: its preemptor is the earliest
        # team-b container started at or after that stop (the pods that did
        # not need a victim wait for the partitioner to add slices instead)
        b_ts = sorted((self.runtime.tenants[k] for k in b if k in self.runtime.tenants), key=lambda t: t.t_start)
        used: set[int] = set()
        pairs = []
        for st in stops:
            j = next((i for i, t in enumerate(b_ts) if i not in used and t.t_start >= st - 1e-3), None)
            if j is not None:
                used.add(j)
                pairs.append((st, b_ts[j]))
        cp = [t.t_start - st for st, t in pairs]
        up = [t.t_ready - t.t_start for _, t in pairs if t.t_ready is not None]
        lat = [t.t_ready - st for st, t in pairs if t.t_ready is not None]
        others = [t for i, t in enumerate(b_ts) if i not in used]
        res["phase_b"] = {"ok": ok, "seconds": round(t2 - t1, 2), "preemptions":
                          self.cl.scheduler.stats.get("preemptions", 0) - p0, "victims": len(stops),
                          # CapacityScheduling may only take back borrowed quota
                          "victims_over_quota_only": {k for kind, k, t in self.events
                                                      if kind == "stop" and t >= t1} <= over_a,
                          "preemption_to_running_s": _stats(lat),
                          "victim_stop_to_preemptor_start_s": _stats(cp),
                          "preemptor_start_to_first_inference_s": _stats(up),
                          # pods placed on slices the partitioner added (batch window + device-plugin delay)
                          "submit_to_start_without_preemption_s": _stats([t.t_start - t1 for t in others]),
                          "timeline_s": {"victim_stops": [round(x - t1, 3) for x in stops],
                                         "team_b_starts": [round(t.t_start - t1, 3) for t in b_ts],
                                         "team_b_first_inference": [round(t.t_ready - t1, 3) for t in b_ts
                                                                    if t.t_ready is not None]},
                          "submit_to_all_running_s": round((b_ready[-1] - t1) if b_ready else -1, 3),
                          **self.snapshot()}
        if sampler is not None:
            res["phase_b"]["gpu_util_pct"] = sampler.mean(t1, t2)[0]
        res["concurrent_tenants"] = len(self.runtime.running())
        return res

    def _labels_settled(self) -> bool:
        for ns in ("team-a", "team-b"):
            if any(v is None for v in self.labels(ns).values()):
                return False
        return True


@dataclass
class ComposedScenario(QuotaScenario):
    """BASELINE config 5 as ONE scenario: "ElasticQuota +
    dynamic partition + CU-mask under bursty synthetic PyTorch-ROCm/RCCL
    tenants".  Two nodes under one control plane:

    * ``mi355x-0`` (cumask, pod server per GPU): per GPU one DP trainer pod
      (``training`` namespace, a 36 GB slice; its own GPU process running
      forward / backward / RCCL all-reduce, models/trainer_pod.py), then
      team-a's inference tenants arriving in ``waves`` bursts (each tenant
      with a duty cycle, ``NOS_AMD_POD_DUTY``), borrowing team-b's quota;
    * ``mi355x-part`` (amdpart, FakeSmi: the mode switch is SIMULATED -- the
      pool has no root to switch an MI355X's compute mode): ``batch`` pods
      requesting CPX partitions it does not have, so the partitioner plans a
      repartition SPX -> CPX and the agent applies it;
    * then team-b claims its min and CapacityScheduling preempts team-a's
      over-quota tenants (the reference flows:
      ``capacity_scheduling.go:468-675``, ``partitioner_controller.go:81-200``).

    Reported per phase: GPU util, running tenants, quota ``status.used``
    against the pod server's measured footprints (``footprint_gb`` sum of the
    namespace's tenants), preemptions, and the repartition count and latency."""

    trainers: bool = True
    trainer_slice_gb: int = 36
    trainer_dim: int = 2048         # NOS_AMD_COLL_DIM of the trainer pods
    waves: int = 3
    wave_gap_s: float = 4.0
    duty: str = "1.5:0.5"
    part_gpus: int = 1
    part_pods: int = 8
    part_resource: str = "amd.com/partition-1xcd.36gb"
    server_stats: object = None     # () -> pod-server stats (live runs), for the footprint comparison
    # team-b on an isolated CU pool (cuPolicy split): its slice profile gets proportional CU masks
    # inside ``isolated_cu_slots`` slots per XCD, team-a's tenants and the trainer share the rest
    isolate_team_b: bool = False
    team_b_gb: int = 0              # team-b's slice profile (0: slice_gb; isolated: a profile of its own)
    isolated_cu_slots: int = 12
    solo_s: float = 8.0             # phase C: team-b alone (team-a deleted), its solo latency
    part_tenants: object = None     # (key) -> env: the repartitioned node's pods as real pod-server tenants

    def _partitioner_config(self) -> GpuPartitionerConfig:
        if not self.isolate_team_b:
            return super()._partitioner_config()
        # spread: every GPU's isolated pool holds its share of team-b's slices (a slot each)
        return GpuPartitionerConfig(cuPolicy="split", isolatedProfiles=[f"{self.team_b_gb}gb"],
                                    isolatedCuSlots=self.isolated_cu_slots, slicePlacement="spread",
                                    batchWindowTimeoutSeconds=int(max(1, self.batch_window_s * 2)),
                                    batchWindowIdleSeconds=int(max(1, self.batch_window_s)))

    def _part_start(self, key: str) -> None:
        """A pod of the repartitioned node: recorded (the partition itself is
        simulated) and, in live runs, also started as a real tenant of the
        GPU's pod server, so the partition pods load the GPU."""
        self.sim_runtime.start(key, {})
        if self.part_tenants is not None:
            self.runtime.start("part/" + key, self.part_tenants(key))

    def _part_stop(self, key: str) -> None:
        self.sim_runtime.stop(key)
        if self.part_tenants is not None:
            self.runtime.stop("part/" + key)

    def tenant_latency(self, since: dict | None) -> dict:
        """Per namespace, the pod server's per-tenant inference latency over
        the interval since ``since`` (a previous :meth:`server_marks`): the
        replay time per completed request (``gpu_s`` / ``completed`` deltas),
        mean over the namespace and its slowest tenant."""
        now = self.server_marks()
        if not now or since is None:
            return {}
        out: dict[str, dict] = {}
        for pod, (done, gpu_s) in now.items():
            d0, g0 = since.get(pod, (0, 0.0))
            if done - d0 <= 0:
                continue
            ns = pod.split("/", 1)[0]
            e = out.setdefault(ns, {"tenants": 0, "requests": 0, "gpu_s": 0.0, "max_ms": 0.0})
            e["tenants"] += 1
            e["requests"] += done - d0
            e["gpu_s"] += gpu_s - g0
            e["max_ms"] = max(e["max_ms"], 1e3 * (gpu_s - g0) / (done - d0))
        return {ns: {"tenants": e["tenants"], "requests": e["requests"],
                     "mean_ms": round(1e3 * e["gpu_s"] / e["requests"], 3), "slowest_tenant_ms": round(e["max_ms"], 3)}
                for ns, e in out.items()}

    def server_marks(self) -> dict:
        if self.server_stats is None:
            return {}
        try:
            st = self.server_stats()
        except Exception:
            return {}
        return {str(t.get("pod")): (int(t.get("completed", 0)), float(t.get("gpu_s", 0.0)))
                for t in st.get("tenants", [])}

    def build(self, runtime):
        from .gpu.fakesmi import FakeSmi

        cl = super().build(runtime)
        self.sim_runtime = RecordingRuntime()
        self.part = cl.add_node("mi355x-part", C.PARTITIONING_AMDPART, gpus=self.part_gpus,
                                smi=FakeSmi(gpus=self.part_gpus, node="mi355x-part"),
                                runtime=lambda pod, conts: self._part_start(ko.key(pod)),
                                on_stop=lambda pod, conts: self._part_stop(ko.key(pod)))
        for ns in ("training", "batch"):
            cl.api.create({"kind": "Namespace", "metadata": {"name": ns}})
        self._settle(30)
        return cl

    def _start(self, pod: dict, conts) -> None:
        env = {}
        for rc in conts:
            env.update(rc.envs)
        if ko.labels(pod).get("nos.nebuly.com/tenant-kind") == "trainer":
            # a GPU process of its own: the slice's GPU instead of the pod-server socket
            sock = env.pop(C.ENV_POD_SERVER, "")
            env.pop(C.ENV_POD_TOKEN, None)
            if env.get(C.ENV_POD_CU_MASK):   # its slice's CU mask (split: the shared pool) for its own process
                env["ROC_GLOBAL_CU_MASK"] = env.pop(C.ENV_POD_CU_MASK)
            gpu = sock.rsplit("gpu-", 1)[-1].split("/", 1)[0] if "gpu-" in sock else "0"
            env.update({"HIP_VISIBLE_DEVICES": gpu, "NOS_AMD_POD_KIND": "trainer", "RANK": "0", "WORLD_SIZE": "1",
                        "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(29600 + int(gpu)),
                        "NOS_AMD_COLL_DIM": str(self.trainer_dim), "NOS_AMD_COLL_BUCKET_MB": "32"})
        key = ko.key(pod)
        self.runtime.start(key, env)
        self.events.append(("start", key, time.monotonic()))

    def _trainer_progress(self, mark: dict) -> dict | None:
        """Training steps the trainer pods completed since ``mark`` (updated
        in place) and their rate: the DP job keeps stepping (forward,
        backward, bucketed all-reduce) while the inference tenants come and go."""
        now = time.monotonic()
        steps = {k: self.runtime.progress(k) for k in self.trainer_keys}
        if not steps or any(v is None for v in steps.values()):
            return None
        done = sum(v - mark.get(k, 0) for k, v in steps.items())
        dt = now - mark.get("_t", now)
        mark.update(steps)
        mark["_t"] = now
        flops = 6.0 * self.trainer_dim ** 3 * 4   # CollectiveTenant: batch = dim, 4 layers, forward + backward
        return {"steps": done, "steps_per_s": round(done / dt, 2) if dt > 0 else None,
                "tflops": round(done * flops / dt / 1e12, 2) if dt > 0 else None, "flops_per_step": flops}

    def _phase_util(self, sampler, t0: float) -> float | None:
        return sampler.mean(t0, time.monotonic())[0] if sampler is not None else None

    def footprints(self) -> dict:
        """Per namespace: the pod server's measured build footprints of its
        tenants (GB), from the server's stats (live runs only)."""
        if self.server_stats is None:
            return {}
        out: dict[str, float] = {}
        try:
            st = self.server_stats()
        except Exception as e:  # reported, not fatal
            return {"error": repr(e)}
        for t in st.get("tenants", []):
            ns = str(t.get("pod", "")).split("/", 1)[0]
            out[ns] = round(out.get(ns, 0.0) + float(t.get("footprint_gb") or 0.0), 3)
        return out

    def quota_vs_footprint(self) -> dict:
        fp = self.footprints()
        snap = self.snapshot()
        return {ns: {"status_used_gb": snap[ns]["status_used_gb"], "slice_gb_running": snap[ns]["tenant_gb"],
                     "server_footprint_gb": fp.get(ns)} for ns in ("team-a", "team-b")}

    def run(self, runtime, phase_timeout_s: float = 600.0, sampler=None) -> dict:
        self.build(runtime)
        res: dict = {"config": {"gpus": self.gpus, "slice_gb": self.slice_gb, "team_a_pods": self.team_a_pods,
                                "team_b_pods": self.team_b_pods, "min_gb": self.min_gb, "max_gb": self.max_gb,
                                "trainers": self.gpus if self.trainers else 0, "waves": self.waves,
                                "duty": self.duty, "part_gpus": self.part_gpus, "part_pods": self.part_pods,
                                "part_resource": self.part_resource,
                                "part_switch": "simulated (FakeSmi; the pool cannot switch MI355X modes)",
                                "part_pods_run_as": "pod-server tenants" if self.part_tenants else "recorded only",
                                "team_b_isolated": self.isolate_team_b, "team_b_gb": self.team_b_gb or self.slice_gb,
                                "isolated_cu_slots_per_xcd": self.isolated_cu_slots if self.isolate_team_b else 0}}
        # phase 0: one DP trainer pod per GPU of the pod-server node
        t0 = time.monotonic()
        tr = []
        if self.trainers:
            for g in range(self.gpus):
                self.cl.submit_pod(f"trainer-{g}", {f"{C.AMD_SLICE_RESOURCE_PREFIX}{self.trainer_slice_gb}gb": 1},
                                   namespace="training", labels={"nos.nebuly.com/tenant-kind": "trainer"})
                tr.append(f"training/trainer-{g}")
            ok = self.drive(lambda: set(tr) <= self.runtime.ready(), phase_timeout_s)
            res["phase_trainers"] = {"ok": ok, "seconds": round(time.monotonic() - t0, 2), "trainers": len(tr),
                                     "gpu_util_pct": self._phase_util(sampler, t0)}
        self.trainer_keys = tr
        mark: dict = {}
        self._trainer_progress(mark)
        if self.isolate_team_b:
            return self._run_isolated(res, mark, phase_timeout_s, sampler)
        # phase A: team-a in bursts, borrowing
        t1 = time.monotonic()
        lat0 = self.server_marks()
        a, per = [], -(-self.team_a_pods // self.waves)
        for w in range(self.waves):
            n = min(per, self.team_a_pods - len(a))
            a += self.submit_range("team-a", len(a), n, "a")
            if w + 1 < self.waves:
                self.drive(lambda: False, self.wave_gap_s)   # the next burst arrives later
        ok = self.drive(lambda: set(a) <= self.runtime.ready() and self._labels_settled(), phase_timeout_s)
        res["phase_a"] = {"ok": ok, "seconds": round(time.monotonic() - t1, 2), **self.snapshot(),
                          "gpu_util_pct": self._phase_util(sampler, t1), "quota_vs_footprint": self.quota_vs_footprint(),
                          "trainer": self._trainer_progress(mark), "latency": self.tenant_latency(lat0)}
        # phase P: pending partition pods force a repartition of the amdpart node
        tp = time.monotonic()
        lat0 = self.server_marks()
        sw0, plans0 = self.part.smi.switches, self.cl.clock.now()
        modes0 = list(self.part.smi.compute)
        keys = []
        for i in range(self.part_pods):
            self.cl.submit_pod(f"p-{i}", {self.part_resource: 1}, namespace="batch")
            keys.append(f"batch/p-{i}")
        ok = self.drive(lambda: set(keys) <= self.sim_runtime.running(), phase_timeout_s)
        res["phase_repartition"] = {"ok": ok, "submit_to_all_running_s": round(time.monotonic() - tp, 2),
                                    "submit_to_all_running_sim_s": round(self.cl.clock.now() - plans0, 2),
                                    "mode_switches": self.part.smi.switches - sw0, "modes_before": modes0,
                                    "modes_after": list(self.part.smi.compute), "pods_running": len(
                                        set(keys) & self.sim_runtime.running()),
                                    "gpu_util_pct": self._phase_util(sampler, tp), "trainer": self._trainer_progress(mark),
                                    "latency": self.tenant_latency(lat0)}
        if self.part_tenants is not None:   # the partition pods' tenants up (a live run): then measure
            self.drive(lambda: {"part/" + k for k in keys} <= self.runtime.ready(), phase_timeout_s)
            lat0 = self.server_marks()
            self.drive(lambda: False, self.wave_gap_s)
            res["phase_repartition"]["latency_with_part_tenants"] = self.tenant_latency(lat0)
        # the batch jobs finish: their pods leave the partitions (and the GPU) before team-b arrives
        for k in keys:
            self.cl.api.delete("Pod", k.split("/", 1)[1], "batch")
        self.drive(lambda: not (set(keys) & self.sim_runtime.running()), phase_timeout_s)
        # phase B: team-b claims its min, preempting team-a's borrowed tenants (team-a keeps bursting)
        b_res = self._phase_b(phase_timeout_s, sampler)
        lat0 = self.server_marks()
        self.drive(lambda: False, self.solo_s)       # a window of team-b beside team-a's in-quota bursts
        res["phase_b"] = {**b_res, "quota_vs_footprint": self.quota_vs_footprint(), "trainer": self._trainer_progress(mark),
                          "latency": self.tenant_latency(lat0)}
        res["concurrent_tenants"] = len(self.runtime.running())
        # phase C: team-a leaves; team-b's latency alone is its solo reference
        tc = time.monotonic()
        for k in list(self.labels("team-a")):
            self.cl.api.delete("Pod", k.split("/", 1)[1], "team-a")
        self.drive(lambda: not any(k.startswith("team-a/") for k in self.runtime.running()), phase_timeout_s)
        lat0 = self.server_marks()
        self.drive(lambda: False, self.solo_s)
        lc = self.tenant_latency(lat0)
        res["phase_c"] = {"seconds": round(time.monotonic() - tc, 2), "latency": lc,
                          "gpu_util_pct": self._phase_util(sampler, tc), "trainer": self._trainer_progress(mark)}
        b_ms = (res["phase_b"].get("latency") or {}).get("team-b", {}).get("mean_ms")
        c_ms = (lc.get("team-b") or {}).get("mean_ms")
        res["team_b_latency_vs_alone"] = round(b_ms / c_ms, 3) if b_ms and c_ms else None
        return res

    def _run_isolated(self, res: dict, mark: dict, phase_timeout_s: float, sampler) -> dict:
        """The isolation variant: team-b's tenants run on
        their own CU slots (a profile of the isolated pool) before team-a
        arrives; their latency alone, then while team-a's tenants burst on the
        shared pool (the trainer there too), then during the repartition.
        Reclaim by preemption needs both teams on one profile (a freed slice
        of another profile does not fit the preemptor: the reference's
        CapacityScheduling semantics) -- the shared variant measures it."""
        t0 = time.monotonic()
        b = self.submit_range("team-b", 0, self.team_b_pods, "b", self.team_b_gb)
        ok = self.drive(lambda: set(b) <= self.runtime.ready() and self._labels_settled(), phase_timeout_s)
        lat0 = self.server_marks()
        self.drive(lambda: False, self.solo_s)
        alone = self.tenant_latency(lat0)
        res["phase_b_alone"] = {"ok": ok, "seconds": round(time.monotonic() - t0, 2), **self.snapshot(),
                                "latency": alone, "gpu_util_pct": self._phase_util(sampler, t0),
                                "trainer": self._trainer_progress(mark)}
        t1 = time.monotonic()
        a, per = [], -(-self.team_a_pods // self.waves)
        lat0 = self.server_marks()
        for w in range(self.waves):
            n = min(per, self.team_a_pods - len(a))
            a += self.submit_range("team-a", len(a), n, "a")
            if w + 1 < self.waves:
                self.drive(lambda: False, self.wave_gap_s)
        ok = self.drive(lambda: set(a) <= self.runtime.ready() and self._labels_settled(), phase_timeout_s)
        self.drive(lambda: False, self.solo_s)        # every wave running and bursting
        during = self.tenant_latency(lat0)
        res["phase_a"] = {"ok": ok, "seconds": round(time.monotonic() - t1, 2), **self.snapshot(),
                          "latency": during, "gpu_util_pct": self._phase_util(sampler, t1),
                          "quota_vs_footprint": self.quota_vs_footprint(), "trainer": self._trainer_progress(mark)}
        b_alone = (alone.get("team-b") or {}).get("mean_ms")
        b_during = (during.get("team-b") or {}).get("mean_ms")
        res["team_b_latency_vs_alone"] = round(b_during / b_alone, 3) if b_alone and b_during else None
        res["concurrent_tenants"] = len(self.runtime.running())
        return res

    def submit_range(self, ns: str, start: int, n: int, prefix: str, gb: int | None = None) -> list[str]:
        keys = []
        for i in range(start, start + n):
            self.cl.submit_pod(f"{prefix}-{i}", {f"{C.AMD_SLICE_RESOURCE_PREFIX}{gb or self.slice_gb}gb": 1},
                               namespace=ns)
            keys.append(f"{ns}/{prefix}-{i}")
        return keys

    def _phase_b(self, phase_timeout_s: float, sampler) -> dict:
        t1 = time.monotonic()
        over_a = {k for k, v in self.labels("team-a").items() if v == "over-quota"}
        p0 = self.cl.scheduler.stats.get("preemptions", 0)
        b = self.submit_range("team-b", 0, self.team_b_pods, "b", self.team_b_gb or None)
        ok = self.drive(lambda: set(b) <= self.runtime.ready() and self._labels_settled(), phase_timeout_s)
        stops = [k for kind, k, t in self.events if kind == "stop" and t >= t1]
        return {"ok": ok, "seconds": round(time.monotonic() - t1, 2),
                "preemptions": self.cl.scheduler.stats.get("preemptions", 0) - p0, "victims": len(stops),
                "victims_over_quota_only": set(stops) <= over_a, **self.snapshot(),
                "gpu_util_pct": self._phase_util(sampler, t1)}


def composed_for(gpus: int, tenant_slots_per_gpu: int = 25, slice_gb: int = 10, isolate_team_b: bool = False,
                 **kw) -> ComposedScenario:
    """A node of ``gpus`` GPUs, each holding one 36 GB trainer slice and
    ``tenant_slots_per_gpu`` 10 GB tenant slices: team-a borrows to 5/7 of
    the tenant slots, team-b then claims its half.  ``isolate_team_b``:
    team-b's pods request a profile of their own (``slice_gb`` + 2 GB) laid
    out on an isolated CU pool (cuPolicy split), as many as its min holds."""
    slots = gpus * tenant_slots_per_gpu
    half = slots // 2
    b_gb = slice_gb + 2 if isolate_team_b else slice_gb
    # isolated: team-b runs 3/4 of its min first, team-a fills what is left of the slots -- borrowing
    # the rest of team-b's min
    b_pods = half * slice_gb // b_gb * 3 // 4 if isolate_team_b else half
    b_per_gpu = -(-b_pods // gpus)
    a_pods = (gpus * ((tenant_slots_per_gpu * slice_gb - b_per_gpu * b_gb) // slice_gb) if isolate_team_b
              else max(half + 1, round(slots * 5 / 7)))
    if isolate_team_b:   # borrowing stops at the quotas' total min (CapacityScheduling's PreFilter)
        a_pods = min(a_pods, (2 * half * slice_gb - b_pods * b_gb) // slice_gb)
    return ComposedScenario(gpus=gpus, slice_gb=slice_gb, team_a_pods=a_pods,
                            team_b_pods=b_pods, min_gb=half * slice_gb, max_gb=slots * slice_gb,
                            tenants_per_gpu=tenant_slots_per_gpu + 1, isolate_team_b=isolate_team_b,
                            team_b_gb=b_gb if isolate_team_b else 0, **kw)


def _stats(v: list[float]) -> dict:
    v = sorted(v)
    return {"n": len(v), "p50": round(v[len(v) // 2], 3) if v else None, "max": round(v[-1], 3) if v else None}


def scenario_for(slices_per_gpu: int, slice_gb: int = 10, **kw) -> QuotaScenario:
    """The default split of a node with ``slices_per_gpu`` slice slots: each
    team's min is half of them, team-a runs 5/7 of them (borrowing), then
    team-b claims its min (preempting team-a's borrowed slices)."""
    half = slices_per_gpu // 2
    return QuotaScenario(slice_gb=slice_gb, team_a_pods=max(half + 1, round(slices_per_gpu * 5 / 7)),
                         team_b_pods=half, min_gb=half * slice_gb, max_gb=slices_per_gpu * slice_gb,
                         tenants_per_gpu=slices_per_gpu, **kw)


def run_cpu_rehearsal(tmp: str | None = None, **kw) -> dict:
    d = tmp or tempfile.mkdtemp(prefix="nos_quota_")
    try:
        sc = QuotaScenario(pod_server_dir=d, **kw)
        return sc.run(RecordingRuntime())
    finally:
        if tmp is None:
            shutil.rmtree(d, ignore_errors=True)


__all__ = ["QuotaScenario", "ComposedScenario", "composed_for", "RecordingRuntime", "ProcessRuntime",
           "run_cpu_rehearsal"]
