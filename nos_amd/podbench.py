"""Steady-state measurement of fractional-GPU pods running as separate processes.

This is the measurement method of the reference's GPU-sharing demo
(``demos/gpu-sharing-comparison/README.md:53-60``: start the pods, let them
warm up, average the inference time over a later window), made exact:

* every pod is its own process (:mod:`nos_amd.models.pod`) started with the
  environment the device plugin allocated to it;
* pods record the completion time of every inference; progress of a pod at
  time ``t`` is interpolated linearly between completions, so the number of
  inferences inside a window ``[t0, t1]`` is exact up to the linearisation of
  the one inference in flight at each edge (:func:`progress`);
* the timed window starts only once *every* pod is warm and running, so all
  of it is measured with all pods co-running;
* mean per-request latency = pods x window / completed inferences -- the
  mean over all requests completed in the window, which makes
  ``pods / latency == throughput`` hold exactly in every row.

:class:`PodFleet` is shared by ``bench.py`` (headline) and
``tools/sharing_table.py`` (latency-vs-pods table).
"""
from __future__ import annotations

import bisect
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from pathlib import Path

from .models.pod import STATE_FAILED, STATE_READY, StatusBoard

REPO = Path(__file__).resolve().parent.parent


def progress(times: list[float], t: float, t_start: float) -> float:
    """Inferences completed by time ``t`` (fractional).  ``times`` are the
    sorted completion times, ``t_start`` the time the first one started."""
    pts = [t_start] + list(times)
    if t <= pts[0]:
        return 0.0
    if t >= pts[-1]:
        return float(len(times))
    j = bisect.bisect_right(pts, t) - 1  # pts[j] <= t < pts[j+1]
    a, b = pts[j], pts[j + 1]
    return j + (t - a) / (b - a)


@dataclass
class PodResult:
    slot: int
    completed: float                  # fractional inferences inside the window
    latency_s: float | None           # window / completed
    max_gap_s: float                  # longest interval without a completion inside the window
    running: bool                     # completed inferences all through the window
    info: dict = field(default_factory=dict)


@dataclass
class WindowStats:
    window_s: float
    pods: list[PodResult]
    sclk_mhz: float | None = None  # mean GFX clock over the window (amd-smi), when sampled

    @property
    def completed(self) -> float:
        """Inferences (trainer pods' iterations are not inferences)."""
        return sum(p.completed for p in self.inference_pods)

    @property
    def inference_pods(self) -> list["PodResult"]:
        return [p for p in self.pods if p.info.get("kind") != "trainer"]

    @property
    def trainer_pods(self) -> list["PodResult"]:
        return [p for p in self.pods if p.info.get("kind") == "trainer"]

    @property
    def throughput(self) -> float:
        return self.completed / self.window_s if self.window_s > 0 else 0.0

    @property
    def concurrent(self) -> int:
        return sum(1 for p in self.pods if p.running)

    @property
    def mean_latency_s(self) -> float | None:
        c = self.completed
        return len(self.inference_pods) * self.window_s / c if c > 0 else None

    def as_dict(self) -> dict:
        lat = [p.latency_s for p in self.inference_pods if p.latency_s]
        return {"pods": len(self.pods), "window_s": round(self.window_s, 3),
                "completed": round(self.completed, 2), "inf_per_s": round(self.throughput, 3),
                "mean_latency_s": None if self.mean_latency_s is None else round(self.mean_latency_s, 5),
                "pod_latency_min_s": round(min(lat), 5) if lat else None,
                "pod_latency_max_s": round(max(lat), 5) if lat else None,
                "concurrent_pods": self.concurrent, "sclk_mhz": self.sclk_mhz,
                # memory isolation evidence: the most any pod allocated vs its slice
                "pod_max_allocated_gb": max((p.info.get("max_allocated_gb") or 0.0 for p in self.pods if p.info),
                                            default=None),
                "pod_memory_limit_gb": next((p.info.get("memory_limit_gb") for p in self.pods
                                             if p.info and p.info.get("memory_limit_gb")), None)}


class _RemoteProc:
    """Popen-like handle of a process started by :class:`PodLauncher`."""

    def __init__(self, launcher: "PodLauncher", pid: int):
        self.launcher, self.pid, self.returncode = launcher, pid, None

    def poll(self) -> int | None:
        if self.returncode is None:
            self.returncode = self.launcher._call({"op": "poll", "pid": self.pid})["rc"]
        return self.returncode

    def wait(self, timeout: float | None = None) -> int:
        deadline = None if timeout is None else time.monotonic() + timeout
        while self.poll() is None:
            if deadline is not None and time.monotonic() > deadline:
                raise subprocess.TimeoutExpired(str(self.pid), timeout)
            time.sleep(0.05)
        return self.returncode

    def kill(self) -> None:
        self.launcher._call({"op": "kill", "pid": self.pid})


class PodLauncher:
    """A clean helper process that starts the pods.

    Started before the orchestrator initialises its own GPU context, so no pod
    is ever forked/exec'd from a process holding a GPU context (the launcher
    never touches the GPU).  Line-delimited JSON over pipes."""

    def __init__(self):
        import threading

        self._lock = threading.Lock()  # one request/reply in flight: callers may be several threads
        self.p = subprocess.Popen([sys.executable, "-u", "-m", "nos_amd.podbench", "--launcher"],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, cwd=str(REPO),
                                  env={**os.environ, "PYTHONPATH": str(REPO) + os.pathsep +
                                       os.environ.get("PYTHONPATH", "")})

    def _call(self, msg: dict) -> dict:
        with self._lock:
            self.p.stdin.write(json.dumps(msg) + "\n")
            self.p.stdin.flush()
            line = self.p.stdout.readline()
        if not line:
            raise RuntimeError("pod launcher died")
        r = json.loads(line)
        if "error" in r:
            raise RuntimeError(f"pod launcher: {r['error']}")
        return r

    def spawn(self, cmd: list[str], env: dict[str, str], log: str, cwd: str) -> _RemoteProc:
        return _RemoteProc(self, self._call({"op": "spawn", "cmd": cmd, "env": env, "log": log, "cwd": cwd})["pid"])

    def close(self) -> None:
        if self.p.poll() is None:
            try:
                self._call({"op": "exit"})
            except Exception:
                pass
            try:
                self.p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                self.p.kill()


def _launcher_main() -> int:
    procs: dict[int, subprocess.Popen] = {}
    for line in sys.stdin:
        msg = json.loads(line)
        op = msg.get("op")
        try:
            if op == "spawn":
                with open(msg["log"], "w") as log:
                    p = subprocess.Popen(msg["cmd"], env=msg["env"], stdout=log, stderr=subprocess.STDOUT,
                                         cwd=msg["cwd"])
                procs[p.pid] = p
                out = {"pid": p.pid}
            elif op == "poll":
                out = {"rc": procs[msg["pid"]].poll()}
            elif op == "kill":
                p = procs[msg["pid"]]
                if p.poll() is None:
                    p.kill()
                    p.wait()
                out = {"rc": p.returncode}
            elif op == "exit":
                for p in procs.values():
                    if p.poll() is None:
                        p.kill()
                        p.wait()
                print(json.dumps({"ok": True}), flush=True)
                return 0
            else:
                out = {"error": f"unknown op {op!r}"}
        except Exception as e:
            out = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    # stdin closed without "exit": the orchestrator died (killed at its time
    # limit, crashed) -- take the pods down with it instead of leaving them on the GPU
    for p in procs.values():
        if p.poll() is None:
            p.kill()
            p.wait()
    return 0


class PodFleet:
    """Start N pod processes with per-pod environments, wait until all are warm,
    then measure windows of wall time while all of them run."""

    def __init__(self, envs: list[dict[str, str]], dtype: str = "fp32", graphs: bool = True,
                 workdir: str | None = None, extra_env: dict[str, str] | None = None, seed0: int = 0,
                 launcher: PodLauncher | None = None, device: str = "cuda"):
        self.envs = envs
        self.dtype = dtype
        self.graphs = graphs
        self._own_dir = workdir is None
        self.dir = Path(workdir or tempfile.mkdtemp(prefix="nos_amd_pods_"))
        self.dir.mkdir(parents=True, exist_ok=True)
        self.extra_env = dict(extra_env or {})
        self.seed0 = seed0
        self.launcher = launcher
        self.device = device
        self.board: StatusBoard | None = None
        self.procs: list[subprocess.Popen] = []
        self.results: dict[int, dict] = {}

    def start(self) -> None:
        self.board = StatusBoard(self.dir / "status.bin", pods=len(self.envs))
        for i, penv in enumerate(self.envs):
            env = dict(os.environ)
            # a pod sees only its own allocation: drop the launcher's rank/device variables
            for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                      "ROC_GLOBAL_CU_MASK", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                      "NOS_AMD_MEMORY_LIMIT_GB", "GROUP_RANK", "ROLE_RANK", "LOCAL_WORLD_SIZE", "GROUP_WORLD_SIZE",
                      "ROLE_WORLD_SIZE", "ROLE_NAME"):
                env.pop(k, None)
            for k in [k for k in env if k.startswith("TORCHELASTIC_")]:
                env.pop(k)  # e.g. TORCHELASTIC_USE_AGENT_STORE: a trainer pod's job must host its own store
            env.update(self.extra_env)
            env.update(penv)
            env["PYTHONPATH"] = str(REPO) + os.pathsep + env.get("PYTHONPATH", "")
            # NOS_AMD_POD_KIND=trainer: the DP trainer tenant (models/trainer_pod.py) instead of a YOLOS pod
            module = "nos_amd.models.trainer_pod" if env.get("NOS_AMD_POD_KIND") == "trainer" else "nos_amd.models.pod"
            cmd = [sys.executable, "-u", "-m", module, "--status", str(self.board.path),
                   "--slot", str(i), "--out", str(self.dir), "--dtype", self.dtype, "--seed", str(self.seed0 + i),
                   "--device", self.device]
            if not self.graphs:
                cmd.append("--no-graphs")
            log = self.dir / f"pod-{i}.err"
            if self.launcher is not None:
                self.procs.append(self.launcher.spawn(cmd, env, str(log), str(REPO)))
            else:
                with open(log, "w") as err:
                    self.procs.append(subprocess.Popen(cmd, env=env, stdout=err, stderr=subprocess.STDOUT,
                                                       cwd=str(REPO)))

    def _failure(self) -> str | None:
        for i, (p, st) in enumerate(zip(self.procs, self.board.states())):
            if st == STATE_FAILED or (p.poll() is not None and st != STATE_READY):
                tail = (self.dir / f"pod-{i}.err").read_text()[-2000:]
                return f"pod {i} failed (exit {p.poll()}):\n{tail}"
        return None

    def wait_ready(self, timeout_s: float = 600.0, poll_s: float = 0.2, progress_cb=None) -> float:
        t0 = time.monotonic()
        last = -1
        while True:
            msg = self._failure()
            if msg:
                raise RuntimeError(msg)
            n = sum(1 for s in self.board.states() if s == STATE_READY)
            if n != last and progress_cb:
                progress_cb(n, len(self.envs))
                last = n
            if n == len(self.envs):
                return time.monotonic() - t0
            if time.monotonic() - t0 > timeout_s:
                raise TimeoutError(f"only {n}/{len(self.envs)} pods ready after {timeout_s} s")
            time.sleep(poll_s)

    def check_alive(self) -> None:
        msg = self._failure()
        if msg:
            raise RuntimeError(msg)

    def stop(self, timeout_s: float = 120.0) -> None:
        if self.board is None:
            return
        self.board.stop()
        deadline = time.monotonic() + timeout_s
        for p in self.procs:
            try:
                p.wait(timeout=max(1.0, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for i in range(len(self.envs)):
            f = self.dir / f"pod-{i}.json"
            self.results[i] = json.loads(f.read_text()) if f.exists() else {"slot": i, "error": "no result"}

    def window(self, t0: float, t1: float) -> WindowStats:
        """Per-pod stats of window [t0, t1] (CLOCK_MONOTONIC seconds)."""
        out = []
        w = t1 - t0
        for i in range(len(self.envs)):
            r = self.results.get(i, {})
            times = r.get("times") or []
            kind = r.get("kind") or ("trainer" if self.envs[i].get("NOS_AMD_POD_KIND") == "trainer" else "inference")
            if not times:
                out.append(PodResult(i, 0.0, None, w, False, {"error": r.get("error"), "kind": kind}))
                continue
            start = r.get("t_ready", times[0])
            c = progress(times, t1, start) - progress(times, t0, start)
            inside = [t0] + [t for t in times if t0 < t < t1] + [t1]
            gap = max(b - a for a, b in zip(inside, inside[1:]))
            # running through the window: warm before it, and never more than a
            # quarter of it without a completion -- the gap list ends at t1, so a
            # pod that stopped early fails it (a bursty pod idling at t1 does not)
            running = times[0] <= t0 and gap < 0.25 * w
            info = {k: r.get(k) for k in ("pid", "multiprocessor_count", "cu_mask", "hip_visible_devices",
                                           "memory_limit_gb", "memory_fraction", "max_allocated_gb", "cu_budget",
                                           "kind", "world_size", "backend", "flops_per_step", "bucket_bytes",
                                           "buckets", "bucket_busbw_gbps", "launched_in_backward", "kernel_config",
                                           "program")}
            info["kind"] = kind
            out.append(PodResult(i, c, (w / c) if c > 0 else None, gap, running, info))
        return WindowStats(w, out)

    def close(self) -> None:
        for p in self.procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        if self._own_dir:
            shutil.rmtree(self.dir, ignore_errors=True)


if __name__ == "__main__" and "--launcher" in sys.argv:
    sys.exit(_launcher_main())

__all__ = ["PodFleet", "PodLauncher", "WindowStats", "PodResult", "progress"]
