"""Sweep the dispatch head-of-line microbenchmark (holbench.hip) over pod
counts, grid sizes and HW-queue settings, one process per pod with the
device plugin's XCD-symmetric CU mask (or no mask).

python tools/hol/run_hol.py --out gpurun_out/hol.json [--pods 1,3,4,5,8] [--grids 0,-4]

Each row: per-pod slot efficiency (workgroup-seconds completed / slot-seconds
the pod's mask owns).  The launcher never touches the GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
BIN = REPO / "build" / "holbench"


def build(force: bool = False) -> Path:
    src = Path(__file__).with_name("holbench.hip")
    if force or not BIN.exists() or BIN.stat().st_mtime < src.stat().st_mtime:
        BIN.parent.mkdir(parents=True, exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", str(src), "-o", str(BIN)],
                       check=True)
    return BIN


def masks(n: int, per_xcd: int, mode: str, starts: list[int] | None = None) -> list[str | None]:
    from nos_amd.gpu.topology import MI355X_CUS, logical_cu
    from nos_amd.ops.streams import mask_hex

    if mode == "none":
        return [None] * n
    out = []
    for k in range(n):
        s0 = starts[k] if starts else k * per_xcd
        slots = range(s0, s0 + per_xcd)
        out.append(mask_hex([logical_cu(x, j) for x in range(8) for j in slots], MI355X_CUS))
    return out


def run_row(n: int, grid: int, hwq: int, mode: str, per_xcd: int, seconds: float, spin_us: float, lds: int,
            depth: int, null_stream: int, timeout: float, phases: int = 0, iters: int = 0,
            starts: list[int] | None = None) -> dict:
    start = time.monotonic_ns() + int(4e9)
    procs = []
    for k, m in enumerate(masks(n, per_xcd, mode, starts)):
        env = dict(os.environ)
        env.pop("ROC_GLOBAL_CU_MASK", None)
        if m:
            env["ROC_GLOBAL_CU_MASK"] = m
        if hwq:
            env["GPU_MAX_HW_QUEUES"] = str(hwq)
        cmd = [str(BIN), "--seconds", str(seconds), "--start-ns", str(start), "--grid", str(grid),
               "--spin-us", str(spin_us), "--lds", str(lds), "--depth", str(depth), "--null-stream", str(null_stream),
               "--phases", str(phases), "--iters", str(iters), "--tag", f"{mode}-n{n}-g{grid}-q{hwq}-d{depth}-ph{phases}-p{k}"]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    pods = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            out, err = p.communicate()
        if p.returncode != 0:
            pods.append({"error": err[-400:], "rc": p.returncode})
            continue
        pods.append(json.loads(out.strip().splitlines()[-1]))
    effs = [q.get("slot_efficiency", 0.0) for q in pods]
    kms = [q.get("kernel_ms", 0.0) for q in pods]
    return {"pods": n, "grid": grid, "hw_queues": hwq, "mask": mode, "per_xcd": per_xcd, "null_stream": null_stream,
            "depth": depth, "phases": phases, "aborted": sum(q.get("barrier_aborted", 0) for q in pods),
            "eff_min": round(min(effs), 3), "eff_max": round(max(effs), 3),
            "eff_mean": round(sum(effs) / len(effs), 3), "iters": iters, "slot_starts": starts,
            "kernel_ms_min": round(min(kms), 4), "kernel_ms_max": round(max(kms), 4), "per_pod": pods}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", default="1,3,4,5,8")
    ap.add_argument("--grids", default="0,-4", help="0 = fit the mask's slots, -k = k x fit, k > 0 = absolute")
    ap.add_argument("--hw-queues", default="0,1")
    ap.add_argument("--masks", default="cumask")
    ap.add_argument("--per-xcd", type=int, default=4)
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--spin-us", type=float, default=50.0)
    ap.add_argument("--lds", type=int, default=40960)
    ap.add_argument("--depth", default="16", help="comma list: kernels queued per host synchronize")
    ap.add_argument("--phases", default="0", help="comma list: 0 = one spin per launch, P = megakernel of P phases")
    ap.add_argument("--null-stream", type=int, default=0)
    ap.add_argument("--iters", type=int, default=0, help="> 0: VALU work per workgroup instead of the realtime spin "
                    "(compare kernel_ms with the 1-pod row)")
    ap.add_argument("--slot-starts", default="", help="';'-separated lists of per-pod first slots, e.g. '0,16;0,4' "
                    "(overrides --pods: one row per list)")
    ap.add_argument("--out", default="gpurun_out/hol.json")
    a = ap.parse_args()
    build()
    rows = []
    for mode in a.masks.split(","):
        for hwq in map(int, a.hw_queues.split(",")):
            for grid in map(int, a.grids.split(",")):
              for depth in map(int, a.depth.split(",")):
               for phases in map(int, a.phases.split(",")):
                layouts = ([[int(x) for x in lst.split(",")] for lst in a.slot_starts.split(";")] if a.slot_starts
                           else [None] * len(a.pods.split(",")))
                for n, starts in zip([len(x) for x in layouts] if a.slot_starts else map(int, a.pods.split(",")),
                                     layouts):
                    r = run_row(n, grid, hwq, mode, a.per_xcd, a.seconds, a.spin_us, a.lds, depth, a.null_stream,
                                timeout=a.seconds + 60, phases=phases, iters=a.iters, starts=starts)
                    print(json.dumps({k: v for k, v in r.items() if k != "per_pod"}), flush=True)
                    rows.append(r)
                    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
                    Path(a.out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
