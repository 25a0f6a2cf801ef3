"""YOLOS pods as separate processes (the real deployment: one container per
slice, CU mask injected by the device plugin as ROC_GLOBAL_CU_MASK) vs. the
in-process CU-masked streams of bench.py.

python tools/pod_procs.py --pods 8 --mode cumask --iters 50
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def _pod(mask_hex: str | None, iters: int, barrier, q, seed: int) -> None:
    if mask_hex:
        os.environ["ROC_GLOBAL_CU_MASK"] = mask_hex
    import torch

    from nos_amd.models.yolos import GraphedTenant, YolosConfig, YolosDetector, demo_input_hw, make_demo_input

    cfg = YolosConfig.small()
    m = YolosDetector(cfg)
    m.reset_parameters(seed)
    m = m.to("cuda", torch.bfloat16).eval()
    x = make_demo_input(cfg, device="cuda", hw=demo_input_hw(), seed=seed)
    s = torch.cuda.Stream()
    t = GraphedTenant(m, s, x)
    with torch.no_grad():
        t.capture()
        for _ in range(3):
            t.launch()
    s.synchronize()
    barrier.wait()
    t0 = time.perf_counter()
    with torch.no_grad():
        for _ in range(iters):
            t.launch()
    s.synchronize()
    q.put((t0, time.perf_counter()))


def run(pods: int, mode: str, iters: int) -> dict:
    from nos_amd.gpu.topology import split_even
    from nos_amd.ops.streams import mask_hex

    ctx = mp.get_context("spawn")
    barrier = ctx.Barrier(pods)
    q = ctx.Queue()
    procs = []
    for i, s in enumerate(split_even(pods)):
        m = mask_hex(s.cus(), 256) if mode == "cumask" else None
        p = ctx.Process(target=_pod, args=(m, iters, barrier, q, i))
        p.start()
        procs.append(p)
    spans = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    t0 = min(a for a, _ in spans)
    t1 = max(b for _, b in spans)
    lat = [(b - a) / iters * 1e3 for a, b in spans]
    return {"pods": pods, "mode": mode, "procs": True, "img_per_s": pods * iters / (t1 - t0),
            "pod_latency_ms": sum(lat) / len(lat)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", default="4,8")
    ap.add_argument("--modes", default="cumask,shared")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--out", default="gpurun_out/pod_procs.json")
    a = ap.parse_args()
    res = []
    for mode in a.modes.split(","):
        for p in map(int, a.pods.split(",")):
            r = run(p, mode, a.iters)
            print(json.dumps(r), flush=True)
            res.append(r)
            Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
