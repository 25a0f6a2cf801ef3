"""Feasibility probe for an MPS-style pod server: N YOLOS-small fp32 tenants
inside ONE process (one HIP context, one KFD process = one HWS slot), each on
its own stream and HIP graph, one launcher thread per tenant.  Prints one JSON
line per N: aggregate inf/s, per-tenant latency spread, SCLK.

  python tools/mps_probe.py --tenants 8,16,28 --mask none --window 8
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def _cus_for(i: int, n: int, num_cus: int) -> list[int]:
    """Equal CU shares spread over the XCDs (logical CU c lives on XCD c % 8)."""
    per = num_cus // n
    order = sorted(range(num_cus), key=lambda c: (c // 8, c % 8))  # round-robin XCDs
    return order[i * per:(i + 1) * per]


def run(n: int, mask: str, window: float, warmup_s: float) -> dict:
    from nos_amd.models.pod import _build, kernel_config
    from nos_amd.models.yolos import GraphedTenant, demo_input_hw
    from nos_amd import ops
    from nos_amd.ops.streams import CUMaskedStream, device_info

    info = device_info(0)
    cfg = kernel_config(1.0 / n, {}, info["num_cus"] // n if mask == "equal" else 0)
    ops.set_gemm_f32_policy(cfg["gemm_f32"])
    ops.set_attention_f32_variant(cfg["attention_f32"])
    ops.set_f32_math(cfg["f32_math"])
    ops.set_gemm_f32x6_tile(cfg["gemm_f32x6_tile"])
    if mask == "equal":
        ops.set_cu_budget(info["num_cus"] // n)
    tenants, streams = [], []
    t0 = time.time()
    for i in range(n):
        m, x = _build("fp32", i, demo_input_hw(), "cuda")
        cus = _cus_for(i, n, info["num_cus"]) if mask == "equal" else None
        s = CUMaskedStream(cus, info["num_cus"])
        streams.append(s)
        t = GraphedTenant(m, s.torch, x)
        with torch.no_grad():
            t.capture()
        tenants.append(t)
    build_s = time.time() - t0
    stop = threading.Event()
    counts = [0] * n
    marks: list[list[float]] = [[] for _ in range(n)]

    def loop(i: int) -> None:
        t, s = tenants[i], streams[i]
        with torch.no_grad():
            while not stop.is_set():
                t.launch()
                s.synchronize()
                counts[i] += 1
                marks[i].append(time.monotonic())

    th = [threading.Thread(target=loop, args=(i,), daemon=True) for i in range(n)]
    for x in th:
        x.start()
    time.sleep(warmup_s)
    w0 = time.monotonic()
    time.sleep(window)
    w1 = time.monotonic()
    stop.set()
    for x in th:
        x.join()
    done = [sum(1 for m in mk if w0 <= m < w1) for mk in marks]
    lat = [window / d if d else None for d in done]
    for s in streams:
        s.close()
    ok = [v for v in lat if v]
    return {"tenants": n, "mask": mask, "window_s": round(w1 - w0, 3), "build_s": round(build_s, 1),
            "inf_per_s": round(sum(done) / (w1 - w0), 2), "min_done": min(done), "max_done": max(done),
            "lat_ms_min": round(1e3 * min(ok), 2) if ok else None, "lat_ms_max": round(1e3 * max(ok), 2) if ok else None,
            "kernel_config": cfg, "mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tenants", default="8,16,28")
    ap.add_argument("--mask", choices=["none", "equal"], default="none")
    ap.add_argument("--window", type=float, default=8.0)
    ap.add_argument("--warmup", type=float, default=2.0)
    a = ap.parse_args()
    torch.backends.cuda.matmul.allow_tf32 = False
    for n in (int(v) for v in a.tenants.split(",")):
        print(json.dumps(run(n, a.mask, a.window, a.warmup)), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
