"""Why do many CU-mask slices lose throughput?  Same 8 YOLOS pods, different
mask layouts (in-process CU-masked streams).

python tools/cumask_layouts.py --pods 8 --steps 20
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from nos_amd.gpu.topology import logical_cu, split_even  # noqa: E402
from nos_amd.models.tenants import InferenceTenants, TenantSpec  # noqa: E402
from nos_amd.models.yolos import YolosConfig, demo_input_hw  # noqa: E402
from nos_amd.ops.streams import device_info  # noqa: E402


def strided(n: int) -> list[list[int]]:
    """slice i owns local CU slots i, i+n, i+2n, ... on every XCD"""
    return [sorted(logical_cu(x, j) for x in range(8) for j in range(i, 32, n)) for i in range(n)]


def paired(n: int) -> list[list[int]]:
    """n/2 distinct masks, two pods per mask"""
    base = [s.cus() for s in split_even(max(1, n // 2))]
    return [base[i // 2] for i in range(n)]


def overlapped(n: int, k: int) -> list[list[int]]:
    """slice i owns the k consecutive fair shares starting at share i (wrapping):
    every CU is shared by k pods, every pod is guaranteed 1/k of its mask"""
    per = 32 // n
    out = []
    for i in range(n):
        slots = {(i * per + j) % 32 for j in range(per * k)}
        out.append(sorted(logical_cu(x, j) for x in range(8) for j in slots))
    return out


def measure(name: str, masks, steps: int, num_cus: int) -> dict:
    ts = InferenceTenants([TenantSpec(f"p{i}", m) for i, m in enumerate(masks)], num_cus,
                          YolosConfig.small(), demo_input_hw(), use_graphs=True)
    ts.prepare()
    with torch.no_grad():
        ts.run(3)
        dt = ts.run(steps)
    ts.close()
    del ts
    torch.cuda.empty_cache()
    n = len(masks)
    return {"layout": name, "pods": n, "img_per_s": n * steps / dt, "pod_latency_ms": dt / steps * 1e3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/cumask_layouts.json")
    ap.add_argument("--layouts", default="")
    a = ap.parse_args()
    num_cus = device_info(0)["num_cus"]
    n = a.pods
    layouts = {
        "contiguous": [s.cus() for s in split_even(n)],
        "strided": strided(n),
        "paired": paired(n),
        "shared": [None] * n,
        "full_mask": [list(range(num_cus))] * n,
        "overlap2": overlapped(n, 2),
        "overlap4": overlapped(n, 4),
    }
    if a.layouts:
        layouts = {k: v for k, v in layouts.items() if k in a.layouts.split(",")}
    res = []
    for name, masks in layouts.items():
        r = measure(name, masks, a.steps, num_cus)
        print(json.dumps(r), flush=True)
        res.append(r)
        Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
