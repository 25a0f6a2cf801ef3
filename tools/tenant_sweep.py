"""Sweep pods-per-GPU x sharing mode for YOLOS-small tenants on one MI355X.

python tools/tenant_sweep.py --out gpurun_out/sweep.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from nos_amd.gpu.topology import split_even  # noqa: E402
from nos_amd.models.tenants import InferenceTenants, TenantSpec  # noqa: E402
from nos_amd.models.yolos import YolosConfig, demo_input_hw  # noqa: E402
from nos_amd.ops.streams import device_info  # noqa: E402


def measure(mode: str, pods: int, steps: int, num_cus: int, graphs: bool = True) -> dict:
    if mode == "cumask":
        masks = [s.cus() for s in split_even(pods)]
    else:
        masks = [None] * pods
    ts = InferenceTenants([TenantSpec(f"p{i}", m) for i, m in enumerate(masks)], num_cus,
                          YolosConfig.small(), demo_input_hw(), use_graphs=graphs)
    ts.prepare()
    with torch.no_grad():
        ts.run(3)
        dt = ts.run(steps)
    ts.close()
    del ts
    torch.cuda.empty_cache()
    return {"mode": mode, "pods": pods, "graphs": graphs, "img_per_s": pods * steps / dt,
            "pod_latency_ms": dt / steps * 1e3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/sweep.json")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--pods", default="1,2,4,7,8,16,28")
    ap.add_argument("--modes", default="cumask,shared")
    a = ap.parse_args()
    info = device_info(0)
    res = []
    for mode in a.modes.split(","):
        for p in map(int, a.pods.split(",")):
            if mode == "cumask" and p > 32:
                continue
            r = measure(mode, p, a.steps, info["num_cus"])
            print(json.dumps(r), flush=True)
            res.append(r)
            Path(a.out).parent.mkdir(parents=True, exist_ok=True)
            Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
