"""Latency-vs-pods table of the reference demo (README.md:63-71) on MI355X.

Each row: N pod processes started with the device plugin's env for the mode
(shared = memory-capped slices on all CUs, the MPS analogue; cumask = exclusive
XCD-symmetric CU slices), all warm, then one steady-state window of
``--window`` seconds (aligned: it starts only when every pod runs).  mean
latency = pods x window / completed inferences, so pods / latency ==
throughput in every row.

python tools/sharing_table.py --pods 1,3,5,7 --modes shared,cumask --window 10 --out gpurun_out/table.json
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", default="1,3,5,7")
    ap.add_argument("--modes", default="shared,cumask")
    ap.add_argument("--window", type=float, default=10.0)
    ap.add_argument("--warmup", type=float, default=2.0)
    ap.add_argument("--slice-gb", type=int, default=36)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--hw-queues", default="0", help="comma list of GPU_MAX_HW_QUEUES values (0 = default)")
    ap.add_argument("--pod-env", action="append", default=[], help="extra KEY=VALUE for every pod (repeatable)")
    ap.add_argument("--out", default="gpurun_out/sharing_table.json")
    a = ap.parse_args()

    import bench
    from nos_amd.podbench import PodLauncher

    launcher = PodLauncher()
    d = bench.Dist()
    plans = {}
    for mode in a.modes.split(","):
        for n in map(int, a.pods.split(",")):
            envs, info = bench.plan(None, 1, 0, a.slice_gb, n, mode)
            plans[(mode, n)] = (envs, info)
    d.init_gpu()
    sampler = bench.UtilSampler(d.device)
    rows = []
    for hq in map(int, a.hw_queues.split(",")):
        extra = {"GPU_MAX_HW_QUEUES": str(hq)} if hq else {}
        extra.update(kv.split("=", 1) for kv in a.pod_env)
        for mode in a.modes.split(","):
            for n in map(int, a.pods.split(",")):
                envs, info = plans[(mode, n)]
                t = time.monotonic()
                w, util, n_util, ready, _ = bench.run_fleet(d, launcher, envs, a.dtype, True, extra, 1, 1, a.window,
                                                         sampler)
                w0 = bench.time.monotonic()
                row = {"mode": mode, "hw_queues": hq, "pod_env": a.pod_env, "dtype": a.dtype, **w.as_dict(), "gpu_util_pct": util,
                       "util_samples": n_util, "pods_ready_s": round(ready, 1),
                       "cus_per_pod": [p.info.get("cu_mask") for p in w.pods][:2],
                       "wall_s": round(w0 - t, 1)}
                print(json.dumps(row), flush=True)
                rows.append(row)
                Path(a.out).write_text(json.dumps(rows, indent=1))
    sampler.close()
    launcher.close()


if __name__ == "__main__":
    main()
