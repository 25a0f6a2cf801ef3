"""Per-pod kernel time vs dispatch gaps from a rocprofv3 kernel trace
(diagnostic for CU-mask slice flatness, docs/status.md item 6).

python tools/trace_gaps.py <rocprofv3 output dir> [--json out.json]

For every process that ran the YOLOS forward (kernels of libnos_hip), over
its graph replays: the mean duration of each kernel kind, and the gap between
a kernel's end and the next kernel's start on the same queue (dispatch /
command-processor delay).  Comparing a 1-pod run with a 7-pod run tells
contention inside the kernels (durations grow: shared L2 / HBM / clock)
from contention in getting them dispatched (gaps grow: queues sharing the
command processor's pipes).
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import statistics
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel)", name)
    base = m.group(1) if m else name.split("(")[0][-40:]
    t = re.search(r"<([^>]*)>", name)
    return f"{base}<{t.group(1)[:40]}>" if t else base


def load(root: Path) -> dict:
    rows = []
    for f in root.rglob("*kernel_trace.csv"):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    by_q: dict[tuple, list] = defaultdict(list)
    for r in rows:
        pid = r.get("Process_Id") or r.get("Pid") or "?"
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        by_q[(pid, q)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    out = {"queues": len(by_q), "per_kernel_us": {}, "gap_us": {}}
    dur: dict[str, list] = defaultdict(list)
    gaps: list[float] = []
    for key, ks in by_q.items():
        ks.sort()
        if not any("f32x6" in k[2] or "attn" in k[2] for k in ks):
            continue
        for (s0, e0, n0), (s1, _e1, _n1) in zip(ks, ks[1:]):
            g = (s1 - e0) / 1e3
            if 0 <= g < 200:  # inside a replay (a host round trip between inferences is longer)
                gaps.append(g)
        for s, e, n in ks:
            if "f32x6" in n or "attn" in n:
                dur[short(n)].append((e - s) / 1e3)
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        out["per_kernel_us"][k] = {"calls": len(v), "mean": round(statistics.mean(v), 2),
                                   "median": round(statistics.median(v), 2)}
    if gaps:
        gs = sorted(gaps)
        out["gap_us"] = {"n": len(gs), "mean": round(statistics.mean(gs), 2), "median": round(gs[len(gs) // 2], 2),
                         "p90": round(gs[int(0.9 * len(gs))], 2)}
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = load(Path(a.root))
    print(json.dumps(res, indent=1))
    if a.json:
        Path(a.json).write_text(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
