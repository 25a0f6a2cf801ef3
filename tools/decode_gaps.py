"""Per-kernel time and launch gaps of a decode tenant's steps from a
rocprofv3 kernel trace (``--kernel-trace --output-format csv``): the last
``--tail`` dispatches (steady-state decode) -> busy time per kernel name and
the idle gap between one kernel's end and the next one's start."""
import argparse
import collections
import csv
import json


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=int, default=5000)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.tail:]
    busy = collections.defaultdict(lambda: [0, 0.0])
    gaps = []
    for i, r in enumerate(rows):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = r["Kernel_Name"][:70] + (f" grid {r['Grid_Size']}" if "Grid_Size" in r else "")
        busy[k][0] += 1
        busy[k][1] += (e - s) / 1e3
        if i:
            gaps.append((s - int(rows[i - 1]["End_Timestamp"])) / 1e3)
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    tot = sum(v[1] for v in busy.values())
    steps = busy.get(next((k for k in busy if "argmax" in k), ""), [0])[0] or 1
    gs = sorted(gaps)
    out = {"dispatches": len(rows), "span_us": round(span, 1), "kernel_busy_us": round(tot, 1),
           "steps": steps, "us_per_step": round(span / steps, 1), "busy_us_per_step": round(tot / steps, 1),
           "gap_us": {"mean": round(sum(gs) / len(gs), 2), "p50": round(gs[len(gs) // 2], 2),
                      "p90": round(gs[int(len(gs) * 0.9)], 2)},
           "per_kernel": {k: {"calls": v[0], "us_per_call": round(v[1] / v[0], 2), "us_per_step": round(v[1] / steps, 1)}
                          for k, v in sorted(busy.items(), key=lambda kv: -kv[1][1])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
