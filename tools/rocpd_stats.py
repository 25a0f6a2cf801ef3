"""Kernel statistics from a rocprofv3 rocpd database (``*_results.db``).

python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--top 25] [--csv out.csv]
"""
from __future__ import annotations

import argparse
import csv
import sqlite3


def kernel_stats(db: str) -> list[dict]:
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                     f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [{"kernel": r[0], "calls": r[1], "total_us": r[2] / 1e3, "avg_us": r[3] / 1e3, "min_us": r[4] / 1e3,
             "max_us": r[5] / 1e3, "pct": 100.0 * r[2] / total} for r in rows]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--csv")
    a = ap.parse_args()
    st = kernel_stats(a.db)
    for r in st[: a.top]:
        print(f"{r['pct']:6.2f}% {r['calls']:6d} {r['avg_us']:10.2f} us  {r['kernel'][:110]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0].keys()))
            w.writeheader()
            w.writerows(st)


if __name__ == "__main__":
    main()
