"""Sum rocprofv3 counter_collection.csv rows per kernel (name prefix) over passes.

python tools/pmc_table.py gpurun_out/pmc_gemm_f32 [--match gemm_f32]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
from pathlib import Path


def table(root: str, match: str = "") -> dict:
    agg: dict = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in sorted(Path(root).rglob("*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if match and match not in name:
                continue
            key = name.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
            if "<" in name:
                key = name[:name.index(">") + 1].replace("void ", "").replace("(anonymous namespace)::", "")
            agg[key][row["Counter_Name"]] += float(row["Counter_Value"])
    return {k: dict(v) for k, v in agg.items()}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    print(json.dumps(table(a.root, a.match), indent=1))


if __name__ == "__main__":
    main()
