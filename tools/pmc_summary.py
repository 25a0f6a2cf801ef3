"""Summarise rocprofv3 --pmc CSV passes per kernel (sum over dispatches).

python tools/pmc_summary.py gpurun_out/pmc_probes --out profiles/r02_pmc_probes.json
Derived: MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs... reported raw too),
VALU per MFMA instruction, L2 hit %, FETCH/WRITE bytes (gfx950 FETCH_SIZE reads half of wide
streaming loads: MI355X_MICROARCH.md, HBM section).
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path


def load(root: Path) -> dict[str, dict[str, float]]:
    agg: dict[str, dict[str, float]] = defaultdict(lambda: defaultdict(float))
    calls: dict[str, set] = defaultdict(set)
    for f in root.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name") or row.get("kernel_name") or "?"
                name = row.get("Counter_Name") or row.get("counter_name")
                val = float(row.get("Counter_Value") or row.get("counter_value") or 0)
                agg[k][name] += val
                calls[k].add((str(f.parent), row.get("Dispatch_Id") or row.get("dispatch_id")))
    return {k: dict(v) for k, v in agg.items()}


def derive(c: dict[str, float], cus: int = 256) -> dict[str, float]:
    out = {}
    if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
        # the rounds-1..5 figure, kept for comparison: busy / (GRBM_GUI_ACTIVE x CUs)
        out["mfma_busy_pct_of_cu_cycles"] = 100.0 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] * cus)
        # the matrix-pipe utilisation itself: SQ_VALU_MFMA_BUSY_CYCLES counts SIMD
        # cycles (32 per 32x32x16 MFMA) summed over the chip's 4 x CUs SIMDs, and
        # rocprofv3's GRBM_GUI_ACTIVE is the sum over the 8 XCDs (MI355X_MICROARCH.md,
        # DVFS note), so the elapsed cycles are GUI / 8 and the pipe-cycles available
        # GUI / 8 x 4 x CUs.  (The old figure is half of this: it divided by GUI x CUs.)
        out["mfma_util_pct"] = 100.0 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 4 * cus)
    if c.get("SQ_INSTS_MFMA"):
        out["valu_per_mfma"] = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_INSTS_MFMA"]
    h, m = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
    if h is not None and m is not None and h + m > 0:
        out["l2_hit_pct"] = 100.0 * h / (h + m)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    data = load(Path(a.root))
    res = {}
    for k, c in sorted(data.items()):
        if a.filter and a.filter not in k:
            continue
        res[k[:120]] = {"counters": c, "derived": derive(c)}
        print(k[:100], json.dumps(derive(c)))
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
