"""Run the gpuagent's slice prober on this GPU for a few slice profiles.

python tools/probe_run.py --profiles 36gb,72gb,288gb --out gpurun_out/probe.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--profiles", default="36gb,72gb,288gb")
    ap.add_argument("--no-loaded", action="store_true")
    ap.add_argument("--out", default="gpurun_out/probe.json")
    a = ap.parse_args()
    from nos_amd.agents.probe import SliceProber
    from nos_amd.gpu.amdsmi import AmdSmi

    smi = AmdSmi.real()
    idx = {g.hip_id: g.index for g in smi.gpus()}.get(0, 0)
    prober = SliceProber(smi, loaded=not a.no_loaded)
    rows = []
    for prof in a.profiles.split(","):
        r = prober(0, prof)
        r["sclk_after"] = smi.clock(idx)
        rows.append({"profile": prof, **{k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}})
        print(json.dumps(rows[-1]), flush=True)
    Path(a.out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
