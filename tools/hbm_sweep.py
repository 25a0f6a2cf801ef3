"""HBM probe variants x grid sizes on the full GPU (gpuagent probe tuning).

python tools/hbm_sweep.py --out gpurun_out/hbm_sweep.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/hbm_sweep.json")
    ap.add_argument("--gb", type=float, default=2.0)
    a = ap.parse_args()
    import torch

    from nos_amd.ops import probes

    s = torch.cuda.current_stream().cuda_stream
    rows = []
    for mode in ("copy", "copy_nt", "read"):
        for nwg in (512, 1024, 2048, 4096, 8192):
            g = probes.hbm_mode_gbps(s, mode, int(a.gb * (1 << 30)), 5, nwg)
            rows.append({"mode": mode, "nwg": nwg, "gbps": round(g, 1)})
            print(json.dumps(rows[-1]), flush=True)
    Path(a.out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
