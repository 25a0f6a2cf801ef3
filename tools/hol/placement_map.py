"""Which physical CUs does each XCD-symmetric CU-mask slot set really get?

For slot sets S (local CU slots per XCD, bit = slot * 8 + xcd), run the
placement probe on a stream created with that mask and record the
(XCC, SE, SH, CU) of every workgroup; report each set's CUs and the overlap
between sets.  Two device-plugin slices must never share a physical CU.

python tools/hol/placement_map.py --out gpurun_out/placement_map.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

SETS = {"s0_3": range(0, 4), "s4_7": range(4, 8), "s8_11": range(8, 12), "s12_15": range(12, 16),
        "s16_19": range(16, 20), "s20_23": range(20, 24), "s24_27": range(24, 28), "s28_31": range(28, 32),
        "s0": range(0, 1), "s1": range(1, 2), "s2": range(2, 3), "s3": range(3, 4), "s4": range(4, 5),
        "s8": range(8, 9), "s15": range(15, 16), "s16": range(16, 17), "s17": range(17, 18), "s31": range(31, 32),
        "s0_15": range(0, 16), "s16_31": range(16, 32)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/placement_map.json")
    ap.add_argument("--nwg", type=int, default=4096)
    a = ap.parse_args()
    import torch

    from nos_amd.gpu.topology import MI355X_CUS, logical_cu
    from nos_amd.ops import probes
    from nos_amd.ops.streams import CUMaskedStream

    torch.cuda.set_device(0)
    res = {}
    full = probes.placement(nwg=a.nwg)
    res["all"] = sorted({r.cu_key for r in full})
    for name, slots in SETS.items():
        cus = [logical_cu(x, j) for x in range(8) for j in slots]
        s = CUMaskedStream(cus, MI355X_CUS)
        recs = probes.placement(stream=s.handle, nwg=a.nwg)
        res[name] = sorted({r.cu_key for r in recs})
        s.close()
        print(name, len(res[name]), flush=True)
    names = [n for n in SETS]
    overlaps = {}
    for i, x in enumerate(names):
        for y in names[i + 1:]:
            o = set(map(tuple, res[x])) & set(map(tuple, res[y]))
            if o and not (set(SETS[x]) & set(SETS[y])):
                overlaps[f"{x}&{y}"] = len(o)
    out = {"distinct_cus": {k: len(v) for k, v in res.items()}, "overlaps_between_disjoint_slot_sets": overlaps,
           "cus": {k: v[:64] for k, v in res.items()}}
    print(json.dumps({"distinct_cus": out["distinct_cus"], "overlaps": overlaps}))
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
