"""Where do the workgroups of CO-RUNNING CU-masked queues land?

N streams (one HW queue each, hipExtStreamCreateWithCUMask) with disjoint
XCD-symmetric masks of 4 CUs per XCD each run the placement probe at the same
time (every workgroup spins long enough for all launches to overlap).  For
each stream: the physical CUs (XCC, SE, SH, CU) its workgroups ran on, whether
they stayed inside its own mask's CUs (measured alone), and which other
streams' CUs they used.  Answers whether queues sharing a command-processor
pipe (5+ masked queues per XCD) still honour their own masks.

python tools/hol/pair_placement.py --streams 5 --out gpurun_out/pair_placement.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=5)
    ap.add_argument("--per-xcd", type=int, default=4)
    ap.add_argument("--nwg", type=int, default=512)
    ap.add_argument("--spin-ms", type=float, default=20.0)
    ap.add_argument("--out", default="gpurun_out/pair_placement.json")
    a = ap.parse_args()
    import torch

    from nos_amd.gpu.topology import MI355X_CUS, logical_cu
    from nos_amd.ops import _lib, probes
    from nos_amd.ops.streams import CUMaskedStream

    torch.cuda.set_device(0)
    streams, alone = [], []
    for k in range(a.streams):
        cus = [logical_cu(x, j) for x in range(8) for j in range(k * a.per_xcd, (k + 1) * a.per_xcd)]
        s = CUMaskedStream(cus, MI355X_CUS)
        streams.append(s)
        alone.append({r.cu_key for r in probes.placement(stream=s.handle, nwg=a.nwg, spin_ticks=2000)})
    # all streams at once: each workgroup spins spin_ms so every launch overlaps the others
    ticks = int(a.spin_ms * 1e5)
    bufs = [torch.zeros((a.nwg, 4), dtype=torch.int32, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    for s, b in zip(streams, bufs):
        _lib.check(_lib.lib().nos_probe_placement(b.data_ptr(), a.nwg, ticks, s.handle), "probe_placement")
    torch.cuda.synchronize()
    together = []
    for b in bufs:
        recs = set()
        for xcc, hw, _blk, _t in b.cpu().tolist():
            se, sh, cu = probes.decode_hw_id(hw & 0xFFFFFFFF)
            recs.add((xcc & 0xF, se, sh, cu))
        together.append(recs)
    rows = []
    for k in range(a.streams):
        outside = together[k] - alone[k]
        rows.append({"stream": k, "cus_alone": len(alone[k]), "cus_together": len(together[k]),
                     "cus_outside_own_mask": len(outside),
                     "borrowed_from": {j: len(outside & alone[j]) for j in range(a.streams)
                                       if j != k and outside & alone[j]}})
    out = {"streams": a.streams, "per_xcd": a.per_xcd, "nwg": a.nwg, "rows": rows}
    print(json.dumps(out))
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(out, indent=1))
    for s in streams:
        s.close()


if __name__ == "__main__":
    main()
