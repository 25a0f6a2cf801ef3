"""Do N CU-masked queues run concurrently?  In-process streams vs. one process per slice.

Every slice runs the same fixed MFMA work (probe_mfma_peak, 2 WGs per CU of
the slice); if N slices execute concurrently the wall time stays ~flat as N
grows (each slice has 1/N of the CUs but also 1/N of the total work).

python tools/cumask_concurrency.py --out gpurun_out/cumask_conc.json
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

TOTAL_WG = 512      # 2 per CU of the whole GPU
ITERS = 200000


def inproc(n: int, masked: bool) -> dict:
    import torch

    from nos_amd.gpu.topology import split_even
    from nos_amd.ops import _lib
    from nos_amd.ops.streams import CUMaskedStream

    L = _lib.lib()
    slices = split_even(n)
    streams = [CUMaskedStream(s.cus() if masked else None, 256) for s in slices]
    scratch = torch.zeros(TOTAL_WG, device="cuda")
    per = TOTAL_WG // n
    for s in streams:  # warm-up
        L.nos_probe_mfma_peak_launch(s.handle, per, 50, scratch.data_ptr())
    for s in streams:
        s.synchronize()
    t = time.perf_counter()
    for s in streams:
        L.nos_probe_mfma_peak_launch(s.handle, per, ITERS, scratch.data_ptr())
    for s in streams:
        s.synchronize()
    dt = time.perf_counter() - t
    for s in streams:
        s.close()
    return {"n": n, "masked": masked, "mode": "inproc", "wall_ms": dt * 1e3}


def _child(mask_hex: str | None, per: int, barrier, q) -> None:
    if mask_hex:
        os.environ["ROC_GLOBAL_CU_MASK"] = mask_hex
    import torch

    from nos_amd.ops import _lib

    L = _lib.lib()
    scratch = torch.zeros(TOTAL_WG, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    L.nos_probe_mfma_peak_launch(s, per, 50, scratch.data_ptr())
    torch.cuda.synchronize()
    barrier.wait()
    t = time.perf_counter()
    L.nos_probe_mfma_peak_launch(s, per, ITERS, scratch.data_ptr())
    torch.cuda.synchronize()
    q.put((t, time.perf_counter()))


def multiproc(n: int, masked: bool) -> dict:
    from nos_amd.gpu.topology import split_even
    from nos_amd.ops.streams import mask_hex

    ctx = mp.get_context("spawn")
    barrier = ctx.Barrier(n)
    q = ctx.Queue()
    per = TOTAL_WG // n
    procs = []
    for s in split_even(n):
        m = mask_hex(s.cus(), 256) if masked else None
        p = ctx.Process(target=_child, args=(m, per, barrier, q))
        p.start()
        procs.append(p)
    spans = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    t0 = min(a for a, _ in spans)
    t1 = max(b for _, b in spans)
    return {"n": n, "masked": masked, "mode": "multiproc", "wall_ms": (t1 - t0) * 1e3,
            "per_proc_ms": sorted(round((b - a) * 1e3, 2) for a, b in spans)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/cumask_conc.json")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--skip-multiproc", action="store_true")
    a = ap.parse_args()
    res = []
    for n in map(int, a.ns.split(",")):
        for masked in (True, False):
            r = inproc(n, masked)
            print(json.dumps(r), flush=True)
            res.append(r)
    if not a.skip_multiproc:
        for n in map(int, a.ns.split(",")):
            for masked in (True, False):
                r = multiproc(n, masked)
                print(json.dumps(r), flush=True)
                res.append(r)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
