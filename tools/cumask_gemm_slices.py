"""BASELINE config 4: CU-mask fractional sharing (the MPS equivalent) with 4
slices per GPU running the bf16 GEMM probe, and per-slice rocprof counters.

The 4 slices are laid out by the device plugin's allocator
(``gpu/topology.py:layout_slots``, ``cuPolicy: proportional``: 72 GB of 288 GB
= 8 of 32 CUs on every XCD) and run on CU-masked HIP streams, the gpuagent
probe's own mechanism.  Phase ``run`` times each slice alone, all 4 at once,
and the unmasked GPU; phase ``pmc`` launches a few GEMMs per slice for a
``rocprofv3 --pmc`` pass, whose per-dispatch counters are split by HSA queue
(one queue per CU-masked stream) into per-slice numbers.

python tools/cumask_gemm_slices.py run --out gpurun_out/cumask4.json
rocprofv3 --pmc SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE ... -- python3 tools/cumask_gemm_slices.py pmc
python tools/cumask_gemm_slices.py summarize gpurun_out/cumask4_pmc --out profiles/...
"""
from __future__ import annotations

import argparse
import csv
import json
import sys
import time
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

N = 4096
SLICES = 4
SLICE_GB = 72


def _slices() -> list[list[int]]:
    from nos_amd.gpu.topology import MI355X_MEMORY_GB, MI355X_XCDS, layout_slots, logical_cu

    slots, bad = layout_slots([(f"s{i}", SLICE_GB) for i in range(SLICES)], {}, "proportional", MI355X_MEMORY_GB)
    assert not bad
    return [sorted(logical_cu(x, j) for x in range(MI355X_XCDS) for j in slots[f"s{i}"]) for i in range(SLICES)]


def _setup():
    import torch

    from nos_amd import ops
    from nos_amd.ops.streams import CUMaskedStream, device_info

    num_cus = device_info(0)["num_cus"]
    streams = [CUMaskedStream(c, num_cus) for c in _slices()]
    g = torch.Generator(device="cuda").manual_seed(0)
    bufs = []
    for _ in streams:
        x = torch.randn(N, N, device="cuda", dtype=torch.bfloat16, generator=g)
        w = torch.randn(N, N, device="cuda", dtype=torch.bfloat16, generator=g) * N ** -0.5
        bufs.append((x, w, torch.empty(N, N, device="cuda", dtype=torch.bfloat16)))
    torch.cuda.synchronize()
    return ops, streams, bufs, num_cus


def _gemms(ops, stream, buf, k: int) -> None:
    import torch

    x, w, o = buf
    with torch.cuda.stream(stream.torch):
        for _ in range(k):
            ops.linear(x, w, out=o)


def run(out: str, iters: int) -> None:
    import torch

    ops, streams, bufs, num_cus = _setup()
    flop = 2.0 * N ** 3
    for s, b in zip(streams, bufs):  # warm-up, every slice
        _gemms(ops, s, b, 2)
    torch.cuda.synchronize()
    res = {"what": f"{SLICES} CU-mask slices x {SLICE_GB} GB (proportional: {len(streams[0].cus)} CUs each), "
                   f"bf16 GEMM probe {N}^3 (csrc/hip/gemm.hip)", "slice_cus": [len(s.cus) for s in streams]}
    alone = []
    for s, b in zip(streams, bufs):
        t0 = time.perf_counter()
        _gemms(ops, s, b, iters)
        torch.cuda.synchronize()
        alone.append(iters * flop / (time.perf_counter() - t0) / 1e12)
    res["alone_tflops"] = [round(v, 1) for v in alone]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in streams]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for (a, e), s, b in zip(ev, streams, bufs):
        a.record(s.torch)
        _gemms(ops, s, b, iters)
        e.record(s.torch)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    res["corun_tflops"] = [round(iters * flop / (a.elapsed_time(e) / 1e3) / 1e12, 1) for a, e in ev]
    res["corun_aggregate_tflops"] = round(SLICES * iters * flop / wall / 1e12, 1)
    x, w, o = bufs[0]
    t0 = time.perf_counter()
    for _ in range(iters):
        ops.linear(x, w, out=o)
    torch.cuda.synchronize()
    res["whole_gpu_tflops"] = round(iters * flop / (time.perf_counter() - t0) / 1e12, 1)
    print(json.dumps(res), flush=True)
    Path(out).parent.mkdir(parents=True, exist_ok=True)
    Path(out).write_text(json.dumps(res, indent=1))


def pmc(k: int) -> None:
    """A few GEMMs per slice, serially per stream, then on the unmasked default stream."""
    import torch

    ops, streams, bufs, _ = _setup()
    for s, b in zip(streams, bufs):
        _gemms(ops, s, b, k)
        torch.cuda.synchronize()
    x, w, o = bufs[0]
    for _ in range(k):
        ops.linear(x, w, out=o)
    torch.cuda.synchronize()
    print("queues in launch order: slices 0..3, then the unmasked stream")


def summarize(root: str, out: str | None) -> None:
    per: dict = defaultdict(lambda: defaultdict(float))
    order: list = []
    for f in sorted(Path(root).rglob("*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "gemm_bf16" not in row["Kernel_Name"]:
                    continue
                q = int(row["Queue_Id"])
                if q not in order:
                    order.append(q)
                per[q][row["Counter_Name"]] += float(row["Counter_Value"])
                per[q]["_dispatches_x_counters"] += 1
    names = [f"slice{i}" for i in range(SLICES)] + ["unmasked"]
    res = {}
    whole = None
    for name, q in zip(names, order):
        c = dict(per[q])
        d = {"queue": q, "counters": {k: v for k, v in c.items() if not k.startswith("_")}}
        if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_BUSY_CU_CYCLES") is not None:
            d["busy_cu_cycles_per_gui_cycle"] = c["SQ_BUSY_CU_CYCLES"] / c["GRBM_GUI_ACTIVE"]
        if c.get("SQ_INSTS_MFMA"):
            d["mfma_per_gui_cycle"] = c["SQ_INSTS_MFMA"] / c["GRBM_GUI_ACTIVE"]
        res[name] = d
        if name == "unmasked":
            whole = d
    if whole and whole.get("busy_cu_cycles_per_gui_cycle"):
        for name, d in res.items():
            if "busy_cu_cycles_per_gui_cycle" in d:
                d["busy_cus_relative_to_unmasked"] = round(
                    d["busy_cu_cycles_per_gui_cycle"] / whole["busy_cu_cycles_per_gui_cycle"], 3)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "counters"} for k, v in res.items()}, indent=1))
    if out:
        Path(out).write_text(json.dumps(res, indent=1))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("phase", choices=["run", "pmc", "summarize"])
    ap.add_argument("root", nargs="?")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.phase == "run":
        run(a.out or "gpurun_out/cumask4.json", a.iters)
    elif a.phase == "pmc":
        pmc(3)
    else:
        summarize(a.root, a.out)


if __name__ == "__main__":
    main()
