"""Sweep the pod-server program fuzzer without stopping at the first failure.

The GPU property test (tests/test_program_fuzz_gpu.py) stops and shrinks at
the first failing program; this tool draws the same derandomized examples,
runs each one on one GPU pod server beside a YOLOS co-tenant and records EVERY
failure (program, error) as a JSON line, so one GPU call finds all of them.

    python tools/fuzz_sweep.py --examples 300 --out gpurun_out/fuzz.jsonl
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import tempfile
import traceback

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--examples", type=int, default=300)
    ap.add_argument("--out", default="gpurun_out/fuzz.jsonl")
    ap.add_argument("--device", default="cuda")
    args = ap.parse_args()

    import torch
    from hypothesis import HealthCheck, given, settings

    from nos_amd import ops
    from nos_amd.models.yolos_program import demo_tenant
    from nos_amd.podserver import program as PG
    from nos_amd.podserver.client import PodClient, PodServerError
    from nos_amd.podserver.server import PodServer
    from program_fuzz import programs, tolerance

    if args.device == "cuda":
        ops.set_f32_math("h3")
    tmp = tempfile.mkdtemp()
    srv = PodServer(os.path.join(tmp, "s.sock"), device=args.device, lanes=4, memory_gb=200).start()
    y = PodClient(srv.path, connect_timeout_s=60)
    y.register("yolos", *demo_tenant("fp32", 0, small=True), memory_limit_gb=4)
    first = y.infer(outputs=True)[0]
    stats: collections.Counter = collections.Counter()
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    out = open(args.out, "w")

    def record(kind, prog, err):
        stats["fail"] += 1
        out.write(json.dumps({"kind": kind, "error": err[-2000:], "program": prog}) + "\n")
        out.flush()

    @settings(max_examples=args.examples, deadline=None, derandomize=True, database=None,
              suppress_health_check=list(HealthCheck))
    @given(case=programs(gpu=True))
    def sweep(case):
        prog, w, data, fam = case
        stats["drawn"] += 1
        print(stats["drawn"], fam, prog["name"], file=sys.stderr, flush=True)
        try:
            p = PG.parse(prog, w, gpu=args.device == "cuda")
        except PG.ProgramError:
            p = None
        c = PodClient(srv.path, connect_timeout_s=30)
        try:
            if p is None:
                try:
                    c.register("fz", prog, w, memory_limit_gb=4)
                    record("accepted-by-server", prog, "server accepted a program the validator refused")
                except PodServerError as e:
                    if "ProgramError" not in str(e):
                        record("refusal", prog, str(e))
                stats["refused"] += 1
                return
            try:
                c.register("fz", prog, w, memory_limit_gb=4)
                outs, _ = c.infer(data, outputs=True)
            except Exception as e:   # noqa: BLE001 -- every failure is recorded
                record("run", prog, f"{type(e).__name__}: {e}")
                return
        finally:
            c.close()
        x = p.input_tensor("cpu", data)
        with torch.no_grad():
            ref = p.reference(x)
        rel, ab = tolerance(p.values[p.outputs[0]].dtype)
        for g, r in zip(outs, ref):
            g, r = torch.from_numpy(g).float(), r.float()
            if g.shape != r.shape:
                record("shape", prog, f"{tuple(g.shape)} vs {tuple(r.shape)}")
                return
            err = float((g - r).nan_to_num().abs().max()) if r.numel() else 0.0
            lim = rel * float(r.nan_to_num().abs().max()) + ab
            if err > lim or not torch.equal(torch.isnan(g), torch.isnan(r)):
                record("numerics", prog, f"err {err:.3e} > {lim:.3e}")
                return
        stats["ran"] += 1
        stats[fam] += 1
        yy = y.infer(outputs=True)[0]
        if not all(np.array_equal(a, b) for a, b in zip(yy, first)):
            record("co-tenant", prog, "the YOLOS co-tenant's output changed")

    try:
        sweep()
    except Exception:   # noqa: BLE001
        traceback.print_exc()
    finally:
        out.close()
        y.close()
        srv.stop()
    print(json.dumps(dict(stats)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
