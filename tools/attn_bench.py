"""Attention kernel throughput (HIP-graph timed), fp32 and bf16, batch sweep.

python tools/attn_bench.py --dtype fp32 --batches 1,8
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--batches", default="1,8")
    ap.add_argument("--S", type=int, default=3401)
    ap.add_argument("--H", type=int, default=6)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--variant", default="auto")
    a = ap.parse_args()
    import torch

    from nos_amd import ops

    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[a.dtype]
    ops.set_attention_f32_variant(a.variant)
    for B in map(int, a.batches.split(",")):
        qkv = torch.randn(B, a.S, 3 * a.H * 64, device="cuda", dtype=dt)
        out = torch.empty(B, a.S, a.H * 64, device="cuda", dtype=dt)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            ops.attention_qkv(qkv, a.H, out=out)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(10):
                    ops.attention_qkv(qkv, a.H, out=out)
            g.replay()
            s.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.iters // 10):
                g.replay()
            e1.record(s)
            s.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (a.iters // 10 * 10)
        fl = 4.0 * B * a.H * a.S * a.S * 64
        print(json.dumps({"dtype": a.dtype, "variant": a.variant, "B": B, "S": a.S, "H": a.H, "us": round(us, 2),
                          "tflops": round(fl / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
