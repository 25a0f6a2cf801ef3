"""One attention call per dtype at batch B (for rocprofv3 --pmc passes).

python tools/attn_once.py --B 8
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--dtypes", default="fp32,bf16")
    ap.add_argument("--variant", default="auto", help="fp32 attention tiling (ops.set_attention_f32_variant)")
    a = ap.parse_args()
    import torch

    from nos_amd import ops

    ops.set_attention_f32_variant(a.variant)

    for dt in a.dtypes.split(","):
        t = {"fp32": torch.float32, "bf16": torch.bfloat16}[dt]
        qkv = torch.randn(a.B, 3401, 3 * 384, device="cuda", dtype=t)
        out = torch.empty(a.B, 3401, 384, device="cuda", dtype=t)
        for _ in range(2):
            ops.attention_qkv(qkv, 6, out=out)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
