"""A few GEMM launches per tile config for rocprofv3 PMC passes (tools/gpu/pmc_gemm.sh).

Runs the 4096^3 GEMM with the base (128x128) and big (256x256) tile configs,
and the batch-8 YOLOS fc2 (+residual) and fc1 (+LN +GELU) shapes with the
default tile choice (256x192 and 256x256) and the base tile, plus torch
(hipBLASLt) on each; kernel names tell the configs apart (Cfg<BM,BN,...>, Cijk_*).
"""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    import torch

    from nos_amd import ops

    torch.manual_seed(0)
    dev = "cuda"
    n = 4096
    x = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, n, device=dev, dtype=torch.bfloat16) * 0.02
    o = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    for pol in ("throughput", "big"):
        ops.set_gemm_policy(pol)
        for _ in range(5):
            ops.linear(x, w, out=o)
    for _ in range(5):
        torch.nn.functional.linear(x, w)
    ops.set_gemm_policy("throughput")
    M, hid, mlp = 8 * 3401, 384, 1536
    h = torch.randn(M, mlp, device=dev, dtype=torch.bfloat16)
    w2 = torch.randn(hid, mlp, device=dev, dtype=torch.bfloat16) * 0.02
    b2 = torch.randn(hid, device=dev, dtype=torch.bfloat16)
    r = torch.randn(M, hid, device=dev, dtype=torch.bfloat16)
    o2 = torch.empty(M, hid, device=dev, dtype=torch.bfloat16)
    for pol in ("throughput", "narrow"):
        ops.set_gemm_policy(pol)
        for _ in range(5):
            ops.linear(h, w2, b2, residual=r, out=o2)
    for _ in range(5):
        torch.nn.functional.linear(h, w2, b2)
    ops.set_gemm_policy("throughput")
    # fc1 + LN + GELU (K = 384 -> N = 1536)
    x1 = torch.randn(M, hid, device=dev, dtype=torch.bfloat16)
    w1 = torch.randn(mlp, hid, device=dev, dtype=torch.bfloat16) * 0.05
    b1 = torch.randn(mlp, device=dev, dtype=torch.bfloat16)
    g = torch.randn(hid, device=dev, dtype=torch.bfloat16)
    be = torch.randn(hid, device=dev, dtype=torch.bfloat16)
    wg, c1, c2 = ops.fold_layernorm(w1, b1, g, be)
    o1 = torch.empty(M, mlp, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        ops.linear_ln(x1, wg, c1, c2, act="gelu", out=o1)
        torch.nn.functional.linear(x1, w1, b1)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
