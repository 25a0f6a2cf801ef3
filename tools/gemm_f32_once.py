"""A few fp32 GEMM launches (exact-f32 MFMA and bf16x6 split, small and
throughput tiles) at the batch-8 YOLOS qkv shape, for rocprofv3 PMC passes
(tools/gpu/pmc_gemm_f32.sh); kernel names tell the configs apart."""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    import torch

    from nos_amd import ops

    torch.manual_seed(0)
    M, N, K = 8 * 3401, 1152, 384
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * 0.05
    o = torch.empty(M, N, device="cuda")
    for math_ in ("exact", "x6"):
        ops.set_f32_math(math_)
        for pol in ("small", "throughput"):
            ops.set_gemm_f32_policy(pol)
            for _ in range(3):
                ops.linear(x, w, out=o)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
