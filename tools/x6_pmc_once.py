"""x6 kernels at batch-8 YOLOS shapes for rocprofv3 PMC passes
(tools/gpu/pmc_x6.sh): the x6 GEMM (128x128 4x1 waves) pipelined and plain
at the qkv and fc2 shapes, and the x6 attention without key splits; three
launches each, told apart by kernel name (the PIPE template argument) and
dispatch order."""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    import torch

    from nos_amd import ops
    from nos_amd.ops import _lib

    torch.manual_seed(0)
    S, hid = 3401, 384
    M = 8 * S
    ops.set_f32_math("x6")
    _lib.check(_lib.lib().nos_gemm_f32x6_set_tile(5), "set_tile")
    for N, K in ((1152, 384), (384, 1536)):
        x = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda") * 0.05
        o = torch.empty(M, N, device="cuda")
        for pipe in (True, False):
            ops.set_gemm_f32x6_pipeline(pipe)
            for _ in range(3):
                ops.linear(x, w, out=o)
    ops.set_gemm_f32x6_pipeline(True)
    ops.set_attention_f32_variant("x6n")
    qkv = torch.randn(8, S, 3 * hid, device="cuda")
    for _ in range(3):
        ops.attention_qkv(qkv, 6)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
