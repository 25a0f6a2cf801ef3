"""h3 kernels at batch-8 YOLOS shapes for rocprofv3 PMC passes
(tools/gpu/pmc_h3.sh): the h3 GEMM (2x2 and 4x1 waves) at the qkv and fc2
shapes, the LN row-split pre-pass and the h3 attention without key splits;
three launches each, told apart by kernel name and dispatch order."""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    import torch

    from nos_amd import ops

    torch.manual_seed(0)
    S, hid, H = 3401, 384, 6
    M = 8 * S
    ops.set_f32_math("h3")
    for N, K in ((1152, 384), (384, 1536)):
        x = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda") * 0.05
        o = torch.empty(M, N, device="cuda")
        for lay in ("2x2", "4x1"):
            ops.set_gemm_f32h3_layout(lay)
            for _ in range(3):
                ops.linear(x, w, out=o)
    ops.set_gemm_f32h3_layout("2x2")
    ops.set_attention_f32_variant("h3n")
    x = torch.randn(8, S, hid, device="cuda")
    w = torch.randn(3 * hid, hid, device="cuda") * 0.05
    wg, c1, c2 = ops.fold_layernorm(w, torch.zeros(3 * hid, device="cuda"), torch.ones(hid, device="cuda"),
                                    torch.zeros(hid, device="cuda"))
    for _ in range(3):
        qkv, ws, sc = ops.linear_ln_qkv_h3(x, wg, c1, c2, H)
        ops.attention_presplit_h3(qkv, ws, sc, H)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
