"""bf16 attention: the ping-pong schedule against the lockstep one (bit for
bit: same per-tile operations in the same order per wave group) and against
an fp32 CPU reference, over odd sizes and a peaky rescale case.

python tools/attn_pp_check.py
"""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    import torch

    from nos_amd import ops

    bad = 0
    torch.manual_seed(0)
    cases = [(1, 3401, 6), (2, 200, 2), (1, 64, 1), (1, 1000, 3), (1, 65, 2), (1, 1, 1), (3, 129, 4), (1, 777, 2)]
    for B, S, H in cases:
        qkv = torch.randn(B, S, 3 * H * 64, device="cuda", dtype=torch.bfloat16)
        if S == 777:  # peaky, growing maxima: the deferred-rescale branch
            qkv[..., : H * 64] *= 6.0
            ramp = torch.linspace(0.2, 3.0, S, device="cuda").view(1, S, 1)
            qkv[..., H * 64: 2 * H * 64] = (qkv[..., H * 64: 2 * H * 64].float() * ramp).bfloat16()
        outs = {}
        for v in ("lockstep", "pingpong"):
            ops.set_attention_bf16_variant(v)
            outs[v] = ops.attention_qkv(qkv, H)
        ops.set_attention_bf16_variant("lockstep")
        torch.cuda.synchronize()
        ref = ops.attention_qkv(qkv.cpu().float(), H)
        err = (outs["pingpong"].float().cpu() - ref).abs().max().item()
        same = torch.equal(outs["pingpong"], outs["lockstep"])
        ok = same and err < 2e-2
        bad += not ok
        print(f"B={B} S={S} H={H}: bit-identical={same} max_err={err:.3e} {'ok' if ok else 'FAIL'}", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
