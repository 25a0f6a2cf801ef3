"""Per-shape timing of the LayerNorm hand-off kernels against the split-pass
path (YOLOS-small encoder shapes, batch 1 and 8; CUDA events, median of
``--iters``): the residual GEMMs (proj, fc2) with and without the row
statistics epilogue, and the LN-GEMMs (QKV with the attention's K / V planes,
fc1 with GELU into fc2's planes) as split pass + GEMM vs LN in the A load.
Prints one JSON line.  usage (GPU box): python tools/ln_handoff_bench.py"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batches", default="1,8")
    a = ap.parse_args()
    import torch

    from nos_amd import ops

    ops.set_f32_math("h3")
    ops.set_attention_f32_variant("h3n")
    torch.manual_seed(0)
    S, D, H = 3401, 384, 6

    def timed1(fn) -> float:
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        t = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev)
        return t[len(t) // 2]

    def timed(fn, setup=None) -> float:
        """min over 5 rounds of the median of ``iters`` (rounds interleave with
        the other configurations' through the caller's order)"""
        best = []
        for _ in range(5):
            if setup:
                setup()
            best.append(timed1(fn))
        return round(min(best), 1)

    res = {}
    for B in (int(b) for b in a.batches.split(",")):
        M = B * S
        row = {}
        for name, N, K in (("proj", D, D), ("fc2", D, 4 * D)):
            x = torch.randn(M, K, device="cuda")
            w = torch.randn(N, K, device="cuda") / K ** 0.5
            b = torch.randn(N, device="cuda")
            r = torch.randn(M, N, device="cuda")
            p, ri = ops._split_rows_h3(x, ln=False)
            A = ops.H3Planes(p, ri, 0.0, (M, K))
            row[name] = {
                "plain_reg_epi_us": timed(lambda: ops.linear_planes(A, w, b, residual=r),
                                          lambda: ops.set_gemm_f32h3_lds_epilogue(False)),
                "plain_lds_epi_us": timed(lambda: ops.linear_planes(A, w, b, residual=r),
                                          lambda: ops.set_gemm_f32h3_lds_epilogue(True)),
                "stats_us": timed(lambda: ops.linear_planes(A, w, b, residual=r, row_stats=True))}
        x = torch.randn(B, S, D, device="cuda") * 2 + 1
        wq = torch.randn(3 * D, D, device="cuda") / D ** 0.5
        cq = torch.randn(3 * D, device="cuda") * 0.1
        w1 = torch.randn(4 * D, D, device="cuda") / D ** 0.5
        c1 = torch.randn(4 * D, device="cuda") * 0.1
        x2 = x.view(M, D)
        st = ops._row_stats(x2)
        for on in (False, True):
            ops.set_ln_handoff(on)
            tag = "lna" if on else "split"
            pre = st if on else None
            row.setdefault("qkv", {})[tag + "_us"] = timed(lambda: ops.linear_ln_qkv_h3(x, wq, wq.sum(1), cq, H,
                                                                                          pre=pre))
            row.setdefault("fc1", {})[tag + "_us"] = timed(
                lambda: ops.linear_ln_to_planes(x, w1, w1.sum(1), c1, act="gelu", pre=pre))
        ops.set_ln_handoff(False)
        row["split_pass_us"] = timed(lambda: ops._split_rows_h3(x2, ln=True, eps=1e-12))
        row["row_stats_us"] = timed(lambda: ops._row_stats(x2))
        res[f"batch{B}"] = row
    print(json.dumps(res))


if __name__ == "__main__":
    main()
