"""Per-kernel timing at the YOLOS-small shapes (one process, interleaved rounds).

python tools/kernel_bench.py [--only attn,gemm] [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from nos_amd import ops  # noqa: E402


def timeit(fn, iters):
    """GPU time per call: `iters` calls captured in one HIP graph and replayed,
    so host launch overhead (~10 us per eager ctypes/torch call) is excluded
    -- this is how the tenants run (graph replay per pod)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    g.replay()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="attn,gemm,torch")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--out", default="")
    ap.add_argument("--rounds", type=int, default=1, help="interleaved rounds per impl (median reported)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"], help="GEMM dtype")
    ap.add_argument("--square", type=int, default=0, help="time one n x n x n GEMM instead of the YOLOS shapes")
    ap.add_argument("--persist", default="0", help="comma list of bf16 GEMM persistent grids (workgroups/CU, 0 = off)")
    ap.add_argument("--policies", default="latency", help="comma list of GEMM tile policies to A/B "
                    "(throughput, latency)")
    ap.add_argument("--x6-tile", type=int, default=-1, help="x6 GEMM tile override (3: 128x64 4x1 waves)")
    ap.add_argument("--stage", type=int, default=0, help="x6 GEMM K-stage config (1: BK32 3-deep, 2: BK64)")
    ap.add_argument("--f32-math", default="exact", choices=["exact", "x6", "h3"], help="fp32 GEMM math (ops.set_f32_math)")
    ap.add_argument("--attn-f32", default="x6n,x6", help="fp32 attention variants to time (--dtype fp32)")
    ap.add_argument("--pipeline", type=int, default=1, help="x6 GEMM software-pipelined K loop (1) or plain (0)")
    a = ap.parse_args()
    ops.set_f32_math(a.f32_math)
    ops.set_gemm_f32x6_pipeline(bool(a.pipeline))
    if a.x6_tile >= 0:
        ops._lib.check(ops._lib.lib().nos_gemm_f32x6_set_tile(a.x6_tile), "nos_gemm_f32x6_set_tile")
    if a.stage:
        ops._lib.check(ops._lib.lib().nos_gemm_f32x6_set_stage(a.stage), "nos_gemm_f32x6_set_stage")
    torch.manual_seed(0)
    S, H, hid, mlp = 3401, 6, 384, 1536
    B = a.batch
    res = {}
    if "attn" in a.only:
        adt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
        qkv = torch.randn(B, S, 3 * hid, device="cuda", dtype=adt)
        out = torch.empty(B, S, hid, device="cuda", dtype=adt)
        fl = B * 4 * S * S * hid
        variants = a.attn_f32.split(",") if a.dtype == "fp32" else [""]
        for v in variants:
            if v:
                ops.set_attention_f32_variant(v)
            us = timeit(lambda: ops.attention_qkv(qkv, H, out=out), a.iters)
            sfx = f"_{v}" if v else ""
            res[f"attn{sfx}_us"] = us
            res[f"attn{sfx}_tflops"] = fl / us / 1e6
        ops.set_attention_f32_variant("auto")
    if "torch" in a.only:
        qkv = torch.randn(B, S, 3, H, 64, device="cuda", dtype=torch.bfloat16)
        q, k, v = (t.transpose(1, 2).contiguous() for t in qkv.unbind(2))
        us = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v), a.iters)
        res["sdpa_us"] = us
        res["sdpa_tflops"] = B * 4 * S * S * hid / us / 1e6
    if "gemm" in a.only:
        M = B * S
        gdt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
        torch.backends.cuda.matmul.allow_tf32 = False
        shapes = {
            "qkv_ln": (3 * hid, hid, None, True, False),
            "fc1_ln_gelu": (mlp, hid, "gelu", True, False),
            "fc1_ln_noact": (mlp, hid, None, True, False),
            "proj_resid": (hid, hid, None, False, True),
            "fc2_resid": (hid, mlp, None, False, True),
            "qkv_plain": (3 * hid, hid, None, False, False),
        }
        if a.square:
            shapes = {f"square{a.square}": (a.square, a.square, None, False, False)}
        for name, (N, K, act, ln, resid) in shapes.items():
            M = a.square or B * S
            xa = torch.randn(M, K, device="cuda", dtype=gdt)
            w = torch.randn(N, K, device="cuda", dtype=gdt) * 0.05
            b = torch.randn(N, device="cuda", dtype=gdt)
            r = torch.randn(M, N, device="cuda", dtype=gdt)
            outg = torch.empty(M, N, device="cuda", dtype=gdt)
            if ln:
                g = torch.randn(K, device="cuda", dtype=gdt)
                be = torch.randn(K, device="cuda", dtype=gdt)
                wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
                fn = lambda: ops.linear_ln(xa, wg, c1, c2, act=act, out=outg)  # noqa: E731
            else:
                fn = lambda: ops.linear(xa, w, b, act=act, residual=r if resid else None, out=outg)  # noqa: E731
            impls = [(int(pe), po) for pe in a.persist.split(",") for po in a.policies.split(",")]
            times = {im: [] for im in impls}
            for _ in range(a.rounds):
                for pe, po in impls:
                    if a.dtype == "fp32":
                        ops.set_gemm_f32_policy(po)
                    else:
                        ops.set_gemm_policy(po)
                        ops.set_gemm_persistent(pe)
                    times[(pe, po)].append(timeit(fn, a.iters))
            ops.set_gemm_policy("throughput")
            ops.set_gemm_persistent(0)
            ops.set_gemm_f32_policy("latency")
            for im in impls:
                t = sorted(times[im])[len(times[im]) // 2]
                sfx = "" if im == impls[0] else f"_p{im[0]}_{im[1]}"
                res[f"{name}{sfx}_us"] = t
                res[f"{name}{sfx}_tflops"] = 2 * M * N * K / t / 1e6
            tus = timeit(lambda: torch.nn.functional.linear(xa, w, b), a.iters)
            res[f"{name}_torch_us"] = tus
    print(json.dumps(res), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
