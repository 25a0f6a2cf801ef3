"""First-contact GPU checks: CU-mask -> XCD mapping, kernel numerics, timings.

Run on an MI355X box:  python tools/gpu_explore.py --out gpurun_out/explore.json
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from nos_amd import ops  # noqa: E402
from nos_amd.ops import probes, streams  # noqa: E402


def log(*a):
    print(*a, flush=True)


def check_numerics(res: dict) -> None:
    torch.manual_seed(0)
    dev = "cuda"
    out = {}
    for (M, N, K, act) in [(3401, 1152, 384, None), (3401, 1536, 384, "gelu"), (3401, 384, 1536, None),
                           (100, 4, 384, "relu"), (257, 200, 128, None)]:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
        b = torch.randn(N, device=dev, dtype=torch.bfloat16)
        r = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        y = ops.linear(x, w, b, act=act, residual=r)
        ref = ops.linear_ref(x.cpu(), w.cpu(), b.cpu(), act=act, residual=r.cpu()).float()
        err = (y.float().cpu() - ref).abs().max().item()
        out[f"gemm_{M}x{N}x{K}_{act}"] = err
    for (M, N, K, act) in [(3401, 1152, 384, None), (3401, 1536, 384, "gelu"), (77, 100, 128, None)]:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16) * 2 + 0.5
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
        b = torch.randn(N, device=dev, dtype=torch.bfloat16)
        g = torch.randn(K, device=dev, dtype=torch.bfloat16)
        be = torch.randn(K, device=dev, dtype=torch.bfloat16)
        wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
        y = ops.linear_ln(x, wg, c1, c2, act=act)
        ln = torch.nn.functional.layer_norm(x.float().cpu(), (K,), g.float().cpu(), be.float().cpu(), 1e-12)
        ref = ops.linear_ref(ln.bfloat16(), w.cpu(), b.cpu(), act=act).float()
        out[f"gemm_ln_{M}x{N}x{K}_{act}"] = (y.float().cpu() - ref).abs().max().item()
    for (B, S, H) in [(1, 3401, 6), (2, 200, 2), (1, 64, 1), (1, 1000, 3), (1, 65, 2)]:
        qkv = torch.randn(B, S, 3 * H * 64, device=dev, dtype=torch.bfloat16)
        o = ops.attention_qkv(qkv, H)
        ref = ops.attention_qkv(qkv.cpu().float(), H)
        out[f"attn_B{B}_S{S}_H{H}"] = (o.float().cpu() - ref).abs().max().item()
    x = torch.randn(3401, 384, device=dev, dtype=torch.bfloat16)
    r = torch.randn(3401, 384, device=dev, dtype=torch.bfloat16)
    g = torch.randn(384, device=dev, dtype=torch.bfloat16)
    bb = torch.randn(384, device=dev, dtype=torch.bfloat16)
    y, s = ops.layernorm(x, g, bb, 1e-12, residual=r)
    yr, sr = ops.layernorm_ref(x.cpu(), g.cpu(), bb.cpu(), 1e-12, residual=r.cpu())
    out["ln"] = (y.float().cpu() - yr.float()).abs().max().item()
    out["ln_sum"] = (s.float().cpu() - sr.float()).abs().max().item()
    res["numerics_maxabs"] = out
    log("numerics", json.dumps(out))


def check_masks(res: dict, num_cus: int) -> None:
    out = {}
    base = probes.placement(None, nwg=4096)
    out["default"] = probes.placement_summary(base)
    trials = {
        "bits0_31": list(range(32)),
        "bits_mod8_eq0": list(range(0, num_cus, 8)),
        "bits0_7": list(range(8)),
        "bits0_63": list(range(64)),
        "bit0": [0],
        "bit1": [1],
        "bit8": [8],
        "bit32": [32],
    }
    for name, cus in trials.items():
        st = streams.CUMaskedStream(cus, num_cus)
        recs = probes.placement(st.handle, nwg=1024)
        out[name] = probes.placement_summary(recs)
        out[name]["mask_readback"] = st.get_mask()[:8]
        st.close()
    res["cumask"] = out
    log("cumask", json.dumps(out))


def time_fn(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def check_model(res: dict) -> None:
    from nos_amd.models.yolos import YolosConfig, YolosDetector, make_demo_input, flops_per_image, demo_input_hw
    cfg = YolosConfig.small()
    m = YolosDetector(cfg).to("cuda", torch.bfloat16).eval()
    x = make_demo_input(cfg, device="cuda")
    with torch.no_grad():
        m.backend = "native"
        ln, bn = m(x)
        m.backend = "torch"
        lt, bt = m(x)
        res["model_parity"] = {"logits_maxabs": (ln.float() - lt.float()).abs().max().item(),
                               "boxes_maxabs": (bn - bt).abs().max().item(),
                               "logits_scale": lt.float().abs().max().item()}
        log("parity", res["model_parity"])
        fl = flops_per_image(cfg, demo_input_hw())
        for be in ("torch", "native"):
            m.backend = be
            t = time_fn(lambda: m(x))
            res[f"yolos_{be}_eager_ms"] = t * 1e3
            log(be, "eager ms", t * 1e3, "TFLOPs", fl / t / 1e12)
        # graphed single tenant
        m.backend = "native"
        from nos_amd.models.yolos import GraphedTenant
        s = torch.cuda.Stream()
        ten = GraphedTenant(m, s, x)
        ten.capture()
        t = time_fn(ten.launch)
        res["yolos_native_graph_ms"] = t * 1e3
        log("native graph ms", t * 1e3, "TFLOPs", fl / t / 1e12)


def check_probes(res: dict, num_cus: int) -> None:
    s = torch.cuda.current_stream().cuda_stream
    res["probe_hbm_gbps_full"] = probes.hbm_gbps(s, 1 << 30, 5, 4096)
    res["probe_mfma_peak_tflops_full"] = probes.mfma_peak_tflops(s, num_cus * 2, 20000)
    res["probe_gemm_tflops_full_4096"] = probes.gemm_tflops(s, 4096, 5)
    res["probe_gemm_tflops_full_8192"] = probes.gemm_tflops(s, 8192, 3)
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    t = time_fn(lambda: a @ b.t(), iters=5)
    res["torch_gemm_tflops_8192"] = 2 * 8192 ** 3 / t / 1e12
    log("probes", {k: v for k, v in res.items() if k.startswith(("probe", "torch_gemm"))})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/explore.json")
    ap.add_argument("--skip", default="")
    a = ap.parse_args()
    res: dict = {}
    info = streams.device_info(0)
    res["device"] = info
    log("device", info, torch.cuda.get_device_name(0))
    steps = [("numerics", lambda: check_numerics(res)),
             ("masks", lambda: check_masks(res, info["num_cus"])),
             ("probes", lambda: check_probes(res, info["num_cus"])),
             ("model", lambda: check_model(res))]
    for name, fn in steps:
        if name in a.skip.split(","):
            continue
        try:
            fn()
        except Exception as e:  # keep going: record the failure
            res[f"{name}_error"] = repr(e)
            log("ERROR", name, repr(e))
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(res, indent=1))
    log(json.dumps(res))


if __name__ == "__main__":
    main()
