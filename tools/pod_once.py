"""One YOLOS-small pod in this process, for profiling (no subprocesses, so it
can run under rocprofv3 directly).

rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python tools/pod_once.py --dtype fp32 --iters 30
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--seconds", type=float, default=0.0, help="keep inferring for this long instead of --iters "
                    "(a co-running background pod)")
    ap.add_argument("--memory-fraction", type=float, default=None, help="as a fractional pod (kernel_config)")
    ap.add_argument("--cu-mask", default="", help="a CU-mask slice (hex, ROC_GLOBAL_CU_MASK) with its CU budget: "
                    "the cumask process pod of the latency table, e.g. 0xffffffff for 32 CUs")
    a = ap.parse_args()
    import os

    if a.cu_mask:  # before HIP initialises: the runtime reads it at queue creation
        os.environ["ROC_GLOBAL_CU_MASK"] = a.cu_mask
    import torch

    from nos_amd.models.pod import _build
    from nos_amd.models.yolos import GraphedTenant, demo_input_hw

    torch.backends.cuda.matmul.allow_tf32 = False
    import os

    from nos_amd import ops
    from nos_amd.models.pod import kernel_config

    from nos_amd.models.pod import slice_cu_budget

    budget = slice_cu_budget(os.environ)
    cfg = kernel_config(a.memory_fraction, os.environ, budget)  # the pod's kernel choices (NOS_AMD_* overrides apply)
    if budget:
        ops.set_cu_budget(budget)
    ops.set_gemm_policy(cfg["gemm_bf16"])
    ops.set_gemm_f32_policy(cfg["gemm_f32"])
    ops.set_attention_f32_variant(cfg["attention_f32"])
    ops.set_f32_math(cfg["f32_math"])
    ops.set_ln_handoff(cfg["ln_handoff"] == "on")
    ops.set_gemm_f32h3_layout(cfg["h3_layout"])
    ops.set_gemm_f32h3_hot_ring(int(cfg["h3_hot_ring"]))
    ops.set_gemm_f32h3_hot_bn(int(cfg["h3_hot_bn"]))
    ops.set_gemm_f32h3_lna_wide(cfg["h3_lna_wide"] == "on")
    print("kernel config", cfg, flush=True)
    m, x = _build(a.dtype, 0, demo_input_hw())
    s = torch.cuda.Stream()
    t = GraphedTenant(m, s, x)
    with torch.no_grad():
        if not a.no_graphs:
            t.capture()
        for _ in range(3):
            t.launch()
        s.synchronize()
        t0 = time.perf_counter()
        n = 0
        while n < a.iters if a.seconds <= 0 else time.perf_counter() - t0 < a.seconds:
            t.launch()
            n += 1
            if a.seconds > 0 and n % 32 == 0:
                s.synchronize()
        s.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"{a.dtype}: {dt * 1e3:.3f} ms/inference ({1 / dt:.1f} inf/s), cu budget {budget}", flush=True)


if __name__ == "__main__":
    main()
