"""GPU-sharing comparison client (the reference's
``demos/gpu-sharing-comparison/client/main.py``): one YOLOS-small inference
loop per pod, exposing the Prometheus summary ``inference_time_seconds`` on
:8000 so the per-pod latency of the three sharing modes can be compared with
the same query as the reference demo.

MI355X-native: the hustvl/yolos-small architecture (random init -- no
checkpoint download; pass --hf-checkpoint to load real weights with
safetensors) in fp32 like the reference (``--dtype bf16`` for the bf16
kernels), the 800x1066 demo input size, the gfx950 kernels replayed as a HIP
graph, and the slice's memory cap from the device plugin applied.
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--iterations", type=int, default=0, help="0 = run forever")
    ap.add_argument("--hf-checkpoint", default="", help="safetensors file of hustvl/yolos-small")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    a = ap.parse_args(argv)
    import torch
    from prometheus_client import Summary, start_http_server

    from nos_amd.models.yolos import GraphedTenant, YolosConfig, YolosDetector, demo_input_hw, make_demo_input
    from nos_amd.utils.memlimit import apply_memory_limit

    inference_time = Summary("inference_time_seconds", "Time required for running a single inference")
    frac = apply_memory_limit(0)
    print(f"memory cap: {frac if frac is not None else 'none'}", flush=True)
    cfg = YolosConfig.small()
    model = YolosDetector(cfg)
    if a.hf_checkpoint:
        from safetensors.torch import load_file

        model.load_hf_state_dict(load_file(a.hf_checkpoint))
    else:
        model.reset_parameters(0)
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    model = model.to("cuda", dt).eval()
    x = make_demo_input(cfg, device="cuda", dtype=dt, hw=demo_input_hw())
    stream = torch.cuda.Stream()
    tenant = GraphedTenant(model, stream, x)
    with torch.no_grad():
        tenant.capture()
    print(f"Starting Prometheus server on port {a.port}...", flush=True)
    start_http_server(a.port)
    i = 0
    while a.iterations == 0 or i < a.iterations:
        t0 = time.perf_counter()
        tenant.launch()
        stream.synchronize()
        inference_time.observe(time.perf_counter() - t0)
        i += 1
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
