"""One pod server with N YOLOS-small fp32 tenants in this process, driven by
client threads over its Unix socket for a fixed window: the pod-server fleet
in a single process, for ``rocprofv3 --kernel-trace --stats`` (the bench runs
the server as its own process, under the clean pod launcher).

  python tools/podserver_once.py --tenants 28 --lanes 16 --window 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


_CACHE: dict = {}


def make(kind: str, dtype: str, seed: int):
    """(program, weights) of one tenant kind."""
    from nos_amd.models.yolos_program import demo_tenant

    if kind == "yolos":
        return demo_tenant(dtype, seed)
    if kind == "bert":  # BERT-base trunk: 12 x (768 hidden, 12 heads, 3072 MLP) at seq 512
        from nos_amd.models.encoder_program import encoder_program, random_encoder_weights

        return encoder_program(random_encoder_weights(12, 768, 3072, seed), 12, 12, (1, 512, 768), "fp32")
    if kind == "mlp":
        from nos_amd.podserver.program import mlp_program

        return mlp_program(dim=4096, layers=4, batch=256, dtype="bf16", seed=seed)
    if kind == "resnet":  # ResNet-18 at 224x224 (torch.fx export), one program shared by the pods
        if "resnet" not in _CACHE:
            from nos_amd.models.resnet import resnet_tenant

            _CACHE["resnet"] = resnet_tenant(dtype, 0)
        return _CACHE["resnet"]
    if kind == "llama-var":  # the decoder registered at seq 512 / 256 / 128 (shape variants, one weight payload)
        if "llama-var" not in _CACHE:
            from nos_amd.models.llama_program import llama_config, llama_model, llama_program

            m = llama_model(llama_config(True), 0)
            progs = [llama_program(m, s_, rope_len=512, dtype=dtype) for s_ in (512, 256, 128)]
            _CACHE["llama-var"] = (progs[0][0], progs[0][1], [p for p, _ in progs[1:]])
        return _CACHE["llama-var"]
    if kind == "llama-dec":  # that decoder as a STATEFUL generation tenant: 128-token prompts, 1024-row K / V caches
        if "llama-dec" not in _CACHE:
            from nos_amd.models.llama_program import llama_config, llama_decode_programs, llama_model

            progs, w = llama_decode_programs(llama_model(llama_config(True), 0), 128, 1024, dtype=dtype)
            _CACHE["llama-dec"] = (progs[0], w, progs[1:])
        return _CACHE["llama-dec"]
    if kind == "llama-ft":  # the same decoder as a TRAINING tenant (next-token cross entropy, AdamW)
        return make("llama", "fp32", seed)
    if kind == "llama":  # a random-init Llama decoder (1024 hidden, 8 layers, head_dim 128, GQA) at seq 512
        if "llama" not in _CACHE:
            from nos_amd.models.llama_program import llama_tenant

            _CACHE["llama"] = llama_tenant(dtype, 0)
        return _CACHE["llama"]
    raise SystemExit(f"unknown tenant kind {kind!r}")


def _lat_summary(lat, kinds, w0: float, w1: float) -> dict | None:
    """Per-token round trips of the decode tenants inside the window."""
    xs = sorted(d for i, ls in enumerate(lat) if kinds[i] == "llama-dec" for t, d in ls if w0 <= t < w1)
    if not xs:
        return None
    q = lambda f: round(1e3 * xs[min(len(xs) - 1, int(f * len(xs)))], 3)  # noqa: E731
    return {"tokens": len(xs), "mean": round(1e3 * sum(xs) / len(xs), 3), "p50": q(0.5), "p90": q(0.9), "p99": q(0.99)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tenants", type=int, default=28)
    ap.add_argument("--lanes", type=int, default=16)
    ap.add_argument("--priority-lanes", type=int, default=0, help="high-priority lanes for the decode tenants")
    ap.add_argument("--latency-cus", type=int, default=0, help="CUs reserved for the priority lanes (multiple of 8)")
    ap.add_argument("--masked-queues", type=int, default=8, help="CU-masked streams the throughput lanes share "
                    "(with --latency-cus)")
    ap.add_argument("--hw-queues", type=int, default=0, help="GPU_MAX_HW_QUEUES (0: lanes + priority lanes)")
    ap.add_argument("--gen-chunk", type=int, default=1, help="llama-dec: tokens per request (> 1: the server's "
                    "generate loop, ids fed back on the device; per-token latency = request time / tokens)")
    ap.add_argument("--window", type=float, default=8.0)
    ap.add_argument("--warmup", type=float, default=2.0)
    ap.add_argument("--slice-gb", type=float, default=10.0)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--pipeline", type=int, default=1, help="x6 GEMM software-pipelined K loop (1) or plain (0)")
    ap.add_argument("--h3-layout", default=None, choices=["4x1", "2x2", "256x128", "4x1r3", "4x1k16", "2x2k16", "2x2r3", "2x2n64"],
                    help="h3 GEMM tile / wave layout / ring (NOS_AMD_H3_LAYOUT: the server's kernel config)")
    ap.add_argument("--h3-hot-ring", default=None, choices=["2", "3"],
                    help="LDS ring of the residual / row-statistics h3 GEMMs (NOS_AMD_H3_HOT_RING)")
    ap.add_argument("--h3-hot-bn", default=None, choices=["64", "128"],
                    help="tile width of the LN hand-off h3 GEMMs (NOS_AMD_H3_HOT_BN)")
    ap.add_argument("--h3-lna-wide", default=None, choices=["on", "off"],
                    help="fc1-class LN-GEMMs on 128 x 256 tiles, 8 waves (NOS_AMD_H3_LNA_WIDE)")
    ap.add_argument("--h3-attn-waves", type=int, default=8, choices=[4, 8], help="h3 attention waves per workgroup")
    ap.add_argument("--lds-epi", type=int, default=None, help="plain fp32-C h3 GEMMs store C through LDS (1) or "
                    "from the MFMA registers (0) (NOS_AMD_H3_EPILOGUE: the server's kernel config)")
    ap.add_argument("--mix", default="", help="heterogeneous tenants instead of --tenants YOLOS pods, e.g. "
                    "yolos:20,bert:4,mlp:4 (bert = BERT-base-shaped fp32 encoder at seq 512, mlp = bf16 GEMM-MLP "
                    "probe, resnet = ResNet-18 at 224x224, llama = Llama decoder at seq 512, llama-ft = that decoder "
                    "fine-tuned in the server: a training tenant, its rate in optimisation steps/s; llama-var = that "
                    "decoder registered at seq 512 / 256 / 128, requests cycling through the three shapes; llama-dec = "
                    "that decoder generating token by token over its K / V cache: prefill 128, decode to 1024); per-kind "
                    "rates in the output")
    a = ap.parse_args()
    kinds = ([k for spec in a.mix.split(",") for k in [spec.split(":")[0]] * int(spec.split(":")[1])]
             if a.mix else ["yolos"] * a.tenants)
    a.tenants = len(kinds)
    # one hardware queue per lane: before anything initialises HIP (cmd/podserver.py)
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(a.hw_queues or (a.lanes + a.priority_lanes), 32))
    # kernel-config A/B knobs go through the server's config (env), which it re-applies around every
    # capture -- a process-wide setter called after start() would be undone by the first registration
    if a.h3_layout is not None:
        os.environ["NOS_AMD_H3_LAYOUT"] = a.h3_layout
    if a.h3_hot_ring is not None:
        os.environ["NOS_AMD_H3_HOT_RING"] = a.h3_hot_ring
    if a.h3_lna_wide is not None:
        os.environ["NOS_AMD_H3_LNA_WIDE"] = a.h3_lna_wide
    if a.h3_hot_bn is not None:
        os.environ["NOS_AMD_H3_HOT_BN"] = a.h3_hot_bn
    if a.lds_epi is not None:
        os.environ["NOS_AMD_H3_EPILOGUE"] = "lds" if a.lds_epi else "reg"
    from nos_amd.models.yolos_program import demo_tenant
    from nos_amd.podserver.client import PodClient
    from nos_amd.podserver.server import PodServer

    path = Path(tempfile.mkdtemp(prefix="nos_ps_", dir="/tmp")) / "gpu-0" / "server.sock"
    srv = PodServer(path, device="cuda", lanes=a.lanes, priority_lanes=a.priority_lanes, latency_cus=a.latency_cus,
                    masked_queues=a.masked_queues, max_tenants=max(48, a.tenants)).start()
    from nos_amd import ops

    ops.set_gemm_f32x6_pipeline(bool(a.pipeline))  # process-wide: every capture below
    ops.set_attention_f32h3_waves(a.h3_attn_waves)
    try:
        t0 = time.monotonic()
        clients = [PodClient(path, connect_timeout_s=30) for _ in range(a.tenants)]
        progs = [make(k, a.dtype, i) for i, k in enumerate(kinds)]
        t_built = time.monotonic()
        train = {"loss": "cross_entropy", "optimizer": "adamw", "lr": 1e-4}
        reps = [c.register(f"pod-{i}", *progs[i][:2], memory_limit_gb=a.slice_gb,
                           train=train if kinds[i].endswith("-ft") else None,
                           variants=progs[i][2] if len(progs[i]) > 2 else None) for i, c in enumerate(clients)]
        batches = {}
        for i, k in enumerate(kinds):
            if k.endswith("-ft"):
                import numpy as np

                shp = reps[i]["input_shape"]
                ids = np.random.default_rng(i).integers(0, 32000, (shp[0], shp[1] + 1)).astype(np.int32)
                batches[i] = (ids[:, :-1], ids[:, 1:])
        shapes = {}
        for i, r in enumerate(reps):
            if len(r.get("input_shapes", [])) > 1:
                import numpy as np

                g = np.random.default_rng(i)
                shapes[i] = [g.integers(0, 32000, tuple(sh)).astype(np.int32) for sh in r["input_shapes"]]
        build_s = time.monotonic() - t_built
        srv_build_ms = sorted(r["compile"].get("build_ms", 0) for r in reps)
        stop = threading.Event()
        marks: list[list[float]] = [[] for _ in clients]

        lat: list[list[float]] = [[] for _ in clients]   # decode tenants: per-token round trips

        def loop(i: int) -> None:
            k = 0
            if kinds[i] == "llama-dec":   # generation: a prompt, then one token per request until the cache fills
                import numpy as np

                g = np.random.default_rng(i)
                while not stop.is_set():
                    outs, _ = clients[i].infer(g.integers(0, 32000, (1, 128)).astype(np.int32), outputs=[1])
                    tok = outs[0].reshape(1, 1).astype(np.int32)
                    marks[i].append(time.monotonic())
                    left = 1024 - 128 - 1
                    while left > 0 and not stop.is_set():
                        n = min(a.gen_chunk, left)
                        t0 = time.monotonic()
                        if n > 1:   # the server's decode loop: one request, n tokens
                            rep, data = clients[i]._call({"op": "generate", "steps": n, "output": 1, "shape": [1, 1],
                                                          "dtype": "i32"}, tok.tobytes())
                            from nos_amd.podserver import protocol as P

                            tok = P.unpack_arrays(rep["outputs"], data)[0].reshape(-1)[-1:].reshape(1, 1).astype(np.int32)
                        else:
                            outs, _ = clients[i].infer(tok, outputs=[1])
                            tok = outs[0].reshape(1, 1).astype(np.int32)
                        t1 = time.monotonic()
                        left -= n
                        for _ in range(n):
                            marks[i].append(t1)
                            lat[i].append((t0, (t1 - t0) / n))
                return
            while not stop.is_set():
                if i in batches:
                    clients[i].train_step(*batches[i])
                elif i in shapes:
                    clients[i].infer(shapes[i][k % len(shapes[i])])
                    k += 1
                else:
                    clients[i].infer()
                marks[i].append(time.monotonic())

        th = [threading.Thread(target=loop, args=(i,), daemon=True) for i in range(a.tenants)]
        for t in th:
            t.start()
        time.sleep(a.warmup)
        w0 = time.monotonic()
        clocks = []
        try:
            from nos_amd.gpu.amdsmi import AmdSmi

            smi = AmdSmi.real()
            while time.monotonic() - w0 < a.window:
                clocks.append(smi.clock(0)["sclk_mhz"])
                time.sleep(0.1)
        except Exception:  # no amd-smi: just wait
            time.sleep(max(0.0, a.window - (time.monotonic() - w0)))
        w1 = time.monotonic()
        sclk = round(sum(clocks) / len(clocks)) if clocks else None
        stop.set()
        for t in th:
            t.join(timeout=30)
        done = [sum(1 for m in mk if w0 <= m < w1) for mk in marks]
        solo = sum(t.solo_completed for t in srv.tenants.values())
        for c in clients:
            c.close()
        print(json.dumps({"tenants": a.tenants, "lanes": a.lanes, "window_s": round(w1 - w0, 3),
                          "build_s": round(build_s, 1), "programs_s": round(t_built - t0, 1),
                          "decode_token_latency_ms": _lat_summary(lat, kinds, w0, w1),
                          "per_kind": {k: {"tenants": kinds.count(k),
                                           "inf_per_s": round(sum(d for d, kk in zip(done, kinds) if kk == k)
                                                              / (w1 - w0), 2),
                                           "program": next(r["program"] for r, kk in zip(reps, kinds) if kk == k),
                                           "footprint_gb": max(r["footprint_gb"] for r, kk in zip(reps, kinds)
                                                               if kk == k)}
                                       for k in sorted(set(kinds))},
                          "server_build_ms_p50": srv_build_ms[len(srv_build_ms) // 2],
                          "server_compile_ms_p50": sorted(r["compile"].get("compile_ms", 0) for r in reps)[len(reps) // 2],
                          "inf_per_s": round(sum(done) / (w1 - w0), 2),
                          "min_done": min(done), "max_done": max(done), "solo_replays": solo,
                          "kernel_config": srv.kernel_config, "pipeline": a.pipeline, "h3_layout": a.h3_layout, "lds_epi": a.lds_epi,
                          "sclk_mhz": sclk}), flush=True)
    finally:
        srv.stop()


if __name__ == "__main__":
    main()
