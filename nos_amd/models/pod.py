"""One fractional-GPU tenant pod as its own process (the demo's client container).

The reference's demo pod (``demos/gpu-sharing-comparison/client/main.py:14-25``)
loads YOLOS-small in fp32 and runs inferences back to back forever; the
"average inference time" of the published table is taken over the last
2 minutes of that loop (``README.md:53-60``).  This is the MI355X pod:

* it runs with exactly the environment the nos-amd device plugin allocated
  (``HIP_VISIBLE_DEVICES``, ``ROC_GLOBAL_CU_MASK`` for CU-mask slices,
  ``NOS_AMD_MEMORY_LIMIT_GB``, see ``deviceplugin/plugin.py:allocate``) -- the
  parent does not touch the mask, HIP applies it to every queue of the pod;
* the memory cap is enforced through the caching allocator
  (:func:`nos_amd.utils.memlimit.apply_memory_limit`);
* every inference is one HIP-graph replay of the whole forward followed by a
  stream synchronize, and its completion time (CLOCK_MONOTONIC, comparable
  across processes) is recorded, so the orchestrator
  (:mod:`nos_amd.podbench`) can integrate exact fractional progress over any
  wall-clock window.

Precision: ``fp32`` (default, the reference's HF default precision) runs
exact fp32: the gfx950 fp32-MFMA GEMMs with fused epilogues
(``csrc/hip/gemm_f32.hip``) and flash attention
(``csrc/hip/attention_f32.hip``) of ``libnos_hip.so``; ``bf16`` runs the bf16
gfx950 kernels (fused-epilogue GEMMs, bf16 flash attention, LayerNorm).

Status protocol (``--status``: a float64 memory-mapped file, see
:class:`StatusBoard`): row 0 = [stop flag, ...]; row 1+slot = [state, count,
last completion time, pid].  On stop the pod writes all completion times to
``<out>/pod-<slot>.json`` and exits 0.  A pod whose launcher is gone (the
orchestrator was killed) exits too: the kernel sends it SIGTERM
(``PR_SET_PDEATHSIG``) and the loop checks its parent, so no orphan keeps
running kernels on the GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path
from typing import Callable

import numpy as np

STATE_STARTING, STATE_READY, STATE_FAILED, STATE_DONE = 0.0, 1.0, 2.0, 3.0
_COLS = 4


class StatusBoard:
    """Shared float64 table in a file (mmap), one writer per row."""

    def __init__(self, path: str | os.PathLike, pods: int | None = None):
        self.path = Path(path)
        if pods is not None:
            np.zeros((1 + pods, _COLS), dtype=np.float64).tofile(self.path)
        self.arr = np.memmap(self.path, dtype=np.float64, mode="r+")
        self.arr = self.arr.reshape(-1, _COLS)

    @property
    def pods(self) -> int:
        return self.arr.shape[0] - 1

    def stop(self) -> None:
        self.arr[0, 0] = 1.0
        self.arr.flush()

    def stopped(self) -> bool:
        return bool(self.arr[0, 0])

    def row(self, slot: int) -> np.ndarray:
        return self.arr[1 + slot]

    def states(self) -> list[float]:
        return [float(self.arr[1 + i, 0]) for i in range(self.pods)]

    def counts(self) -> list[float]:
        return [float(self.arr[1 + i, 1]) for i in range(self.pods)]


def _build(dtype: str, seed: int, hw, device: str = "cuda"):
    import torch

    from .yolos import YolosConfig, YolosDetector, make_demo_input

    cfg = YolosConfig.small() if device == "cuda" else YolosConfig.test()
    if dtype == "fp32":  # exact fp32: the gfx950 fp32-MFMA GEMMs and attention
        if device == "cuda":
            from ..ops import _lib

            _lib.require_native_on_gpu()
        m = YolosDetector(cfg, backend="native" if device == "cuda" else "torch")
        tdt = torch.float32
    elif dtype == "bf16":
        from ..ops import _lib

        _lib.require_native_on_gpu()
        m = YolosDetector(cfg, backend="native")
        tdt = torch.bfloat16
    else:
        raise ValueError(f"dtype {dtype!r}")
    m.reset_parameters(seed)
    m = m.to(device, tdt).eval()
    x = make_demo_input(cfg, device=device, dtype=tdt, hw=hw if device == "cuda" else cfg.image_size, seed=seed)
    return m, x


def _die_with_parent() -> Callable[[], bool]:
    """SIGTERM this process when its parent exits (Linux prctl), and return a
    check for the case the signal cannot cover (parent gone before prctl)."""
    ppid0 = os.getppid()
    try:
        import ctypes
        import signal

        ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGTERM), 0, 0, 0)  # PR_SET_PDEATHSIG
    except Exception:  # not Linux / no libc symbol: the getppid check below still works
        pass
    return lambda: os.getppid() != ppid0


def kernel_config(memory_fraction: float | None, env: dict | None = None, cu_budget: int = 0) -> dict[str, str]:
    """Kernel configs a pod picks from its slice (and ``NOS_AMD_*`` overrides
    for A/B runs).

    A pod owning the whole GPU wants the fewest rounds of tiles (bf16 GEMM
    latency policy: fc2 19.7 -> 14.2 us at batch 1) and two attention wave
    groups when its grid leaves CUs idle (the kernel's auto rule).  A
    fractional slice that SHARES the CUs with other pods wants small
    per-workgroup footprints: bf16 least-work tiles, fp32 GEMMs on 64x64
    tiles (33 KB LDS, <= 64 VGPRs; 8 pods: 318.0 / 318.1 vs 317.3 / 314.2
    inf/s, profiles/r02_f32_gemm_policy_fleet_ab.json) and fp32 attention with
    one wave group on 32-key tiles (317 vs 310 inf/s for 64-key tiles,
    profiles/r02_attention_f32_tilings.json).  A CU-mask slice (``cu_budget``
    CUs of its own, persistent grids) plans for its own CUs: budget-aware
    latency tiles and the auto attention rule, which picks the register-capped
    32-key tiling (4 waves per SIMD) -- 7 exclusive 32-CU pods 217.6 -> 231.0
    inf/s, solo 29.0 -> 27.2 ms (profiles/r03_cumask_kernel_configs.json).

    fp32 math: every pod runs the bf16x6 split kernels (fp32 operands as three
    exact bf16 pieces, six piece products on the bf16 matrix pipes; error vs
    fp64 <= the exact-f32 MFMA's, tests/test_kernels_gpu.py): attention
    (attention_f32x.hip) for every slice kind -- 8-pod fleet 318 -> 407 inf/s
    -- and the GEMMs (gemm_f32x.hip) -> 415 inf/s
    (profiles/r03_f32x6_fleet_ab.json).  A whole-GPU pod splits the keys
    when its grid leaves CU slots empty (``x6``: batch-1 attention 164 -> 133
    us); fractional pods never split (``x6n``: the co-tenants fill the slots,
    8 pods 410 vs 399 inf/s with the split) and run the x6 GEMMs on 128x128
    tiles with 4 x 1 waves (466 vs 448 for 128x64 and 425 for 64x64 tiles).  Since then the
    default is the fp16x3 split (``h3``: two fp16 pieces per operand on
    power-of-two scales, three fp16 MFMAs per product, errors vs fp64 at or
    below the exact-f32 kernels'): 28-tenant fleet 482 (x6) -> 640 inf/s
    (profiles/r04_h3_fleet_ab.json); ``h3`` splits keys for a whole-GPU pod,
    ``h3n`` never.  ``NOS_AMD_F32_MATH=x6|exact`` /
    ``NOS_AMD_ATTN_F32_VARIANT=x6|<tiling>`` select the bf16x6 or exact-f32
    MFMA kernels."""
    env = os.environ if env is None else env
    whole = memory_fraction is None or memory_fraction >= 0.99
    if cu_budget and not whole:
        gf = "latency"
    else:
        gf = "latency" if whole else "small"
    return {"gemm_bf16": env.get("NOS_AMD_GEMM_POLICY") or ("latency" if whole else "throughput"),
            "gemm_f32": env.get("NOS_AMD_GEMM_F32_POLICY") or gf,
            "attention_f32": env.get("NOS_AMD_ATTN_F32_VARIANT") or ("h3" if whole else "h3n"),
            "f32_math": env.get("NOS_AMD_F32_MATH") or "h3",
            "gemm_f32x6_tile": env.get("NOS_AMD_X6_TILE") or ("policy" if whole else "128x128"),
            # LayerNorm hand-off (ops.set_ln_handoff): residual GEMMs write row
            # statistics, LN-GEMMs normalise in their A load -- no split pass;
            # 28-tenant fleet 799 (on) vs 784 (off) inf/s (profiles/r05_lna_fleet_ab.json)
            "ln_handoff": env.get("NOS_AMD_LN_HANDOFF") or "on",
            # plain fp32-C h3 GEMMs store C through LDS (float4 rows): 801 vs 799 inf/s
            "h3_epilogue": env.get("NOS_AMD_H3_EPILOGUE") or "lds",
            # h3 GEMM tile layout (ops.set_gemm_f32h3_layout; the LN hand-off GEMMs keep 2x2)
            "h3_layout": env.get("NOS_AMD_H3_LAYOUT") or "2x2",
            # LDS ring of the residual (row-statistics) h3 GEMMs: "2" or "3" stages
            "h3_hot_ring": env.get("NOS_AMD_H3_HOT_RING") or "2",
            # tile width of the residual (row-statistics) h3 GEMMs: 128 x 128 (two workgroups per CU);
            # 128 x 64 (48 KiB, three) measured 2 % slower with the LN hand-off (profiles/r06_hot_bn_ab.json)
            "h3_hot_bn": env.get("NOS_AMD_H3_HOT_BN") or "128",
            # fc1-class LN-GEMMs (plane outputs) on 128 x 256 tiles, 8 waves
            "h3_lna_wide": env.get("NOS_AMD_H3_LNA_WIDE") or "off"}


def slice_cu_budget(env: dict | None = None) -> int:
    """CUs of the pod's CU-mask slice (popcount of ``ROC_GLOBAL_CU_MASK``), 0
    for an unmasked pod.  ``NOS_AMD_CU_BUDGET`` overrides it (A/B runs: "0"
    keeps one workgroup per tile on a masked slice)."""
    env = os.environ if env is None else env
    if env.get("NOS_AMD_CU_BUDGET") is not None:
        return int(env["NOS_AMD_CU_BUDGET"])
    m = env.get("ROC_GLOBAL_CU_MASK")
    if not m:
        return 0
    try:
        return bin(int(m, 16)).count("1")
    except ValueError:
        return 0


class _ServerTenant:
    """A pod on a pod-server slice: its inferences run in the GPU's pod server
    (nos_amd/podserver); this process never opens the GPU."""

    def __init__(self, client):
        self.client = client

    def launch(self) -> None:
        self.client.infer()

    def synchronize(self) -> None:  # infer() returns when the server's replay has finished
        pass


class _CpuTenant:
    def __init__(self, model, x):
        self.model, self.x = model, x

    def launch(self) -> None:
        self.model(self.x)

    def synchronize(self) -> None:
        pass


def run_pod(status: str, slot: int, out: str, dtype: str = "fp32", graphs: bool = True, seed: int = 0,
            warmup: int = 3, device: str = "cuda") -> int:
    """``device="cpu"`` runs the tiny test config on the CPU (protocol tests)."""
    orphaned = _die_with_parent()
    board = StatusBoard(status)
    row = board.row(slot)
    row[3] = os.getpid()
    client = None
    try:
        from ..api import constants as C

        if os.environ.get(C.ENV_POD_SERVER):
            # pod-server slice: ship the model to the server as a program (op
            # graph + weights, built with numpy: this process never imports
            # torch or opens the GPU), then infer through it
            from ..podserver.client import PodClient

            prefix = os.environ.get("NOS_AMD_POD_PROGRAM")
            if prefix:  # a prebuilt program (a conv net, a decoder LLM, ...): save_program's files
                from ..podserver.program import load_program

                program, weights = load_program(prefix)
            else:
                from .yolos_program import demo_tenant

                program, weights = demo_tenant(dtype, seed, small=device == "cuda")
            client = PodClient.from_env(reconnect_s=float(os.environ.get("NOS_AMD_POD_RECONNECT_S", "0")))
            rep = client.register(os.environ.get("NOS_AMD_POD_NAME") or f"pod-{slot}", program, weights)
            s = t = _ServerTenant(client)
            for _ in range(warmup):
                t.launch()
            srv = rep.get("server") or {}
            info = {"slot": slot, "pid": os.getpid(), "dtype": dtype, "graphs": graphs, "memory_fraction": None,
                    "program": rep.get("program"),
                    "device": srv.get("device"), "multiprocessor_count": srv.get("multiprocessor_count"),
                    "cu_mask": os.environ.get(C.ENV_POD_CU_MASK), "cu_budget": 0,
                    "kernel_config": srv.get("kernel_config"), "hip_visible_devices": None,
                    "memory_limit_gb": os.environ.get(C.ENV_MEMORY_LIMIT_GB),
                    "max_allocated_gb": rep.get("footprint_gb"), "pod_server": os.environ[C.ENV_POD_SERVER],
                    "server_lanes": srv.get("lanes"), "server_tenant": rep.get("tenant")}
            return _loop(board, row, slot, out, t, s, info, orphaned, gpu=False)
        import torch

        from ..utils.memlimit import apply_memory_limit
        from .yolos import GraphedTenant, demo_input_hw

        gpu = device == "cuda"
        frac = None
        if gpu:
            torch.cuda.set_device(0)  # the device plugin's HIP_VISIBLE_DEVICES leaves exactly the slice's GPU
            frac = apply_memory_limit(0)
            torch.backends.cuda.matmul.allow_tf32 = False  # true fp32 GEMMs (no reduced-precision shortcut)
            from ..ops import (set_attention_f32_variant, set_cu_budget, set_f32_math, set_gemm_f32_policy,
                               set_gemm_f32h3_hot_bn, set_gemm_f32h3_hot_ring, set_gemm_f32h3_layout,
                               set_gemm_f32h3_lna_wide, set_gemm_f32x6_tile, set_gemm_policy, set_ln_handoff)

            budget = slice_cu_budget(os.environ)
            cfg = kernel_config(frac, os.environ, budget)
            set_gemm_policy(cfg["gemm_bf16"])
            set_gemm_f32_policy(cfg["gemm_f32"])
            set_attention_f32_variant(cfg["attention_f32"])
            set_f32_math(cfg["f32_math"])
            set_gemm_f32x6_tile(cfg["gemm_f32x6_tile"])
            set_ln_handoff(cfg["ln_handoff"] == "on")
            set_gemm_f32h3_layout(cfg["h3_layout"])
            set_gemm_f32h3_hot_ring(int(cfg["h3_hot_ring"]))
            set_gemm_f32h3_hot_bn(int(cfg["h3_hot_bn"]))
            set_gemm_f32h3_lna_wide(cfg["h3_lna_wide"] == "on")
            if budget:  # CU-mask slice: slice-sized persistent grids (ops.set_cu_budget)
                set_cu_budget(budget)
        m, x = _build(dtype, seed, demo_input_hw(), device)
        if gpu:
            s = torch.cuda.Stream()
            t = GraphedTenant(m, s, x)
        else:
            s = t = _CpuTenant(m, x)
        with torch.no_grad():
            if graphs and gpu:
                t.capture()
            for _ in range(warmup):
                t.launch()
            s.synchronize()
        props = torch.cuda.get_device_properties(0) if gpu else None
        info = {"slot": slot, "pid": os.getpid(), "dtype": dtype, "graphs": graphs and gpu, "memory_fraction": frac,
                "device": props.name if gpu else "cpu",
                "multiprocessor_count": props.multi_processor_count if gpu else 0,
                "cu_mask": os.environ.get("ROC_GLOBAL_CU_MASK"),
                "cu_budget": slice_cu_budget(os.environ) if gpu else 0,
                "kernel_config": cfg if gpu else None,
                "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES"),
                "memory_limit_gb": os.environ.get("NOS_AMD_MEMORY_LIMIT_GB"),
                "max_allocated_gb": None}
        torch.set_grad_enabled(False)  # inference only (eager CPU tenants; graphs were captured without grad)
        return _loop(board, row, slot, out, t, s, info, orphaned, gpu)
    except Exception as e:  # the orchestrator sees the failure in the board and in the file
        Path(out, f"pod-{slot}.json").write_text(json.dumps({"slot": slot, "error": repr(e)}))
        row[0] = STATE_FAILED
        print(f"[pod {slot}] failed: {e!r}", file=sys.stderr, flush=True)
        return 1
    finally:
        if client is not None:
            client.close()


def _loop(board: StatusBoard, row, slot: int, out: str, t, s, info: dict, orphaned, gpu: bool) -> int:
    """Back-to-back inferences until the board says stop; completion times to
    ``<out>/pod-<slot>.json``."""
    row[0] = STATE_READY
    times: list[float] = []
    info["t_ready"] = time.monotonic()
    # bursty tenants (NOS_AMD_POD_DUTY="on_s:off_s"): infer for on_s, idle
    # for off_s, with a per-pod phase so the pods do not burst in step
    duty = os.environ.get("NOS_AMD_POD_DUTY")
    on_s, off_s = (float(v) for v in duty.split(":")) if duty else (0.0, 0.0)
    phase0 = time.monotonic() - (on_s + off_s) * ((slot * 0.618) % 1.0)
    while not board.stopped():
        if orphaned():
            print(f"[pod {slot}] launcher gone: exiting", file=sys.stderr, flush=True)
            return 1
        if off_s > 0 and (time.monotonic() - phase0) % (on_s + off_s) >= on_s:
            time.sleep(0.005)
            continue
        t.launch()
        s.synchronize()
        now = time.monotonic()
        times.append(now)
        row[1] = len(times)
        row[2] = now
    if gpu:
        import torch

        info["max_allocated_gb"] = round(torch.cuda.max_memory_allocated(0) / 2 ** 30, 3)
    info["times"] = times
    Path(out, f"pod-{slot}.json").write_text(json.dumps(info))
    row[0] = STATE_DONE
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="nos-amd fractional-GPU YOLOS pod")
    ap.add_argument("--status", required=True)
    ap.add_argument("--slot", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    a = ap.parse_args(argv)
    return run_pod(a.status, a.slot, a.out, a.dtype, not a.no_graphs, a.seed, device=a.device)


if __name__ == "__main__":
    sys.exit(main())
