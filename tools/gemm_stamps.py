"""Per-workgroup time breakdown of the register-epilogue GEMM from in-kernel
s_memtime stamps (diagnostic build: tools/variants/gemm_stamps.py).

NOS_AMD_HIP_LIB=build/variants/stamps/libnos_hip.so python tools/gemm_stamps.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nos_amd import ops  # noqa: E402
from nos_amd.ops import _lib  # noqa: E402


def read(nwg: int) -> np.ndarray:
    buf = (ctypes.c_uint64 * (nwg * 8))()
    rc = _lib.lib().nos_dbg_read(buf, nwg * 8)
    assert rc == 0, rc
    return np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 8).astype(np.float64)


def analyse(d: np.ndarray) -> dict:
    t0, t1, t2, t3, t4, r0, r4, xcc = d.T
    clk = np.median((t4 - t0) / np.maximum(r4 - r0, 1)) * 100.0  # MHz (memrealtime = 100 MHz)
    us = 1.0 / clk  # us per cycle
    # entry/exit relative to the earliest entry, via the 100 MHz realtime (global across CUs)
    start = (r0 - r0.min()) / 100.0
    end = (r4 - r0.min()) / 100.0

    def q(x):
        return {"p10": round(float(np.percentile(x, 10)), 2), "p50": round(float(np.median(x)), 2),
                "p90": round(float(np.percentile(x, 90)), 2), "max": round(float(x.max()), 2)}

    return {"clock_mhz": round(float(clk), 0), "workgroups": int(len(d)),
            "prologue_us": q((t1 - t0) * us), "kloop_us": q((t2 - t1) * us), "ln_stats_us": q((t3 - t2) * us),
            "epilogue_us": q((t4 - t3) * us), "wg_total_us": q((t4 - t0) * us),
            "wg_start_us": q(start), "wg_end_us": q(end), "span_us": round(float(end.max()), 2),
            "xcc_histogram": np.bincount(xcc.astype(int), minlength=8).tolist()}


def main() -> int:
    assert "stamps" in os.environ.get("NOS_AMD_HIP_LIB", ""), "run with the stamps variant"
    lib = _lib.lib()
    lib.nos_dbg_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    torch.manual_seed(0)
    S, hid, mlp = 3401, 384, 1536
    out = {}
    for B in (1, 8):
        M = B * S
        for name, (N, K, ln, act, resid) in {"qkv_ln": (3 * hid, hid, True, None, False),
                                             "fc1_ln_gelu": (mlp, hid, True, "gelu", False),
                                             "proj_resid": (hid, hid, False, None, True),
                                             "fc2_resid": (hid, mlp, False, None, True)}.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
            b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
            r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            if ln:
                g = torch.randn(K, device="cuda", dtype=torch.bfloat16)
                be = torch.randn(K, device="cuda", dtype=torch.bfloat16)
                wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
                fn = lambda: ops.linear_ln(x, wg, c1, c2, act=act, out=y)  # noqa: E731
            else:
                fn = lambda: ops.linear(x, w, b, act=act, residual=r if resid else None, out=y)  # noqa: E731
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            nwg = ((M + 127) // 128) * ((N + 127) // 128)
            out[f"{name}_b{B}"] = analyse(read(min(nwg, 4096)))
            print(name, B, json.dumps(out[f"{name}_b{B}"]), flush=True)
    if len(sys.argv) > 1:
        Path(sys.argv[1]).write_text(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
