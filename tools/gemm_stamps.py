"""Per-phase cycle split of the x6 fp32 GEMM from an s_memtime-stamped build
(python tools/build_variant.py stamps tools/patches/gemm_f32x_stamps.py, loaded via
NOS_AMD_HIP_LIB; stamps go to a device array of their own, never to outputs).

NOS_AMD_HIP_LIB=build/variants/stamps/libnos_hip.so python tools/gemm_stamps.py --batch 1
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--policy", default="small")
    a = ap.parse_args()
    import torch

    from nos_amd import ops
    from nos_amd.ops import _lib

    L = _lib.lib()
    fn = L.nos_gemm_f32x6_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    fn.restype = ctypes.c_int
    buf = (ctypes.c_ulonglong * 8)()
    ops.set_f32_math("x6")
    ops.set_gemm_f32_policy(a.policy)
    S, hid, mlp = 3401, 384, 1536
    M = a.batch * S
    out = {}
    for name, (N, K, ln) in {"qkv_ln": (3 * hid, hid, True), "proj": (hid, hid, False),
                             "fc1_ln": (mlp, hid, True), "fc2": (hid, mlp, False)}.items():
        x = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda") * 0.05
        b = torch.randn(N, device="cuda")
        if ln:
            wg, c1, c2 = ops.fold_layernorm(w, b, torch.randn(K, device="cuda"), torch.randn(K, device="cuda"))
            f = lambda: ops.linear_ln(x, wg, c1, c2)  # noqa: E731
        else:
            f = lambda: ops.linear(x, w, b)  # noqa: E731
        f()
        torch.cuda.synchronize()
        fn(buf, 1)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(5):
            f()
        en.record()
        torch.cuda.synchronize()
        fn(buf, 1)
        waves = buf[5] or 1
        tot = sum(buf[i] for i in range(5)) or 1
        out[name] = {"us": round(st.elapsed_time(en) / 5 * 1e3, 1), "waves": waves,
                     "cycles_per_wave": round(tot / waves),
                     "split_pct": {k: round(100.0 * buf[i] / tot, 1) for i, k in
                                   enumerate(("prologue", "wait_barrier", "dma_issue", "compute", "epilogue"))}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
