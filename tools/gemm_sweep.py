"""GEMM time vs K and vs grid size (fixed cost vs per-k-tile cost).

python tools/gemm_sweep.py --out gpurun_out/gemm_sweep.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from nos_amd import ops  # noqa: E402


sys.path.insert(0, str(Path(__file__).resolve().parent))
from kernel_bench import timeit  # noqa: E402  (HIP-graph timing: no host launch overhead)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/gemm_sweep.json")
    a = ap.parse_args()
    res = []
    for M, N, K in [(128, 128, 64), (128, 128, 384), (3401, 128, 384), (3401, 1152, 64), (3401, 1152, 128),
                    (3401, 1152, 384), (3401, 1152, 768), (3401, 1152, 1536), (3401, 1152, 3072),
                    (6802, 1152, 384), (3401, 2304, 384), (8192, 8192, 8192)]:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        us = timeit(lambda: ops.linear(x, w, None, out=out), 20 if K == 8192 else 100)
        tus = timeit(lambda: torch.matmul(x, w.t()), 20 if K == 8192 else 100)
        r = {"M": M, "N": N, "K": K, "wg": ((M + 127) // 128) * ((N + 127) // 128), "us": round(us, 2),
             "tflops": round(2 * M * N * K / us / 1e6, 1), "torch_us": round(tus, 2)}
        print(json.dumps(r), flush=True)
        res.append(r)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
