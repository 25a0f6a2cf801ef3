"""What one CU-mask slice delivers: the gpuagent's probes (MFMA peak, HBM
stream, tiled GEMM) on the first slice of an n-way XCD-symmetric split, for
n = 1..32 -- the numbers the gpuagent publishes as node annotations.

python tools/slice_probe.py --out gpurun_out/slice_probe.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from nos_amd.gpu.topology import split_even  # noqa: E402
from nos_amd.ops import probes  # noqa: E402
from nos_amd.ops.streams import CUMaskedStream, device_info  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/slice_probe.json")
    ap.add_argument("--splits", default="1,2,4,8,16,32")
    a = ap.parse_args()
    info = device_info(0)
    res = {"device": info, "slices": []}
    for n in map(int, a.splits.split(",")):
        cus = split_even(n)[0].cus()
        s = CUMaskedStream(cus, info["num_cus"])
        try:
            pl = probes.placement_summary(probes.placement(s.handle, nwg=len(cus) * 8))
            tf = probes.mfma_peak_tflops(s.handle, nwg=len(cus) * 4, iters=20000)
            gb = probes.hbm_gbps(s.handle, bytes_=1 << 30, iters=5, nwg=len(cus) * 8)
            gemm = probes.gemm_tflops(s.handle, n=4096, iters=5, max_wg=len(cus) * 2)
        finally:
            s.close()
        r = {"slices_per_gpu": n, "cus": len(cus), "distinct_cus_seen": pl["distinct_cus"],
             "xccs_seen": len(pl["xccs"]), "mfma_peak_tflops": round(tf, 1), "hbm_gbps": round(gb, 1),
             "gemm4096_tflops": round(gemm, 1)}
        print(json.dumps(r), flush=True)
        res["slices"].append(r)
        Path(a.out).write_text(json.dumps(res, indent=1))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
