"""Each gpuagent probe kernel once on the whole GPU (for rocprofv3 --pmc passes).

rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES ... --output-format csv -d gpurun_out/pmc1 -- \
    python tools/probe_kernels_once.py
"""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    import torch

    from nos_amd.ops import probes

    s = torch.cuda.current_stream().cuda_stream
    print("mfma_peak_tflops", probes.mfma_peak_tflops(s, nwg=1024, iters=4000))
    print("gemm_tflops", probes.gemm_tflops(s, n=4096, iters=2))
    print("hbm_read_gbps", probes.hbm_mode_gbps(s, "read", 1 << 30, 2, 8192))
    print("hbm_copy_gbps", probes.hbm_mode_gbps(s, "copy", 1 << 30, 2, 512))


if __name__ == "__main__":
    main()
