"""Python side of the gpuagent probe kernels (csrc/hip/probes.hip)."""
from __future__ import annotations

import ctypes
from collections import Counter
from dataclasses import dataclass

import torch

from . import _lib


@dataclass
class Placement:
    xcc: int
    se: int
    sh: int
    cu: int
    block: int

    @property
    def cu_key(self) -> tuple[int, int, int, int]:
        return (self.xcc, self.se, self.sh, self.cu)


def decode_hw_id(hw_id: int) -> tuple[int, int, int]:
    """gfx9 HW_REG_HW_ID: CU_ID[11:8], SH_ID[12], SE_ID[15:13] -> (se, sh, cu)."""
    return (hw_id >> 13) & 0x7, (hw_id >> 12) & 0x1, (hw_id >> 8) & 0xF


def placement(stream: int | None = None, nwg: int = 2048, spin_ticks: int = 2000) -> list[Placement]:
    """Run probe_placement on `stream` (hipStream_t handle); returns one record per WG."""
    buf = torch.zeros((nwg, 4), dtype=torch.int32, device="cuda")
    s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.lib().nos_probe_placement(buf.data_ptr(), nwg, spin_ticks, s), "probe_placement")
    torch.cuda.synchronize()
    out = []
    for xcc, hw, blk, _t in buf.cpu().tolist():
        se, sh, cu = decode_hw_id(hw & 0xFFFFFFFF)
        out.append(Placement(xcc & 0xF, se, sh, cu, blk))
    return out


def placement_summary(recs: list[Placement]) -> dict:
    cus = {r.cu_key for r in recs}
    per_xcc = Counter(r.xcc for r in recs)
    cus_per_xcc = Counter(k[0] for k in cus)
    return {"distinct_cus": len(cus), "xccs": sorted(per_xcc), "wg_per_xcc": dict(sorted(per_xcc.items())),
            "cus_per_xcc": dict(sorted(cus_per_xcc.items()))}


def hbm_gbps(stream: int, bytes_: int = 1 << 30, iters: int = 5, nwg: int = 2048) -> float:
    v = ctypes.c_double()
    _lib.check(_lib.lib().nos_probe_hbm(stream, bytes_, iters, nwg, ctypes.byref(v)), "probe_hbm")
    return v.value


HBM_MODES = {"copy": 0, "copy_nt": 1, "read": 2}


def hbm_mode_gbps(stream: int, mode: str = "copy_nt", bytes_: int = 1 << 30, iters: int = 5, nwg: int = 2048) -> float:
    v = ctypes.c_double()
    _lib.check(_lib.lib().nos_probe_hbm_mode(stream, bytes_, iters, nwg, HBM_MODES[mode], ctypes.byref(v)),
               "probe_hbm_mode")
    return v.value


def mfma_peak_tflops(stream: int, nwg: int, iters: int = 20000) -> float:
    v = ctypes.c_double()
    _lib.check(_lib.lib().nos_probe_mfma_peak(stream, nwg, iters, ctypes.byref(v)), "probe_mfma_peak")
    return v.value


def gemm_tflops(stream: int, n: int = 4096, iters: int = 5, max_wg: int = 0) -> float:
    v = ctypes.c_double()
    _lib.check(_lib.lib().nos_probe_gemm(stream, n, iters, max_wg, ctypes.byref(v)), "probe_gemm")
    return v.value
